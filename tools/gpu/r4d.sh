# round-4 GPU session d: NaN probe (C4 repeated calls) + f64 train-step test after the RoIAlign contraction fix
set -o pipefail
run(){ t=$1; shift; timeout -k 10 $t "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
mkdir -p gpurun_out/r4d
run 200 python -u tools/nan_probe.py --preset b7 --dtype bf16 > gpurun_out/r4d/nan_b7_bf16.log 2>&1
run 200 python -u tools/nan_probe.py --preset b7 --dtype f32 > gpurun_out/r4d/nan_b7_f32.log 2>&1
run 200 python -u tools/nan_probe.py --preset b0 --dtype bf16 > gpurun_out/r4d/nan_b0_bf16.log 2>&1
run 200 python -u tools/nan_probe.py --preset b1 --dtype bf16 > gpurun_out/r4d/nan_b1_bf16.log 2>&1
run 300 python -u -m pytest -v -s --tb=short --timeout 300 --timeout-method thread tests/test_gpu_c1_u4_f64.py tests/test_gpu_parity.py -k "f64 or c1 or roi" > gpurun_out/r4d/f64.log 2>&1
