set -o pipefail
run(){ t=$1; shift; timeout -k 10 $t "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
mkdir -p gpurun_out/r4g
P="python -u -m pytest -v -s --tb=short --timeout 300 --timeout-method thread"
run 300 $P tests/test_gpu_pw_forms.py > gpurun_out/r4g/pw_forms.log 2>&1
run 300 python -u tools/nan_probe.py --preset b1 --calls 2 --fill --check-fwd > gpurun_out/r4g/b1_fill.log 2>&1
run 300 python -u tools/nan_probe.py --preset b7 --calls 2 --fill --check-fwd > gpurun_out/r4g/b7_fill.log 2>&1
run 400 $P tests/test_gpu_parity.py -k "bf16_logits_error or preset" tests/test_gpu_c1_u4_f64.py > gpurun_out/r4g/parity.log 2>&1
run 400 $P tests/test_gpu_ddp.py -k "world2" > gpurun_out/r4g/ddp2.log 2>&1
run 300 $P tests/test_gpu_ddp.py -k graphed > gpurun_out/r4g/ddp_graphed.log 2>&1
