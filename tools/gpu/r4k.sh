set -o pipefail
run(){ t=$1; shift; timeout -k 10 $t "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
mkdir -p gpurun_out/r4k
P="python -u -m pytest -v -s --tb=short --timeout 300 --timeout-method thread"
run 100 python -u tools/roi_probe.py > gpurun_out/r4k/roi_probe.log 2>&1
run 300 $P tests/test_gpu_c1_u4_f64.py > gpurun_out/r4k/c1u4.log 2>&1
run 300 $P tests/test_gpu_parity.py -k roi > gpurun_out/r4k/roi_tests.log 2>&1
