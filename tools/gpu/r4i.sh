set -o pipefail
run(){ t=$1; shift; timeout -k 10 $t "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
mkdir -p gpurun_out/r4i
P="python -u -m pytest -v -s --tb=short --timeout 300 --timeout-method thread"
run 100 python -u tools/roi_probe.py > gpurun_out/r4i/roi_probe.log 2>&1
run 300 $P tests/test_gpu_churn.py > gpurun_out/r4i/churn.log 2>&1
run 400 python -u tools/churn_control.py > gpurun_out/r4i/churn_control.log 2>&1
run 200 python -u tools/host_bound.py --train b0 --graphed --ddp --steps 10 > gpurun_out/r4i/host_bound_ddp.log 2>&1
