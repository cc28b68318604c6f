# round-4 GPU session a: full GPU suite (strict descriptor pointers), DDP tests, churn control, host-bound DDP
set -o pipefail
run(){ t=$1; shift; timeout -k 10 $t "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
mkdir -p gpurun_out/r4a
run 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_ddp.py tests/test_gpu_export.py > gpurun_out/r4a/ddp.log 2>&1
run 600 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests --deselect tests/test_gpu_ddp.py > gpurun_out/r4a/full.log 2>&1
run 200 python -u tools/churn_control.py > gpurun_out/r4a/churn_control.log 2>&1
run 200 python -u tools/host_bound.py --train b0 --graphed --ddp --steps 10 > gpurun_out/r4a/host_bound_ddp.log 2>&1
run 200 python -u tools/host_bound.py --train b0 --graphed --steps 10 > gpurun_out/r4a/host_bound.log 2>&1
