set -o pipefail
run(){ t=$1; shift; timeout -k 10 $t "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
mkdir -p gpurun_out/r4h
P="python -u -m pytest -v -s --tb=short --timeout 300 --timeout-method thread"
run 300 $P tests/test_gpu_c1_u4_f64.py > gpurun_out/r4h/c1u4.log 2>&1
run 700 python -u -m pytest -q --tb=short -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/r4h/full.log 2>&1
run 200 python -u tools/churn_control.py > gpurun_out/r4h/churn_control.log 2>&1
run 200 python -u tools/host_bound.py --train b0 --graphed --steps 10 > gpurun_out/r4h/host_bound.log 2>&1
run 200 python -u tools/host_bound.py --train b0 --graphed --ddp --steps 10 > gpurun_out/r4h/host_bound_ddp.log 2>&1
