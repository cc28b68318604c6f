# round-4 GPU session b: export + DDP tests with tracebacks, then the full suite
set -o pipefail
run(){ t=$1; shift; timeout -k 10 $t "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
mkdir -p gpurun_out/r4b
P="python -u -m pytest -v --tb=short --timeout 300 --timeout-method thread"
run 300 $P tests/test_gpu_export.py > gpurun_out/r4b/export.log 2>&1
run 400 $P tests/test_gpu_ddp.py -k "world2" > gpurun_out/r4b/ddp2.log 2>&1
run 600 python -u -m pytest -q --tb=short -m gpu --timeout 200 --timeout-method thread tests --deselect tests/test_gpu_ddp.py > gpurun_out/r4b/full.log 2>&1
run 300 $P tests/test_gpu_ddp.py -k "graphed" > gpurun_out/r4b/ddp_graphed.log 2>&1
