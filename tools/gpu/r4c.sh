# round-4 GPU session c: DDP + C1/U4/f64 diagnostics
set -o pipefail
run(){ t=$1; shift; timeout -k 10 $t "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
mkdir -p gpurun_out/r4c
P="python -u -m pytest -v -s --tb=short --timeout 300 --timeout-method thread"
run 300 $P tests/test_gpu_c1_u4_f64.py > gpurun_out/r4c/c1u4.log 2>&1
run 400 $P tests/test_gpu_ddp.py -k "world2" > gpurun_out/r4c/ddp2.log 2>&1
run 300 $P tests/test_gpu_ddp.py -k "graphed" > gpurun_out/r4c/ddp_graphed.log 2>&1
