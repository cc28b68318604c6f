# round 5: the r5ag sequence with -s (see the exception before the RCCL abort)
set -o pipefail
mkdir -p gpurun_out/r5ai
cd $GRAFT_REPO_ROOT
NCCL_DEBUG=WARN timeout -k 10 900 python3 -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_distill.py tests/test_gpu_c1_u4_f64.py tests/test_gpu_ddp.py > gpurun_out/r5ai/tests.txt 2>&1; echo "rc=$?" >> gpurun_out/r5ai/tests.txt
