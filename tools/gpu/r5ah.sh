# round 5: the graphed RCCL DDP test alone (abort in r5ag), with and without the halo weight-gradient tile
set -o pipefail
mkdir -p gpurun_out/r5ah
cd $GRAFT_REPO_ROOT
HISEG_WGRAD_HWC=0 NCCL_DEBUG=WARN AMD_LOG_LEVEL=1 timeout -k 10 300 python3 -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_ddp.py -k "rccl" > gpurun_out/r5ah/hwc0.txt 2>&1; echo "rc=$?" >> gpurun_out/r5ah/hwc0.txt
NCCL_DEBUG=WARN AMD_LOG_LEVEL=1 timeout -k 10 300 python3 -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_ddp.py -k "rccl" > gpurun_out/r5ah/hwc1.txt 2>&1; echo "rc=$?" >> gpurun_out/r5ah/hwc1.txt
