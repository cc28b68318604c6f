# round 5: stream -> hardware-queue overlap table; distillation step per teacher side stream
set -o pipefail
mkdir -p gpurun_out/r5z
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u tools/stream_map.py --distill 0,1,2,3,4,5 > gpurun_out/r5z/map.txt 2> gpurun_out/r5z/err.txt
