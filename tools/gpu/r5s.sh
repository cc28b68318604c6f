# round 5: kernel-level stats of the unfrozen distillation leg
set -o pipefail
mkdir -p gpurun_out/r5s
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5s/prof -o du -- python3 bench.py --leg distill_unfrozen --steps 8 --warmup 2 > gpurun_out/r5s/du.log 2>&1 || exit $?
find gpurun_out/r5s -name "*kernel_trace.csv" -delete
