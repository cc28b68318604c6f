# distillation step trace with the concurrent teacher (per-queue timelines)
set -o pipefail
mkdir -p gpurun_out/r4qq
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r4qq/prof -o d -- python3 bench.py --leg distill --steps 6 > gpurun_out/r4qq/prof.log 2>&1 || exit $?
