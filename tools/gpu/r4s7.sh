# round 4 final tree: rocprofv3 kernel-trace --stats of the default bench command
set -o pipefail
mkdir -p gpurun_out/r4s7
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/r4s7/prof -o bench --output-format csv -- python3 bench.py > gpurun_out/r4s7/bench.log 2>&1 || exit $?
