# round 4: rocprofv3 kernel-trace --stats of the default bench command (profiles/r4_bench_kernel_stats.csv)
set -o pipefail
mkdir -p gpurun_out/r4z
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/r4z/prof -o bench --output-format csv -- python3 bench.py > gpurun_out/r4z/bench.log 2>&1 || exit $?
