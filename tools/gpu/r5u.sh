# round 5: the default bench command, and its rocprofv3 kernel trace (dominant-class average from the trace)
set -o pipefail
mkdir -p gpurun_out/r5u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u bench.py > gpurun_out/r5u/bench.json 2> gpurun_out/r5u/bench.err || exit $?
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5u/prof -o bench -- python3 bench.py > gpurun_out/r5u/bench_under_rocprof.json 2> gpurun_out/r5u/bench_under_rocprof.err || exit $?
T=$(find gpurun_out/r5u/prof -name "*kernel_trace.csv" | head -1)
python3 tools/dominant_from_trace.py $T --last 90 > gpurun_out/r5u/dominant_kernel.json
rm -f $T
