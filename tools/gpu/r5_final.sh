# round 5 final: the default bench command; rocprofv3 kernel trace + stats of its inference leg's command
# (bench.py --leg infer, the child process that measures `value`) and the dominant-class average from that trace
set -o pipefail
mkdir -p gpurun_out/r5final
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u bench.py > gpurun_out/r5final/bench.json 2> gpurun_out/r5final/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5final_prof -o infer -- python3 bench.py --leg infer > gpurun_out/r5final/infer_under_rocprof.json 2> gpurun_out/r5final/infer_under_rocprof.err || exit $?
T=$(find /tmp/r5final_prof -name "*kernel_trace.csv" | head -1)
S=$(find /tmp/r5final_prof -name "*kernel_stats.csv" | head -1)
python3 tools/dominant_from_trace.py $T --last 90 > gpurun_out/r5final/dominant_kernel.json || exit $?
cp $S gpurun_out/r5final/infer_kernel_stats.csv
