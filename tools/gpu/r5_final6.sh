# round 5 final (6): full GPU suite, then the default bench command and the rocprofv3 summary of its inference leg
set -o pipefail
mkdir -p gpurun_out/r5final6
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r5final6/suite.txt 2>&1 || exit $?
timeout -k 10 600 python3 -u bench.py > gpurun_out/r5final6/bench.json 2> gpurun_out/r5final6/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5final6_prof -o infer -- python3 bench.py --leg infer > gpurun_out/r5final6/infer_under_rocprof.json 2> gpurun_out/r5final6/infer_under_rocprof.err || exit $?
T=$(find /tmp/r5final6_prof -name "*kernel_trace.csv" | head -1)
S=$(find /tmp/r5final6_prof -name "*kernel_stats.csv" | head -1)
python3 tools/dominant_from_trace.py $T --last 90 > gpurun_out/r5final6/dominant_kernel.json || exit $?
cp $S gpurun_out/r5final6/infer_kernel_stats.csv
