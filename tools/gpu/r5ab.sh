# round 5: distillation leg alone under role streams: touch / HIP graph-queue knobs
set -o pipefail
mkdir -p gpurun_out/r5ab
cd $GRAFT_REPO_ROOT
export HISEG_BENCH_STEP_TIMES=1
run() { tag=$1; shift; env "$@" timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --leg distill --steps 10 --warmup 3 > gpurun_out/r5ab/$tag.json 2> gpurun_out/r5ab/$tag.err; }
run base HISEG_X=0 || exit $?
run notouch HISEG_STREAM_TOUCH=0 || exit $?
run dyn DEBUG_HIP_DYNAMIC_QUEUES=1 || exit $?
run gq1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1 || exit $?
run gq2 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 || exit $?
run gq4 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 || exit $?
run serial HISEG_SERIAL_TEACHER=1 || exit $?
AMD_LOG_LEVEL=3 timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --leg distill --steps 2 --warmup 1 > /tmp/log3.txt 2>&1 || exit $?
grep -iE "parallel stream|hipGraph\]|queue" /tmp/log3.txt | sort | uniq -c | sort -rn | head -40 > gpurun_out/r5ab/log3_summary.txt
ls -la /tmp/log3.txt >> gpurun_out/r5ab/log3_summary.txt
for f in gpurun_out/r5ab/*.json; do echo "$f $(grep -o '"distill": {[^{]*"ms_per_step": [0-9.]*' $f | grep -o 'ms_per_step": [0-9.]*')"; done > gpurun_out/r5ab/summary.txt
