# round 5: kernel stats of the train and distillation legs (current tree)
set -o pipefail
mkdir -p gpurun_out/r5al
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5al/train -o t --output-format csv -- python3 bench.py --no-cpu-baseline --leg train --steps 8 --warmup 2 > gpurun_out/r5al/train.json 2> gpurun_out/r5al/train.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5al/distill -o t --output-format csv -- python3 bench.py --no-cpu-baseline --leg distill --steps 8 --warmup 2 > gpurun_out/r5al/distill.json 2> gpurun_out/r5al/distill.err || exit $?
for d in train distill; do f=$(find gpurun_out/r5al/$d -name "*kernel_stats.csv" | head -1); head -45 $f > gpurun_out/r5al/${d}_stats.csv; done
find gpurun_out/r5al -name "*kernel_trace.csv" -delete
