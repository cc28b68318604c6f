# round 5: hardware-queue mapping of the graphed distillation step alone vs after the C4 leg; C4 probe after warm-up
set -o pipefail
mkdir -p gpurun_out/r5c
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5c/alone -o t -- python3 tools/queue_probe.py run > gpurun_out/r5c/alone.txt 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5c/after -o t -- python3 tools/queue_probe.py run --train-first > gpurun_out/r5c/after.txt 2>&1 || exit $?
for f in $(find gpurun_out/r5c -name "*kernel_trace.csv"); do python3 tools/queue_probe.py parse $f --last 3500 > $f.summary.txt; rm -f $f; done
timeout -k 10 300 python3 -u bench.py --leg c4 --steps 10 --warmup 3 > gpurun_out/r5c/c4.json 2> gpurun_out/r5c/c4.err || exit $?
