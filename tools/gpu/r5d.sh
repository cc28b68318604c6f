# round 5: leg-order sensitivity of the graphed distillation step / inference, no profiler
set -o pipefail
mkdir -p gpurun_out/r5d
cd $GRAFT_REPO_ROOT
export HISEG_BENCH_STEP_TIMES=1
timeout -k 10 200 python3 -u tools/queue_probe.py run --infer-after > gpurun_out/r5d/alone.txt 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/queue_probe.py run --b0-first > gpurun_out/r5d/b0first.txt 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/queue_probe.py run --infer-first --b0-first > gpurun_out/r5d/infer_b0_first.txt 2>&1 || exit $?
