# round 5: distillation leg after other legs, caching-allocator blocks kept vs returned between legs
set -o pipefail
mkdir -p gpurun_out/r5v
cd $GRAFT_REPO_ROOT
export HISEG_BENCH_STEP_TIMES=1
HISEG_BENCH_EMPTY_CACHE=0 timeout -k 10 300 python3 -u tools/queue_probe.py run --train-first > gpurun_out/r5v/c4_keep.txt 2>&1 || exit $?
HISEG_BENCH_EMPTY_CACHE=1 timeout -k 10 300 python3 -u tools/queue_probe.py run --train-first > gpurun_out/r5v/c4_empty.txt 2>&1 || exit $?
HISEG_BENCH_EMPTY_CACHE=0 timeout -k 10 300 python3 -u tools/queue_probe.py run > gpurun_out/r5v/alone.txt 2>&1 || exit $?
