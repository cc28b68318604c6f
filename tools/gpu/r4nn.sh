# distill in the bench sequence with 8 hardware queues per process
set -o pipefail
mkdir -p gpurun_out/r4nn
GPU_MAX_HW_QUEUES=8 HISEG_BENCH_STEP_TIMES=1 timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-presets --steps 10 > gpurun_out/r4nn/bench8.log 2>&1 || exit $?
