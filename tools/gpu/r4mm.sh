# distill in the bench sequence: per-replay times
set -o pipefail
mkdir -p gpurun_out/r4mm
HISEG_BENCH_STEP_TIMES=1 timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-presets --steps 10 > gpurun_out/r4mm/bench.log 2>&1 || exit $?
HISEG_BENCH_STEP_TIMES=1 timeout -k 10 300 python -u bench.py --leg distill --steps 10 > gpurun_out/r4mm/leg.log 2>&1 || exit $?
