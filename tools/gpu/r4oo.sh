# full default bench with the distillation leg first
set -o pipefail
mkdir -p gpurun_out/r4oo
timeout -k 10 900 python -u bench.py > gpurun_out/r4oo/bench.log 2>&1 || exit $?
