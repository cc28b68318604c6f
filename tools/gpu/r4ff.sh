# round 4: split-K 3x3 small images -- full GPU suite, C4 leg
set -o pipefail
mkdir -p gpurun_out/r4ff
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=10 -v -k "parity or train or distill" --tb=short --timeout 300 --timeout-method thread > gpurun_out/r4ff/gpu_suite.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --leg c4 --steps 6 > gpurun_out/r4ff/c4.log 2>&1 || exit $?
