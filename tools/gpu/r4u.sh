# round 4: full GPU suite, default bench, rocprof summary of the bench
set -o pipefail
mkdir -p gpurun_out/r4u
timeout -k 10 200 python -u tools/gated_bench.py > gpurun_out/r4u/gated_bench0.log 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --tb=short --timeout 300 --timeout-method thread > gpurun_out/r4u/gpu_suite.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r4u/bench.log 2>&1 || exit $?
