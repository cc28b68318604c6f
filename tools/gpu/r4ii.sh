# round 4: 3x3 split-K restricted to small-batch train calls; concurrent teacher in the full bench
set -o pipefail
mkdir -p gpurun_out/r4ii
timeout -k 10 600 python -u -m pytest tests -m gpu -v --tb=short --timeout 300 --timeout-method thread -k "parity or train or distill" > gpurun_out/r4ii/tests.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py > gpurun_out/r4ii/bench.log 2>&1 || exit $?
