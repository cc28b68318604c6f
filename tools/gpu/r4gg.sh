# round 4 final: full GPU suite, smoke, default bench
set -o pipefail
mkdir -p gpurun_out/r4gg
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --tb=short --timeout 300 --timeout-method thread > gpurun_out/r4gg/gpu_suite.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4gg/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py > gpurun_out/r4gg/bench.log 2>&1 || exit $?
