set -o pipefail
mkdir -p gpurun_out/r4n
timeout -k 10 900 python -u -m pytest -q --tb=short -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/r4n/full.log 2>&1
timeout -k 10 600 python -u bench.py > gpurun_out/r4n/bench.log 2>&1
