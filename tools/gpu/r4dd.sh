# round 4: tap-major wgrad reduce -- train tests, legs
set -o pipefail
mkdir -p gpurun_out/r4dd
timeout -k 10 600 python -u -m pytest -v --tb=short --timeout 200 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_distill.py > gpurun_out/r4dd/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --leg c4 --steps 6 > gpurun_out/r4dd/c4.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --leg train --steps 6 > gpurun_out/r4dd/train.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --leg c3 --steps 6 > gpurun_out/r4dd/c3.log 2>&1 || exit $?
