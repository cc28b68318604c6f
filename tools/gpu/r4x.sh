# round 4: parallel wgrad reduce, B-prefetch default -- train tests, wgrad bench, train leg
set -o pipefail
mkdir -p gpurun_out/r4x
timeout -k 10 600 python -u -m pytest -v --tb=short --timeout 200 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_norm_act.py > gpurun_out/r4x/train_tests.log 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/wgrad_bench.py > gpurun_out/r4x/wgrad_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --leg train --steps 6 > gpurun_out/r4x/train.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --leg c3 --steps 6 > gpurun_out/r4x/c3.log 2>&1 || exit $?
