set -o pipefail
mkdir -p gpurun_out/r4m
timeout -k 10 500 python -u -m pytest -q --tb=short --timeout 200 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_norm_act.py tests/test_gpu_distill.py tests/test_gpu_optim.py tests/test_gpu_churn.py > gpurun_out/r4m/train_tests.log 2>&1
timeout -k 10 300 python -u bench.py --distill-only > gpurun_out/r4m/distill.log 2>&1
