set -o pipefail
mkdir -p gpurun_out/r4l
timeout -k 10 200 python -u -m pytest -v --tb=short --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "hwt" > gpurun_out/r4l/hwt_test.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/conv_bench.py --variants 97,103 --shapes res256_3x3_64x48,res128_3x3_128x96,c128to256_3x3_64x48 --reps 20 --rounds 3 --bitref 97 > gpurun_out/r4l/bench.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest -q --tb=short --timeout 200 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_norm_act.py tests/test_gpu_distill.py tests/test_gpu_optim.py tests/test_gpu_churn.py > gpurun_out/r4l/train_tests.log 2>&1
timeout -k 10 300 python -u bench.py --distill-only > gpurun_out/r4l/distill.log 2>&1
