# round 5: adaptive wgrad reduce -- tests + timing
set -o pipefail
mkdir -p gpurun_out/r5ar
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train.py -k "wgrad or train_step" > gpurun_out/r5ar/tests.txt 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/wgrad_bench.py --shapes w256_3x3_64x48,w128_3x3_128x96,w128to256_3x3_64x48,w64_3x3_64x48,w128_3x3_64x48 > gpurun_out/r5ar/wgrad.txt 2>&1 || exit $?
