# round 5: conv_hwc on 64-Cout tiles (variant 107) -- bit-identity tests, timing vs conv_hwr 100, train leg
set -o pipefail
mkdir -p gpurun_out/r5au
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_train.py -k "hwc or fused_bn" > gpurun_out/r5au/tests.txt 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/conv_bench.py --variants 100,107 --bitref 100 --shapes res64_3x3_64x48,c256to64_3x3_64x48,dec2_up128+64to64_3x3_120x160 --reps 20 --rounds 4 > gpurun_out/r5au/bench.txt 2>&1 || exit $?
export HISEG_BENCH_STEP_TIMES=1
timeout -k 10 500 python3 -u bench.py --no-cpu-baseline --order train,c3 > gpurun_out/r5au/train.json 2> gpurun_out/r5au/train.err || exit $?
