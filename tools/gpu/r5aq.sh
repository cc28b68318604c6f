# round 5: wgrad reduce (16 split groups) tests + timing; the teacher's 1x1 expansions on every conv kernel
set -o pipefail
mkdir -p gpurun_out/r5aq
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train.py -k "wgrad or train_step or fused_bn or finalize" > gpurun_out/r5aq/tests.txt 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/wgrad_bench.py --shapes w256_3x3_64x48,w128_3x3_128x96,w128to256_3x3_64x48,w64_3x3_64x48,w128_3x3_64x48 > gpurun_out/r5aq/wgrad.txt 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/conv_bench.py --variants 0,90,-1,1,2,4,6 --bitref 0 --shapes b7exp_48to288_1x1_160x160,b7exp_80to480_1x1_80x80,b7exp_160to960_1x1_40x40,b7exp_224to1344_1x1_40x40,b7exp_384to2304_1x1_20x20 --reps 20 --rounds 3 > gpurun_out/r5aq/pw.txt 2>&1 || exit $?
