# round 5: the teacher's 1x1 expansion layers on every applicable conv kernel
set -o pipefail
mkdir -p gpurun_out/r5ap
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u tools/conv_bench.py --variants 0,90,-1,1,2,4,6 --bitref 0 --shapes b7exp_48to288_1x1_160x160,b7exp_80to480_1x1_80x80,b7exp_160to960_1x1_40x40,b7exp_224to1344_1x1_40x40,b7exp_384to2304_1x1_20x20 --reps 20 --rounds 3 > gpurun_out/r5ap/res.txt 2>&1 || exit $?
