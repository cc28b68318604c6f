# round 5: conv_hwc halo DMA issue points (DIAG variants, bit-identical forms), alternating rounds
set -o pipefail
mkdir -p gpurun_out/r5ao
cd $GRAFT_REPO_ROOT
HISEG_LIB=$PWD/human-instance-segmentation_amd/hiseg/libhiseg_diag.so timeout -k 10 300 python3 -u tools/conv_bench.py --variants 104,662,1174,1686 --bitref 104 --shapes res256_3x3_64x48,res128_3x3_128x96,c256to256_3x3_64x48 --reps 10 --rounds 4 > gpurun_out/r5ao/res.txt 2>&1 || exit $?
