# round 5: conv_hwc with the first round's workgroups in 4 start phases (DIAG 2198 / 4246, bit-identical timing forms)
set -o pipefail
mkdir -p gpurun_out/r5ax
cd $GRAFT_REPO_ROOT
HISEG_LIB=$PWD/human-instance-segmentation_amd/hiseg/libhiseg_diag.so timeout -k 10 300 python3 -u tools/conv_bench.py --variants 104,2198,4246 --bitref 104 --shapes res256_3x3_64x48,res128_3x3_128x96 --reps 10 --rounds 4 > gpurun_out/r5ax/res.txt 2>&1 || exit $?
