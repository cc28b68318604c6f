# round 5: BatchNorm element-wise passes and depthwise conv at the train / distillation shapes
set -o pipefail
mkdir -p gpurun_out/r5bd
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 -u tools/bn_bench.py > gpurun_out/r5bd/bn.txt 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/dw_bench.py > gpurun_out/r5bd/dw.txt 2>&1 || exit $?
