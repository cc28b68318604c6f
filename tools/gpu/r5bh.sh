# round 5: LDS-tiled (XCD-major order) vs gather depthwise kernel per layer shape, to re-derive the selection rule
set -o pipefail
mkdir -p gpurun_out/r5bh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do timeout -k 10 200 python3 -u tools/dw_bench.py --modes 2,0,1 >> gpurun_out/r5bh/dw.txt 2>&1 || exit $?; done
