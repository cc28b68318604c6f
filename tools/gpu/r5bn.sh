# round 5: LDS-tiled depthwise conv without per-tap bounds tests (k3 layers, packed FMAs): parity + timing A/B
set -o pipefail
mkdir -p gpurun_out/r5bn
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "dwconv or dw_ or depthwise or mbconv" > gpurun_out/r5bn/tests.txt 2>&1 || exit $?
for v in 0 1 0 1; do echo "HISEG_DWCONV_ZP=$v" >> gpurun_out/r5bn/dw.txt; HISEG_DWCONV_ZP=$v timeout -k 10 200 python3 -u tools/dw_bench.py --modes 2 >> gpurun_out/r5bn/dw.txt 2>&1 || exit $?; done
