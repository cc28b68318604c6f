# round 5: XCD-major block order for the LDS-tiled depthwise conv, tile-fastest (1) and channel-group-fastest (2) vs launched order (0)
set -o pipefail
mkdir -p gpurun_out/r5bg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "dwconv or dw_ or depthwise or mbconv" > gpurun_out/r5bg/tests.txt 2>&1 || exit $?
HISEG_DWCONV_XCD=2 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "dwconv or dw_ or depthwise or mbconv" > gpurun_out/r5bg/tests2.txt 2>&1 || exit $?
for v in 0 1 2 0 1 2; do echo "HISEG_DWCONV_XCD=$v" >> gpurun_out/r5bg/dw.txt; HISEG_DWCONV_XCD=$v timeout -k 10 200 python3 -u tools/dw_bench.py --modes 1 >> gpurun_out/r5bg/dw.txt 2>&1 || exit $?; done
for v in 0 1 2; do for c in FETCH_SIZE WRITE_SIZE; do
HISEG_DWCONV_XCD=$v timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/r5bg/${c}_$v -o pmc --output-format csv -- python3 tools/dw_bench.py --modes 1 --reps 3 > gpurun_out/r5bg/${c}_$v.log 2>&1 || exit $?
done
python3 tools/pmc_hbm.py gpurun_out/r5bg/FETCH_SIZE_$v gpurun_out/r5bg/WRITE_SIZE_$v --match dwconv_t > gpurun_out/r5bg/hbm_$v.txt || exit $?
done
