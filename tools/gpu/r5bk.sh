# round 5: block order of the gather depthwise kernel (dwconv_q_kernel), HISEG_DWCONV_QXCD 0 / 1 / 2 -- parity,
# timing (dw_bench --modes 0: gather forced), HBM bytes
set -o pipefail
mkdir -p gpurun_out/r5bk
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 1 2; do HISEG_DWCONV_QXCD=$v timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "dwconv or dw_ or depthwise or mbconv" > gpurun_out/r5bk/tests_$v.txt 2>&1 || exit $?; done
for v in 0 1 2 0 1 2; do echo "HISEG_DWCONV_QXCD=$v" >> gpurun_out/r5bk/dw.txt; HISEG_DWCONV_QXCD=$v timeout -k 10 200 python3 -u tools/dw_bench.py --modes 0 >> gpurun_out/r5bk/dw.txt 2>&1 || exit $?; done
for v in 0 1 2; do for c in FETCH_SIZE WRITE_SIZE; do
HISEG_DWCONV_QXCD=$v timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/r5bk/${c}_$v -o pmc --output-format csv -- python3 tools/dw_bench.py --modes 0 --reps 3 > gpurun_out/r5bk/${c}_$v.log 2>&1 || exit $?
done
python3 tools/pmc_hbm.py gpurun_out/r5bk/FETCH_SIZE_$v gpurun_out/r5bk/WRITE_SIZE_$v --match dwconv_q > gpurun_out/r5bk/hbm_$v.txt || exit $?
rm -rf gpurun_out/r5bk/FETCH_SIZE_$v gpurun_out/r5bk/WRITE_SIZE_$v
done
