# round 5: the zero-pad LDS tile on k5 layers too (HISEG_DWCONV_ZP=2, one window row's reads live at a time) vs k3 only
set -o pipefail
mkdir -p gpurun_out/r5bo
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
HISEG_DWCONV_ZP=2 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "dwconv or dw_ or depthwise or mbconv" > gpurun_out/r5bo/tests.txt 2>&1 || exit $?
for v in 1 2 1 2; do echo "HISEG_DWCONV_ZP=$v" >> gpurun_out/r5bo/dw.txt; HISEG_DWCONV_ZP=$v timeout -k 10 200 python3 -u tools/dw_bench.py --modes 2 >> gpurun_out/r5bo/dw.txt 2>&1 || exit $?; done
for r in 1 2; do for v in 1 2; do
HISEG_DWCONV_ZP=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg infer > gpurun_out/r5bo/infer_${v}_$r.json 2> gpurun_out/r5bo/infer_${v}_$r.err || exit $?
HISEG_DWCONV_ZP=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg distill > gpurun_out/r5bo/distill_${v}_$r.json 2> gpurun_out/r5bo/distill_${v}_$r.err || exit $?
done; done
