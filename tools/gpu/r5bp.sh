# round 5: the gather depthwise kernel without its per-tap column test (HISEG_DWCONV_QZP 0 / 1): parity, timing, pipelines
set -o pipefail
mkdir -p gpurun_out/r5bp
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_distill.py -k "dwconv or dw_ or depthwise or mbconv or student or teacher" > gpurun_out/r5bp/tests.txt 2>&1 || exit $?
for v in 0 1 0 1; do echo "HISEG_DWCONV_QZP=$v" >> gpurun_out/r5bp/dw.txt; HISEG_DWCONV_QZP=$v timeout -k 10 200 python3 -u tools/dw_bench.py --modes 0 >> gpurun_out/r5bp/dw.txt 2>&1 || exit $?; done
for r in 1 2; do for v in 0 1; do
HISEG_DWCONV_QZP=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg infer > gpurun_out/r5bp/infer_${v}_$r.json 2> gpurun_out/r5bp/infer_${v}_$r.err || exit $?
HISEG_DWCONV_QZP=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg distill > gpurun_out/r5bp/distill_${v}_$r.json 2> gpurun_out/r5bp/distill_${v}_$r.err || exit $?
done; done
