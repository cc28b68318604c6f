# round 5: BN statistics fused into conv_hwc's epilogue -- GPU suite, train legs (A/B vs HISEG_FUSED_BN_STATS=0)
set -o pipefail
mkdir -p gpurun_out/r5r
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_train.py -k "fused_bn" > gpurun_out/r5r/fused.txt 2>&1 || exit $?
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_c1_u4_f64.py tests/test_gpu_distill.py > gpurun_out/r5r/suite.txt 2>&1 || exit $?
for leg in train c3; do
  timeout -k 10 300 python3 -u bench.py --leg $leg --steps 20 --warmup 3 > gpurun_out/r5r/$leg.json 2> gpurun_out/r5r/$leg.err || exit $?
  HISEG_FUSED_BN_STATS=0 timeout -k 10 300 python3 -u bench.py --leg $leg --steps 20 --warmup 3 > gpurun_out/r5r/${leg}_nofuse.json 2> gpurun_out/r5r/${leg}_nofuse.err || exit $?
done
