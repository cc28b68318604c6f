# round 5: BatchNorm backward reduction in the data-gradient epilogue -- tests, train legs
set -o pipefail
mkdir -p gpurun_out/r5aw
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py -k "fused_bn or train_step or residual or bf16 or wgrad_hwc" > gpurun_out/r5aw/tests.txt 2>&1 || exit $?
export HISEG_BENCH_STEP_TIMES=1
for f in 1 0; do
  HISEG_FUSED_BN_BWD=$f timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg train > gpurun_out/r5aw/train_$f.json 2> gpurun_out/r5aw/train_$f.err || exit $?
done
HISEG_FUSED_BN_BWD=1 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg train > gpurun_out/r5aw/train_1b.json 2> gpurun_out/r5aw/train_1b.err || exit $?
