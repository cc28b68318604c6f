# round 5: shared side / aux streams (<= 4 normal-priority streams per process): tests, bench both orders, legs alone
set -o pipefail
mkdir -p gpurun_out/r5ac
cd $GRAFT_REPO_ROOT
export HISEG_BENCH_STEP_TIMES=1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_distill.py tests/test_gpu_ddp.py tests/test_gpu_train.py -k "concurrent or graph or ddp or pipelined or finalize_n or fused_bn" > gpurun_out/r5ac/tests.txt 2>&1 || exit $?
timeout -k 10 120 python3 -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_parity.py -k pipelined >> gpurun_out/r5ac/tests.txt 2>&1 || exit $?
timeout -k 10 500 python3 -u bench.py > gpurun_out/r5ac/default.json 2> gpurun_out/r5ac/default.err || exit $?
timeout -k 10 500 python3 -u bench.py --no-cpu-baseline --order distill_unfrozen,distill,c4,c3,train,infer > gpurun_out/r5ac/reversed.json 2> gpurun_out/r5ac/reversed.err || exit $?
for leg in distill distill_unfrozen infer train; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg $leg > gpurun_out/r5ac/alone_$leg.json 2> gpurun_out/r5ac/alone_$leg.err || exit $?
done
