# round 5: DDP across progressive unfreezing; the unfrozen distillation leg; leg-order check (full bench both orders + each leg alone)
set -o pipefail
mkdir -p gpurun_out/r5e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ddp.py > gpurun_out/r5e/ddp_tests.txt 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --leg distill_unfrozen --steps 20 --warmup 3 > gpurun_out/r5e/distill_unfrozen.json 2> gpurun_out/r5e/distill_unfrozen.err || exit $?
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5e/bench_fwd.json 2> gpurun_out/r5e/bench_fwd.err || exit $?
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --order distill_unfrozen,distill,c4,c3,train,infer > gpurun_out/r5e/bench_rev.json 2> gpurun_out/r5e/bench_rev.err || exit $?
for leg in infer train c3 c4 distill; do
  timeout -k 10 300 python3 -u bench.py --leg $leg --steps 40 --warmup 5 > gpurun_out/r5e/alone_$leg.json 2> gpurun_out/r5e/alone_$leg.err || exit $?
done
