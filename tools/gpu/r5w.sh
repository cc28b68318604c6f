# round 5: which earlier leg slows the distillation leg in the full bench (cache kept between legs)
set -o pipefail
mkdir -p gpurun_out/r5w
cd $GRAFT_REPO_ROOT
export HISEG_BENCH_STEP_TIMES=1
for order in infer,distill train,distill train,c3,c4,distill; do
  HISEG_BENCH_EMPTY_CACHE=0 timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --steps 10 --warmup 3 --order $order > gpurun_out/r5w/$order.json 2> gpurun_out/r5w/$order.err || exit $?
done
HISEG_BENCH_EMPTY_CACHE=1 timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --steps 10 --warmup 3 --order train,c3,c4,distill > gpurun_out/r5w/empty_train,c3,c4,distill.json 2> gpurun_out/r5w/empty.err || exit $?
