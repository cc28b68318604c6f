# round 5: full bench in the default and the reversed leg order, legs released with the quiescence wait
set -o pipefail
mkdir -p gpurun_out/r5x
cd $GRAFT_REPO_ROOT
export HISEG_BENCH_STEP_TIMES=1
timeout -k 10 500 python3 -u bench.py > gpurun_out/r5x/default.json 2> gpurun_out/r5x/default.err || exit $?
timeout -k 10 500 python3 -u bench.py --no-cpu-baseline --order distill,c4,c3,train,infer > gpurun_out/r5x/reversed.json 2> gpurun_out/r5x/reversed.err || exit $?
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --order infer,distill > gpurun_out/r5x/infer_distill.json 2> gpurun_out/r5x/infer_distill.err || exit $?
