# round 5: bench legs in child processes, both orders; wide vs transposed-read weight gradient on 128->256
set -o pipefail
mkdir -p gpurun_out/r5ad
cd $GRAFT_REPO_ROOT
export HISEG_BENCH_STEP_TIMES=1
for w in 1 0; do
  HISEG_WGRAD_WIDE=$w timeout -k 10 200 python3 -u tools/wgrad_bench.py --shapes w128to256_3x3_64x48,w256_3x3_64x48,w64_3x3_64x48 > gpurun_out/r5ad/wgrad_wide$w.txt 2>&1 || exit $?
done
timeout -k 10 600 python3 -u bench.py > gpurun_out/r5ad/default.json 2> gpurun_out/r5ad/default.err || exit $?
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline --order distill_unfrozen,distill,c4,c3,train,infer > gpurun_out/r5ad/reversed.json 2> gpurun_out/r5ad/reversed.err || exit $?
