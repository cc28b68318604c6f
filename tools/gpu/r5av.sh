# round 5: distillation teacher branch on a high-priority stream (A/B, alternating, one process per run)
set -o pipefail
mkdir -p gpurun_out/r5av
cd $GRAFT_REPO_ROOT
export HISEG_BENCH_STEP_TIMES=1
for rep in 1 2; do for h in 0 1; do
  HISEG_TEACHER_HIGH=$h timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg distill --steps 10 > gpurun_out/r5av/d_${h}_$rep.json 2> gpurun_out/r5av/d_${h}_$rep.err || exit $?
  HISEG_TEACHER_HIGH=$h timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg distill_unfrozen --steps 10 > gpurun_out/r5av/u_${h}_$rep.json 2> gpurun_out/r5av/u_${h}_$rep.err || exit $?
done; done
