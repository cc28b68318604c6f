# round 5: distillation step as three graphs (teacher / student forwards side by side), A/B against one graph
set -o pipefail
mkdir -p gpurun_out/r5ba
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_distill.py -k "branch_graphs or concurrent" > gpurun_out/r5ba/tests.txt 2>&1 || exit $?
export HISEG_BENCH_STEP_TIMES=1
for rep in 1 2; do for v in 0 1; do
  HISEG_DISTILL_BRANCH_GRAPHS=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg distill --steps 10 > gpurun_out/r5ba/d_${v}_$rep.json 2> gpurun_out/r5ba/d_${v}_$rep.err || exit $?
  HISEG_DISTILL_BRANCH_GRAPHS=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg distill_unfrozen --steps 10 > gpurun_out/r5ba/u_${v}_$rep.json 2> gpurun_out/r5ba/u_${v}_$rep.err || exit $?
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r5ba_t -o t -- python3 bench.py --no-cpu-baseline --leg distill --steps 6 --warmup 2 > gpurun_out/r5ba/trace.json 2> gpurun_out/r5ba/trace.err || exit $?
T=$(find /tmp/r5ba_t -name "*kernel_trace.csv" | head -1)
python3 tools/step_timeline.py $T > gpurun_out/r5ba/timeline.txt 2>&1 || exit $?
