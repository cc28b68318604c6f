# round 5: distillation teacher pipelined one batch ahead (GraphedBranchStep handoff), parity + A/B
set -o pipefail
mkdir -p gpurun_out/r5bc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_distill.py -k "branch_graphs or concurrent or pipelined" > gpurun_out/r5bc/tests.txt 2>&1 || exit $?
export HISEG_BENCH_STEP_TIMES=1
for rep in 1 2; do for v in 0 1; do
  HISEG_DISTILL_PIPELINE=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg distill --steps 10 > gpurun_out/r5bc/d_${v}_$rep.json 2> gpurun_out/r5bc/d_${v}_$rep.err || exit $?
  HISEG_DISTILL_PIPELINE=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg distill_unfrozen --steps 10 > gpurun_out/r5bc/u_${v}_$rep.json 2> gpurun_out/r5bc/u_${v}_$rep.err || exit $?
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r5bc_t -o t -- python3 bench.py --no-cpu-baseline --leg distill --steps 6 --warmup 2 > gpurun_out/r5bc/trace.json 2> gpurun_out/r5bc/trace.err || exit $?
T=$(find /tmp/r5bc_t -name "*kernel_trace.csv" | head -1)
python3 tools/step_timeline.py $T > gpurun_out/r5bc/timeline.txt 2>&1 || exit $?
