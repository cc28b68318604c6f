# round 5: which branch of the distillation step is captured first / lands on the launch queue (A/B)
set -o pipefail
mkdir -p gpurun_out/r5az
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
HISEG_STUDENT_SIDE=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_distill.py -k "concurrent" > gpurun_out/r5az/tests.txt 2>&1 || exit $?
export HISEG_BENCH_STEP_TIMES=1
for rep in 1 2; do for v in 0 1; do
  HISEG_STUDENT_SIDE=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg distill --steps 10 > gpurun_out/r5az/d_${v}_$rep.json 2> gpurun_out/r5az/d_${v}_$rep.err || exit $?
  HISEG_STUDENT_SIDE=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg distill_unfrozen --steps 10 > gpurun_out/r5az/u_${v}_$rep.json 2> gpurun_out/r5az/u_${v}_$rep.err || exit $?
done; done
HISEG_STUDENT_SIDE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r5az_t -o t -- python3 bench.py --no-cpu-baseline --leg distill --steps 6 --warmup 2 > gpurun_out/r5az/trace.json 2> gpurun_out/r5az/trace.err || exit $?
T=$(find /tmp/r5az_t -name "*kernel_trace.csv" | head -1)
python3 tools/step_timeline.py $T > gpurun_out/r5az/timeline.txt 2>&1 || exit $?
