# round 5: per-queue timeline of one replayed distillation step (decoder-only and unfrozen)
set -o pipefail
mkdir -p gpurun_out/r5ay
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for leg in distill distill_unfrozen; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r5ay_$leg -o t -- python3 bench.py --no-cpu-baseline --leg $leg --steps 6 --warmup 2 > gpurun_out/r5ay/$leg.json 2> gpurun_out/r5ay/$leg.err || exit $?
  T=$(find /tmp/r5ay_$leg -name "*kernel_trace.csv" | head -1)
  python3 tools/step_timeline.py $T > gpurun_out/r5ay/timeline_$leg.txt 2>&1 || exit $?
done
