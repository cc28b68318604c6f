# round 5: PMC HBM bytes per kernel class per step for the distillation legs (dispatches matched in Dispatch_Id order)
set -o pipefail
mkdir -p gpurun_out/r5bj /tmp/r5bj
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for leg in distill distill_unfrozen; do
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d /tmp/r5bj/f_$leg -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --leg $leg --steps 4 --warmup 1 --eager-train > gpurun_out/r5bj/f_$leg.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d /tmp/r5bj/w_$leg -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --leg $leg --steps 4 --warmup 1 --eager-train > gpurun_out/r5bj/w_$leg.log 2>&1 || exit $?
  python3 tools/pmc_classes.py /tmp/r5bj/f_$leg /tmp/r5bj/w_$leg --json gpurun_out/r5bj/traffic.json --leg $leg > gpurun_out/r5bj/classes_$leg.txt 2>&1 || exit $?
  rm -rf /tmp/r5bj/f_$leg /tmp/r5bj/w_$leg
done
