# round 5: PMC HBM bytes per kernel class per step for the train / C3 / C4 / distillation legs (current tree)
set -o pipefail
mkdir -p gpurun_out/r5at
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for leg in train c3 c4 distill; do
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d /tmp/r5at/f_$leg -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --leg $leg --steps 4 --warmup 1 --eager-train > gpurun_out/r5at/f_$leg.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d /tmp/r5at/w_$leg -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --leg $leg --steps 4 --warmup 1 --eager-train > gpurun_out/r5at/w_$leg.log 2>&1 || exit $?
  python3 tools/pmc_classes.py /tmp/r5at/f_$leg /tmp/r5at/w_$leg --json gpurun_out/r5at/traffic.json --leg $leg > gpurun_out/r5at/classes_$leg.txt 2>&1 || exit $?
  rm -rf /tmp/r5at/f_$leg /tmp/r5at/w_$leg
done
