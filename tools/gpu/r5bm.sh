# round 5 final tree: PMC HBM bytes per kernel class per step for the train / C3 / C4 legs (Dispatch_Id matching)
set -o pipefail
mkdir -p gpurun_out/r5bm /tmp/r5bm
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for leg in train c3 c4; do
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d /tmp/r5bm/f_$leg -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --leg $leg --steps 4 --warmup 1 --eager-train > gpurun_out/r5bm/f_$leg.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d /tmp/r5bm/w_$leg -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --leg $leg --steps 4 --warmup 1 --eager-train > gpurun_out/r5bm/w_$leg.log 2>&1 || exit $?
  python3 tools/pmc_classes.py /tmp/r5bm/f_$leg /tmp/r5bm/w_$leg --json gpurun_out/r5bm/traffic.json --leg $leg > gpurun_out/r5bm/classes_$leg.txt 2>&1 || exit $?
  rm -rf /tmp/r5bm/f_$leg /tmp/r5bm/w_$leg
done
