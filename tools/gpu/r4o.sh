# round 4: per-leg class profiles (new call_profile) and PMC HBM bytes per class per step
set -o pipefail
mkdir -p gpurun_out/r4o
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for leg in train c3 c4 distill; do
  timeout -k 10 300 python3 -u bench.py --leg $leg --steps 6 > gpurun_out/r4o/leg_$leg.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/r4o/pmcf_$leg -o pmc --output-format csv -- python3 bench.py --leg $leg --steps 4 --warmup 1 --eager-train > gpurun_out/r4o/pmcf_$leg.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/r4o/pmcw_$leg -o pmc --output-format csv -- python3 bench.py --leg $leg --steps 4 --warmup 1 --eager-train > gpurun_out/r4o/pmcw_$leg.log 2>&1 || exit $?
done
