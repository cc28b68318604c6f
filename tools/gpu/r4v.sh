# gated projections: split-count sweep (HISEG_SPLITK forces the split on every layer the plan applies to)
set -o pipefail
mkdir -p gpurun_out/r4v
for sp in 0 4 6 12 16 24; do
  echo "== HISEG_SPLITK=$sp" >> gpurun_out/r4v/sweep.log
  HISEG_SPLITK=$sp timeout -k 10 120 python -u tools/gated_bench.py >> gpurun_out/r4v/sweep.log 2>&1 || exit $?
done
