# round 5: which weight-gradient kernel takes every layer of each train leg (HISEG_LOG_WGRAD names the generic fallbacks)
set -o pipefail
mkdir -p gpurun_out/r5a
cd $GRAFT_REPO_ROOT
for leg in c4 train c3 distill; do
  HISEG_LOG_WGRAD=1 HISEG_LOG_PLACEMENT=1 timeout -k 10 300 python3 -u bench.py --leg $leg --steps 10 --warmup 3 > gpurun_out/r5a/$leg.json 2> gpurun_out/r5a/$leg.err || exit $?
done
