# round 5: halo weight-gradient tile variants (setprio, stagger), alternating runs
set -o pipefail
mkdir -p gpurun_out/r5ak
cd $GRAFT_REPO_ROOT
for rep in 1 2; do for v in 0 1 2 3; do
  echo "var=$v rep=$rep" >> gpurun_out/r5ak/var.txt
  HISEG_WGRAD_HWC_VAR=$v timeout -k 10 120 python3 -u tools/wgrad_bench.py --shapes w256_3x3_64x48,w128_3x3_128x96 --reps 20 2>&1 | grep -v amdgpu.ids >> gpurun_out/r5ak/var.txt || exit $?
done; done
