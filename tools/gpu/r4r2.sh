# wide wgrad shared-tap DMA addressing: bit-identity tests, then A/B timing on the ROI head's shapes
set -o pipefail
mkdir -p gpurun_out/r4r2
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_train.py -k "wgrad_wide" > gpurun_out/r4r2/tests.txt 2>&1 || exit $?
for v in 2 1 0 2 1 0; do
  HISEG_WGRAD_SHT=$v timeout -k 10 120 python3 -u tools/wgrad_bench.py --reps 10 --shapes w256_3x3_64x48,w128_3x3_64x48 >> gpurun_out/r4r2/bench.txt 2>&1 || exit $?
done
