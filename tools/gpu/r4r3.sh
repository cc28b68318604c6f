# conv_wgrad_tr_kernel incremental DMA offsets: bit-identity tests, then A/B timing on the ROI head's shapes
set -o pipefail
mkdir -p gpurun_out/r4r3
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_train.py -k "wgrad" > gpurun_out/r4r3/tests.txt 2>&1 || exit $?
for v in 1 0 1 0; do
  HISEG_WGRAD_INC=$v timeout -k 10 120 python3 -u tools/wgrad_bench.py --reps 10 >> gpurun_out/r4r3/bench.txt 2>&1 || exit $?
done
