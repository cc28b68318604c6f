# round 5: halo weight-gradient tile -- parity tests, timing against the transposed-read / wide tiles
set -o pipefail
mkdir -p gpurun_out/r5ae
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py -k "wgrad_hwc" > gpurun_out/r5ae/tests.txt 2>&1 || exit $?
for h in 1 0; do
  HISEG_WGRAD_HWC=$h timeout -k 10 200 python3 -u tools/wgrad_bench.py --shapes w256_3x3_64x48,w128_3x3_128x96,w128to256_3x3_64x48,w64_3x3_64x48,w128_3x3_64x48 > gpurun_out/r5ae/wgrad_hwc$h.txt 2>&1 || exit $?
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_kernel_paths.py -k "wgrad or paths or train_step or bf16" >> gpurun_out/r5ae/tests.txt 2>&1 || exit $?
