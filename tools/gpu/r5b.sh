# round 5: far-apart two-source weight gradients on the transposed-read tile (no generic fallback)
set -o pipefail
mkdir -p gpurun_out/r5b
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernel_paths.py "tests/test_gpu_train.py::test_two_source_results_do_not_depend_on_operand_placement" > gpurun_out/r5b/tests.txt 2>&1 || exit $?
for leg in c4 train; do
  HISEG_LOG_WGRAD=1 timeout -k 10 300 python3 -u bench.py --leg $leg --steps 10 --warmup 3 > gpurun_out/r5b/$leg.json 2> gpurun_out/r5b/$leg.err || exit $?
done
