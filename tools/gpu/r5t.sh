# round 5: unfrozen-distillation small kernels (depthwise weight gradient splits, SE backward) -- tests, leg, kernel stats
set -o pipefail
mkdir -p gpurun_out/r5t
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_distill.py tests/test_gpu_kernel_paths.py tests/test_gpu_norm_act.py tests/test_gpu_parity.py tests/test_gpu_ddp.py > gpurun_out/r5t/tests.txt 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --leg distill_unfrozen --steps 20 --warmup 3 > gpurun_out/r5t/du.json 2> gpurun_out/r5t/du.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5t/prof -o du -- python3 bench.py --leg distill_unfrozen --steps 8 --warmup 2 > gpurun_out/r5t/du_prof.log 2>&1 || exit $?
find gpurun_out/r5t -name "*kernel_trace.csv" -delete
