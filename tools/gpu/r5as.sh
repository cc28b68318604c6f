# round 5: halo weight-gradient tile on concat layers -- tests, train legs
set -o pipefail
mkdir -p gpurun_out/r5as
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_kernel_paths.py -k "wgrad or paths or train_step or placement or far" > gpurun_out/r5as/tests.txt 2>&1 || exit $?
export HISEG_BENCH_STEP_TIMES=1
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline --order train,c3,c4 > gpurun_out/r5as/train.json 2> gpurun_out/r5as/train.err || exit $?
