# round 5: bench with the halo weight-gradient tile (train legs), GPU train tests
set -o pipefail
mkdir -p gpurun_out/r5ag
cd $GRAFT_REPO_ROOT
export HISEG_BENCH_STEP_TIMES=1
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline --order train,c3,c4,distill_unfrozen > gpurun_out/r5ag/train.json 2> gpurun_out/r5ag/train.err || exit $?
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_distill.py tests/test_gpu_c1_u4_f64.py tests/test_gpu_ddp.py > gpurun_out/r5ag/tests.txt 2>&1 || exit $?
