# round 4: 32-bit pack indices -- train tests, C4 leg, C4 trace
set -o pipefail
mkdir -p gpurun_out/r4ee
timeout -k 10 600 python -u -m pytest -v --tb=short --timeout 200 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_optim.py > gpurun_out/r4ee/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --leg c4 --steps 6 > gpurun_out/r4ee/c4.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r4ee/prof -o c4 -- python3 bench.py --leg c4 --steps 6 > gpurun_out/r4ee/prof.log 2>&1 || exit $?
