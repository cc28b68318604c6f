# ubf two-pixel loop: bit identity, train leg A/B, trace
set -o pipefail
mkdir -p gpurun_out/r4pp
timeout -k 10 400 python -u -m pytest -v --tb=short --timeout 200 --timeout-method thread tests/test_gpu_train.py -k "ubf or graphed or train_step" > gpurun_out/r4pp/tests.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r4pp/p1 -o t -- python3 bench.py --leg train --steps 6 > gpurun_out/r4pp/p1.log 2>&1 || exit $?
HISEG_UBF_U2=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r4pp/p0 -o t -- python3 bench.py --leg train --steps 6 > gpurun_out/r4pp/p0.log 2>&1 || exit $?
