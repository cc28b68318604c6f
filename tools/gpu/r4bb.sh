# round 4: concurrent teacher stream -- test, distill leg A/B (serial vs concurrent), trace
set -o pipefail
mkdir -p gpurun_out/r4bb
timeout -k 10 400 python -u -m pytest -v --tb=short --timeout 200 --timeout-method thread tests/test_gpu_distill.py > gpurun_out/r4bb/tests.log 2>&1 || exit $?
HISEG_SERIAL_TEACHER=0 timeout -k 10 300 python -u bench.py --leg distill --steps 10 > gpurun_out/r4bb/distill_conc.log 2>&1 || exit $?
HISEG_SERIAL_TEACHER=1 timeout -k 10 300 python -u bench.py --leg distill --steps 10 > gpurun_out/r4bb/distill_serial.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
HISEG_SERIAL_TEACHER=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r4bb/prof -o distill -- python3 bench.py --leg distill --steps 6 > gpurun_out/r4bb/prof.log 2>&1 || exit $?
