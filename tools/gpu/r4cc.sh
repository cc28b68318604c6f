# round 4: 64/128 tiles for ragged wide Cout -- parity / train tests, C3 + C4 legs with top layers
set -o pipefail
mkdir -p gpurun_out/r4cc
timeout -k 10 600 python -u -m pytest -v --tb=short --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_train.py tests/test_gpu_pw_forms.py > gpurun_out/r4cc/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --leg c3 --steps 6 > gpurun_out/r4cc/c3.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --leg c4 --steps 6 > gpurun_out/r4cc/c4.log 2>&1 || exit $?
