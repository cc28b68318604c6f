# generic conv kernel: tap-mask gather for k x k layers (HISEG_IGEMM_LIN=2 vs 1) -- bit-identity tests, legs
set -o pipefail
mkdir -p gpurun_out/r4s4
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "igemm_linear or splitk or conv3x3 or generic" > gpurun_out/r4s4/tests.txt 2>&1 || exit $?
for leg in c3 c4 train; do
  timeout -k 10 300 python3 -u bench.py --leg $leg --steps 20 --warmup 5 > gpurun_out/r4s4/$leg.txt 2>&1 || exit $?
  HISEG_IGEMM_LIN=1 timeout -k 10 300 python3 -u bench.py --leg $leg --steps 20 --warmup 5 > gpurun_out/r4s4/${leg}_lin1.txt 2>&1 || exit $?
done
