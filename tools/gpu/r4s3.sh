# generic conv kernel: 1x1 gather through buffer offsets (HISEG_IGEMM_LIN) -- bit-identity tests, gated timing, legs
set -o pipefail
mkdir -p gpurun_out/r4s3
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "igemm_linear or splitk or gated or pw" > gpurun_out/r4s3/tests.txt 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/gated_bench.py > gpurun_out/r4s3/gated.txt 2>&1 || exit $?
for leg in distill c3 c4; do
  timeout -k 10 300 python3 -u bench.py --leg $leg --steps 20 --warmup 5 > gpurun_out/r4s3/$leg.txt 2>&1 || exit $?
  HISEG_IGEMM_LIN=0 timeout -k 10 300 python3 -u bench.py --leg $leg --steps 20 --warmup 5 > gpurun_out/r4s3/${leg}_nolin.txt 2>&1 || exit $?
done
