set -o pipefail
mkdir -p gpurun_out/r4p
timeout -k 10 300 python -u -m pytest -v --tb=short --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "se_two or dwconv or dw_ or norm_act or efficientnet or se_ or preset or bf16_logits" > gpurun_out/r4p/dw_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/dw_bench.py > gpurun_out/r4p/dw_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --leg distill --steps 10 > gpurun_out/r4p/distill_t.log 2>&1 || exit $?
