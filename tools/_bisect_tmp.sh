set -o pipefail
for i in 1 2 3; do
timeout -k 10 200 python -u -m pytest tests/test_gpu_train.py -q --timeout 120 --timeout-method thread -k "not recaptures and not side_stream and not fragment_order" > gpurun_out/bis3_$i.log 2>&1 || true
grep -E "passed|failed" gpurun_out/bis3_$i.log | tail -1
done
