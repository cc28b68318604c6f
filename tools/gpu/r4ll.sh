# concurrent teacher after the train leg / after the inference leg in one process
set -o pipefail
mkdir -p gpurun_out/r4ll
timeout -k 10 400 python -u tools/stream_probe.py 0 --train-first >> gpurun_out/r4ll/probe.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/stream_probe.py 0 --infer-first >> gpurun_out/r4ll/probe.log 2>&1 || exit $?
