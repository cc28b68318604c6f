# concurrent teacher: high-priority stream first, cached memory
set -o pipefail
mkdir -p gpurun_out/r4kk
timeout -k 10 200 python -u tools/stream_probe.py 0 --hiprio-first >> gpurun_out/r4kk/probe.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/stream_probe.py 4 --hiprio-first >> gpurun_out/r4kk/probe.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/stream_probe.py 0 --mem >> gpurun_out/r4kk/probe.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-presets --steps 6 > gpurun_out/r4kk/bench_nopresets.log 2>&1 || exit $?
