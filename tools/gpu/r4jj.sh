# concurrent teacher vs the number of streams in the process
set -o pipefail
mkdir -p gpurun_out/r4jj
for k in 0 3 7 11; do
  timeout -k 10 200 python -u tools/stream_probe.py $k >> gpurun_out/r4jj/probe.log 2>&1 || exit $?
done
timeout -k 10 200 python -u tools/stream_probe.py 11 --prio >> gpurun_out/r4jj/probe.log 2>&1 || exit $?
