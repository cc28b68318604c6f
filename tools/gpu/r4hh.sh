# distill slowdown in the full bench: leg alone (concurrent), full bench with a serial teacher
set -o pipefail
mkdir -p gpurun_out/r4hh
timeout -k 10 300 python -u bench.py --leg distill --steps 10 > gpurun_out/r4hh/leg_conc.log 2>&1 || exit $?
HISEG_SERIAL_TEACHER=1 timeout -k 10 900 python -u bench.py > gpurun_out/r4hh/bench_serial.log 2>&1 || exit $?
