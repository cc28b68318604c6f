# round-4 GPU session e: bisect the bf16 NaN gradients (round-3 tree vs HEAD), B1 at several batch sizes
set -o pipefail
run(){ t=$1; shift; timeout -k 10 $t "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
mkdir -p gpurun_out/r4e
run 200 python -u _r3/tools/nan_probe.py --preset b1 --dtype bf16 > gpurun_out/r4e/r3_b1.log 2>&1
run 200 python -u _r3/tools/nan_probe.py --preset b7 --dtype bf16 > gpurun_out/r4e/r3_b7.log 2>&1
run 200 python -u tools/nan_probe.py --preset b1 --dtype bf16 --n 8 > gpurun_out/r4e/b1_n8.log 2>&1
run 200 python -u tools/nan_probe.py --preset b1 --dtype bf16 --n 32 --hw 320,320 > gpurun_out/r4e/b1_n32.log 2>&1
