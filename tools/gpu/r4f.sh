set -o pipefail
run(){ t=$1; shift; timeout -k 10 $t "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
mkdir -p gpurun_out/r4f
run 200 python -u tools/poison_conv.py > gpurun_out/r4f/poison_conv.log 2>&1
run 200 python -u tools/nan_probe.py --preset b1 --calls 1 --fill --check-fwd > gpurun_out/r4f/b1_fill.log 2>&1
run 200 python -u tools/nan_probe.py --preset b7 --calls 2 --check-fwd > gpurun_out/r4f/b7_check.log 2>&1
