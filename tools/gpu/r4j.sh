set -o pipefail
run(){ t=$1; shift; timeout -k 10 $t "$@"; rc=$?; echo "step rc=$rc: $*"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
mkdir -p gpurun_out/r4j
run 200 python -u tools/host_bound.py --train b0 --graphed --steps 5 > gpurun_out/r4j/hb.log 2>&1
run 200 python -u tools/host_bound.py --train b0 --graphed --ddp --steps 5 > gpurun_out/r4j/hb_ddp.log 2>&1
HB_NO_COUNT_SYNC=1 run 200 python -u tools/host_bound.py --train b0 --graphed --ddp --steps 5 > gpurun_out/r4j/hb_ddp_nocount.log 2>&1
HB_BUCKET_MB=1000 HB_NO_COUNT_SYNC=1 run 200 python -u tools/host_bound.py --train b0 --graphed --ddp --steps 5 > gpurun_out/r4j/hb_ddp_onebucket.log 2>&1
