# round 5: gather depthwise block order in the pipelines (HISEG_DWCONV_QXCD 0 / 2), then the distillation leg's PMC
# HBM bytes per kernel class on the final tree
set -o pipefail
mkdir -p gpurun_out/r5bl /tmp/r5bl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do for v in 0 2; do
HISEG_DWCONV_QXCD=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg infer > gpurun_out/r5bl/infer_${v}_$r.json 2> gpurun_out/r5bl/infer_${v}_$r.err || exit $?
HISEG_DWCONV_QXCD=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg distill > gpurun_out/r5bl/distill_${v}_$r.json 2> gpurun_out/r5bl/distill_${v}_$r.err || exit $?
HISEG_DWCONV_QXCD=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg c4 > gpurun_out/r5bl/c4_${v}_$r.json 2> gpurun_out/r5bl/c4_${v}_$r.err || exit $?
done; done
leg=distill
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d /tmp/r5bl/f_$leg -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --leg $leg --steps 4 --warmup 1 --eager-train > gpurun_out/r5bl/f_$leg.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d /tmp/r5bl/w_$leg -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --leg $leg --steps 4 --warmup 1 --eager-train > gpurun_out/r5bl/w_$leg.log 2>&1 || exit $?
python3 tools/pmc_classes.py /tmp/r5bl/f_$leg /tmp/r5bl/w_$leg --json gpurun_out/r5bl/traffic.json --leg $leg > gpurun_out/r5bl/classes_$leg.txt 2>&1 || exit $?
