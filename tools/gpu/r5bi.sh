# round 5: depthwise block order in the full pipelines (C2 inference, distillation): HISEG_DWCONV_XCD 0 / 2, with the
# rocprofv3 kernel statistics of the inference leg for each
set -o pipefail
mkdir -p gpurun_out/r5bi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do for v in 0 2; do
HISEG_DWCONV_XCD=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg infer > gpurun_out/r5bi/infer_${v}_$r.json 2> gpurun_out/r5bi/infer_${v}_$r.err || exit $?
HISEG_DWCONV_XCD=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg distill > gpurun_out/r5bi/distill_${v}_$r.json 2> gpurun_out/r5bi/distill_${v}_$r.err || exit $?
done; done
for v in 0 2; do
HISEG_DWCONV_XCD=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5bi_$v -o s -- python3 bench.py --no-cpu-baseline --leg infer > gpurun_out/r5bi/prof_$v.json 2> gpurun_out/r5bi/prof_$v.err || exit $?
S=$(find /tmp/r5bi_$v -name "*kernel_stats.csv" | head -1); cp $S gpurun_out/r5bi/stats_$v.csv || exit $?
done
