# round 5: role streams -- stream-touching GPU tests, bench default / reversed order / legs alone; conv_hwc stagger
set -o pipefail
mkdir -p gpurun_out/r5aa
cd $GRAFT_REPO_ROOT
export HISEG_BENCH_STEP_TIMES=1
HISEG_LIB=$PWD/human-instance-segmentation_amd/hiseg/libhiseg_diag.so timeout -k 10 300 python3 -u tools/conv_bench.py --variants 104,214,278 --bitref 104 --shapes res256_3x3_64x48,res128_3x3_128x96 --reps 10 --rounds 4 > gpurun_out/r5aa/stagger.txt 2>&1 || exit $?
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_distill.py tests/test_gpu_ddp.py -k "concurrent or graph or ddp or pipelined" > gpurun_out/r5aa/tests.txt 2>&1 || exit $?
timeout -k 10 500 python3 -u bench.py > gpurun_out/r5aa/default.json 2> gpurun_out/r5aa/default.err || exit $?
timeout -k 10 500 python3 -u bench.py --no-cpu-baseline --order distill,c4,c3,train,infer > gpurun_out/r5aa/reversed.json 2> gpurun_out/r5aa/reversed.err || exit $?
for leg in distill infer; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --leg $leg > gpurun_out/r5aa/alone_$leg.json 2> gpurun_out/r5aa/alone_$leg.err || exit $?
done
