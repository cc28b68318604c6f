# round 5: halo weight-gradient tile timing (one-round splits) + SQ counters of it and of the dominant conv (conv_hwc)
set -o pipefail
mkdir -p gpurun_out/r5af
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 -u tools/wgrad_bench.py --shapes w256_3x3_64x48,w128_3x3_128x96,w128to256_3x3_64x48,w64_3x3_64x48,w128_3x3_64x48 > gpurun_out/r5af/wgrad.txt 2>&1 || exit $?
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES"
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace -d gpurun_out/r5af/w1 -o p --output-format csv -- python3 tools/wgrad_bench.py --shapes w256_3x3_64x48 --reps 2 > gpurun_out/r5af/w1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-trace -d gpurun_out/r5af/w2 -o p --output-format csv -- python3 tools/wgrad_bench.py --shapes w256_3x3_64x48 --reps 2 > gpurun_out/r5af/w2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace -d gpurun_out/r5af/c1 -o p --output-format csv -- python3 tools/conv_bench.py --variants 104 --shapes res256_3x3_64x48 --reps 2 --rounds 1 > gpurun_out/r5af/c1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-trace -d gpurun_out/r5af/c2 -o p --output-format csv -- python3 tools/conv_bench.py --variants 104 --shapes res256_3x3_64x48 --reps 2 --rounds 1 > gpurun_out/r5af/c2.log 2>&1 || exit $?
for d in w1 w2 c1 c2; do f=$(find gpurun_out/r5af/$d -name "*counter_collection.csv" | head -1); python3 tools/pmc_kernels.py $f hiseg > gpurun_out/r5af/$d.summary.txt; done
