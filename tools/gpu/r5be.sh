# round 5: SQ counters of the LDS-tiled depthwise conv (k5 s1, the headline path's C2 shape and the B7 teacher's)
set -o pipefail
mkdir -p gpurun_out/r5be
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM"
P2="SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_SMEM"
for sh in c2_b0_s3_k5s1_c240 b7_s3_k5s1_c480; do
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace -d gpurun_out/r5be/${sh}_1 -o p --output-format csv -- python3 tools/dw_bench.py --shapes $sh --modes 1 --reps 3 > gpurun_out/r5be/${sh}_1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-trace -d gpurun_out/r5be/${sh}_2 -o p --output-format csv -- python3 tools/dw_bench.py --shapes $sh --modes 1 --reps 3 > gpurun_out/r5be/${sh}_2.log 2>&1 || exit $?
done
for d in c2_b0_s3_k5s1_c240_1 c2_b0_s3_k5s1_c240_2 b7_s3_k5s1_c480_1 b7_s3_k5s1_c480_2; do f=$(find gpurun_out/r5be/$d -name "*counter_collection.csv" | head -1); python3 tools/pmc_kernels.py $f dwconv > gpurun_out/r5be/$d.summary.txt || exit $?; done
