# wgrad_wide / wgrad_tr counters after the addressing changes (SHT 2, TOG, INC)
set -o pipefail
mkdir -p gpurun_out/r4s2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python3 -u tools/wgrad_bench.py --shapes w256_3x3_64x48,w128_3x3_128x96 > gpurun_out/r4s2/bench.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/r4s2/p1 -o p --output-format csv -- python3 tools/wgrad_bench.py --shapes w256_3x3_64x48,w128_3x3_128x96 --reps 2 > gpurun_out/r4s2/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES --kernel-trace -d gpurun_out/r4s2/p2 -o p --output-format csv -- python3 tools/wgrad_bench.py --shapes w256_3x3_64x48,w128_3x3_128x96 --reps 2 > gpurun_out/r4s2/p2.log 2>&1 || exit $?
