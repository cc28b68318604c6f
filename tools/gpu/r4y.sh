# train leg kernel trace (wgrad reduce / BN / loss finalize after round-4 changes), same-box A/B of the B prefetch
set -o pipefail
mkdir -p gpurun_out/r4y
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u bench.py --leg train --steps 6 > gpurun_out/r4y/train_a.log 2>&1 || exit $?
HISEG_WGRAD_BPRE=0 timeout -k 10 300 python3 -u bench.py --leg train --steps 6 > gpurun_out/r4y/train_b.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --leg train --steps 6 > gpurun_out/r4y/train_c.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4y/prof -o train -- python3 bench.py --leg train --steps 6 > gpurun_out/r4y/prof_train.log 2>&1 || exit $?
