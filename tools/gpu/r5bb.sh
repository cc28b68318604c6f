# round 5: overlap of the distillation step's teacher / student forward graphs
set -o pipefail
mkdir -p gpurun_out/r5bb
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u tools/distill_branches.py > gpurun_out/r5bb/d.txt 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/distill_branches.py --unfrozen 2 > gpurun_out/r5bb/u.txt 2>&1 || exit $?
HISEG_SERIAL_TEACHER=1 timeout -k 10 300 python3 -u tools/distill_branches.py > gpurun_out/r5bb/d_serialflag.txt 2>&1 || exit $?
