# round 5: where the distillation step's device copies come from
set -o pipefail
mkdir -p gpurun_out/r5am
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u tools/copy_probe.py > gpurun_out/r5am/copies.txt 2>&1 || exit $?
