# round 4: C3 / C4 leg kernel traces (outliers)
set -o pipefail
mkdir -p gpurun_out/r4aa
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r4aa/c3 -o c3 -- python3 bench.py --leg c3 --steps 6 > gpurun_out/r4aa/c3.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r4aa/c4 -o c4 -- python3 bench.py --leg c4 --steps 6 > gpurun_out/r4aa/c4.log 2>&1 || exit $?
