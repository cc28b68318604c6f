# round 5: full GPU suite on the current tree
set -o pipefail
mkdir -p gpurun_out/r5aj
cd $GRAFT_REPO_ROOT
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r5aj/suite.txt 2>&1; echo "rc=$?" >> gpurun_out/r5aj/suite.txt
