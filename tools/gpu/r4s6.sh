# round 4 final: full GPU suite, smoke, the default bench line
set -o pipefail
mkdir -p gpurun_out/r4s6
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/r4s6/suite.txt 2>&1 || exit $?
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4s6/smoke.txt 2>&1 || exit $?
timeout -k 10 900 python3 -u bench.py > gpurun_out/r4s6/bench.txt 2>&1 || exit $?
