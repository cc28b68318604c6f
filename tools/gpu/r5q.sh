# round 5: conv_hwc automatic -- full GPU suite, inference leg, PMC HBM bytes of the dominant kernel through the bench command
set -o pipefail
mkdir -p gpurun_out/r5q
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r5q/suite.txt 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --leg infer --steps 20 --warmup 5 > gpurun_out/r5q/infer.json 2> gpurun_out/r5q/infer.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r5q/pmc_f -o pmc -- python3 bench.py --leg infer --steps 6 --warmup 2 > gpurun_out/r5q/pmc_f.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/r5q/pmc_w -o pmc -- python3 bench.py --leg infer --steps 6 --warmup 2 > gpurun_out/r5q/pmc_w.log 2>&1 || exit $?
F=$(dirname $(find gpurun_out/r5q/pmc_f -name "pmc_counter_collection.csv" | head -1))
W=$(dirname $(find gpurun_out/r5q/pmc_w -name "pmc_counter_collection.csv" | head -1))
python3 tools/pmc_hbm.py $F $W --top 40 > gpurun_out/r5q/pmc_hbm.txt 2>&1
find gpurun_out/r5q -name "*.csv" -size +20M -delete
