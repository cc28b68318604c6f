# training legs after the weight-gradient addressing change
set -o pipefail
mkdir -p gpurun_out/r4r5
cd $GRAFT_REPO_ROOT
for leg in train c3 c4; do
  timeout -k 10 300 python3 -u bench.py --leg $leg --steps 20 --warmup 5 > gpurun_out/r4r5/$leg.txt 2>&1 || exit $?
done
