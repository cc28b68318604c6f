# round 5: which HIP API calls launch the distillation leg's copyBuffer kernels
set -o pipefail
mkdir -p gpurun_out/r5an
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d /tmp/r5an -o t --output-format csv -- python3 bench.py --no-cpu-baseline --leg distill --steps 4 --warmup 2 > gpurun_out/r5an/distill.json 2> gpurun_out/r5an/distill.err || exit $?
python3 tools/copy_sources.py /tmp/r5an > gpurun_out/r5an/sources.txt 2>&1 || exit $?
