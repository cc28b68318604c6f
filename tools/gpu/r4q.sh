# round 4: depthwise LDS tiles, two-launch SE, RoIAlign whole-pixel stores -- tests, microbenchmarks, distill leg
set -o pipefail
mkdir -p gpurun_out/r4q
timeout -k 10 400 python -u -m pytest -v --tb=short --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "roi or se_two or dwconv or dw_ or norm_act or efficientnet or se_ or preset or bf16_logits" > gpurun_out/r4q/tests.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/roi_bench.py > gpurun_out/r4q/roi_bench.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/dw_bench.py > gpurun_out/r4q/dw_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --leg distill --steps 10 > gpurun_out/r4q/distill.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4q/prof -o distill -- python3 bench.py --leg distill --steps 6 > gpurun_out/r4q/prof_distill.log 2>&1 || exit $?
