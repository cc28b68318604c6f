# round 4: pipelined dwconv_t window, LDS-tiled SE W2, tree-merged BN reductions -- tests, microbenchmarks, legs
set -o pipefail
mkdir -p gpurun_out/r4t
timeout -k 10 400 python -u -m pytest -v --tb=short --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "roi or se_two or dwconv or dw_ or norm_act or efficientnet or se_ or preset or bf16_logits" > gpurun_out/r4t/tests.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -v --tb=short --timeout 200 --timeout-method thread tests/test_gpu_train.py > gpurun_out/r4t/train_tests.log 2>&1 || exit $?

timeout -k 10 300 python -u bench.py --leg distill --steps 10 > gpurun_out/r4t/distill.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --leg train --steps 6 > gpurun_out/r4t/train.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4t/prof -o distill -- python3 bench.py --leg distill --steps 6 > gpurun_out/r4t/prof_distill.log 2>&1 || exit $?
