#!/bin/bash
# One GPU job on a gpurun box (developer tool; replaces the per-lease scripts of earlier rounds).
#   bash tools/gpu_job.sh <out-dir> <job> [args...]
# jobs:
#   tests  [pytest args]        pytest -m gpu (thread timeout per test), log in <out>/tests.txt
#   bench  [bench.py args]      bench.py, line in <out>/bench.txt (detail file under gpurun_out/)
#   prof   [bench.py args]      rocprofv3 --kernel-trace --stats (csv) of bench.py, into <out>/prof
#   pmc    <counter> [args]     one rocprofv3 --pmc pass (one counter group) of bench.py --leg ..., into <out>/pmc_<counter>
#   tool   <script.py> [args]   python tools/<script.py> args, log in <out>/<script>.txt
#   env    <VAR=VAL> <job> ...  run <job> with VAR=VAL set (A/B knobs such as HISEG_PW_RB)
# Every GPU step runs under its own timeout; the first failure ends the job (no retries).
set -o pipefail
out=gpurun_out/$1; shift
job=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
case "$job" in
  tests) timeout -k 10 900 python3 -u -m pytest -x -v -m gpu --timeout 240 --timeout-method thread "${@:-tests}" > "$out/tests.txt" 2>&1 ;;
  bench) timeout -k 10 600 python3 -u bench.py "$@" > "$out/bench.txt" 2> "$out/bench.err" ;;
  prof)  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- python3 bench.py "$@" > "$out/prof.log" 2>&1 ;;
  pmc)   c=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$c" --kernel-trace --output-format csv -d "$out/pmc_$c" -o pmc -- python3 bench.py "$@" > "$out/pmc_$c.log" 2>&1 ;;
  tool)  t=$1; shift; timeout -k 10 300 python3 -u "tools/$t" "$@" > "$out/${t%.py}.txt" 2>&1 ;;
  env)   kv=$1; shift; export "$kv"; sub=$1; shift; bash "$0" "${out#gpurun_out/}" "$sub" "$@" ;;
  *) echo "unknown job $job" >&2; exit 2 ;;
esac
