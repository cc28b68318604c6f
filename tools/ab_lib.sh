#!/bin/bash
# A/B of libhiseg builds on conv_bench shapes, alternating processes on one box (developer tool).
#   bash tools/ab_lib.sh <out-dir> <lib1,lib2,...> <rounds> [conv_bench args...]
set -o pipefail
out=gpurun_out/$1; libs=$2; n=$3; shift 3
mkdir -p "$out"
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
for i in $(seq 1 "$n"); do
  for L in ${libs//,/ }; do
    echo "== $L round $i" >> "$out/ab.txt"
    HISEG_LIB="$L" timeout -k 10 240 python3 -u tools/conv_bench.py "$@" >> "$out/ab.txt" 2>&1 || exit 1
  done
done
