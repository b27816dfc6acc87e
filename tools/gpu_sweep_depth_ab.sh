#!/bin/bash
# Sweep ring depth A/B on the GPU box (tools/sweep_lib_ab.py over the shipped build and
# DEIG_AB_SWEEP_DEPTH builds in tools/ab_libs).  usage: bash tools/gpu_sweep_depth_ab.sh <tag> libs...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for c in "8192 80 bf16x3" "8192 80 bf16x5" "8192 80 bf16x6" "16384 128 bf16x3" "16384 128 bf16x6" "3072 32 bf16x3"; do
  timeout -k 10 240 python -u tools/sweep_lib_ab.py 7 $c "$@" >> $OUT/ab.log 2>&1 || { echo "failed at $c"; tail -20 $OUT/ab.log; exit 1; }
done
cat $OUT/ab.log
