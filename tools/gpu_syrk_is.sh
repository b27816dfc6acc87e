#!/bin/bash
# correctness (poisoned workspace vs float64) then interleaved timing of SYRK variants
# usage (GPU box): bash tools/gpu_syrk_is.sh <tag> <variants...>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 200 python3 tools/syrk_ab.py check "$@" --n 131071 --d 8192 > $OUT/check.log 2>&1 || { echo "check failed"; tail $OUT/check.log; exit 1; }
timeout -k 10 200 python3 tools/syrk_ab.py check "$@" --n 70001 --d 8000 >> $OUT/check.log 2>&1 || { echo "check2 failed"; tail $OUT/check.log; exit 1; }
cat $OUT/check.log | grep check
timeout -k 10 300 python3 tools/syrk_ab.py run "$@" --rounds 3 > $OUT/ab.log 2>&1 || { echo "ab failed"; tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
