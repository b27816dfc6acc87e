#!/bin/bash
# r03p: Oja knock-out / prefetch-depth A/B at config 4's shape
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03p
mkdir -p $OUT
cd $R
timeout -k 10 400 python3 -u tools/oja_ab.py run 0 256 8 264 56 63 --rounds 7 > $OUT/oja_ab.log 2>&1 \
  || { echo "oja ab failed"; tail -20 $OUT/oja_ab.log; exit 1; }
tail -14 $OUT/oja_ab.log
