#!/bin/bash
# r04i: the k = 160 projector average under DEIG_DEBUG, block vs scalar Jacobi.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04i
mkdir -p $OUT
timeout -k 10 300 python -u tools/diag_projavg160.py tools/ab_libs/libdeig_rrscalarj.so > $OUT/diag.log 2>&1
rc=$?
cat $OUT/diag.log | cut -c1-260
exit $rc
