#!/bin/bash
# r04u: config-3 shard covariance - the staggered-phase kernel's phase counts and DMA
# spreads (1PQR0: P phases per K-tile, next K-tile's pieces over Q of them, R prio)
# against the shipped quarter-refill ring, interleaved in one process.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04u
mkdir -p $OUT
L=tools/ab_libs
timeout -k 10 900 python -u tools/syrk_ab.py --reps 4 shipped $L/libdeig_syrk12100.so $L/libdeig_syrk12110.so $L/libdeig_syrk14100.so $L/libdeig_syrk14300.so $L/libdeig_syrk18100.so $L/libdeig_syrk18400.so $L/libdeig_syrk18700.so > $OUT/syrk_ab.log 2>&1 || { tail -20 $OUT/syrk_ab.log; exit 1; }
grep -v amdgpu.ids $OUT/syrk_ab.log | cut -c1-160
