#!/bin/bash
# r04w: config-3 shard covariance - the two-phase half-refill ring (30000) against
# the shipped two-phase staggered kernel (12100) and the r03 quarter ring (20100),
# interleaved in one process, twice (two orders).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04w
mkdir -p $OUT
L=tools/ab_libs
timeout -k 10 600 python -u tools/syrk_ab.py --reps 5 shipped $L/libdeig_syrk30000.so $L/libdeig_syrk20100.so > $OUT/syrk_ab.log 2>&1 || { tail -20 $OUT/syrk_ab.log; exit 1; }
grep -v amdgpu.ids $OUT/syrk_ab.log | cut -c1-220
timeout -k 10 600 python -u tools/syrk_ab.py --reps 5 $L/libdeig_syrk30000.so shipped $L/libdeig_syrk20100.so > $OUT/syrk_ab2.log 2>&1 || { tail -20 $OUT/syrk_ab2.log; exit 1; }
grep -v amdgpu.ids $OUT/syrk_ab2.log | cut -c1-220
