#!/bin/bash
# r04y: config 2 (2^20 x 3072) covariance - the fused split (shipped for d <= 4096)
# against the split pass + half-ring SYRK (30000), interleaved A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04y
mkdir -p $OUT
timeout -k 10 300 python -u tools/syrk_ab.py --n 1048576 --d 3072 --reps 5 shipped tools/ab_libs/libdeig_syrk30000all.so > $OUT/syrk_c2_ab.log 2>&1 || { tail -20 $OUT/syrk_c2_ab.log; exit 1; }
grep -v amdgpu.ids $OUT/syrk_c2_ab.log
timeout -k 10 300 python -u tools/syrk_ab.py --n 524288 --d 4096 --reps 5 shipped tools/ab_libs/libdeig_syrk30000all.so > $OUT/syrk_d4096_ab.log 2>&1 || { tail -20 $OUT/syrk_d4096_ab.log; exit 1; }
grep -v amdgpu.ids $OUT/syrk_d4096_ab.log
timeout -k 10 300 python -u tools/syrk_ab.py --n 2097152 --d 2048 --reps 5 shipped tools/ab_libs/libdeig_syrk30000all.so > $OUT/syrk_d2048_ab.log 2>&1 || { tail -20 $OUT/syrk_d2048_ab.log; exit 1; }
grep -v amdgpu.ids $OUT/syrk_d2048_ab.log
