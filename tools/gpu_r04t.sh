#!/bin/bash
# r04t: config-3 shard covariance - the shipped SYRK against the other schedules of
# the same kernel family (s_setprio, 2-phase staggering, XCD pacing every 128 / 32
# K-tiles), interleaved in one process.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04t
mkdir -p $OUT
timeout -k 10 600 python -u tools/syrk_ab.py --reps 4 shipped tools/ab_libs/libdeig_syrk20110.so tools/ab_libs/libdeig_syrk12100.so tools/ab_libs/libdeig_pace128.so tools/ab_libs/libdeig_pace32.so > $OUT/syrk_ab.log 2>&1 || { tail -20 $OUT/syrk_ab.log; exit 1; }
grep -v amdgpu.ids $OUT/syrk_ab.log
