#!/bin/bash
# r04zl: XCD pacing interval with the half-ring SYRK (shipped 64 K-tiles vs 32 / 128),
# interleaved A/B at the config-3 shard; then the PMC records of the current
# syrk_split.hip (tools/gpu_r04v.sh, TAG=r04zl: c3 / c2 traffic, SQ pass, c3 driver bench).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04zl
mkdir -p $OUT
timeout -k 10 400 python -u tools/syrk_ab.py --n 2097152 --d 8192 --reps 5 shipped tools/ab_libs/libdeig_pace32.so tools/ab_libs/libdeig_pace128.so > $OUT/syrk_pace_ab.log 2>&1 || { tail -20 $OUT/syrk_pace_ab.log; exit 1; }
grep -v amdgpu.ids $OUT/syrk_pace_ab.log | python -c "
import json,sys
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.strip()); continue
    print(d['lib'][-28:], round(d['ms_median'],2), d['ms'], d['max_rel_diff_vs_first'])"
TAG=r04zl bash tools/gpu_r04v.sh
