#!/bin/bash
# r04za: remainder schedule of the half-ring SYRK - shipped (global numbering, remainder
# unpaced) vs rem1 (remainder rounds paced), rem2 (XCD-major items), rem3 (both),
# interleaved A/B at config 2, d = 4096, d = 5120 and the config-3 shard.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04za
mkdir -p $OUT
LIBS="shipped tools/ab_libs/libdeig_rem1.so tools/ab_libs/libdeig_rem2.so tools/ab_libs/libdeig_rem3.so"
for cfg in "c2 1048576 3072" "d4096 524288 4096" "d5120 1048576 5120" "c3 2097152 8192"; do
  set -- $cfg
  timeout -k 10 400 python -u tools/syrk_ab.py --n $2 --d $3 --reps 5 $LIBS > $OUT/syrk_$1_ab.log 2>&1 || { tail -20 $OUT/syrk_$1_ab.log; exit 1; }
  echo "== $1"; grep -v amdgpu.ids $OUT/syrk_$1_ab.log | python -c "
import json,sys
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.strip()); continue
    print(d['lib'][-24:], round(d['ms_median'],2), d['ms'], d['max_rel_diff_vs_first'])"
done
