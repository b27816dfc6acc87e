#!/bin/bash
# r04zb: the split pass with 16-B loads per lane vs the r03 scalar-load split pass
# (both with remainder pacing), interleaved A/B at config 2 and the config-3 shard,
# then the covariance GPU tests on the shipped library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04zb
mkdir -p $OUT
LIBS="shipped tools/ab_libs/libdeig_splitscalar.so"
for cfg in "c2 1048576 3072" "c3 2097152 8192"; do
  set -- $cfg
  timeout -k 10 400 python -u tools/syrk_ab.py --n $2 --d $3 --reps 7 $LIBS > $OUT/syrk_$1_ab.log 2>&1 || { tail -20 $OUT/syrk_$1_ab.log; exit 1; }
  echo "== $1"; grep -v amdgpu.ids $OUT/syrk_$1_ab.log | python -c "
import json,sys
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.strip()); continue
    print(d['lib'][-28:], round(d['ms_median'],2), d['ms'], d['max_rel_diff_vs_first'])"
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_syrk_chunks.py tests/test_gpu_kernels.py > $OUT/cov_tests.log 2>&1 || { tail -30 $OUT/cov_tests.log; exit 1; }
tail -2 $OUT/cov_tests.log
