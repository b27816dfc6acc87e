#!/bin/bash
# r04b: RR v2 A/B against r03's small solve (tools/rr_ab.py), under rocprofv3 for the
# per-kernel averages; then the new parity tests and the whole GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/rr_ab.py run --reps 3 > $OUT/rr_ab.log 2>&1 || { tail -30 $OUT/rr_ab.log; exit 1; }
cat $OUT/rr_ab.log | grep case
timeout -k 10 200 python -u tools/u8_mirror_ab.py run > $OUT/u8_mirror_ab.log 2>&1 || { tail -20 $OUT/u8_mirror_ab.log; exit 1; }
cat $OUT/u8_mirror_ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_rr -o rr -- python -u tools/rr_ab.py run --reps 2 > $OUT/rr_ab_prof.log 2>&1 || { tail -20 $OUT/rr_ab_prof.log; exit 1; }
find $OUT/prof_rr -name "*kernel_stats.csv" -exec cp {} $OUT/rr_ab_kernel_stats.csv \;
grep -i "rr_small\|rr_update" $OUT/rr_ab_kernel_stats.csv | cut -c1-160
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_gpu_syrk_chunks.py tests/test_gpu_integration_stub.py \
  tests/test_gpu_general_solver.py tests/test_gpu_solver_robust.py tests/test_gpu_batch_solver.py > $OUT/new_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR" $OUT/new_tests.log | tail -60
tail -3 $OUT/new_tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
  --durations=15 > $OUT/gputests.log 2>&1
rc=$?
tail -30 $OUT/gputests.log
exit $rc
