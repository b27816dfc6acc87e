#!/bin/bash
# r04d: RR phase timings (shipped v2 vs the r03 small solve), then the tests that
# failed in r04b, then the whole GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04d
mkdir -p $OUT
timeout -k 10 500 python -u tools/rr_phases_ab.py tools/ab_libs/libdeig_rrv1.so tools/ab_libs/libdeig_rrjlow.so > $OUT/rr_phases.log 2>&1 || { tail -30 $OUT/rr_phases.log; exit 1; }
cat $OUT/rr_phases.log
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_gpu_syrk_chunks.py tests/test_gpu_integration_stub.py \
  tests/test_gpu_general_solver.py tests/test_gpu_solver_robust.py > $OUT/new_tests.log 2>&1
rc=$?
grep -E "FAIL|ERROR" $OUT/new_tests.log | tail -30
tail -2 $OUT/new_tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
  > $OUT/gputests.log 2>&1
rc=$?
tail -15 $OUT/gputests.log
exit $rc
