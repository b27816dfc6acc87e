#!/bin/bash
# r04h: the RR Jacobi step with the column pair rotation hoisted (vs -DDEIG_AB_RR_JOLD),
# the solver and u8 tests, c1 / c5.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04h
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_general_solver.py tests/test_gpu_solver_robust.py tests/test_gpu_batch_solver.py tests/test_gpu_u8.py > $OUT/tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|Error" $OUT/tests.log | tail -40
[ $rc -eq 0 ] || exit 1
timeout -k 10 500 python -u tools/rr_phases_ab.py tools/ab_libs/libdeig_rrjold.so > $OUT/rr_phases.log 2>&1 || { tail -30 $OUT/rr_phases.log; exit 1; }
cat $OUT/rr_phases.log
for c in c1 c5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err \
    || { echo "bench $c failed"; tail -20 $OUT/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['value']/1e6,3), d['step_ms']['median'], d['breakdown'])"
done
