#!/bin/bash
# r04l: Chebyshev from resid <= 0.1 by default and the ballot rotation count - the whole
# GPU suite, c1 / c5 / c2, RR phases vs the r04h Jacobi (-DDEIG_AB_RR_JOLD = r03 step).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04l
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $OUT/gputests.log 2>&1
rc=$?
tail -15 $OUT/gputests.log
[ $rc -eq 0 ] || exit 1
for c in c1 c5 c2; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err \
    || { echo "bench $c failed"; tail -20 $OUT/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['value']/1e6,3), d['step_ms']['median'], d['breakdown'])"
done
timeout -k 10 500 python -u tools/rr_phases_ab.py tools/ab_libs/libdeig_rrjold.so > $OUT/rr_phases.log 2>&1 || { tail -30 $OUT/rr_phases.log; exit 1; }
grep -E "^#|median|RRs" $OUT/rr_phases.log
