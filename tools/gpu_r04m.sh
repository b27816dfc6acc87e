#!/bin/bash
# r04m: the Chebyshev threshold on the spiked sweep-count test matrix (wall time), then
# c1 / c5 / c2 benches and the RR phases against the r04h Jacobi.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04m
mkdir -p $OUT
timeout -k 10 300 python -u tools/cheb_probe_spiked.py > $OUT/cheb_probe.log 2>&1 || { tail -20 $OUT/cheb_probe.log; exit 1; }
grep -v amdgpu.ids $OUT/cheb_probe.log
for c in c1 c5 c2; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err \
    || { echo "bench $c failed"; tail -20 $OUT/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['value']/1e6,3), d['step_ms']['median'], d['breakdown'])"
done
timeout -k 10 500 python -u tools/rr_phases_ab.py tools/ab_libs/libdeig_rrjold.so > $OUT/rr_phases.log 2>&1 || { tail -30 $OUT/rr_phases.log; exit 1; }
grep -E "^#|median|RRs" $OUT/rr_phases.log
