#!/bin/bash
# r04s: the fused one-workgroup CholQR in the Oja loop - Oja tests, c4 bench, a c4
# kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04s
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -k "oja or Oja or stream" tests/ -m gpu > $OUT/tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR" $OUT/tests.log | tail -30
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --config c4 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -20 $OUT/bench_c4.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_c4.json')); print('c4', round(d['value']/1e6,3), d['step_ms'], d['breakdown'], d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c4 -- python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/c4_kernel_stats.csv \;
rm -rf $OUT/prof
python - <<PY
import csv
for r in list(csv.DictReader(open("$OUT/c4_kernel_stats.csv")))[:10]:
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us avg")
PY
