#!/bin/bash
# r03n: Oja with unpredicated loads: Oja GPU tests, c4 bench + kernel trace
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03n
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "oja or Oja or streaming" tests/ > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python3 bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err \
  || { echo "bench c4 failed"; tail $OUT/bench_c4.err; exit 1; }
python3 -c "import json; r=json.load(open('$OUT/bench_c4.json')); print('c4', r['value'], r['ms_per_step'], r['roofline'])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4trace -o p -- \
  python3 $R/bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_c4_rocprof.json 2> $OUT/c4trace.err \
  || { echo "c4 trace failed"; tail $OUT/c4trace.err; exit 1; }
python3 -c "
import csv
r=list(csv.DictReader(open('$OUT/c4trace/p_kernel_stats.csv')))
for x in r[:10]: print(x['Name'][:70], x['Calls'], round(float(x['AverageNs'])/1e3,2))
"
