#!/bin/bash
# r03v: u8 exactness diagnosis; pinned status kernel + RQ v3 + direct u8: benches and c1 trace
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03v
mkdir -p $OUT
cd $R

timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread > $OUT/gputests.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 $OUT/gputests.log; exit 1; }
tail -2 $OUT/gputests.log
for c in c1 c1g c5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-alt --steps 10 > $OUT/bench_$c.json 2> $OUT/bench_$c.err \
    || { echo "bench $c failed"; tail $OUT/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d['breakdown'])"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c1 -o p -- \
  python3 $R/bench.py --config c1 --no-cpu-baseline --no-alt --steps 10 > $OUT/c1_rocprof.json 2> $OUT/c1_rocprof.err \
  || { echo "c1 trace failed"; tail $OUT/c1_rocprof.err; exit 1; }
python3 -c "
import csv
r=list(csv.DictReader(open('$OUT/trace_c1/p_kernel_stats.csv')))
for x in r[:18]: print(x['Name'][:80], x['Calls'], round(float(x['AverageNs'])/1e3,2), x['Percentage'])
" | tee $OUT/c1_kernels.txt
