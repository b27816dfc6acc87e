#!/bin/bash
# r03s: where c1's step goes (kernel trace, batched solve) + worker-mode A/B at c1 / c5
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03s
mkdir -p $OUT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c1 -o p -- \
  python3 $R/bench.py --config c1 --no-cpu-baseline --no-alt --steps 10 > $OUT/c1_rocprof.json 2> $OUT/c1_rocprof.err \
  || { echo "c1 trace failed"; tail $OUT/c1_rocprof.err; exit 1; }
python3 -c "
import csv
r=list(csv.DictReader(open('$OUT/trace_c1/p_kernel_stats.csv')))
for x in r[:16]: print(x['Name'][:80], x['Calls'], round(float(x['AverageNs'])/1e3,2), x['Percentage'])
" | tee $OUT/c1_kernels.txt
cd $R
for m in "" "--threaded-workers"; do
  for c in c1 c5; do
    timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-alt --steps 10 $m > $OUT/ab_${c}${m}.json 2> $OUT/ab_${c}${m}.err \
      || { echo "bench $c $m failed"; tail $OUT/ab_${c}${m}.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/ab_${c}${m}.json')); print('$c', '$m', d['value'], d['ms_per_step'], d['breakdown'])"
  done
done
