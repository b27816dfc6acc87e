#!/bin/bash
# r04zo: rocprof kernel summary of the c5 bench (where the batched worker solve's
# 12 ms per worker goes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r04zo
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p -o p -- python3 -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-alt > $OUT/prof_c5.json 2> $OUT/prof_c5.err || { tail -20 $OUT/prof_c5.err; exit 1; }
f=$(find $OUT/p -name "*kernel_stats.csv" | head -1); cp $f $OUT/c5_kernel_stats.csv; rm -rf $OUT/p
python3 -c "
import csv
rows=list(csv.DictReader(open('$OUT/c5_kernel_stats.csv')))
for r in rows[:24]: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', round(float(r['TotalDurationNs'])/1e6,2), 'ms')"
