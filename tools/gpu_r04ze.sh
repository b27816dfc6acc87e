#!/bin/bash
# r04ze: phase timeline of the resident Oja kernel (trace build) + rocprof kernel
# stats of the config-4 A/B (resident vs two-pass).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r04ze
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/oja_trace.py > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
grep -v amdgpu.ids $OUT/trace.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p -o p -- python3 $R/tools/oja_resident_ab.py 3 > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
f=$(find $OUT/p -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv; rm -rf $OUT/p
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us', round(float(r['TotalDurationNs'])/1e6,2), 'ms')"
