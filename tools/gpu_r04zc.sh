#!/bin/bash
# r04zc: Oja batch-size scaling - per-kernel averages (rocprofv3 --kernel-trace
# --stats) of oja_nn_kernel / oja_tn_kernel at b = 1024 .. 32768 rows (d = 3072,
# k = 32), to separate each pass's fixed cost from its per-byte cost.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r04zc
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in "1024 256" "2048 128" "4096 64" "8192 32" "16384 16" "32768 8"; do
  set -- $cfg
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p_$1 -o p -- python3 $R/tools/time_oja.py $1 3072 32 $2 > $OUT/t_$1.log 2>&1 || { tail -5 $OUT/t_$1.log; exit 1; }
  f=$(find $OUT/p_$1 -name "*kernel_stats.csv" | head -1)
  cp $f $OUT/stats_$1.csv
  rm -rf $OUT/p_$1
  echo "b=$1 $(grep 'us/batch' $OUT/t_$1.log)"
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/stats_$1.csv')):
    if 'oja' in r['Name'] or 'img' in r['Name']: print('   ', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')"
done
