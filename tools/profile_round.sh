#!/bin/bash
# rocprofv3 kernel-trace/stats of the default bench + PMC traffic passes of the
# covariance op.  usage: [SKIP_TRACE=1] bash tools/profile_round.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
if [ -z "$SKIP_TRACE" ]; then
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o p -- \
  python3 $R/bench.py --no-cpu-baseline --no-alt > $OUT/bench_under_rocprof.json 2> $OUT/bench_under_rocprof.err \
  || { echo "trace pass failed rc=$?"; tail -20 $OUT/bench_under_rocprof.err; exit 1; }
fi
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o p -- \
  python3 $R/tools/run_syrk_once.py > $OUT/fetch.log 2>&1 || { echo "fetch pass failed"; tail $OUT/fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o p -- \
  python3 $R/tools/run_syrk_once.py > $OUT/write.log 2>&1 || { echo "write pass failed"; tail $OUT/write.log; exit 1; }
python3 $R/tools/pmc_traffic.py $OUT/fetch $OUT/write $OUT/pmc_syrk_c3_split3.json 2097152 8192 \
  "covariance split3 (split_kernel + syrks_h_kernel + syrks_reduce_kernel + diag_corr_kernel)" > /dev/null \
  && python3 - $OUT/pmc_syrk_c3_split3.json $TAG <<'PY'
import json, sys, time
p, tag = sys.argv[1:3]
r = json.load(open(p))
r["measured"] = f"profile round {tag}, {time.strftime('%Y-%m-%d')}"
json.dump(r, open(p, "w"), indent=1)
PY
[ -z "$SKIP_TRACE" ] && ls $OUT/trace
# config 2 (2^20 x 3072, split pass + half ring since r04): its own PMC record for bench.py --config c2
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_c2 -o p -- \
  python3 $R/tools/run_syrk_once.py 1048576 3072 > $OUT/fetch_c2.log 2>&1 || { echo "c2 fetch pass failed"; tail $OUT/fetch_c2.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_c2 -o p -- \
  python3 $R/tools/run_syrk_once.py 1048576 3072 > $OUT/write_c2.log 2>&1 || { echo "c2 write pass failed"; tail $OUT/write_c2.log; exit 1; }
python3 $R/tools/pmc_traffic.py $OUT/fetch_c2 $OUT/write_c2 $OUT/pmc_syrk_c2_split3.json 1048576 3072 \
  "covariance split3 (split_kernel + syrks_h_kernel + syrks_reduce_kernel + diag_corr_kernel)" > /dev/null \
  && python3 - $OUT/pmc_syrk_c2_split3.json $TAG <<'PY'
import json, sys, time
p, tag = sys.argv[1:3]
r = json.load(open(p))
r["measured"] = f"profile round {tag}, {time.strftime('%Y-%m-%d')}"
json.dump(r, open(p, "w"), indent=1)
PY
