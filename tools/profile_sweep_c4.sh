#!/bin/bash
# rocprofv3: PMC traffic of the sweep kernel (d=8192 p=80, prepared image) and a
# kernel trace of the Oja bench (config 4).  usage: bash tools/profile_sweep_c4.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/sw_fetch -o p -- \
  python3 $R/tools/time_sweep.py 8192:80 > $OUT/sw_fetch.log 2>&1 || { echo "sweep fetch pass failed"; tail $OUT/sw_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/sw_write -o p -- \
  python3 $R/tools/time_sweep.py 8192:80 > $OUT/sw_write.log 2>&1 || { echo "sweep write pass failed"; tail $OUT/sw_write.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4 -o p -- \
  python3 $R/bench.py --config c4 --no-cpu-baseline > $OUT/c4.json 2> $OUT/c4.err || { echo "c4 trace failed"; tail $OUT/c4.err; exit 1; }
echo done
