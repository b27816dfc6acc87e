#!/bin/bash
# PMC traffic (FETCH_SIZE, WRITE_SIZE: separate passes) of the sweep chain at d=8192,
# p=80 (tools/time_sweep_chain.py), summarised per kernel by tools/pmc_sweep.py.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmcsweep}
mkdir -p $OUT
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o p -- python3 $R/tools/time_sweep_chain.py 8192:80 > $OUT/fetch.log 2>&1 || { echo "fetch pass failed"; tail $OUT/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o p -- python3 $R/tools/time_sweep_chain.py 8192:80 > $OUT/write.log 2>&1 || { echo "write pass failed"; tail $OUT/write.log; exit 1; }
python3 $R/tools/pmc_sweep.py $OUT/fetch $OUT/write $OUT/pmc_sweep_d8192_p80.json 8192 80
