#!/bin/bash
# r03q: Oja batch kernels under PMC counters (separate passes) + kernel trace
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03q
mkdir -p $OUT
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o p -- python3 $R/tools/time_oja.py 4096 3072 32 16 > $OUT/trace.log 2>&1 || { echo trace failed; tail $OUT/trace.log; exit 1; }
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc$i -o p -- python3 $R/tools/time_oja.py 4096 3072 32 16 > $OUT/pmc$i.log 2>&1 || { echo "pmc $pmc failed"; tail $OUT/pmc$i.log; exit 1; }
done
python3 $R/tools/pmc_oja.py $OUT/pmc1 $OUT/pmc2 $OUT/pmc3 $OUT/pmc4 $OUT/pmc5 | tee $OUT/pmc_summary.txt
python3 -c "
import csv
r=list(csv.DictReader(open('$OUT/trace/p_kernel_stats.csv')))
for x in r[:8]: print(x['Name'][:70], x['Calls'], round(float(x['AverageNs'])/1e3,2))
"
