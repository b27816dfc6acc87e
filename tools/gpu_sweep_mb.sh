#!/bin/bash
# v3 sweep with 2 vs 4 m-blocks per wave (DEIG_SWEEP_MB) and ring depths
# (DEIG_SWEEP_DEPTH), every mode on v3 (DEIG_SWEEP_KERNEL=3): parity tests per
# setting, then chain / apply timings and rocprof kernel averages.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-swmb}
mkdir -p $OUT
cd $R
for cfg in ${CFGS:-"2 6" "2 8"}; do
  set -- $cfg
  DEIG_SWEEP_KERNEL=3 DEIG_SWEEP_MB=$1 DEIG_SWEEP_DEPTH=$2 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sym_apply or sym_power or topk" > $OUT/t_$1_$2.log 2>&1 || { echo "tests MB=$1 D=$2 failed"; tail -30 $OUT/t_$1_$2.log; exit 1; }
  echo "tests MB=$1 D=$2: $(tail -1 $OUT/t_$1_$2.log)"
done
cd /tmp
for cfg in "0 4 3" ${TCFGS:-"3 2 5" "3 2 6" "3 2 8"}; do
  set -- $cfg
  DEIG_SWEEP_KERNEL=$1 DEIG_SWEEP_MB=$2 DEIG_SWEEP_DEPTH=$3 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$1_$2_$3 -o p -- python3 $R/tools/time_sweep_chain.py 8192:80 16384:128 3072:32 > $OUT/sweep_$1_$2_$3.log 2>&1 || { tail $OUT/sweep_$1_$2_$3.log; exit 1; }
  echo "== KERNEL=$1 MB=$2 DEPTH=$3"; grep "d=" $OUT/sweep_$1_$2_$3.log
  python3 - $OUT/prof_$1_$2_$3 <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "sweep2" in n or "sweep3" in n:
        print(f"   {n[:80]:80s} calls={r['Calls']:>5s} avg={float(r['AverageNs'])/1e3:8.1f} us")
PY
done
