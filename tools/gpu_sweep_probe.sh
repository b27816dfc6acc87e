# Knock-out kernel timing (rocprofv3 kernel trace) of sweep2 at d=8192 p=80.
# DEIG_SWEEP_PROBE bits: 1 no MFMA, 2 no S loads, 4 no Q loads.  usage: bash tools/gpu_sweep_probe.sh <tag> [probes...]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-swp}; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
for pr in "${@:-0}"; do
  DEIG_SWEEP_PROBE=$pr timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p$pr -o p -- \
    python3 $R/tools/time_sweep.py ${SWEEP_CASES:-8192:80} > $OUT/p$pr.log 2>&1 || { tail $OUT/p$pr.log; exit 1; }
  echo "probe=$pr"; grep bf16x6 $OUT/p$pr.log
  python3 - $OUT/p$pr <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "sweep" in n or "split_q" in n:
        print(f"   {n[:60]:60s} calls={r['Calls']:>5s} avg={float(r['AverageNs'])/1e3:8.1f} us")
PY
done
