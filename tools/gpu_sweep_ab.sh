# Sweep kernel A/B: parity tests of the default kernel, then rocprof kernel times
# of each version (DEIG_SWEEP_KERNEL / DEIG_SWEEP_DEPTH) at the bench shapes.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-swab}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sym_apply" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
cd /tmp
for v in ${VARIANTS:-3:3 3:4 2:3}; do
  ver=${v%:*}; dep=${v#*:}
  DEIG_SWEEP_KERNEL=$ver DEIG_SWEEP_DEPTH=$dep timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/v$ver-$dep -o p -- \
    python3 $R/tools/time_sweep.py ${SWEEP_CASES:-8192:80 3072:32 16384:128} > $OUT/v$ver-$dep.log 2>&1 || { tail $OUT/v$ver-$dep.log; exit 1; }
  echo "version=$ver depth=$dep"; grep bf16x6 $OUT/v$ver-$dep.log
  python3 - $OUT/v$ver-$dep <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "sweep" in n or "split_q" in n:
        print(f"   {n[:60]:60s} calls={r['Calls']:>5s} avg={float(r['AverageNs'])/1e3:8.1f} us")
PY
done
