set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in "DEIG_OJA_KERNEL=1" "DEIG_OJA_PROBE=0" "DEIG_OJA_PROBE=1" "DEIG_OJA_PROBE=2" "DEIG_OJA_PROBE=8" "DEIG_OJA_PROBE=11" "DEIG_OJA_TN_SLICES=2" "DEIG_OJA_TN_SLICES=4" "DEIG_OJA_TN_SLICES=8" "DEIG_OJA_TN_SLICES=12"; do
  env $cfg timeout -k 10 120 python3 tools/time_oja.py || exit 1
done
mkdir -p gpurun_out/ojaab
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ojaab/p -o p -- python3 tools/time_oja.py > /dev/null 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/ojaab/p/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>6s} avg={float(r['AverageNs'])/1e3:8.2f} us")
PY
