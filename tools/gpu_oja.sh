set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/oja
timeout -k 10 300 python -u -m pytest tests -m gpu -k "oja or c4 or streaming" -x -q --timeout 120 --timeout-method thread > gpurun_out/oja/tests.log 2>&1 || { tail -30 gpurun_out/oja/tests.log; exit 1; }
tail -2 gpurun_out/oja/tests.log
timeout -k 10 300 python -u bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/oja/bench_c4.json 2> gpurun_out/oja/bench_c4.err || { tail gpurun_out/oja/bench_c4.err; exit 1; }
python -c "import json;L=json.load(open('gpurun_out/oja/bench_c4.json'));print(L['value'],L['roofline']['achieved'],L['roofline']['frac'],L['breakdown'],L['accuracy'])"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/oja/prof -o p -- python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/oja/prof.log 2>&1 || { tail gpurun_out/oja/prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/oja/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>6s} avg={float(r['AverageNs'])/1e3:8.2f} us tot%={r.get('Percentage','')}")
PY
