#!/bin/bash
# Oja (config 4): parity tests, then the c4 bench line under rocprofv3 kernel stats.
# usage: bash tools/gpu_oja_round.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-oja}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "oja or Oja or c4 or streaming or skinny or server or projavg or golden" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o p -- \
  python3 $R/bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > $OUT/c4.json 2> $OUT/c4.err || { tail $OUT/c4.err; exit 1; }
python3 -c "import json; r=json.load(open('$OUT/c4.json')); print(r['value'], r['roofline']['frac'], r['breakdown'])"
python3 - $OUT/prof <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(f"   {r['Name'][:75]:75s} calls={r['Calls']:>5s} avg={float(r['AverageNs'])/1e3:8.1f} us")
PY
