#!/bin/bash
# Fused sweep chain: solver / sweep parity tests, per-kernel rocprof times of the
# sweep chain and the standalone apply, then a c3 bench line.
# usage: bash tools/gpu_sweep_chain.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-swchain}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_solver_robust.py tests/test_gpu_cifar.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
cd /tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o p -- \
  python3 $R/tools/time_sweep_chain.py ${SWEEP_CASES:-8192:80 16384:128 3072:32} > $OUT/sweep.log 2>&1 || { tail $OUT/sweep.log; exit 1; }
grep "d=" $OUT/sweep.log
python3 - $OUT/prof <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "sweep" in n or "split_q" in n:
        print(f"   {n[:75]:75s} calls={r['Calls']:>5s} avg={float(r['AverageNs'])/1e3:8.1f} us")
PY
cd $R
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt > $OUT/c3.json 2> $OUT/c3.err || { tail $OUT/c3.err; exit 1; }
python3 -c "import json; r=json.load(open('$OUT/c3.json')); print(r['value'], r['breakdown'], json.dumps(r['sweep'])[:900])"
