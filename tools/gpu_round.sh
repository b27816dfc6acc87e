#!/bin/bash
# End-of-round evidence on one MI355X: the whole GPU suite, smoke, every bench line
# (the driver's default command first), and a rocprofv3 kernel-trace summary of the
# default command.  Usage: bash tools/gpu_round.sh TAG  (outputs under gpurun_out/TAG)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $OUT/gputests.log 2>&1
rc=$?
tail -4 $OUT/gputests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err \
  || { echo "driver bench failed"; tail -20 $OUT/bench_driver.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_driver.json')); print('c3', round(d['value']/1e6,3), d['step_ms']['median'], d['roofline']['frac'], d['roofline']['launch_ms'])"
for c in c1 c1g c2 c4 c5; do
  timeout -k 10 400 python -u bench.py --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err \
    || { echo "bench $c failed"; tail -20 $OUT/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['value']/1e6,3), d['step_ms']['median'], d['roofline']['frac'])"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python -u bench.py --steps 5 --warmup 2 > $OUT/prof_bench.log 2>&1 \
  || { echo "rocprof failed"; tail -20 $OUT/prof_bench.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/c3_kernel_stats.csv \;
rm -rf $OUT/prof
python - <<PY
import csv
rows = list(csv.DictReader(open("$OUT/c3_kernel_stats.csv")))
for r in rows[:8]:
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms avg")
PY
