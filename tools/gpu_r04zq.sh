#!/bin/bash
# r04zq: f64-MFMA Rayleigh quotients - the whole GPU suite, the c5 per-step timeline,
# the c5 and c1 bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/${TAG:-r04zq}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gputests.log 2>&1 || { tail -30 $OUT/gputests.log; exit 1; }
tail -2 $OUT/gputests.log
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/p -o p -- python3 -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-alt > $OUT/prof_c5.json 2> $OUT/prof_c5.err || { tail -20 $OUT/prof_c5.err; exit 1; }
f=$(find $OUT/p -name "*kernel_trace.csv" | head -1)
python3 tools/step_timeline.py $f --first-kernel split_kernel --per-step 8 > $OUT/timeline.txt
rm -rf $OUT/p
sed -n 1,12p $OUT/timeline.txt
for c in c5 c1; do
  timeout -k 10 400 python -u bench.py --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -20 $OUT/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['value']/1e6,3), d['step_ms']['median'], d['breakdown'])"
done
