#!/bin/bash
# r04c: bench lines of every config on the current tree, and kernel traces (begin /
# end timestamps) of the c1 and c5 steps for the overlap analysis of the batched
# worker solves (tools/trace_overlap.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04c
mkdir -p $OUT
export TMPDIR=/tmp
for c in c1 c1g c2 c4 c5; do
  timeout -k 10 300 python -u bench.py --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err \
    || { echo "bench $c failed"; tail -20 $OUT/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['value']/1e6,3), d['step_ms']['median'], d['breakdown'])"
done
for c in c1 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$c -o tr -- python -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-alt > $OUT/trace_$c.log 2>&1 \
    || { echo "trace $c failed"; tail -20 $OUT/trace_$c.log; exit 1; }
  find $OUT/trace_$c -name "*kernel_stats.csv" -exec cp {} $OUT/${c}_kernel_stats.csv \;
  find $OUT/trace_$c -name "*kernel_trace.csv" -exec cp {} $OUT/${c}_kernel_trace.csv \;
  rm -rf $OUT/trace_$c
done
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err \
  || { echo "driver bench failed"; tail -20 $OUT/bench_driver.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_driver.json')); print('c3', round(d['value']/1e6,3), d['roofline']['frac'], d.get('time_to_eigenspace_16M_rows_1gpu',{}).get('sigma_hat_rel_err_vs_f64_sampled'))"
