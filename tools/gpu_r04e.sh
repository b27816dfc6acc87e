#!/bin/bash
# r04e: batched sweeps across the worker problems of solve_batch - bit-identity and
# parity tests, then c1 / c1g with the shipped slicing and the DEIG_AB_BATCH_KS variant.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04e
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_gpu_batch_solver.py tests/test_gpu_general_solver.py > $OUT/tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR" $OUT/tests.log | tail -30
[ $rc -eq 0 ] || exit 1
for c in c1 c1g; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err \
    || { echo "bench $c failed"; tail -20 $OUT/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['value']/1e6,3), d['step_ms'], d['breakdown'])"
  DEIG_LIB_PATH=tools/ab_libs/libdeig_batchks.so timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $OUT/bench_${c}_batchks.json 2> $OUT/bench_${c}_batchks.err \
    || { echo "bench $c batchks failed"; tail -20 $OUT/bench_${c}_batchks.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_${c}_batchks.json')); print('$c batchks', round(d['value']/1e6,3), d['step_ms'], d['breakdown'])"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c1 -o tr -- python -u bench.py --config c1 --steps 2 --warmup 1 --no-cpu-baseline --no-alt > $OUT/trace_c1.log 2>&1 \
  || { echo "trace c1 failed"; tail -20 $OUT/trace_c1.log; exit 1; }
find $OUT/trace_c1 -name "*kernel_stats.csv" -exec cp {} $OUT/c1_kernel_stats.csv \;
find $OUT/trace_c1 -name "*kernel_trace.csv" -exec cp {} $OUT/c1_kernel_trace.csv \;
rm -rf $OUT/trace_c1
head -25 $OUT/c1_kernel_stats.csv
