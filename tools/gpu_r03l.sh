#!/bin/bash
# r03l: batched worker solves + Oja v3 tests, c1 / c1g / c4 bench lines, SYRK DMA-schedule A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03l
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_batch_solver.py tests/test_gpu_configs.py tests/test_gpu_distributed.py \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for c in c4 c1 c1g; do
  timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err \
    || { echo "bench $c failed"; tail $OUT/bench_$c.err; exit 1; }
  python3 -c "import json,sys; r=json.load(open('$OUT/bench_$c.json')); print('$c', r['value'], r['ms_per_step'], r.get('roofline',{}).get('frac'), r.get('breakdown'))"
done
bash tools/gpu_syrk_is.sh r03j 20000 20100 20010 20110
