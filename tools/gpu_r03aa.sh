#!/bin/bash
# r03aa: GPU tests (symmetric-half RQ), then worker-mode A/B (batched vs threaded Slave workers) at c5 / c1 / c1g on the final kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03aa
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread > $OUT/gputests.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 $OUT/gputests.log; exit 1; }
tail -1 $OUT/gputests.log
for rep in 1; do
for m in "" "--threaded-workers"; do
  for c in c5 c1 c1g; do
    timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-alt --steps 10 $m > $OUT/ab_${c}${m}_$rep.json 2> $OUT/ab_${c}${m}_$rep.err \
      || { echo "bench $c $m failed"; tail $OUT/ab_${c}${m}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/ab_${c}${m}_$rep.json')); print('$c', '$m', round(d['value']/1e6,3), round(d['step_ms']['median'],2), round(d['step_ms']['spread_pct'],1), d['breakdown']['syrk_ms_per_worker'], d['breakdown']['worker_eig_ms_per_worker'], d['accuracy'].get('sigma_hat_rel_err_vs_f64_sampled'))"
  done
done
done
