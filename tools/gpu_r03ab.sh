#!/bin/bash
# r03ab: final-tree round (symmetric-half RQ): GPU tests, smoke, driver bench, configs;
# then the batched vs threaded worker A/B at c5 / c1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
DRIVER=1 bash tools/gpu_round.sh r03ab c1 c1g c4 c2 c5 || exit 1
OUT=$R/gpurun_out/r03ab
for c in c5 c1; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-alt --steps 10 --threaded-workers > $OUT/ab_${c}_threaded.json 2> $OUT/ab_${c}_threaded.err \
    || { echo "bench $c threaded failed"; tail $OUT/ab_${c}_threaded.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/ab_${c}_threaded.json')); print('$c threaded', round(d['value']/1e6,3), round(d['step_ms']['median'],2), round(d['step_ms']['spread_pct'],1), d['breakdown']['syrk_ms_per_worker'], d['breakdown']['worker_eig_ms_per_worker'])"
done
