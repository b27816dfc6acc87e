#!/bin/bash
# Rayleigh-Ritz spacing A/B (DEIG_RR_EVERY: sweeps per RR step while there are >= 16
# guard columns): c1 / c1g / c2 / c3 worker solves.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/${1:-rrevery}
mkdir -p $OUT
for e in 4 6 8; do
  for c in c1 c1g c2 c3; do
    DEIG_RR_EVERY=$e timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-alt > $OUT/b_${c}_$e.json 2> $OUT/b_${c}_$e.err || { tail $OUT/b_${c}_$e.err; exit 1; }
    python3 -c "import json; r=json.load(open('$OUT/b_${c}_$e.json')); a=r['accuracy']; print('rr_every=$e $c', round(r['value']), round(r['breakdown']['worker_eig_ms_per_worker'],3), r['breakdown']['worker_sweeps'], a.get('P_dist_last_worker_vs_f64_eigh'), a.get('sin_theta_server_vs_planted'), a['worker_resid'])"
  done
done
