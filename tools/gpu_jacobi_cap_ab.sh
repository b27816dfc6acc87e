#!/bin/bash
# Jacobi sweep cap A/B for the Rayleigh-Ritz small solve (DEIG_JACOBI_EARLY sweeps
# while the residual is above DEIG_JACOBI_EARLY_ABOVE): parity tests per setting,
# c1 / c2 bench lines.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-jcap}
mkdir -p $OUT
cd $R
# CFGS: space-separated sweeps:threshold pairs
for cfg in ${CFGS:-3:1e-2 2:1e-4 1:1e-3 2:1e-5}; do
  set -- ${cfg/:/ }
  tag=$1_$2
  DEIG_JACOBI_EARLY=$1 DEIG_JACOBI_EARLY_ABOVE=$2 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "topk or golden or robust or cifar or solver or sym_power" > $OUT/t_$tag.log 2>&1 || { echo "tests $tag failed"; tail -30 $OUT/t_$tag.log; exit 1; }
  echo "tests jcap=$1 above=$2: $(tail -1 $OUT/t_$tag.log)"
  for c in c1 c1g c2; do
    DEIG_JACOBI_EARLY=$1 DEIG_JACOBI_EARLY_ABOVE=$2 timeout -k 10 200 python -u bench.py --config $c --steps 3 --warmup 1 > $OUT/${c}_$tag.json 2> $OUT/${c}_$tag.err || { echo "bench $c failed"; tail $OUT/${c}_$tag.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/${c}_$tag.json') if l.startswith('{')][-1]); b=d['breakdown']; a=d['accuracy']; print('$c $tag', round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],2), 'ms/step eig/worker', round(b['worker_eig_ms_per_worker'],3), 'sweeps', b['worker_sweeps'], 'resid', a.get('worker_resid'), 'Pdist', a.get('P_dist_last_worker_vs_f64_eigh'))"
  done
done
