#!/bin/bash
# r04o: a looser rotation threshold in the capped (early) small solves, A/B against
# the shipped library: worker solves (tools/rr_ab.py) and the c1 / c5 bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04o
mkdir -p $OUT
for v in jrel4 jrel5; do
  timeout -k 10 400 python -u tools/rr_ab.py run --reps 5 --other tools/ab_libs/libdeig_$v.so > $OUT/rr_ab_$v.log 2>&1 || { tail -20 $OUT/rr_ab_$v.log; exit 1; }
  echo "## $v"; grep -v amdgpu.ids $OUT/rr_ab_$v.log | cut -c1-330
done
for c in c1 c5; do
  for v in shipped jrel4 jrel5; do
    if [ $v = shipped ]; then L=""; else L=tools/ab_libs/libdeig_$v.so; fi
    DEIG_LIB_PATH=$L timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $OUT/bench_${c}_$v.json 2> $OUT/bench_${c}_$v.err \
      || { echo "bench $c $v failed"; tail -20 $OUT/bench_${c}_$v.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_${c}_$v.json')); print('$c $v', round(d['value']/1e6,3), round(d['step_ms']['median'],3), round(d['breakdown']['worker_eig_ms_per_worker'],3), d['breakdown']['worker_sweeps'], d.get('accuracy'))"
  done
done
