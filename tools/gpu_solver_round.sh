#!/bin/bash
# Solver change check: solver / CIFAR / config / pipeline parity tests, RR phase
# log at the c1 / c2 shapes, then c1 and c1g bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/${1:-solver}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver_robust.py tests/test_gpu_cifar.py tests/test_gpu_configs.py tests/test_gpu_kernels.py tests/test_gpu_pipeline.py tests/test_gpu_u8.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 200 python -u tools/diag_rr_phases.py > $OUT/rr.log 2>&1 || { tail $OUT/rr.log; exit 1; }
grep "===\|deflated" $OUT/rr.log
for c in c1 c1g; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-alt > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail $OUT/bench_$c.err; exit 1; }
  python3 -c "import json; r=json.load(open('$OUT/bench_$c.json')); print('$c', r['value'], r['breakdown'], r['accuracy'])"
done
