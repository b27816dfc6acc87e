#!/bin/bash
# r04g: pipelined split pass (split of chunk c + 1 on a side stream under the SYRK of
# chunk c) - interleaved A/B against the sequential pass and 8 chunks at the config-3
# shard, the covariance tests, then the c3 bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04g
mkdir -p $OUT
timeout -k 10 300 python -u tools/syrk_ab.py --reps 4 shipped tools/ab_libs/libdeig_pipe1.so tools/ab_libs/libdeig_pipe8.so > $OUT/syrk_ab.log 2>&1 \
  || { tail -20 $OUT/syrk_ab.log; exit 1; }
cat $OUT/syrk_ab.log
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_gpu_syrk_chunks.py tests/test_gpu_kernels.py > $OUT/tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR" $OUT/tests.log | tail -30
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err \
  || { echo "bench failed"; tail -20 $OUT/bench_c3.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_c3.json')); print('c3', round(d['value']/1e6,3), d['roofline']['launch_ms'], d['roofline']['frac'], d['step_ms'])"
