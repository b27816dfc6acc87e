#!/bin/bash
# r04zw: non-temporal split-pass stores - covariance GPU tests, the c2 bench line, then
# the PMC records of the new syrk_split.hip and the c3 driver bench (tools/gpu_r04v.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04zw
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_syrk_chunks.py tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_f64flow.py > $OUT/cov_tests.log 2>&1 || { tail -30 $OUT/cov_tests.log; exit 1; }
tail -1 $OUT/cov_tests.log
timeout -k 10 400 python -u bench.py --config c2 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_c2.json')); print('c2', round(d['value']/1e6,3), d['ms_per_step'], d['roofline'].get('frac'))"
TAG=r04zw bash tools/gpu_r04v.sh
