#!/bin/bash
# r04z: after moving the fused-split threshold to d <= 2048 - the covariance / chunk
# GPU tests, the c2 bench line, then the PMC records for the new syrk_split.hip
# (tools/gpu_r04v.sh with TAG=r04z: c3 + c2 traffic, c3 SQ pass, c3 driver bench).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04z
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_syrk_chunks.py tests/test_gpu_kernels.py tests/test_gpu_configs.py > $OUT/cov_tests.log 2>&1 || { tail -30 $OUT/cov_tests.log; exit 1; }
tail -2 $OUT/cov_tests.log
timeout -k 10 400 python -u bench.py --config c2 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_c2.json')); print('c2', round(d['value']/1e6,3), d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('launch_ms'))"
TAG=r04z bash tools/gpu_r04v.sh
