#!/bin/bash
# r04zn: parallel diag_corr_kernel - covariance GPU tests, the c2 bench line, then the
# PMC records of the new syrk_split.hip and the c3 driver bench (tools/gpu_r04v.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04zn
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_syrk_chunks.py tests/test_gpu_kernels.py tests/test_gpu_f64flow.py > $OUT/cov_tests.log 2>&1 || { tail -30 $OUT/cov_tests.log; exit 1; }
tail -2 $OUT/cov_tests.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/p -o p -- python3 -u bench.py --config c2 --no-cpu-baseline > $OUT/prof_c2.json 2> $OUT/prof_c2.err || { tail -20 $OUT/prof_c2.err; exit 1; }
f=$(find $R/$OUT/p -name "*kernel_stats.csv" | head -1); cp $f $OUT/c2_kernel_stats.csv; rm -rf $R/$OUT/p
grep -E "diag_corr|syrks_h|split_kernel" $OUT/c2_kernel_stats.csv | cut -c1-140
timeout -k 10 400 python -u bench.py --config c2 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_c2.json')); print('c2', round(d['value']/1e6,3), d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('launch_ms'))"
TAG=r04zn bash tools/gpu_r04v.sh
