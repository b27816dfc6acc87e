#!/bin/bash
# r04zh: the resident Oja path as the c4 default - every Oja GPU test, the c4 bench
# line and its rocprof kernel summary.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r04zh
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_oja_resident.py tests/test_gpu_configs.py tests/test_gpu_distributed.py -k "oja or c4 or Oja" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 400 python -u bench.py --config c4 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -20 $OUT/bench_c4.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_c4.json')); print('c4', round(d['value']/1e6,2), 'M/s', d['roofline']['frac'], d['breakdown'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p -o p -- python3 -u bench.py --config c4 --no-cpu-baseline > $OUT/prof_c4.json 2> $OUT/prof_c4.err || { tail -20 $OUT/prof_c4.err; exit 1; }
f=$(find $OUT/p -name "*kernel_stats.csv" | head -1); cp $f $OUT/c4_kernel_stats.csv; rm -rf $OUT/p
head -8 $OUT/c4_kernel_stats.csv | cut -c1-160
