#!/bin/bash
# r03x: isolated traces of the c1 / c5 worker pieces (u8 covariance, RQ), u8 tests, c1 / c5 lines
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03x
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_u8.py tests/test_gpu_cifar.py tests/test_gpu_f64flow.py tests/test_gpu_general_solver.py tests/test_gpu_configs.py -q -x --timeout 240 --timeout-method thread > $OUT/gputests.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 $OUT/gputests.log; exit 1; }
tail -2 $OUT/gputests.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_parts -o p -- \
  python3 $R/tools/time_solve_parts.py > $OUT/parts.log 2>&1 || { echo "parts trace failed"; tail $OUT/parts.log; exit 1; }
cat $OUT/parts.log | grep -v amdgpu.ids
python3 -c "
import csv
r=list(csv.DictReader(open('$OUT/trace_parts/p_kernel_stats.csv')))
for x in r[:22]: print(x['Name'][:80], x['Calls'], round(float(x['AverageNs'])/1e3,2), x['Percentage'])
" | tee $OUT/parts_kernels.txt
cd $R
for c in c1 c5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-alt --steps 10 > $OUT/bench_$c.json 2> $OUT/bench_$c.err \
    || { echo "bench $c failed"; tail $OUT/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d['step_ms'], d['breakdown'])"
done
