#!/bin/bash
# r03ae: LDS-transposed mirror stores in the direct uint8 SYRK: u8 / CIFAR / f64-flow tests, isolated trace, c1 / c1g
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03ae
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_u8.py tests/test_gpu_cifar.py tests/test_gpu_f64flow.py -q -x --timeout 240 --timeout-method thread > $OUT/gputests.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 $OUT/gputests.log; exit 1; }
tail -1 $OUT/gputests.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_parts -o p -- \
  python3 $R/tools/time_solve_parts.py > $OUT/parts.log 2>&1 || { echo "parts trace failed"; tail $OUT/parts.log; exit 1; }
python3 -c "
import csv
r=list(csv.DictReader(open('$OUT/trace_parts/p_kernel_trace.csv')))
print('u8_syrk us', [round((int(x['End_Timestamp'])-int(x['Start_Timestamp']))/1e3,1) for x in r if 'u8_syrk' in x['Kernel_Name']])
"
cd $R
for c in c1 c1g; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-alt --steps 10 > $OUT/bench_$c.json 2> $OUT/bench_$c.err \
    || { echo "bench $c failed"; tail $OUT/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['value']/1e6,3), round(d['step_ms']['median'],2), d['breakdown']['syrk_ms_per_worker'])"
done
