#!/bin/bash
# r04zp: per-step kernel timeline of the c5 bench (batched worker solves): where the
# 8 x 12 ms of worker solve go.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r04zp
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/p -o p -- python3 -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-alt > $OUT/prof_c5.json 2> $OUT/prof_c5.err || { tail -20 $OUT/prof_c5.err; exit 1; }
f=$(find $OUT/p -name "*kernel_trace.csv" | head -1)
python3 tools/step_timeline.py $f --first-kernel split_kernel --per-step 8 > $OUT/timeline.txt
rm -rf $OUT/p
head -60 $OUT/timeline.txt
