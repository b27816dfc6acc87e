#!/bin/bash
# r03y: isolated worker-piece trace, then the full round (GPU tests, smoke, driver bench, configs)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03y
mkdir -p $OUT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_parts -o p -- \
  python3 $R/tools/time_solve_parts.py > $OUT/parts.log 2>&1 || { echo "parts trace failed"; tail $OUT/parts.log; exit 1; }
grep -v amdgpu.ids $OUT/parts.log | grep solve
cd $R
DRIVER=1 bash tools/gpu_round.sh r03y c1 c1g c4 c2 c5
