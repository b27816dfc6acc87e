#!/bin/bash
# One GPU-box pass: parity tests, then bench lines.  Each step has its own time
# limit; the first failure ends the script (no retries).
# usage: bash tools/gpu_round.sh <tag> [configs...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > $OUT/gputests.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $OUT/gputests.log; exit 1; }
tail -3 $OUT/gputests.log
for c in "$@"; do
  timeout -k 10 420 python -u bench.py --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err \
    || { echo "bench $c failed rc=$?"; tail -20 $OUT/bench_$c.err; exit 1; }
  cat $OUT/bench_$c.json
done
