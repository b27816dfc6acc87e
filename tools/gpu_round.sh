#!/bin/bash
# One GPU-box pass: parity tests, then bench lines.  Each step has its own time
# limit; the first failure ends the script (no retries).
# usage: [DRIVER=1] [GLOO=1] bash tools/gpu_round.sh <tag> [configs...]
#   DRIVER=1: also the driver's exact bench command (python bench.py --gpus 1
#             --steps 20 --warmup 5, default config c3)
#   GLOO=1:   also a 2-rank gloo rehearsal of the N > 1 path (c2, ranks share cuda:0)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  --durations=15 > $OUT/gputests.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -40 $OUT/gputests.log; exit 1; }
tail -3 $OUT/gputests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
  || { echo "smoke failed rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
if [ "${DRIVER:-0}" = 1 ]; then
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json \
    2> $OUT/bench_driver.err || { echo "driver bench failed rc=$?"; tail -20 $OUT/bench_driver.err; exit 1; }
  cat $OUT/bench_driver.json
fi
if [ "${GLOO:-0}" = 1 ]; then
  timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --config c2 --steps 3 --warmup 1 \
    > $OUT/bench_gloo2_c2.json 2> $OUT/bench_gloo2_c2.err \
    || { echo "gloo bench failed rc=$?"; tail -20 $OUT/bench_gloo2_c2.err; exit 1; }
  cat $OUT/bench_gloo2_c2.json
fi
for c in "$@"; do
  timeout -k 10 420 python -u bench.py --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err \
    || { echo "bench $c failed rc=$?"; tail -20 $OUT/bench_$c.err; exit 1; }
  cat $OUT/bench_$c.json
done
