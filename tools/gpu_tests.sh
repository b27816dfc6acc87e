#!/bin/bash
# GPU tests in one process per group, each step time-limited; stops at the first
# step that fails (no retries).  usage: bash tools/gpu_tests.sh <tag> [pytest args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread \
  --durations=20 "$@" > $OUT/gputests.log 2>&1
rc=$?
tail -40 $OUT/gputests.log
exit $rc
