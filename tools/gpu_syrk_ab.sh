#!/bin/bash
# SYRK variant A/B on the GPU box: split3 parity tests, then interleaved timing of
# the given settings (tools/time_syrk_variants.py) at config-3 and config-2 shapes.
# usage: bash tools/gpu_syrk_ab.sh <tag> [settings...]   (default: 163 162)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-syrkab}; shift
SET=${*:-163 162}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "syrk or worker_path" > $OUT/t.log 2>&1 || { echo "tests failed"; tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 300 python -u tools/time_syrk_variants.py 2097152 8192 $SET > $OUT/ab_c3.log 2>&1 \
  || { echo "ab c3 failed"; tail -20 $OUT/ab_c3.log; exit 1; }
cat $OUT/ab_c3.log
timeout -k 10 120 python -u tools/time_syrk_variants.py 1048576 3072 $SET > $OUT/ab_c2.log 2>&1 \
  || { echo "ab c2 failed"; tail -20 $OUT/ab_c2.log; exit 1; }
cat $OUT/ab_c2.log
