#!/bin/bash
# The GPU suite against A/B builds of libdeig (DEIG_LIB_PATH), one pytest process per
# build, each time-limited; stops at the first failing build.
# usage: bash tools/gpu_lib_tests.sh <tag> lib.so [lib.so ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for lib in "$@"; do
  name=$(basename $lib .so)
  DEIG_LIB_PATH=$R/$lib timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 240 \
    --timeout-method thread > $OUT/tests_$name.log 2>&1
  rc=$?
  echo "$name: $(tail -1 $OUT/tests_$name.log)"
  [ $rc -eq 0 ] || exit 1
done
