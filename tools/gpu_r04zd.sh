#!/bin/bash
# r04zd: first GPU run of the block-resident Oja kernel - its tests (vs the two-pass
# path and ref_cpu.oja_epoch, NaN-poisoned workspace), then the interleaved A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04zd
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_oja_resident.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -8 $OUT/tests.log
timeout -k 10 200 python -u tools/oja_resident_ab.py 7 > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
grep -v amdgpu.ids $OUT/ab.log
