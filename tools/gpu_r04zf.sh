#!/bin/bash
# r04zf: resident Oja after the step-3 / step-4 restructure: its tests, the phase
# trace and the interleaved A/B against the two-pass path.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/${TAG:-r04zf}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_oja_resident.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 120 python -u tools/oja_trace.py > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
grep -v amdgpu.ids $OUT/trace.log
timeout -k 10 200 python -u tools/oja_resident_ab.py 7 > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
grep -v amdgpu.ids $OUT/ab.log
