#!/bin/bash
# r04x: the half-refill ring as the default - covariance tests, s_setprio variant A/B,
# then the PMC / SQ passes and the c3 line (tools/gpu_r04v.sh with TAG=r04x).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04x
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_gpu_syrk_chunks.py tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_f64flow.py > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u tools/syrk_ab.py --reps 5 shipped tools/ab_libs/libdeig_syrk30010.so > $OUT/syrk_ab.log 2>&1 || { tail -20 $OUT/syrk_ab.log; exit 1; }
grep -v amdgpu.ids $OUT/syrk_ab.log | cut -c1-200
TAG=r04x bash tools/gpu_r04v.sh
