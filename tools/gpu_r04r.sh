#!/bin/bash
# r04r: solver schedule options (Chebyshev from higher residuals, RR spacing, early
# Jacobi cap) at the c5 / c3 / c1 worker shapes against float64 eigh.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04r
mkdir -p $OUT
timeout -k 10 600 python -u tools/solver_opts_sweep.py --reps 3 --cases c5n,c3,c2,c1 > $OUT/opts.log 2>&1
rc=$?
grep -v amdgpu.ids $OUT/opts.log
exit $rc
