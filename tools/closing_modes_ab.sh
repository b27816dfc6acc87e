# Interleaved A/B of the solver's closing-mode switch points (deig_solver_opts
# fast_until / round_until) on the c3 / c5 worker phases; measurement tooling.
set -o pipefail
OUT=gpurun_out/${1:-closing_ab}
mkdir -p $OUT
for c in c3 c5; do
  for rep in 1 2; do
    for o in "" "--opt fast_until=3e-4" "--opt fast_until=1e-4" "--opt round_until=1e-5" "--opt fast_until=1e-4 --opt round_until=1e-5"; do
      timeout -k 10 300 python -u tools/cu_split_probe.py serial --case $c --reps 3 $o 2>&1 | grep -v amdgpu.ids >> $OUT/ab.log || exit 1
    done
  done
done
