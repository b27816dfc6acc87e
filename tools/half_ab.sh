# Interleaved A/B of the solver's one-product early sweeps (deig_solver_opts.half_until)
# on the c5 and c3 worker phases (covariances + batched solves): python processes in
# turn, off / on / off / on.  Measurement tooling; output gpurun_out/half_ab/half_ab.log.
set -o pipefail
mkdir -p gpurun_out/half_ab
for c in c5 c3; do
  for h in 0 1e-2 0 1e-2; do
    timeout -k 10 300 python -u tools/cu_split_probe.py serial --case $c --reps 3 --half-until $h 2>&1 \
      | grep -v amdgpu.ids >> gpurun_out/half_ab/half_ab.log || exit 1
  done
done
