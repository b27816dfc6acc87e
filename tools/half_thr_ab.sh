set -o pipefail
mkdir -p gpurun_out/r06bf
for c in c5 c3; do
  for h in 1e-2 5e-3 3e-3 1e-2 5e-3 3e-3; do
    timeout -k 10 300 python -u tools/cu_split_probe.py serial --case $c --reps 3 --half-until $h 2>&1 | grep -v amdgpu.ids >> gpurun_out/r06bf/thr.log || exit 1
  done
done
