set -o pipefail
mkdir -p gpurun_out/r06ax
for c in c5 c3; do
for lib in shipped tools/ab_libs/libdeig_half_1e-2.so tools/ab_libs/libdeig_half_3e-2.so shipped; do
  if [ $lib = shipped ]; then unset DEIG_LIB_PATH; else export DEIG_LIB_PATH=$lib; fi
  timeout -k 10 300 python -u tools/cu_split_probe.py serial --case $c --reps 3 2>&1 | grep -v amdgpu.ids >> gpurun_out/r06ax/half_ab.log || exit 1
done
done
