# Interleaved A/B of the batched solve's stream-group count (measurement builds
# DEIG_AB_BATCH_GROUPS=3/4 vs the in-tree 2) on the c5 / c3 worker phases.
set -o pipefail
OUT=gpurun_out/${1:-groups_ab}
mkdir -p $OUT
DEIG_LIB_PATH=tools/ab_libs/libdeig_g4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_batch_solver.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $OUT/tests_g4.log 2>&1 || { tail -20 $OUT/tests_g4.log; exit 1; }
tail -1 $OUT/tests_g4.log
for c in c5 c3; do
  for lib in shipped tools/ab_libs/libdeig_g3.so tools/ab_libs/libdeig_g4.so shipped tools/ab_libs/libdeig_g3.so tools/ab_libs/libdeig_g4.so; do
    if [ $lib = shipped ]; then unset DEIG_LIB_PATH; else export DEIG_LIB_PATH=$lib; fi
    timeout -k 10 300 python -u tools/cu_split_probe.py serial --case $c --reps 3 2>&1 | grep -v amdgpu.ids >> $OUT/ab.log || exit 1
  done
done
