#!/bin/bash
# r04zv: (1) non-temporal split-pass stores vs shipped (config-3 shard, config 2);
# (2) the CholQR apply as a triangular solve with the image fused (trsm_img_kernel)
# vs the inverse + skinny apply + img_kernel: Oja GPU tests, interleaved config-4 A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/r04zv
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_oja_resident.py tests/test_gpu_configs.py tests/test_gpu_distributed.py -k "oja or c4 or Oja" > $OUT/oja_tests.log 2>&1 || { tail -30 $OUT/oja_tests.log; exit 1; }
tail -1 $OUT/oja_tests.log
timeout -k 10 200 python -u tools/oja_lib_ab.py 7 shipped tools/ab_libs/libdeig_pretrsm.so > $OUT/oja_trsm_ab.log 2>&1 || { tail -20 $OUT/oja_trsm_ab.log; exit 1; }
grep -v amdgpu.ids $OUT/oja_trsm_ab.log
timeout -k 10 400 python -u tools/syrk_ab.py --n 2097152 --d 8192 --reps 5 shipped tools/ab_libs/libdeig_splitnt.so > $OUT/split_nt_c3.log 2>&1 || { tail -20 $OUT/split_nt_c3.log; exit 1; }
timeout -k 10 300 python -u tools/syrk_ab.py --n 1048576 --d 3072 --reps 7 shipped tools/ab_libs/libdeig_splitnt.so > $OUT/split_nt_c2.log 2>&1 || { tail -20 $OUT/split_nt_c2.log; exit 1; }
grep -hv amdgpu.ids $OUT/split_nt_c3.log $OUT/split_nt_c2.log | cut -c1-200
