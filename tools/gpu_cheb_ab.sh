set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; OUT=gpurun_out/r02p_cheb; mkdir -p $OUT
for a in 0.01 0.1 0.3; do
  DEIG_CHEB_ABOVE=$a timeout -k 10 400 python -u -m pytest tests/test_gpu_solver_robust.py tests/test_gpu_cifar.py tests/test_gpu_configs.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t_$a.log 2>&1 || { echo "tests failed at $a"; tail -20 $OUT/t_$a.log; exit 1; }
  echo "cheb_above=$a tests: $(tail -n 1 $OUT/t_$a.log)"
  for c in c1 c1g c2; do
    DEIG_CHEB_ABOVE=$a timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-alt > $OUT/b_${c}_$a.json 2> $OUT/b_${c}_$a.err || { tail $OUT/b_${c}_$a.err; exit 1; }
    python3 -c "import json; r=json.load(open('$OUT/b_${c}_$a.json')); a=r['accuracy']; print('  $c', round(r['value']), round(r['breakdown']['worker_eig_ms_per_worker'],3), r['breakdown']['worker_sweeps'], a.get('P_dist_last_worker_vs_f64_eigh'), a.get('sin_theta_server_vs_planted'), a['worker_resid'])"
  done
done
