# A/B of the Rayleigh-Ritz small solve: phase timings (DEIG_DEBUG) with the
# residual-relative Jacobi threshold on (default) and off (DEIG_JACOBI_REL=0),
# then the solver / CIFAR / kernel GPU tests.
mkdir -p gpurun_out/rr2
for jr in def 0; do
  if [ $jr = def ]; then unset DEIG_JACOBI_REL; else export DEIG_JACOBI_REL=$jr; fi
  timeout -k 10 120 python -u tools/diag_rr_phases.py > gpurun_out/rr2/phases_$jr.log 2>&1 || exit 1
done
unset DEIG_JACOBI_REL
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solver_robust.py tests/test_gpu_cifar.py tests/test_gpu_kernels.py > gpurun_out/rr2/tests.log 2>&1 || exit 1
timeout -k 10 240 python -u bench.py --config c1 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/rr2/c1.json 2> gpurun_out/rr2/c1.err
