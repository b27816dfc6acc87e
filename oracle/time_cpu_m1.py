"""Test / measurement infrastructure (bench.py cpu_baseline leg only): times the float64
oracle's one-worker path (ref_cpu.sigma_hat = reference/distributed.py:59-70, then
ref_cpu.top_k_eigh = :22-29) on a sample saved by bench.py, in a CHILD process whose
BLAS thread count is fixed by the environment before numpy loads.

Why a child: OpenBLAS sizes its thread buffers when it initialises (OMP_NUM_THREADS,
16 on the GPU box); raising the count later with threadpool_limits crashed the
bench process on the 256-CPU host.  Never touches the GPU.

usage: python oracle/time_cpu_m1.py SAMPLE.npy K EIG_D  -> one JSON line on stdout
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    path, k, eig_d = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    import numpy as np

    from oracle import ref_cpu
    try:
        from threadpoolctl import threadpool_info
        threads = max((i.get("num_threads", 1) for i in threadpool_info()
                       if i.get("user_api") == "blas"), default=None)
    except Exception:  # pragma: no cover
        threads = None
    xs = np.load(path, allow_pickle=False)
    ref_cpu.top_k_eigh(np.eye(8) + 0.1, 2)  # first-call (lazy load) costs out of the timing
    ref_cpu.sigma_hat(xs[:64])
    t0 = time.perf_counter()
    S = ref_cpu.sigma_hat(xs)
    t_cov = time.perf_counter() - t0
    t0 = time.perf_counter()
    ref_cpu.top_k_eigh(S[:eig_d, :eig_d], k)
    t_eig = time.perf_counter() - t0
    print(json.dumps({"t_cov_s": t_cov, "t_eig_s": t_eig, "blas_threads": threads}), flush=True)


if __name__ == "__main__":
    main()
