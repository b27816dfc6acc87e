#!/usr/bin/env python
"""Benchmark: distributed eigenspace estimation on MI355X.

Default workload (BASELINE.json configs[2], the metric's "d=8192, k=64" config):
each GPU holds one worker's shard of 2^21 synthetic spiked-covariance rows x
d = 8192 (fp32, 64 GiB, resident in HBM before timing); k = 64.  At N GPUs the
job covers N * 2^21 rows (N = 8 -> 16,777,216 = config 3), so scaling is "weak".

One step of a one-shot config = time-to-eigenspace of the whole pipeline:
  workers: Sigma_hat = X^T X / n (SYRK kernel) -> top-k eigenpairs (subspace
  iteration), W logical workers per GPU back to back ; exchange: all-gather of
  the d x k bases (RCCL, N > 1) ; server: top-k of the projector average
  (implicit operator) on rank 0.
value = samples ingested per second over the whole job = N * rows / t_step.

Other configs (--config; each prints its own JSON line, the driver's default
line is c3):
  c2  configs[1]: d = 3072, n = 2^20 rows per GPU, k = 16, one worker per GPU;
  c5  configs[4] (stress) per GPU: 8 logical workers x 65,536 rows, d = 16384,
      k = 128 (64 workers on 8 GPUs); server over all workers' bases;
  c1  configs[0] shape: 50,000 x 3072 uint8 bytes per GPU, 8 logical workers,
      k = 10, exact int8-MFMA covariance of the bytes (csrc/syrk_u8.hip);
  c1g the reference's own CIFAR preprocessing: 60,000 x 32x32x3 uint8 pixels,
      grayscale fused into the covariance (d = 1024), 8 workers, k = 10;
  c4  configs[3] (online): per GPU a stream of 4096 x 3072 batches, Oja steps
      (k = 32), aggregation (all-gather + server solve + broadcast) every 64
      batches; one step = 64 batches + one aggregation.

Extra objects on the JSON line: ``roofline`` (the dominant kernel vs the peak of
the instructions it runs, timed with HIP events on the launch stream),
``sweep`` (one subspace-iteration sweep S*Q vs the HBM roof, both sweep
kernels), ``cpu_baseline`` (the float64 oracle on a bounded sample of the same
workload, rank 0 at N = 1 only), ``breakdown`` and ``accuracy``.

Covariance algorithm (--syrk-algo, default auto = split3 at these sizes): fp32
samples split into bf16 hi/lo pairs, 3 bf16 MFMA products per fp32 product,
fp32 accumulation (include/deig.h); "fp32" = the f32 MFMA kernel.  The fp32
kernel is also timed once outside the timed region (``roofline.fp32_kernel``).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c1|c1g|c4|c5]
       [--syrk-algo auto|split3|fp32]
       (N > 1: either under python -m torch.distributed.run --nproc-per-node N, or
       plain ``python bench.py --gpus N``, which starts the N ranks itself)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
FP32_MFMA_PEAK = 157.3e12  # MI355X_MICROARCH.md: FP32 matrix, dense
BF16_MFMA_PEAK = 2.5e15    # MI355X_MICROARCH.md: BF16 MFMA, dense (16 x the f32 rate)
I8_MFMA_PEAK = 5.0e15      # MI355X_MICROARCH.md: I8 MFMA = 2 x BF16 per clock, dense
HBM_PEAK = 8.0e12

CONFIGS = {
    "c3": dict(kind="oneshot", rows=1 << 21, d=8192, k=64, workers=1, full_rows=1 << 24,
               label="synthetic spiked d=8192 k=64, 2^21 rows/GPU (config 3 shard)"),
    "c2": dict(kind="oneshot", rows=1 << 20, d=3072, k=16, workers=1,
               label="synthetic spiked d=3072 n=2^20 k=16 per GPU (config 2)"),
    "c5": dict(kind="oneshot", rows=8 * 65536, d=16384, k=128, workers=8,
               label="stress: synthetic spiked d=16384 k=128, 8 logical workers x 65536 rows "
                     "per GPU (config 5)"),
    "c1": dict(kind="oneshot", rows=50000, d=3072, k=10, workers=8, u8="raw",
               label="configs[0] shape: CIFAR-10 train 50000 x 3072 uint8 bytes (synthetic "
                     "spiked), 8 threaded workers, k=10, exact int8-MFMA covariance"),
    "c1g": dict(kind="oneshot", rows=60000, d=1024, k=10, workers=8, u8="gray",
                label="CIFAR-10 60000 x 32x32x3 uint8 pixels (synthetic spiked) grayscaled "
                      "in the covariance kernel (distributed.py:170-173), 8 threaded workers, k=10"),
    # orth_every 16 (r05, tools/oja_orth_sweep.py over one 64-batch span vs the float64
    # per-batch-orthonormalised oracle): ||P - P_oracle||_F 1.6e-5 (8: 1.1e-5, 32: 2.8e-5,
    # 64: 2.2e-4 - over the 1e-4 bar), 29.1 us per batch (8: 33.0)
    "c4": dict(kind="oja", rows=4096, d=3072, k=32, agg_every=64, eta=0.02, orth_every=16,
               label="online: Oja mini-batches 4096 x 3072, k=32, aggregation every 64 "
                     "batches (config 4)"),
}
EIGH_MAX_D = 8192  # CPU baseline: larger d times eigh on a leading block and scales by d^3
THREADED_EIGH_MAX_D = 3072  # same for the m concurrent eighs of the threaded variant


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def blas_cores():
    try:
        from threadpoolctl import threadpool_info
        return max((i.get("num_threads", 1) for i in threadpool_info()
                    if i.get("user_api") == "blas"), default=os.cpu_count())
    except Exception:  # pragma: no cover
        return os.cpu_count()


def blas_max_threads() -> int:
    """The smallest compiled thread limit (MAX_THREADS) of the OpenBLAS libraries
    numpy / scipy load (64 if it cannot be read)."""
    import ctypes
    import re
    lim = []
    try:
        import scipy.linalg  # noqa: F401
        from threadpoolctl import threadpool_info
        for i in threadpool_info():
            if i.get("internal_api") != "openblas":
                continue
            lib = ctypes.CDLL(i["filepath"])
            for fn in ("openblas_get_config", "openblas_get_config64_", "scipy_openblas_get_config64_",
                       "scipy_openblas_get_config"):
                f = getattr(lib, fn, None)
                if f is None:
                    continue
                f.restype = ctypes.c_char_p
                m = re.search(rb"MAX_THREADS=(\d+)", f() or b"")
                if m:
                    lim.append(int(m.group(1)))
                break
    except Exception:  # pragma: no cover
        pass
    return min(lim) if lim else 64


def host_info() -> dict:
    """The host the CPU baseline ran on (nproc, CPU model,
    BLAS vendor and version): ``cores`` on a cpu_baseline is the BLAS thread count
    actually used, which is below nproc where OMP_NUM_THREADS caps it (16 on the GPU box)."""
    blas = []
    try:
        import scipy.linalg  # noqa: F401  (scipy's own OpenBLAS, used by the oracle's eigh)
        from threadpoolctl import threadpool_info
        blas = [{"vendor": i.get("internal_api"), "version": i.get("version"),
                 "library": i.get("prefix"), "threads": i.get("num_threads"),
                 "architecture": i.get("architecture")}
                for i in threadpool_info() if i.get("user_api") == "blas"]
    except Exception:  # pragma: no cover
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):  # pragma: no cover
        affinity = None
    return {"nproc": os.cpu_count(), "cpus_in_affinity_mask": affinity,
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"), "blas": blas}


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threaded_oneshot(xs: np.ndarray, n_total: int, k: int, m: int, cores: int,
                         eig_d: int) -> dict:
    """The reference's threaded CPU path (my_threading.Slave workers, each running
    distributed.py:59-70 then :22-29 on its own shard), m Slave threads with
    OPENBLAS threads = cores // m each: the same ``n_total`` rows split over m
    workers.  Timed on the bounded sample ``xs`` in two phases (all covariances,
    then all eighs, each joined); the covariance phase is scaled linearly in rows,
    the eigh phase by (d / eig_d)^3 when it runs on a leading eig_d block."""
    from threadpoolctl import threadpool_limits

    from distributed_eigenspaces_amd.my_threading import Slave
    from oracle import ref_cpu
    d = xs.shape[1]
    shards = np.array_split(xs, m)
    Ss = [None] * m
    with threadpool_limits(limits=max(1, cores // m), user_api="blas"):
        def cov(i):
            Ss[i] = ref_cpu.sigma_hat(shards[i])

        def eig(i):
            ref_cpu.top_k_eigh(Ss[i][:eig_d, :eig_d], k)

        def phase(fn):
            t0 = time.perf_counter()
            ts = [Slave(fn, i) for i in range(m)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            return time.perf_counter() - t0

        t_cov = phase(cov)
        t_eig = phase(eig) * (d / eig_d) ** 3
    t = t_cov * (n_total / xs.shape[0]) + t_eig
    return {"value": n_total / t, "threads": m, "blas_threads_per_worker": max(1, cores // m),
            "t_cov_sample_s": t_cov, "t_eig_s": t_eig, "t_total_s": t,
            "note": (f"{m} my_threading.Slave workers x {max(1, cores // m)} BLAS threads on "
                     f"{xs.shape[0]} rows ({xs.shape[0] // m} per worker): covariance phase "
                     f"{t_cov:.2f}s scaled to {n_total} rows; {m} concurrent top-{k} eighs"
                     + (f" of the leading {eig_d}x{eig_d} block, x (d/{eig_d})^3" if eig_d < d
                        else "") + f" -> {t_eig:.1f}s")}


def cpu_m1_child(xs: np.ndarray, k: int, eig_d: int, threads: int) -> dict | None:
    """oracle/time_cpu_m1.py on ``xs`` in a child process with ``threads`` BLAS threads
    (no GPU use in the child); None if it fails."""
    import subprocess
    import tempfile
    env = dict(os.environ, OMP_NUM_THREADS=str(threads), OPENBLAS_NUM_THREADS=str(threads))
    env.pop("CUDA_VISIBLE_DEVICES", None)
    env["HIP_VISIBLE_DEVICES"] = ""  # the child never touches the GPU
    with tempfile.TemporaryDirectory() as tdir:
        path = os.path.join(tdir, "sample.npy")
        np.save(path, xs)
        try:
            r = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "time_cpu_m1.py"), path,
                                str(k), str(eig_d)], env=env, capture_output=True, text=True,
                               timeout=600)
        except subprocess.TimeoutExpired:
            log("cpu baseline child: timed out")
            return None
    if r.returncode != 0:
        log(f"cpu baseline child failed ({r.returncode}): {r.stderr[-500:]}")
        return None
    return json.loads(r.stdout.strip().splitlines()[-1])


def cpu_baseline_oneshot(xs: np.ndarray, n_worker: int, workers: int, k: int,
                         threads: int = 8):
    """Float64 oracle (oracle/ref_cpu.py) on ``xs``, the first rows of a worker
    shard as the reference's float64 features, two variants:

    * m = 1 worker x all BLAS cores: covariance scaled linearly to the full shard
      (it is linear in n), the top-k eigh timed once and counted per worker;
    * m = ``threads`` my_threading.Slave workers x cores/m BLAS threads each over
      the same rows (cpu_threaded_oneshot).

    ``value`` is the better of the two; both are reported."""
    sample_rows, d = xs.shape
    cores = int(blas_cores())
    de = min(d, EIGH_MAX_D)

    def m1_result(t_cov, t_eig, used, extra=""):
        t_eig = t_eig * (d / de) ** 3
        t_worker = t_cov * (n_worker / sample_rows) + t_eig
        eig_note = (f"eigh top-{k} {t_eig:.2f}s" if de == d else
                    f"eigh top-{k} of the leading {de}x{de} block scaled by (d/{de})^3 -> "
                    f"{t_eig:.1f}s")
        return {"value": workers * n_worker / (workers * t_worker), "threads": 1,
                "blas_threads_per_worker": used,
                "note": (f"1 worker x {used} BLAS threads on {sample_rows} rows x d={d} of a "
                         f"worker shard: sigma_hat {t_cov:.2f}s + {eig_note}; covariance scaled "
                         f"linearly to {n_worker} rows -> {t_worker:.1f}s per worker shard, x "
                         f"{workers} worker(s){extra}")}

    from oracle import ref_cpu
    t0 = time.perf_counter()
    S = ref_cpu.sigma_hat(xs)
    t_cov = time.perf_counter() - t0
    t0 = time.perf_counter()
    ref_cpu.top_k_eigh(S[:de, :de], k)
    t_eig = time.perf_counter() - t0
    del S
    single = m1_result(t_cov, t_eig, cores)
    # SURVEY.md §8(d)'s "m = 1 x all cores": every CPU of the host up to the BLAS's
    # compiled limit (numpy / scipy's OpenBLAS: MAX_THREADS=64), in a child process
    # whose thread count is set before numpy loads (raising it in this process with
    # threadpool_limits crashed OpenBLAS on the 256-CPU GPU host)
    nproc = os.cpu_count() or 1
    want = min(nproc, blas_max_threads())
    allc = None
    if want > cores:
        allc = cpu_m1_child(xs, k, de, want)
        if allc is not None:
            allc = m1_result(allc["t_cov_s"], allc["t_eig_s"], allc.get("blas_threads") or want,
                             f" (child process, OPENBLAS_NUM_THREADS={want}; host nproc {nproc}, "
                             f"BLAS MAX_THREADS {blas_max_threads()})")
    threaded = None
    if threads > 1:
        threaded = cpu_threaded_oneshot(xs, workers * n_worker, k, threads, cores,
                                        min(d, THREADED_EIGH_MAX_D))
    cands = [v for v in (single, allc, threaded) if v is not None]
    best = max(cands, key=lambda v: v["value"])
    return {
        "value": best["value"], "unit": "samples/s", "cores": best["blas_threads_per_worker"]
        * best["threads"], "kind": "port",
        "cpu_model": cpu_model(), "host": host_info(),
        "sample": (f"float64 NumPy/SciPy oracle (distributed.py:59-70 + :22-29) on a bounded "
                   f"sample; best of: " + " and ".join(f"[{v['note']}]" for v in cands)
                   + "; server solve not counted"),
        "variants": {"m1_default_threads": single, "m1_all_cores": allc,
                     f"m{threads}_slave_threads": threaded},
    }


def cpu_baseline_oja(pool, V0: torch.Tensor, eta: float, nb: int):
    from oracle import ref_cpu
    xs = np.concatenate([pool[i].double().cpu().numpy() for i in range(nb)])
    b = pool[0].shape[0]
    t0 = time.perf_counter()
    ref_cpu.oja_epoch(xs, V0.double().cpu().numpy(), eta, b)
    t = time.perf_counter() - t0
    return {
        "value": nb * b / t, "unit": "samples/s", "cores": int(blas_cores()), "kind": "port",
        "cpu_model": cpu_model(), "host": host_info(),
        "sample": (f"float64 NumPy oracle oja_epoch on {nb} batches of {b} x {xs.shape[1]} "
                   f"(k={V0.shape[1]}): {t:.2f}s; aggregation not counted"),
    }


def sin_theta(U: torch.Tensor, V: torch.Tensor) -> float:
    s = torch.linalg.svdvals(U.double().t() @ V.double()).min().clamp(max=1)
    return float(s.pow(2).neg().add(1).clamp(min=0).sqrt())


def time_events(fn, reps: int, stream, trials: int = 1) -> float:
    """Mean ms of fn() over reps launches, HIP events on ``stream``; with trials > 1
    the best of that many such means (the microsecond-scale sweep figures: one
    trial can catch a clock or scheduling dip, r02p's 92.8 us kernel-only sweep)."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    best = float("inf")
    for _ in range(trials):
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps)
    return best


SIGMA_SAMPLED_BAR = 2e-6   # sampled Sigma_hat vs float64 (north_star SYRK bar)
EVAL_REL_BAR = 1e-5        # north_star: top-k eigenvalues to 1e-5 relative


def spiked_block_fn(synthetic, U, first_seed: int = 1, seed0: int = 1000):
    """Row block b of the streamed 16M-row job, generated in place: block 0 is the
    bench shard itself (seed ``first_seed``), block b > 0 seed ``seed0 + b``."""
    def gen(b, out):
        synthetic.spiked_samples(out.shape[0], U, seed=first_seed if b == 0 else seed0 + b,
                                 out=out)
    return gen


def full_time_to_eigenspace(de, gen_block, X, U, n_total: int, k: int, stream,
                            keep_S: bool = False, f64_check: bool = True) -> dict:
    """BASELINE.json north_star's literal target on ONE GPU: the top-k eigenspace of
    n_total = 16,777,216 rows of d = 8192 (reference/distributed.py:66-69 forms
    Sigma_hat of any n in one call, then :22-29 its top-k).  The rows do not fit in HBM
    (512 GiB of fp32), so they stream through the covariance in blocks of X's rows,
    each block accumulated into one Sigma (block 0 overwrites S, the others
    DEIG_SYRK_ACCUMULATE; ``gen_block(b, X)`` regenerates block b in place - a
    data-arrival stand-in, untimed), then one eigensolve.

    Timed: each block's ONE covariance launch (one HIP event pair on the launch
    stream around the single call - r04 timed it with ``time_events``, whose warm-up
    call accumulated every block twice, S = 2 Sigma_hat) + the solve.

    Checked (outside the timed launches; raises if a bar is missed): a float64 X^T X
    of 16 sampled features over all rows vs the same entries of S (<= 2e-6), and -
    after the solve, with the blocks regenerated - the float64 Rayleigh quotients
    v_j^T Sigma v_j and residuals ||Sigma v_j - rq_j v_j|| / lambda_max of the returned
    vectors on the float64 Sigma of ALL rows (never formed: X V, then X^T (X V),
    block by block), against the returned eigenvalues (<= 1e-5 relative)."""
    n, d = X.shape
    blocks = n_total // n
    S = torch.empty((d, d), dtype=torch.float32, device=X.device)
    cols = torch.randperm(d, generator=torch.Generator().manual_seed(7))[:16].to(X.device)
    S64 = torch.zeros((16, 16), dtype=torch.float64, device=X.device)
    syrk_ms = []
    for b in range(blocks):
        gen_block(b, X)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        de.sigma_hat(X, alpha=1.0 / n_total, out=S, accumulate=b > 0)
        e1.record(stream)
        e1.synchronize()
        syrk_ms.append(e0.elapsed_time(e1))
        Xc = X.index_select(1, cols).double()
        S64 += Xc.t() @ Xc
        del Xc
    torch.cuda.synchronize()
    S64 /= n_total
    Sblk = S.index_select(0, cols).index_select(1, cols).double()
    sigma_err = float((Sblk - S64).abs().max() / S64.abs().max())
    t0 = time.perf_counter()
    r = de.topk_eigh(S, k, check_finite=False)
    torch.cuda.synchronize()
    solve_s = time.perf_counter() - t0
    cov_s = float(sum(syrk_ms)) / 1e3
    out = {"rows": n_total, "d": d, "k": k, "blocks": blocks, "rows_per_block": n,
           "covariance_s": cov_s, "covariance_ms_per_block": syrk_ms, "solve_s": solve_s,
           "time_to_eigenspace_s": cov_s + solve_s,
           "samples_per_s": n_total / (cov_s + solve_s), "sweeps": r.sweeps, "resid": r.resid,
           "sin_theta_vs_planted": sin_theta(U, r.V),
           "sigma_hat_rel_err_vs_f64_sampled": sigma_err,
           "evals": [float(v) for v in r.evals.cpu()]}
    if sigma_err > SIGMA_SAMPLED_BAR:
        raise RuntimeError(f"16M-row Sigma_hat: sampled rel err {sigma_err:.3e} > "
                           f"{SIGMA_SAMPLED_BAR:.0e} vs float64 - not the reference's Sigma_hat")
    if f64_check:
        V64 = r.V.double()
        Z = torch.zeros((d, k), dtype=torch.float64, device=X.device)
        ch = 1 << 17
        for b in range(blocks):
            gen_block(b, X)
            for lo in range(0, n, ch):
                Xd = X[lo:lo + ch].double()
                Z.addmm_(Xd.t(), Xd @ V64)
                del Xd
        Z /= n_total
        vn = (V64 * V64).sum(0)
        rq = (V64 * Z).sum(0) / vn
        res = (Z - V64 * rq[None, :]).norm(dim=0) / vn.sqrt()
        lam_max = float(rq.abs().max())
        ev_err = float(((r.evals.double() - rq).abs() / rq.abs()).max())
        out.update({"evals_rel_err_vs_f64_rayleigh_all_rows": ev_err,
                    "resid_vs_f64_sigma_all_rows": float(res.max() / lam_max)})
        if ev_err > EVAL_REL_BAR:
            raise RuntimeError(f"16M-row eigenvalues: rel err {ev_err:.3e} vs the float64 "
                               f"Rayleigh quotients on all rows > {EVAL_REL_BAR:.0e}")
    out["note"] = ("one GPU streams all n_total rows (config 3's 2^24) through one covariance "
                   "(block 0 overwrites, the rest DEIG_SYRK_ACCUMULATE; "
                   "tests/test_gpu_syrk_chunks.py::test_full_time_to_eigenspace_helper); each "
                   "block's single launch timed by one HIP event pair; block regeneration "
                   "between launches is untimed (data arrival); sigma_hat_rel_err_vs_f64_sampled: "
                   "16 sampled features, float64 over all rows (bar 2e-6); "
                   "evals_rel_err_vs_f64_rayleigh_all_rows / resid_vs_f64_sigma_all_rows: the "
                   "returned pairs against the float64 Sigma_hat of ALL rows (bar 1e-5)")
    if keep_S:
        out["S"] = S
        out["V"] = r.V
    return out


def sweep_roofline(de, S: torch.Tensor, p: int, stream) -> dict:
    """One subspace-iteration sweep Y = S Q at the solver's p, both kernels:
    4 d^2 bytes of S (read once), 2 d^2 p flop."""
    d = S.shape[0]
    g = torch.Generator(device=S.device).manual_seed(11)
    Q = torch.randn((d, p), generator=g, device=S.device, dtype=torch.float32)
    Y = torch.empty((d, p), device=S.device, dtype=torch.float32)
    byt, fl = 4.0 * d * d, 2.0 * d * d * p
    out = {"d": d, "p": p, "bound": "hbm", "algorithmic": "4 d^2 bytes (S read once), 2 d^2 p flop",
           "peak_GBs": HBM_PEAK / 1e9}
    for algo in ("bf16x3", "bf16x5", "bf16x6", "fp32"):
        if algo != "fp32":
            # as in the solver: the S images are built once per solve (timed apart),
            # then every sweep streams one; bf16x3 / bf16x5 = the solver's modes (Q
            # rounded in place to two bf16 pieces, idempotent; bf16x3 also reads S as
            # two pieces from the prepared two-piece image: three products)
            rq, fa = algo in ("bf16x3", "bf16x5"), algo == "bf16x3"
            prep_ms = time_events(lambda: de.sym_apply(S, Q, out=Y, round_q=rq, fast=fa), 5,
                                  stream, trials=3)
            ms = time_events(lambda: de.sym_apply(S, Q, out=Y, prepared=True, round_q=rq,
                                                  fast=fa), 20, stream, trials=3)
        else:
            ms = time_events(lambda: de.sym_apply(S, Q, algo=algo, out=Y), 20, stream, trials=3)
        t = ms * 1e-3
        nprod = {"bf16x3": 3, "bf16x5": 5, "bf16x6": 6}.get(algo)
        t_min = max(byt / HBM_PEAK, fl / (BF16_MFMA_PEAK / nprod if nprod else FP32_MFMA_PEAK))
        out[algo] = {"us": ms * 1e3, "hbm_GBs": byt / t / 1e9, "hbm_frac": byt / t / HBM_PEAK,
                     "fp32_equiv_tflops": fl / t / 1e12, "attainable_frac": t_min / t}
        if nprod:
            out[algo]["image_prepare_us_once_per_solve"] = max(prep_ms - ms, 0.0) * 1e3
            # the solver's cost per sweep: inside its chain each basis step is fused
            # with the split-K reduction and the next sweep's Q image (sym_power:
            # sweep kernel + sweep_finish_kernel per sweep, launched from C)
            # (scaled by 1 / lambda_max, from a few torch power steps: the chain's
            # dominant direction keeps unit scale over all trials, nothing under- or
            # overflows)
            v = torch.randn((d, 1), generator=g, device=S.device, dtype=torch.float32)
            for _ in range(30):
                v = S @ v
                v = v / v.norm()
            cs = torch.full((p,), 1.0, device=S.device) / (S @ v).norm()
            Qc = Q.clone()
            nst = 10
            cms = time_events(lambda: de.sym_power(S, Qc, cs, nst, out=Y, prepared=True,
                                                   round_q=rq, fast=fa), 3, stream, trials=3) / nst
            out[algo]["in_solver_chain_us"] = cms * 1e3
            out[algo]["in_solver_chain_hbm_frac"] = byt / (cms * 1e-3) / HBM_PEAK
            # the sweep kernel alone (DEIG_SWEEP_KERNEL_ONLY: on the Q image the last
            # call left, no split of Q, no split-K reduction)
            de.sym_apply(S, Q, out=Y, prepared=True, round_q=rq, fast=fa)
            kms = time_events(lambda: de.sym_apply(S, Q, out=Y, prepared=True, round_q=rq,
                                                   fast=fa, kernel_only=True), 20, stream, trials=3)
            out[algo]["kernel_us"] = kms * 1e3
            out[algo]["kernel_hbm_frac"] = byt / (kms * 1e-3) / HBM_PEAK
    out["kernel"] = ("us: split_q_kernel + sweep2_kernel / sweep3_kernel (+ sweep_reduce_kernel), "
                     "one standalone product; kernel_us: the sweep kernel alone; in_solver_chain_us: sweep kernel "
                     "+ sweep_finish_kernel (split-K reduction, power step and next Q image fused), "
                     "per sweep of a 10-sweep chain; on the S images (sweep_prepare_kernel, once per solve): "
                     "bf16x3 = 3 bf16 MFMA 16x16x32 products of the prepared two-piece S image and "
                     "two-piece Q; bf16x5 / bf16x6 = 5 / 6 products of S rows split into 3 pieces "
                     "in registers and 2- / 3-piece Q; fp32: skinny_kernel<T> f32 MFMA 16x16x4")
    out["solver_uses"] = ("bf16x3 while the residual is above 1e-3, bf16x5 down to 1e-4, "
                          "bf16x6 below")
    return out


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """``--gpus N`` (N > 1) without a launcher: start N rank processes of this same
    command line (one per GPU, torch.distributed env rendezvous on 127.0.0.1) and
    return the worst exit code.  Runs before anything touches the GPU; the ranks
    are children, not an exec of this process."""
    import subprocess
    env = dict(os.environ)
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(n),
               LOCAL_WORLD_SIZE=str(n))
    procs = []
    for r in range(n):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=e))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    if bad:
        log(f"bench: rank exit codes {codes}")
    return bad[0] if bad else 0


def init_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    if args.dist_backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    return world, rank, dev


STEP_MS: dict = {}


def timed_loop(step, args, world, dev):
    for _ in range(args.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    out = None
    ends = []
    for _ in range(args.steps):
        out = step(True)
        ends.append(time.perf_counter())  # every step ends with a device sync
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    per = np.diff(np.array([t0] + ends)) * 1e3
    STEP_MS.update(median=float(np.median(per)), min=float(per.min()), max=float(per.max()),
                   spread_pct=float((per.max() - per.min()) / np.median(per) * 100),
                   note="this rank's host wall time per timed step (each ends with a device sync)")
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, out


def formed_group(args) -> dict:
    """What the job actually ran on: the process group torch.distributed formed (world
    size, backend: "nccl" is RCCL on ROCm), the devices this rank sees, and the
    launcher's WORLD_SIZE - recorded on every line so an N > 1 number can be checked
    against the ranks that really took part."""
    formed = dist.is_available() and dist.is_initialized()
    return {"world_size": dist.get_world_size() if formed else 1,
            "backend": dist.get_backend() if formed else None,
            "requested_backend": args.dist_backend if formed else None,
            "WORLD_SIZE_env": os.environ.get("WORLD_SIZE"),
            "device_count": torch.cuda.device_count(),
            "gpus_arg": args.gpus,
            "note": ("gloo rehearsal: ranks share GPUs, bases staged through host memory - "
                     "control flow only, not a scaling number")
            if formed and dist.get_backend() != "nccl" else None}


def base_line(args, world, elapsed, total, dtype, config):
    return {
        "metric": METRIC,
        "value": total / elapsed,
        "unit": "samples/s",
        "n_gpus": world,
        "process_group": formed_group(args),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "step_ms": dict(STEP_MS),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": dtype,
        "data": "synthetic spiked covariance (planted U, theta 8->4), generated on device",
        "config": config,
    }


# ---------------------------------------------------------------- one-shot configs
def run_oneshot(args, cfg, world, rank, dev):
    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd import synthetic
    from distributed_eigenspaces_amd.estimator import gather_bases
    from distributed_eigenspaces_amd.my_threading import Slave

    n, d, k, W = cfg["rows"], cfg["d"], cfg["k"], cfg["workers"]
    if args.rows:
        n = args.rows
    ni = n // W  # rows per logical worker (distributed.py:99-104 split of the rank block)
    U = synthetic.planted_basis(d, k, seed=0, device=dev)
    u8 = cfg.get("u8")
    if u8:
        # bytes (c1) or interleaved pixels (c1g), resident in HBM like the fp32 shards
        X = synthetic.spiked_bytes(n, U, seed=1 + rank, channels=3 if u8 == "gray" else 0)
    else:
        X = synthetic.spiked_samples(n, U, seed=1 + rank)

    def features(xb):
        """The reference's float64 sample matrix of a block of X (distributed.py:170-173)."""
        xb = xb.double()
        return xb.mean(dim=3).reshape(xb.shape[0], -1) if u8 == "gray" else xb

    S = torch.empty((d, d), dtype=torch.float32, device=dev)
    Wt_local = torch.empty((W * k, d), dtype=torch.float32, device=dev)
    # W > 1 logical workers per GPU: each worker's eigensolve runs in its own
    # my_threading.Slave thread on its own HIP stream, started as soon as its
    # covariance is enqueued, so the latency-bound parts of one solve (the
    # single-workgroup Rayleigh-Ritz step, host syncs) overlap the others' sweeps.
    concurrent = W > 1 and not args.serial_workers and args.threaded_workers
    # default for W > 1: the W covariances back to back, then ONE batched solve
    # (linalg.topk_eigh_batch: each worker's sweeps on its own stream, the small
    # Rayleigh-Ritz solves of all W workers in one launch per step)
    batched = W > 1 and not args.serial_workers and not args.threaded_workers
    Ss = [S] + [torch.empty((d, d), dtype=torch.float32, device=dev)
                for _ in range(W - 1)] if (concurrent or batched) else None
    side = [torch.cuda.Stream(dev) for _ in range(W)] if concurrent else None
    torch.cuda.synchronize()
    m = world * W
    stream = torch.cuda.current_stream(dev)
    rec = {"worker": [], "gather": [], "server": []}
    syrk_ev = []

    def solve_on_side(w, ev):
        with torch.cuda.stream(side[w]):
            side[w].wait_event(ev)
            r = de.topk_eigh(Ss[w], k, check_finite=False)  # synchronises side[w]
            Wt_local[w * k:(w + 1) * k].copy_(r.V.t())
            side[w].synchronize()
        return r

    def step_concurrent(record: bool):
        t0 = time.perf_counter()
        evs, slaves = [], []
        for w in range(W):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            e[0].record(stream)
            de.sigma_hat(X[w * ni:(w + 1) * ni], out=Ss[w], algo=args.syrk_algo)
            e[1].record(stream)
            sl = Slave(solve_on_side, w, e[1])
            sl.start()
            slaves.append((sl, e))
        rs = []
        for sl, e in slaves:
            sl.join()
            if sl.exception is not None:
                raise sl.exception
            rs.append(sl.result)
            evs.append((e, sl.result.sweeps))
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        Wt = gather_bases(Wt_local)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        res = None
        if rank == 0:
            res = de.projavg_topk(Wt, k, 1.0 / m, q0=Wt[:k].t())
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        if record:
            syrk_ev.extend(evs)
            rec["worker"].append(t1 - t0)
            rec["gather"].append(t2 - t1)
            rec["server"].append(t3 - t2)
        return rs[-1], res

    def step_batched(record: bool):
        t0 = time.perf_counter()
        evs = []
        for w in range(W):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            e[0].record(stream)
            de.sigma_hat(X[w * ni:(w + 1) * ni], out=Ss[w], algo=args.syrk_algo)
            e[1].record(stream)
            evs.append(e)
        rs = de.topk_eigh_batch(Ss, k, check_finite=False)
        for w, r in enumerate(rs):
            Wt_local[w * k:(w + 1) * k].copy_(r.V.t())
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        Wt = gather_bases(Wt_local)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        res = None
        if rank == 0:
            res = de.projavg_topk(Wt, k, 1.0 / m, q0=Wt[:k].t())
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        if record:
            syrk_ev.extend((e, r.sweeps) for e, r in zip(evs, rs))
            rec["worker"].append(t1 - t0)
            rec["gather"].append(t2 - t1)
            rec["server"].append(t3 - t2)
        return rs[-1], res

    def step(record: bool):
        if batched:
            return step_batched(record)
        if concurrent:
            return step_concurrent(record)
        t0 = time.perf_counter()
        evs = []
        r = None
        for w in range(W):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            e[0].record(stream)
            de.sigma_hat(X[w * ni:(w + 1) * ni], out=S, algo=args.syrk_algo)
            e[1].record(stream)
            r = de.topk_eigh(S, k, check_finite=False)  # synchronises the stream
            Wt_local[w * k:(w + 1) * k].copy_(r.V.t())
            evs.append((e, r.sweeps))
        t1 = time.perf_counter()
        Wt = gather_bases(Wt_local)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        res = None
        if rank == 0:
            res = de.projavg_topk(Wt, k, 1.0 / m, q0=Wt[:k].t())
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        if record:
            syrk_ev.extend(evs)
            rec["worker"].append(t1 - t0)
            rec["gather"].append(t2 - t1)
            rec["server"].append(t3 - t2)
        return r, res

    elapsed, (r, res) = timed_loop(step, args, world, dev)

    syrk_ms = float(np.mean([a.elapsed_time(b) for (a, b), _ in syrk_ev]))
    sweeps = [s for _, s in syrk_ev]
    flops = float(ni) * d * (d + 1)  # algorithmic, per worker launch: lower triangle incl. diag
    algo = args.syrk_algo
    if u8:
        algo = f"u8-{u8}"
    elif algo == "auto":
        algo = "split3" if ni >= 1024 else "fp32"
    if u8:
        planes = 3 if u8 == "gray" else 1
        mfma_flops, peak = planes * flops, I8_MFMA_PEAK
        kernel = ("covariance u8 (u8_prep_kernel + u8_syrk_kernel v_mfma_i32_16x16x64_i8 + "
                  "u8_finalize_kernel)")
        algorithmic = (f"{planes} * n*d*(d+1) = {planes * flops:.4e} int8 MFMA op per launch "
                       f"(n = {ni} rows" + ("; gray: 3 integer products P_hh, P_ww, P_ll of the "
                                             "pixel-sum digits" if planes == 3 else "") + ")")
    elif algo == "split3":
        mfma_flops, peak = 3.0 * flops, BF16_MFMA_PEAK
        kernel = ("covariance split3 (split_kernel + syrks_h_kernel + syrks_reduce_kernel + "
                  "diag_corr_kernel)" if d > 2048 else
                  "covariance split3, fused split (syrks_kernel<..., true> + syrks_reduce_kernel + "
                  "diag_corr_kernel)")
        algorithmic = (f"3 * n*d*(d+1) = {3 * flops:.4e} bf16 MFMA flop per launch (n = {ni} rows; "
                       f"3 split products per fp32 product)")
    else:
        mfma_flops, peak = flops, FP32_MFMA_PEAK
        kernel = "syrk_kernel (+ syrk_reduce_kernel)"
        algorithmic = f"n*d*(d+1) = {flops:.4e} f32 MFMA flop per launch (n = {ni} rows)"
    achieved = mfma_flops / (syrk_ms * 1e-3)
    # concurrent workers: the in-loop events also span other workers' solve kernels
    # interleaved on their side streams, so the covariance is also timed alone
    syrk_alone_ms = None
    if concurrent:
        syrk_alone_ms = time_events(lambda: de.sigma_hat(X[:ni], out=S, algo=args.syrk_algo),
                                    5, stream)

    # --- outside the timed region: accuracy, alternative kernel, sweep roofline
    if concurrent or batched:
        del Ss[1:-1]  # keep worker 0's (S, reused below) and the last worker's buffer
        torch.cuda.empty_cache()
    Xw = X[(W - 1) * ni:W * ni]
    cols = torch.randperm(d, generator=torch.Generator().manual_seed(7))[:16].to(dev)
    Xs = features(Xw).index_select(1, cols)
    S64 = (Xs.t() @ Xs) / ni
    # the last worker's covariance (Ss[0] is S = worker 0's in the concurrent and
    # batched modes; r03y and before compared it with the last worker's rows there)
    S_last = Ss[-1] if (concurrent or batched) else S
    Sblk = S_last.index_select(0, cols).index_select(1, cols).double()
    sigma_err = float((Sblk - S64).abs().max() / S64.abs().max())
    del Xs
    fp32_kernel = None
    if algo == "split3" and not args.no_alt:
        S2 = torch.empty_like(S)
        ms = time_events(lambda: de.sigma_hat(Xw, out=S2, algo="fp32"), 1, stream)
        fp32_kernel = {"kernel": "syrk_kernel (+ syrk_reduce_kernel), v_mfma_f32_32x32x2_f32",
                       "launch_ms": ms, "tflops": flops / (ms * 1e-3) / 1e12,
                       "frac": flops / (ms * 1e-3) / FP32_MFMA_PEAK,
                       # same shard (the last worker's) through both kernels
                       "max_abs_diff_vs_split3_rel": float((S2 - S_last).abs().max()
                                                           / S_last.abs().max())}
        del S2
    p = de.default_subspace(d, k)
    sweep = sweep_roofline(de, S, p, stream)

    acc_u8 = None
    if u8 and rank == 0:
        # bytes: the covariance is exact, so the last worker's basis is checked
        # against float64 eigh of the same shard (the planted U is not the top-k of
        # an uncentered byte covariance: its mean direction dominates)
        Xf = features(Xw).cpu()
        w64, V64 = torch.linalg.eigh(Xf.t() @ Xf / ni)
        V64 = V64[:, -k:]
        Vr = r.V.double().cpu()
        acc_u8 = {"P_dist_last_worker_vs_f64_eigh": float(torch.linalg.matrix_norm(
                      Vr @ Vr.t() - V64 @ V64.t())),
                  # both ascending (distributed.py:22-29 order)
                  "evals_rel_err_vs_f64_eigh": float(((r.evals.double().cpu() - w64[-k:]).abs()
                                                     / w64[-k:]).max()),
                  "lambda1_over_lambdak": float(w64[-1] / w64[-k])}
        del Xf
    if rank != 0:
        return None
    # HBM-side bytes per covariance launch from the separate rocprofv3 PMC passes
    # (FETCH_SIZE / WRITE_SIZE, gfx950 corrections; tools/profile_round.sh) of this
    # same kernel and shard: tools/ travels to the GPU box, profiles/ does not.
    # The measurement is bound to the kernel it describes: it is reported only while
    # the covariance sources hash as they did when tools/profile_round.sh ran.
    traffic, traffic_note = None, None
    pmc = os.path.join(ROOT, "tools", f"pmc_syrk_{args.config}_{algo}.json")
    if os.path.exists(pmc) and not args.rows:
        try:
            pmc_rec = json.load(open(pmc))
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            from pmc_traffic import source_sha256
            if pmc_rec.get("source_sha256") == source_sha256():
                traffic = pmc_rec.get("hbm_bytes_per_launch")
                traffic_note = pmc_rec.get("measured")
            else:
                traffic_note = "stale: kernel sources changed since the PMC passes"
        except Exception as e:  # pragma: no cover
            traffic_note = f"unreadable ({e})"
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_oneshot(features(X[:min(args.cpu_sample, ni)]).cpu().numpy(),
                                   ni, W, k)
    full = None
    if cfg.get("full_rows") and world == 1 and not args.rows and not args.no_full:
        full = full_time_to_eigenspace(de, spiked_block_fn(synthetic, U), X[:ni], U,
                                       cfg["full_rows"], k, stream)
    line = base_line(args, world, elapsed, float(n) * world * args.steps, "u8" if u8 else "f32", {
        "workload": cfg["label"], "rows_per_gpu": n, "total_rows": n * world, "d": d, "k": k,
        "workers_per_gpu": W, "rows_per_worker": ni, "workers_total": m, "subspace_p": p,
        "parallelism": f"dp{world} ({W} logical worker(s) per GPU, RCCL all-gather of bases)",
        "worker_solves": ("batched (deig_topk_sym_batch)" if batched else
                          "my_threading.Slave threads" if concurrent else "serial")})
    if u8:
        line["data"] = ("synthetic spiked bytes: clip(round(128 + 20 x)) of spiked rows (planted "
                        "U, theta 8->4)" + ("; 3 channels with independent noise" if u8 == "gray"
                                            else "") + ", generated on device")
        line["config"]["image"] = "60000 x 32 x 32 x 3" if u8 == "gray" else None
    line["dtype_note"] = ("uint8 in, exact int32/int64 integer covariance, fp32 out; eigensolver "
                          "fp32 with dominant-pair deflation") if u8 else (
                          "fp32 in / fp32 out / fp32 accumulation; split3 covariance and sweeps "
                          "form each fp32 product from 3 bf16 MFMA products of the split operands "
                          "(hi*hi + hi*lo + lo*hi; covariance restores lo^2 on the diagonal); "
                          "accuracy in accuracy.sigma_hat_rel_err_vs_f64_sampled and the solver "
                          "residuals")
    line["roofline"] = {"bound": "mfma", "kernel": kernel, "achieved": achieved / 1e12,
                        "peak": peak / 1e12, "unit": "TOP/s" if u8 else "TFLOP/s", "frac": achieved / peak,
                        "traffic": traffic,
                        "traffic_source": (f"tools/pmc_syrk_{args.config}_{algo}.json (rocprofv3 "
                                           "FETCH_SIZE x2 + WRITE_SIZE, separate passes of this "
                                           "kernel source (sha256-checked); fabric-side L2 misses "
                                           "incl. Infinity-Cache hits: an upper bound on HBM "
                                           f"bytes; {traffic_note})") if traffic else traffic_note,
                        "traffic_vs_algorithmic": (traffic / (4.0 * ni * d)) if traffic else None,
                        "algorithmic": algorithmic, "launch_ms": syrk_ms,
                        "launch_ms_alone": syrk_alone_ms,
                        "frac_alone": (mfma_flops / (syrk_alone_ms * 1e-3) / peak
                                       if syrk_alone_ms else None),
                        # fp32 products per second delivered by the bf16-split kernel:
                        # a throughput, NOT an fp32-MFMA utilisation (the fp32 MFMA
                        # kernel's own utilisation is fp32_kernel.frac)
                        "fp32_products_tflops": flops / (syrk_ms * 1e-3) / 1e12,
                        "fp32_kernel": fp32_kernel}
    line["sweep"] = sweep
    line["syrk_algo"] = algo
    line["cpu_baseline"] = cpu
    wk = 1e3 * float(np.mean(rec["worker"]))
    line["breakdown"] = {"syrk_ms_per_worker": syrk_ms,
                         "worker_eig_ms_per_worker": wk / W - syrk_ms,
                         "worker_sweeps": sweeps[-W:],
                         "gather_ms": 1e3 * float(np.mean(rec["gather"])),
                         "server_ms": 1e3 * float(np.mean(rec["server"])),
                         "server_sweeps": res.sweeps}
    line["accuracy"] = {"sin_theta_server_vs_planted": None if u8 else sin_theta(U, res.V),
                        "sin_theta_last_worker_vs_planted": None if u8 else sin_theta(U, r.V),
                        "worker_resid": r.resid, "server_resid": res.resid,
                        "sigma_hat_rel_err_vs_f64_sampled": sigma_err}
    if acc_u8:
        line["accuracy"].update(acc_u8)
    if full:
        line["time_to_eigenspace_16M_rows_1gpu"] = full
    return line


# ---------------------------------------------------------------- online (Oja) config
def run_oja(args, cfg, world, rank, dev):
    from distributed_eigenspaces_amd import synthetic
    from distributed_eigenspaces_amd.streaming import StreamingOja

    b, d, k, agg = cfg["rows"], cfg["d"], cfg["k"], cfg["agg_every"]
    eta = args.eta if args.eta > 0 else cfg["eta"]
    if args.rows:
        b = args.rows
    U = synthetic.planted_basis(d, k, seed=0, device=dev)
    pool = synthetic.spiked_samples(agg * b, U, seed=1 + rank)  # 64 distinct batches, resident
    g = torch.Generator(device="cpu").manual_seed(5)
    V0 = torch.linalg.qr(torch.randn(d, k, generator=g, dtype=torch.float64))[0].float().to(dev)
    est = StreamingOja(V0, eta=eta, agg_every=agg)
    stream = torch.cuda.current_stream(dev)
    ev = []

    def step(record: bool):
        # one C call for the 64 batches, then the aggregation (gather + solve + broadcast)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record(stream)
        est.block_fn(pool, est.V, est.eta, b, cfg["orth_every"])
        e[1].record(stream)
        est.batches_seen += agg
        est.aggregate()
        e[2].record(stream)
        torch.cuda.synchronize(dev)
        if record:
            ev.append(e)
        return None

    elapsed, _ = timed_loop(step, args, world, dev)
    oja_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev])) / agg  # per batch
    # the aggregation (gather + server solve + broadcast) on the device timeline, from
    # the last Oja batch's end (r03's host clock started when the 64 batches were
    # enqueued, so it also counted their GPU time)
    agg_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in ev]))
    # an Oja batch's algorithmic HBM bytes are ONE read of Xb (4·b·d);
    # the two-pass path reads it twice (that is its cost, not the algorithm's)
    byt = 4.0 * b * d
    achieved = byt / (oja_ms * 1e-3)
    fl = 4.0 * b * d * k  # Xb·V and Xbᵀ·T: 2·b·d·k flop each
    if rank != 0:
        return None
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_oja([pool[i * b:(i + 1) * b] for i in range(16)], V0, eta, 16)
    line = base_line(args, world, elapsed, float(agg * b) * world * args.steps, "f32", {
        "workload": cfg["label"], "batch_rows": b, "d": d, "k": k, "agg_every": agg, "eta": eta,
        "orth_every": cfg["orth_every"], "batches_per_gpu_per_step": agg,
        "rows_per_gpu_per_step": agg * b,
        "parallelism": f"dp{world} (one Oja stream per GPU; RCCL all-gather + broadcast of "
                       f"bases every {agg} batches)"})
    resident = b == 4096 and d % 512 == 0 and d <= 3072 and k <= 32  # DEIG_OJA_AUTO's choice
    kname = ("Oja steps (oja_blk_kernel: one launch per run of orth_every batches, its 256 "
             "workgroups co-resident (occupancy-checked), Xb held in registers "
             "and read from HBM once per batch, Xb*V and Xb^T*T as bf16x3 split products, "
             "in-launch hand-offs; CholQR every orth_every batches), whole op per batch" if resident else
             "Oja steps (oja_nn_kernel Xb*V + oja_tn_kernel V += c Xb^T*T, bf16x3 split "
             "products; CholQR every orth_every batches), whole op per batch")
    line["roofline"] = {"bound": "hbm", "kernel": kname,
                        "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK, "traffic": None,
                        "algorithmic": f"4*b*d = {byt:.4e} bytes per batch (Xb read from HBM "
                                       "once, SURVEY.md §8(d); V / T are L2-resident)",
                        "launch_ms": oja_ms,
                        "mfma_leg": {"flop_per_batch": fl,
                                     "bf16_mfma_flop_per_batch": 3 * fl,
                                     "achieved_bf16_tflops": 3 * fl / (oja_ms * 1e-3) / 1e12,
                                     "frac_of_bf16_peak": 3 * fl / (oja_ms * 1e-3) / BF16_MFMA_PEAK,
                                     "note": "4·b·d·k fp32-equivalent flop per batch, each formed "
                                             "from 3 bf16 MFMA products (bf16x3)"}}
    line["cpu_baseline"] = cpu
    line["breakdown"] = {"oja_ms_per_batch": oja_ms,
                         "aggregate_ms": agg_ms,
                         "aggregate_timing": "HIP events: end of the 64th Oja batch -> end of the aggregation (all-gather + server solve + broadcast), on the launch stream"}
    line["accuracy"] = {"sin_theta_vs_planted": sin_theta(U, est.V),
                        "batches_seen_per_gpu": est.batches_seen}
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--rows", type=int, default=0, help="override rows per GPU (batch rows for c4)")
    ap.add_argument("--eta", type=float, default=0.0, help="c4 step size (default: config's)")
    ap.add_argument("--cpu-sample", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-alt", action="store_true", help="skip the fp32-kernel comparison launch")
    ap.add_argument("--no-full", action="store_true",
                    help="c3: skip streaming all 2^24 rows through one GPU (time_to_eigenspace)")
    ap.add_argument("--serial-workers", action="store_true",
                    help="W > 1 workers per GPU: run each worker's solve after its covariance on "
                         "one stream (default: one batched solve, deig_topk_sym_batch)")
    ap.add_argument("--threaded-workers", action="store_true",
                    help="W > 1: each worker's solve in a my_threading.Slave thread on its own "
                         "stream (the r02 mode)")
    ap.add_argument("--syrk-algo", default="auto", choices=["auto", "split3", "fp32"])
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo = rehearsal of the N>1 control flow with ranks sharing one GPU")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world, rank, dev = init_dist(args)
    cfg = CONFIGS[args.config]
    if cfg["kind"] == "oja":
        line = run_oja(args, cfg, world, rank, dev)
    else:
        line = run_oneshot(args, cfg, world, rank, dev)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
