#!/usr/bin/env python
"""Benchmark: one-shot distributed eigenspace estimation on MI355X.

Workload (BASELINE.json configs[2], the metric's "d=8192, k=64" config): each GPU
holds one worker's shard of 2^21 synthetic spiked-covariance rows x d = 8192
(fp32, 64 GiB, resident in HBM before timing); k = 64.  At N GPUs the job covers
N * 2^21 rows (N = 8 -> 16,777,216 = config 3), so scaling is "weak".

One step = time-to-eigenspace of the whole pipeline:
  worker: Sigma_hat = X^T X / n (SYRK kernel) -> top-k eigenpairs (subspace
  iteration) ; exchange: all-gather of the d x k bases (RCCL, N > 1) ;
  server: top-k of the projector average (implicit operator) on rank 0.
value = samples ingested per second over the whole job = N * n / t_step.

Extra objects on the JSON line: ``roofline`` (the covariance op vs the MFMA peak
of the instructions it runs, timed with HIP events on the launch stream),
``cpu_baseline`` (the float64 oracle on a bounded sample of the same workload,
rank 0 at N = 1 only), ``breakdown`` and ``accuracy`` (sin theta of the server
basis vs the planted subspace; Sigma_hat vs float64 on a sampled 16 x 16 block).

Covariance algorithm (--syrk-algo, default auto = split3 at these sizes): fp32
samples split into bf16 hi/lo pairs, 3 bf16 MFMA products per fp32 product,
fp32 accumulation (include/deig.h); "fp32" = the f32 MFMA kernel.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2]
       [--syrk-algo auto|split3|fp32]
       (N > 1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N)
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
HBM_PEAK = 8.0e12

CONFIGS = {
    # name: (rows per GPU, d, k, workload label)
    "c3": (1 << 21, 8192, 64, "synthetic spiked d=8192 k=64, 2^21 rows/GPU (config 3 shard)"),
    "c2": (1 << 20, 3072, 16, "synthetic spiked d=3072 n=1M k=16 (config 2)"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(X_dev: torch.Tensor, n_full: int, k: int, sample_rows: int):
    """Float64 oracle (oracle/ref_cpu.py) on the first ``sample_rows`` rows; the
    covariance term is scaled linearly to the full shard (it is linear in n)."""
    from oracle import ref_cpu
    try:
        from threadpoolctl import threadpool_info
        cores = max((i.get("num_threads", 1) for i in threadpool_info()
                     if i.get("user_api") == "blas"), default=os.cpu_count())
    except Exception:  # pragma: no cover
        cores = os.cpu_count()
    xs = X_dev[:sample_rows].double().cpu().numpy()
    t0 = time.perf_counter()
    S = ref_cpu.sigma_hat(xs)
    t_cov = time.perf_counter() - t0
    t0 = time.perf_counter()
    ref_cpu.top_k_eigh(S, k)
    t_eig = time.perf_counter() - t0
    t_full = t_cov * (n_full / sample_rows) + t_eig
    return {
        "value": n_full / t_full, "unit": "samples/s", "cores": int(cores), "kind": "port",
        "sample": (f"float64 NumPy/SciPy oracle on {sample_rows} rows x d={xs.shape[1]} of the "
                   f"same shard: sigma_hat {t_cov:.2f}s + eigh top-{k} {t_eig:.2f}s; covariance "
                   f"scaled linearly to {n_full} rows -> {t_full:.1f}s per worker shard"),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--rows", type=int, default=0, help="override rows per GPU")
    ap.add_argument("--cpu-sample", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--syrk-algo", default="auto", choices=["auto", "split3", "fp32"])
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo = rehearsal of the N>1 control flow with ranks sharing one GPU")
    args = ap.parse_args()

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

    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd import synthetic
    from distributed_eigenspaces_amd.estimator import gather_bases

    n, d, k, label = CONFIGS[args.config]
    if args.rows:
        n = args.rows
    U = synthetic.planted_basis(d, k, seed=0, device=dev)
    X = synthetic.spiked_samples(n, U, seed=1 + rank)
    S = torch.empty((d, d), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    m = world  # one logical worker per GPU
    stream = torch.cuda.current_stream(dev)
    times = {"syrk": [], "worker_eig": [], "gather": [], "server": []}
    syrk_ev = []

    def step(record: bool):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        t0 = time.perf_counter()
        e[0].record(stream)
        de.sigma_hat(X, out=S, algo=args.syrk_algo)
        e[1].record(stream)
        r = de.topk_eigh(S, k, check_finite=False)  # synchronises the stream
        t1 = time.perf_counter()
        Wt_local = r.V.t().contiguous()           # k x d
        Wt = gather_bases(Wt_local)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        res = None
        if rank == 0:
            res = de.projavg_topk(Wt, k, 1.0 / m, q0=Wt[:k].t())
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        if record:
            syrk_ev.append(e)
            times["worker_eig"].append(t1 - t0)
            times["gather"].append(t2 - t1)
            times["server"].append(t3 - t2)
        return r, res

    for _ in range(args.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r, res = step(True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    syrk_ms = float(np.mean([a.elapsed_time(b) for a, b in syrk_ev]))
    flops = float(n) * d * (d + 1)  # algorithmic: lower triangle incl. diagonal
    algo = args.syrk_algo
    if algo == "auto":
        algo = "split3" if n >= 1024 else "fp32"
    if algo == "split3":
        # 3 bf16 MFMA products per fp32 product; peak = dense bf16 MFMA
        mfma_flops, peak = 3.0 * flops, BF16_MFMA_PEAK
        kernel = "covariance split3 (split_kernel + syrks_kernel + syrks_reduce_kernel + diag_corr_kernel)"
        algorithmic = f"3 * n*d*(d+1) = {3 * flops:.4e} bf16 MFMA flop per launch (3 split products per fp32 product)"
    else:
        mfma_flops, peak = flops, FP32_MFMA_PEAK
        kernel = "syrk_kernel (+ syrk_reduce_kernel)"
        algorithmic = f"n*d*(d+1) = {flops:.4e} f32 MFMA flop per launch"
    achieved = mfma_flops / (syrk_ms * 1e-3)
    # Sigma_hat vs float64 on a sampled 16 x 16 block (all n rows)
    cols = torch.randperm(d, generator=torch.Generator().manual_seed(7))[:16].to(dev)
    Xs = X.index_select(1, cols).double()
    S64 = (Xs.t() @ Xs) / n
    Sblk = S.index_select(0, cols).index_select(1, cols).double()
    sigma_err = float((Sblk - S64).abs().max() / S64.abs().max())
    del Xs

    if rank == 0:
        sin_server = float(torch.linalg.svdvals(U.double().t() @ res.V.double()).min().clamp(max=1)
                           .pow(2).neg().add(1).clamp(min=0).sqrt())
        sin_worker = float(torch.linalg.svdvals(U.double().t() @ r.V.double()).min().clamp(max=1)
                           .pow(2).neg().add(1).clamp(min=0).sqrt())
        traffic = None
        pmc = os.path.join(ROOT, "profiles", f"pmc_syrk_{args.config}_{algo}.json")
        if os.path.exists(pmc) and not args.rows:
            try:
                traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(X, n, k, min(args.cpu_sample, n))
        total = float(n) * world * args.steps
        line = {
            "metric": METRIC,
            "value": total / elapsed,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic spiked covariance (planted U, theta 8->4), generated on device",
            "config": {"workload": label, "rows_per_gpu": n, "total_rows": n * world, "d": d,
                       "k": k, "workers": m, "subspace_p": de.default_subspace(d, k),
                       "parallelism": f"dp{world} (one worker per GPU, RCCL all-gather)"},
            "roofline": {"bound": "mfma", "kernel": kernel, "achieved": achieved / 1e12,
                         "peak": peak / 1e12, "unit": "TFLOP/s",
                         "frac": achieved / peak, "traffic": traffic,
                         "algorithmic": algorithmic, "launch_ms": syrk_ms,
                         "fp32_equiv_tflops": flops / (syrk_ms * 1e-3) / 1e12,
                         "fp32_mfma_peak": FP32_MFMA_PEAK / 1e12},
            "syrk_algo": algo,
            "cpu_baseline": cpu,
            "breakdown": {"syrk_ms": syrk_ms,
                          "worker_eig_ms": 1e3 * float(np.mean(times["worker_eig"])) - syrk_ms,
                          "worker_sweeps": r.sweeps,
                          "gather_ms": 1e3 * float(np.mean(times["gather"])),
                          "server_ms": 1e3 * float(np.mean(times["server"])),
                          "server_sweeps": res.sweeps},
            "accuracy": {"sin_theta_server_vs_planted": sin_server,
                         "sin_theta_worker0_vs_planted": sin_worker,
                         "worker_resid": r.resid, "server_resid": res.resid,
                         "sigma_hat_rel_err_vs_f64_sampled": sigma_err},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
