"""Sweep kernel probe: Y = S Q (bf16x6 / x5 / x3 and fp32) at several (d, p), HIP-event
time per launch on the launch stream (bf16x6: S image prepared once, not timed), HBM GB/s on 4 d^2 bytes, and the error
vs a float64 product.  usage: python tools/time_sweep.py [d:p ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import distributed_eigenspaces_amd as de

dev = torch.device("cuda", 0)
st = torch.cuda.current_stream()
cases = [tuple(map(int, a.split(":"))) for a in sys.argv[1:]] or [(3072, 32), (8192, 80), (16384, 128), (1000, 16)]
for d, p in cases:
    g = torch.Generator(device=dev).manual_seed(5)
    A = torch.randn((d, d), generator=g, device=dev)
    S = (A + A.t()) * 0.5
    del A
    Q = torch.randn((d, p), generator=g, device=dev)
    Y = torch.empty((d, p), device=dev)
    ref = (S.double() @ Q.double())
    for mode in ("bf16x6", "bf16x5", "bf16x3", "fp32"):
        # solver modes: bf16x5 = Q rounded in place, five products; bf16x3 = also S
        # as two pieces from the prepared two-piece image, three products
        rq, fa = mode in ("bf16x5", "bf16x3"), mode == "bf16x3"
        algo = "fp32" if mode == "fp32" else "bf16x6"
        Qm = Q.clone() if rq else Q
        de.sym_apply(S, Qm, algo=algo, out=Y, round_q=rq, fast=fa)
        ref = S.double() @ Qm.double()
        err = ((Y.double() - ref).abs().max() / ref.abs().max()).item()
        reps = 30
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):  # the solver's case: S images built once
            de.sym_apply(S, Qm, algo=algo, out=Y, prepared=True, round_q=rq, fast=fa)
        e1.record(st)
        e1.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        print(f"d={d:6d} p={p:4d} {mode:7s} {us:9.1f} us  {4.0*d*d/us/1e3:8.1f} GB/s  "
              f"({4.0*d*d/us/1e3/8000*100:5.1f}% of 8 TB/s)  max rel err {err:.2e}", flush=True)
    del S, Q, Y, ref
    torch.cuda.empty_cache()
