"""Sweep cost inside the solver's chain vs a standalone product: per sweep, HIP
events on the launch stream, at (d, p) in the solver's modes.  chain = sym_power
(power step, split-K reduction and the next sweep's Q image fused into one
kernel after the sweep); apply = sym_apply (split_q + sweep + reduce).
usage: python tools/time_sweep_chain.py [d:p ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import distributed_eigenspaces_amd as de

dev = torch.device("cuda", 0)
st = torch.cuda.current_stream()
cases = [tuple(map(int, a.split(":"))) for a in sys.argv[1:]] or [(8192, 80)]
for d, p in cases:
    g = torch.Generator(device=dev).manual_seed(5)
    A = torch.randn((d, d), generator=g, device=dev)
    S = (A + A.t()) * (0.5 / d ** 0.5)
    del A
    Q = torch.randn((d, p), generator=g, device=dev)
    Y = torch.empty((d, p), device=dev)
    cs = torch.full((p,), 0.5, device=dev)
    for mode in ("bf16x3", "bf16x5", "bf16x6"):
        kw = {"round_q": mode != "bf16x6", "fast": mode == "bf16x3"}
        de.sym_apply(S, Q, out=Y, **kw)  # prepare the images
        steps = 20
        de.sym_power(S, Q, cs, 2, out=Y, prepared=True, **kw)
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(st)
        de.sym_power(S, Q, cs, steps, out=Y, prepared=True, **kw)
        e1.record(st)
        for _ in range(steps):
            de.sym_apply(S, Q, out=Y, prepared=True, **kw)
        e2.record(st)
        e2.synchronize()
        us_c = e0.elapsed_time(e1) / steps * 1e3
        us_a = e1.elapsed_time(e2) / steps * 1e3
        print(f"d={d:6d} p={p:4d} {mode}: chain {us_c:8.1f} us/sweep ({4.0*d*d/us_c/1e3/8000:5.3f} of 8 TB/s)"
              f"   apply {us_a:8.1f} us ({4.0*d*d/us_a/1e3/8000:5.3f})", flush=True)
    del S, Q, Y
    torch.cuda.empty_cache()
