"""CU-partition probe (measurement tooling): can the worker solves run beside the next
workers' covariances on a disjoint set of CUs?

  probe: which XCC / CU a launch on a CU-masked stream lands on (tools/cu_mask_probe.so),
         and whether mask bit i maps to XCC i % 8 (interleaved) or XCC i // 32.
  pipe:  the c5 worker phase with the covariances on a stream masked to 256 - S CUs
         (library built with DEIG_AB_SYRK_G = 256 - S) and the single-problem solves on
         a stream masked to the other S CUs, each solve waiting for its covariance.
  serial: the bench's schedule (covariances back to back, then one batched solve).

  python tools/cu_split_probe.py probe
  DEIG_LIB_PATH=tools/ab_libs/libdeig_syrk_g232.so python tools/cu_split_probe.py pipe --solve-cus 24
  python tools/cu_split_probe.py serial [--case c5|c3] [--half-until 0]
  python tools/cu_split_probe.py solve [--case c5|c3]     (the batched solves alone)
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NXCC, NCU = 8, 256


def load_probe():
    P = ctypes.CDLL(os.path.join(ROOT, "tools", "cu_mask_probe.so"))
    P.cu_probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong]
    P.cu_stream_create.argtypes = [ctypes.POINTER(ctypes.c_uint), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    P.cu_stream_mask.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint)]
    return P


def make_stream(P, bits):
    mask = (ctypes.c_uint * 8)()
    for b in bits:
        mask[b // 32] |= 1 << (b % 32)
    s = ctypes.c_void_p()
    assert P.cu_stream_create(mask, 8, ctypes.byref(s)) == 0
    back = (ctypes.c_uint * 8)()
    assert P.cu_stream_mask(s, 8, back) == 0
    return s.value, [hex(x) for x in back]


def where(P, torch, sptr, nblk=4096):
    """Distinct hardware CUs per XCC that a spread-out launch on the stream used."""
    out = torch.zeros(2 * nblk, dtype=torch.int32, device="cuda")
    assert P.cu_probe_launch(sptr, nblk, out.data_ptr(), 2000) == 0
    torch.cuda.synchronize()
    a = out.cpu().numpy().astype("uint32").reshape(-1, 2)
    per = {}
    for xcc, hw in a:
        per.setdefault(int(xcc) & 0xF, set()).add(int(hw >> 8) & 0xFF)
    return {x: len(per.get(x, ())) for x in range(NXCC)}


def masks(interleaved, solve_cus):
    per = solve_cus // NXCC
    if interleaved:  # bit i -> XCC i % 8, CU i // 8
        solve = [b for b in range(NCU) if b // NXCC >= NCU // NXCC - per]
    else:  # bit i -> XCC i // 32, CU i % 32
        solve = [b for b in range(NCU) if b % 32 >= 32 - per]
    cov = [b for b in range(NCU) if b not in set(solve)]
    return cov, solve


def decide(P, torch):
    full, fm = make_stream(P, range(NCU))
    print("full mask", fm, where(P, torch, full), flush=True)
    # safe under both readings (every XCC keeps >= 1 CU): one bit per 32-bit chunk with
    # residue x in chunk x, plus bits 1 and 2 (interleaved: XCC 1 and 2 get 2 CUs;
    # contiguous: XCC 0 gets 3)
    r_bits = [32 * x + 24 + x for x in range(NXCC)] + [1, 2]
    rs, rm = make_stream(P, r_bits)
    w = where(P, torch, rs)
    print("probe mask", rm, w, flush=True)
    if w[1] == 2 and w[2] == 2 and w[0] == 1:
        return True
    if w[0] == 3 and w[1] == 1:
        return False
    raise SystemExit(f"mask reading not recognised: {w}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["probe", "pipe", "serial", "solve"])
    ap.add_argument("--solve-cus", type=int, default=24)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--case", default="c5")
    ap.add_argument("--half-until", type=float, default=None,
                    help="serial: deig_solver_opts.half_until (default: the library's)")
    ap.add_argument("--opt", action="append", default=[],
                    help="serial: another deig_solver_opts field, NAME=VALUE (repeatable)")
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    P = load_probe()
    if a.mode == "probe":
        inter = decide(P, torch)
        print("interleaved", inter, flush=True)
        for s in (8, 16, 24, 32):
            cov, solve = masks(inter, s)
            cs, cm = make_stream(P, cov)
            ss, sm = make_stream(P, solve)
            print(f"solve {s}: cov", where(P, torch, cs), "solve", where(P, torch, ss), flush=True)
        return
    import distributed_eigenspaces_amd as de
    from distributed_eigenspaces_amd import synthetic
    n, d, k = {"c5": (65536, 16384, 128), "c3": (262144, 8192, 64)}[a.case]
    W = a.workers
    dev = torch.device("cuda", 0)
    U = synthetic.planted_basis(d, k, seed=0, device=dev)
    X = synthetic.spiked_samples(n * W, U, seed=1)
    Ss = [torch.empty((d, d), dtype=torch.float32, device=dev) for _ in range(W)]
    Wt = torch.empty((W * k, d), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()

    def sin_err(V):
        sv = torch.linalg.svdvals(V.double().t() @ U.double()).clamp(max=1)
        return float((1 - sv.min() ** 2).clamp(min=0).sqrt())

    res = {"mode": a.mode, "case": a.case, "lib": os.environ.get("DEIG_LIB_PATH", "shipped")}
    if a.mode == "solve":  # the batched worker solves alone (covariances once, untimed)
        for w in range(W):
            de.sigma_hat(X[w * n:(w + 1) * n], out=Ss[w])
        del X
        ts = []
        for _ in range(a.reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rs = de.topk_eigh_batch(Ss, k, check_finite=False)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        res.update(solve_ms=[round(t, 3) for t in ts[1:]], sweeps=[r.sweeps for r in rs])
        print(json.dumps(res), flush=True)
        return
    if a.mode == "serial":
        st = torch.cuda.current_stream(dev)
        from distributed_eigenspaces_amd import _lib
        extra = {kv.split("=")[0]: float(kv.split("=")[1]) for kv in a.opt}
        opts = _lib.solver_opts(half_until=a.half_until, **extra)
        res["half_until"] = float(opts.half_until)
        res["opts"] = extra

        def step():
            for w in range(W):
                de.sigma_hat(X[w * n:(w + 1) * n], out=Ss[w])
            rs = de.topk_eigh_batch(Ss, k, check_finite=False, opts=opts)
            for w, r in enumerate(rs):
                Wt[w * k:(w + 1) * k].copy_(r.V.t())
            torch.cuda.synchronize()
            return rs
    else:
        inter = decide(P, torch)
        cov, solve = masks(inter, a.solve_cus)
        cs_ptr, _ = make_stream(P, cov)
        ss_ptr, _ = make_stream(P, solve)
        cw, sw = where(P, torch, cs_ptr), where(P, torch, ss_ptr)
        print("cov CUs", cw, "solve CUs", sw, flush=True)
        gexp = (NCU - a.solve_cus) // NXCC
        assert all(v == gexp for v in cw.values()), "covariance stream does not have G/8 CUs per XCC"
        cs = torch.cuda.ExternalStream(cs_ptr, device=dev)
        ss = torch.cuda.ExternalStream(ss_ptr, device=dev)
        st = cs

        def step():
            evs = []
            with torch.cuda.stream(cs):
                for w in range(W):
                    de.sigma_hat(X[w * n:(w + 1) * n], out=Ss[w])
                    e = torch.cuda.Event()
                    e.record(cs)
                    evs.append(e)
            rs = []
            with torch.cuda.stream(ss):
                for w in range(W):
                    ss.wait_event(evs[w])
                    r = de.topk_eigh(Ss[w], k, check_finite=False)
                    Wt[w * k:(w + 1) * k].copy_(r.V.t())
                    rs.append(r)
            torch.cuda.synchronize()
            return rs

    rs = step()  # warm
    ts = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rs = step()
        ts.append((time.perf_counter() - t0) * 1e3)
    res["step_ms"] = round(statistics.median(ts), 2)
    res["step_all"] = [round(t, 2) for t in ts]
    # covariance alone on its stream, and (pipe) one solve alone on the solve stream
    with torch.cuda.stream(st):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for w in range(W):
            de.sigma_hat(X[w * n:(w + 1) * n], out=Ss[w])
        e1.record(st)
    torch.cuda.synchronize()
    res["cov_alone_ms_per_worker"] = round(e0.elapsed_time(e1) / W, 3)
    if a.mode == "pipe":
        with torch.cuda.stream(ss):
            t0 = time.perf_counter()
            r = de.topk_eigh(Ss[0], k, check_finite=False)
            torch.cuda.synchronize()
            res["solve_alone_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
            res["solve_alone_sweeps"] = r.sweeps
    res["sweeps"] = [r.sweeps for r in rs]
    res["sin_theta_last"] = round(sin_err(rs[-1].V), 4)
    res["resid_max"] = max(r.resid for r in rs)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
