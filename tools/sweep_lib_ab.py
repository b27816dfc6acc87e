"""Interleaved A/B of libdeig builds on the solver's sweep chain (deig_sym_power_f32,
prepared images) at (d, p) in one mode: us per sweep by HIP events on the launch
stream, and whether each build reproduces the first one's Y and Q bit for bit
(measurement tooling).
usage: python tools/sweep_lib_ab.py reps d p mode lib [lib ...]
       mode: bf16x3 | bf16x5 | bf16x6;  "shipped" = the in-tree build"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_eigenspaces_amd import _lib  # noqa: E402

reps, d, p, mode = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
libs = []
for path in sys.argv[5:]:
    L = ctypes.CDLL(_lib.LIB_PATH if path == "shipped" else path)
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    libs.append((path, L))
code = _lib.DEIG_SWEEP_BF16X6
if mode != "bf16x6":
    code |= _lib.DEIG_SWEEP_ROUND_Q
if mode == "bf16x3":
    code |= _lib.DEIG_SWEEP_FAST
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)
g = torch.Generator(device=dev).manual_seed(5)
A = torch.randn((d, d), generator=g, device=dev)
S = (A + A.t()) * (0.5 / d ** 0.5)
del A
Q0 = torch.randn((d, p), generator=g, device=dev)
cs = torch.full((p,), 0.5, device=dev)
steps = 20
state = {}
for path, L in libs:
    nbytes = L.deig_sym_apply_workspace(d, p, code)
    ws = torch.empty(nbytes // 4 + 64, dtype=torch.float32, device=dev)
    Q = Q0.clone()
    Y = torch.empty((d, p), device=dev)
    rc = L.deig_sym_apply_f32(S.data_ptr(), d, d, Q.data_ptr(), p, p, Y.data_ptr(), p,
                              ctypes.c_float(1.0), code, ws.data_ptr(), nbytes, stream.cuda_stream)
    assert rc == 0, L.deig_last_error()
    state[path] = (ws, nbytes, Y)
times = {p_: [] for p_, _ in libs}
outs = {}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(reps + 1):
    order = libs if r % 2 == 0 else libs[::-1]
    for path, L in order:
        ws, nbytes, Y = state[path]
        Q = Q0.clone()
        torch.cuda.synchronize()
        e0.record(stream)
        rc = L.deig_sym_power_f32(S.data_ptr(), d, d, Q.data_ptr(), p, p, Y.data_ptr(), p, cs.data_ptr(),
                                  steps, code | _lib.DEIG_SWEEP_PREPARED, ws.data_ptr(), nbytes,
                                  stream.cuda_stream)
        e1.record(stream)
        e1.synchronize()
        assert rc == 0, L.deig_last_error()
        if r:
            times[path].append(e0.elapsed_time(e1) / steps * 1e3)
        outs[path] = (Y.clone(), Q)
ref = outs[libs[0][0]]
for path, ts in times.items():
    st = sorted(ts)
    med = st[len(st) // 2]
    same = torch.equal(outs[path][0], ref[0]) and torch.equal(outs[path][1], ref[1])
    print(f"d={d} p={p} {mode} {path}: median {med:.1f} us/sweep (min {st[0]:.1f}) = "
          f"{4.0 * d * d / med / 1e3 / 8000:.3f} of 8 TB/s; bit-identical to first: {same}", flush=True)
