"""Numpy emulation: how the reference's float64 data flow (distributed.py:169-173 gray
means -> compute_sigma_hat_ :59-70 -> top_k_eigenvectors :22-29) is perturbed by each
precision choice of the GPU path.  Not a test; a design probe.

    python tools/emulate_f64flow.py [n] [d] [k]
"""
import sys

import numpy as np
import scipy.linalg

sys.path.insert(0, ".")
from oracle import ref_cpu  # noqa: E402


def bf16(x):
    """Round float32 array to bf16 (RNE), returned as float32."""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def gray_data(n, d, k, seed):
    rng = np.random.default_rng(seed)
    U = np.linalg.qr(rng.standard_normal((d, k)))[0]
    sig = (rng.standard_normal((n, k)) * np.sqrt(np.linspace(8.0, 4.0, k))) @ U.T
    out = np.empty((n, d, 3), dtype=np.uint8)
    for c in range(3):
        x = rng.standard_normal((n, d), dtype=np.float32) + sig
        out[:, :, c] = np.clip(np.rint(128.0 + 20.0 * x), 0, 255)
    return out.mean(axis=2)  # float64, the reference's data.mean(axis=3) of pixels


def topk(S, k):
    return ref_cpu.top_k_eigh(S, k)


def report(name, S, k, w0, V0):
    w, V = topk(S, k)
    print(f"{name:44s} P {ref_cpu.projector_distance(V, V0):.2e}  "
          f"ev {np.max(np.abs(w - w0) / np.abs(w0)):.2e}")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 7500
    d = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    X = gray_data(n, d, k, 1)
    S64 = ref_cpu.sigma_hat(X)
    w0, V0 = topk(S64, k)
    print(f"n={n} d={d} k={k}  lambda_1/lambda_k = {w0[-1] / w0[0]:.3e}")
    report("S64 -> fp32 storage", S64.astype(np.float32).astype(np.float64), k, w0, V0)
    X32 = X.astype(np.float32)
    report("fp32 input, exact sum", (X32.astype(np.float64).T @ X32.astype(np.float64)) / n, k, w0, V0)
    report("fp32 input, fp32 sum (sgemm)", (X32.T @ X32).astype(np.float64) / n, k, w0, V0)
    mu = X.mean(axis=0)
    C = (X - mu).astype(np.float32)
    s = C.astype(np.float64).sum(axis=0)

    def recon(Sc):
        return Sc + np.outer(mu, mu) + (np.outer(s, mu) + np.outer(mu, s)) / n

    Cd = C.astype(np.float64)
    report("shift: fp32 C, exact sum", recon(Cd.T @ Cd / n), k, w0, V0)
    report("shift: fp32 C, fp32 sum", recon((C.T @ C).astype(np.float64) / n), k, w0, V0)
    hi = bf16(C)
    lo = bf16(C - hi)
    sp = (hi.T @ hi + hi.T @ lo + lo.T @ hi).astype(np.float64)
    sp[np.diag_indices(d)] += (lo.astype(np.float64) ** 2).sum(axis=0)
    Ssp = recon(sp / n)
    report("shift: split3 C, fp32 sum", Ssp, k, w0, V0)
    report("shift: split3 C, fp32 sum, fp32 storage", Ssp.astype(np.float32).astype(np.float64), k, w0, V0)
    hi = bf16(X32)
    lo = bf16(X32 - hi)
    sp = (hi.T @ hi + hi.T @ lo + lo.T @ hi).astype(np.float64)
    sp[np.diag_indices(d)] += (lo.astype(np.float64) ** 2).sum(axis=0)
    report("no shift: split3 X, fp32 sum (r02 path)", sp / n, k, w0, V0)
    # deflation stage 2 on an fp32 image formed from the f64 matrix vs from fp32 S
    for name, Sin in (("f64", Ssp), ("f32", Ssp.astype(np.float32).astype(np.float64))):
        w1, V1 = topk(Sin.astype(np.float32).astype(np.float64), k)
        r = int(np.sum(w1 >= 64 * w1[0]))
        Vd, ld = V1[:, k - r:].astype(np.float32).astype(np.float64), w1[k - r:]
        if name == "f64":
            img = (Sin - (Vd * ld) @ Vd.T).astype(np.float32).astype(np.float64)
        else:
            Sf = Sin.astype(np.float32)
            img = Sf - ((Vd * ld) @ Vd.T).astype(np.float32)  # fp32 subtraction
            img = img.astype(np.float32).astype(np.float64)
        w2, V2 = topk(img, k - r)
        V2 = V2 - Vd @ (Vd.T @ V2)
        V2 /= np.linalg.norm(V2, axis=0)
        V = np.concatenate([V2, Vd], axis=1)
        w = np.concatenate([w2, ld])
        print(f"{'stage-2 deflation (r=%d) image from ' % r + name:44s} P "
              f"{ref_cpu.projector_distance(V, V0):.2e}  ev {np.max(np.abs(w - w0) / np.abs(w0)):.2e}")


if __name__ == "__main__":
    main()
