"""A/B split3 SYRK settings in one process on the config-3 shard.

Each setting is "variant[:ENV=value,...]" where variant is DEIG_SYRK_VARIANT and
the extra pairs are DEIG_SYRK_<ENV> overrides (FLUSH_ROWS, PRIO, PACE).  Also reports
whether each setting reproduces the first setting's Sigma_hat bit for bit (same
accumulation order -> identical; a cheap race screen) and its max deviation.

usage: python tools/time_syrk_variants.py [n] [d] [settings...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distributed_eigenspaces_amd as de  # noqa: E402
from distributed_eigenspaces_amd import synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else (1 << 21)
d = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
settings = sys.argv[3:] or ["162", "22"]
KEYS = ("DEIG_SYRK_VARIANT", "DEIG_SYRK_FLUSH_ROWS", "DEIG_SYRK_PRIO", "DEIG_SYRK_PACE",
        "DEIG_SYRK_SEGS")


def apply(setting):
    for k in KEYS:
        os.environ.pop(k, None)
    v, _, extra = setting.partition(":")
    os.environ["DEIG_SYRK_VARIANT"] = v
    for kv in filter(None, extra.split(",")):
        k, _, val = kv.partition("=")
        os.environ["DEIG_SYRK_" + k.upper()] = val


dev = torch.device("cuda", 0)
U = synthetic.planted_basis(d, 64, 0, dev)
X = synthetic.spiked_samples(n, U, seed=1)
ref = None
for rep in range(2):
    for st in settings:
        apply(st)
        S = de.sigma_hat(X, algo="split3")
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            de.sigma_hat(X, out=S, algo="split3")
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        if ref is None:
            ref = S.clone()
        same = bool(torch.equal(S, ref))
        dev_max = float((S - ref).abs().max() / ref.abs().max())
        tf = 3 * n * d * (d + 1) / (min(ts) * 1e-3) / 1e12
        print(f"{st:28s}: {min(ts):8.2f} ms (median {sorted(ts)[1]:8.2f})  {tf:7.1f} bf16-MFMA TF/s  "
              f"bit-identical={same} maxdev={dev_max:.2e}", flush=True)
