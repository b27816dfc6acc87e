"""A resident-Oja hand-off that waits past its bound is reported as an error, not as a
silent NaN basis (``linalg.oja_steps`` and the
streaming aggregation used to feed the NaN on).

The shipped bound is 2 s, reachable only when other work holds CUs; the test-only
variant ``libdeig_test_oja_timeout.so`` (``_build.build_oja_timeout_lib``: oja.hip built
with a zero spin bound, every other object the shipped library's) makes every hand-off
time out, in a child process so that this process keeps the shipped library."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
from distributed_eigenspaces_amd import linalg, _lib
from distributed_eigenspaces_amd.streaming import StreamingOja
assert _lib.LIB_PATH.endswith("libdeig_test_oja_timeout.so"), _lib.LIB_PATH
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)
b, d, k = 4096, 1024, 16
X = torch.randn((2 * b, d), generator=g, device=dev)
V = torch.linalg.qr(torch.randn((d, k), generator=g, device=dev))[0].t().contiguous().t()
try:
    linalg.oja_steps(X, V, 0.5, b, orth_every=2, algo="resident")
except _lib.DeigTimeoutError as e:
    assert torch.isnan(V).all(), "timeout reported but V is not the NaN poison"
    print("TIMEOUT-RAISED", str(e)[:80])
else:
    raise SystemExit("resident Oja with a zero spin bound returned without an error")
# the two-pass path has no hand-offs: the same variant runs it cleanly
V2 = torch.linalg.qr(torch.randn((d, k), generator=g, device=dev))[0].t().contiguous().t()
linalg.oja_steps(X, V2, 0.5, b, orth_every=2, algo="two_pass")
assert torch.isfinite(V2).all()
# the streaming estimator surfaces it too (its block steps check)
s = StreamingOja(V2.clone(), 0.5, agg_every=2)
try:
    s.partial_fit_block(X, b, orth_every=2)
except _lib.DeigTimeoutError:
    print("STREAM-RAISED")
else:
    raise SystemExit("StreamingOja did not raise")
"""


def test_resident_timeout_raises(cuda):
    from distributed_eigenspaces_amd import _build
    lib = _build.OJA_TIMEOUT_LIB
    if not os.path.exists(lib):
        pytest.fail(f"{lib} missing: build it with `python __graft_entry__.py build`")
    env = dict(os.environ, DEIG_LIB_PATH=lib)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "TIMEOUT-RAISED" in r.stdout and "STREAM-RAISED" in r.stdout, r.stdout


def test_shipped_library_reports_no_timeout(cuda):
    import torch
    from distributed_eigenspaces_amd import linalg
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(4)
    b, d, k = 4096, 1024, 16
    X = torch.randn((2 * b, d), generator=g, device=dev)
    V = torch.linalg.qr(torch.randn((d, k), generator=g, device=dev))[0].t().contiguous().t()
    linalg.oja_steps(X, V, 0.5, b, orth_every=2, algo="resident")  # check=True: raises on timeout
    assert torch.isfinite(V).all()
    linalg.oja_check(dev, b, d, k)
