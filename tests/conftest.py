import functools
import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built libdeig.so")


@functools.lru_cache(maxsize=2)
def _regenerated_samples(n, d, k, seed, grid, sha):
    """Samples of a seeded fixture (cached: d = 8192 takes seconds), read-only."""
    from tests.golden_data import spiked_int_data, xq_digest
    Xq, _ = spiked_int_data(n, d, k, seed, grid=grid)
    assert xq_digest(Xq) == sha, "regenerated samples differ from the fixture's"
    Xq.flags.writeable = False
    return Xq


def load_golden(name):
    """Golden fixture (inputs + reference outputs) as a dict; X as float64 + float32."""
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    out = {k: z[k] for k in z.files}
    if "Xq" not in out and "seed" in out:  # seeded fixture: regenerate the samples
        out["Xq"] = _regenerated_samples(int(out["n"]), int(out["d"]), int(out["k"]),
                                         int(out["seed"]), float(out["grid"]),
                                         str(out["xq_sha256"]))
    if "Xq" in out:
        out["X"] = out["Xq"].astype(np.float64) / float(out["grid"])
    return out


def golden_keys(name):
    """The arrays a fixture stores (no sample regeneration)."""
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return set(z.files)


def golden_d(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return int(z["worker_V"].shape[1]) if "worker_V" in z.files else int(z["Xq"].shape[1])


def golden_names(prefix="spiked", max_d=None):
    names = sorted(os.path.basename(p)[:-4]
                   for p in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))
    return [n for n in names if max_d is None or golden_d(n) <= max_d]


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU visible")
    from distributed_eigenspaces_amd import _lib
    _lib.lib()  # raise loudly if the HIP library is missing
    return torch.device("cuda", 0)
