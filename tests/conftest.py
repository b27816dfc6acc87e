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


def load_golden(name):
    """Golden fixture (inputs + reference outputs) as a dict; X as float64 + float32."""
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    out = {k: z[k] for k in z.files}
    if "Xq" not in out and "seed" in out:  # seeded fixture: regenerate the samples
        from tests.golden_data import spiked_int_data, xq_digest
        Xq, _ = spiked_int_data(int(out["n"]), int(out["d"]), int(out["k"]), int(out["seed"]),
                                grid=float(out["grid"]))
        assert xq_digest(Xq) == str(out["xq_sha256"]), f"{name}: regenerated samples differ"
        out["Xq"] = Xq
    if "Xq" in out:
        out["X"] = out["Xq"].astype(np.float64) / float(out["grid"])
    return out


def golden_names(prefix="spiked"):
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU visible")
    from distributed_eigenspaces_amd import _lib
    _lib.lib()  # raise loudly if the HIP library is missing
    return torch.device("cuda", 0)
