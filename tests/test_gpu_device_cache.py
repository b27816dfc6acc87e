"""SlaveNode reads rows [lo, hi) of its data on every request, like the reference's
``self.data[lo:hi]`` (distributed.py:46): a write to the host array between two
requests is always seen (the former sampled-fingerprint device
cache missed writes that landed between sampled elements)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rows(data, lo, hi):
    from distributed_eigenspaces_amd.distributed import _rows_to_device
    return _rows_to_device(data, lo, hi)


def test_single_unsampled_row_write_is_seen(cuda):
    # a config-3-like shard shape scaled down: one row rewritten in place between
    # requests, far from any element a sampled fingerprint would have looked at
    x = np.zeros((8192, 257), dtype=np.float32)
    a = _rows(x, 0, 8192)
    assert float(a.abs().sum()) == 0.0
    x[4097, 131] = 3.0  # one element of one row
    b = _rows(x, 0, 8192)
    assert float(b[4097, 131]) == 3.0
    assert float(_rows(x, 4000, 4100)[97, 131]) == 3.0


def test_cpu_tensor_written_through_numpy_alias(cuda):
    t = torch.arange(4096 * 8, dtype=torch.float32).reshape(4096, 8)
    assert torch.equal(_rows(t, 0, 4096).cpu(), t)
    t.numpy()[:] += 1.0  # bypasses torch's version counter
    assert torch.equal(_rows(t, 0, 4096).cpu(), t)


def test_readonly_numpy_unlocked_and_written(cuda):
    x = np.arange(4096 * 8, dtype=np.float64).reshape(4096, 8)
    x.flags.writeable = False
    assert np.array_equal(_rows(x, 0, 4096).cpu().numpy(), x)
    x.flags.writeable = True
    x[17] = -x[17]
    x.flags.writeable = False
    r = _rows(x, 0, 4096)
    assert r.dtype == torch.float64
    assert np.array_equal(r.cpu().numpy(), x)


def test_dtypes_and_device_tensor_slice(cuda):
    u = np.arange(64 * 16, dtype=np.uint8).reshape(64, 16)
    assert _rows(u, 3, 9).dtype == torch.uint8
    assert _rows(u.astype(np.int32), 3, 9).dtype == torch.float32
    g = torch.randn(64, 16, device="cuda")
    v = _rows(g, 5, 20)
    assert v.data_ptr() == g[5:20].data_ptr()  # a view: no copy
