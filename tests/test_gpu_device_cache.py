"""SlaveNode's device copy of its data is re-uploaded whenever the host contents
changed, however they were written (a CPU tensor written through
an aliasing numpy array kept torch's version counter, and a read-only numpy array
can be unlocked, written and locked again)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_cpu_tensor_written_through_numpy_alias(cuda):
    from distributed_eigenspaces_amd.distributed import _device_copy, clear_device_cache
    clear_device_cache()
    t = torch.arange(4096 * 8, dtype=torch.float32).reshape(4096, 8)
    a = _device_copy(t)
    assert torch.equal(a.cpu(), t)
    assert _device_copy(t) is a  # unchanged: the cached copy
    v0 = t._version
    t.numpy()[:] += 1.0  # bypasses torch's version counter
    assert t._version == v0
    b = _device_copy(t)
    assert torch.equal(b.cpu(), t), "stale device copy after a write through a numpy alias"


def test_readonly_numpy_unlocked_and_written(cuda):
    from distributed_eigenspaces_amd.distributed import _device_copy, clear_device_cache
    clear_device_cache()
    x = np.arange(4096 * 8, dtype=np.float64).reshape(4096, 8)
    x.flags.writeable = False
    a = _device_copy(x)
    assert np.array_equal(a.cpu().numpy(), x)
    x.flags.writeable = True
    x[:] = -x
    x.flags.writeable = False
    b = _device_copy(x)
    assert np.array_equal(b.cpu().numpy(), x), "stale device copy of a re-locked array"
