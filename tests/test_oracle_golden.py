"""The float64 oracle (oracle/ref_cpu.py) against golden vectors produced by running
the reference itself (tests/golden/gen_golden.py).  CPU only."""
import json
import os

import numpy as np
import pytest

from oracle import ref_cpu
from tests.conftest import GOLDEN, golden_keys, golden_names, load_golden

NAMES = golden_names(max_d=4096)  # d = 8192: oracle eigh too slow for the CPU suite (the GPU tests compare with the reference outputs directly)


def test_fixtures_present():
    assert len(NAMES) >= 5
    assert os.path.exists(os.path.join(GOLDEN, "notebook_online_d64.npz"))


@pytest.mark.parametrize("name", NAMES)
def test_sigma_hat_matches_reference(name):
    g = load_golden(name)
    if "sigma_hat0" not in g:
        pytest.skip("fixture stores no Sigma_hat")
    lo, hi = g["sigma_hat0_range"]
    S = ref_cpu.sigma_hat(g["X"][lo:hi])
    np.testing.assert_allclose(S, g["sigma_hat0"], rtol=1e-12, atol=1e-12)
    assert np.array_equal(S, S.T)


@pytest.mark.parametrize("name", NAMES)
def test_worker_topk_matches_reference(name):
    g = load_golden(name)
    k = int(g["k"])
    for i, (lo, hi) in enumerate(g["ranges"]):
        w, v = ref_cpu.top_k_eigh(ref_cpu.sigma_hat(g["X"][lo:hi]), k)
        np.testing.assert_allclose(w, g["worker_evals"][i], rtol=1e-12)
        np.testing.assert_allclose(ref_cpu.align_signs(v, g["worker_V"][i]), g["worker_V"][i],
                                   rtol=0, atol=1e-12)
        assert v.shape == (g["X"].shape[1], k) and v.flags["F_CONTIGUOUS"]
        assert np.all(np.diff(w) >= 0), "ascending order like eigh(eigvals=...)"


@pytest.mark.parametrize("name", NAMES)
def test_server_matches_reference(name):
    g = load_golden(name)
    k, m = int(g["k"]), int(g["m"])
    w, v = ref_cpu.server_topk(list(g["worker_V"]), k, m)
    np.testing.assert_allclose(w, g["server_evals"], rtol=1e-11)
    np.testing.assert_allclose(ref_cpu.align_signs(v, g["server_V"]), g["server_V"], rtol=0,
                               atol=1e-10)
    if "sigma_tilde" in g:
        np.testing.assert_allclose(ref_cpu.projector_average(list(g["worker_V"]), m),
                                   g["sigma_tilde"], rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("name", [n for n in NAMES if "request_ranges" in golden_keys(n)])
def test_shard_split_and_dispatch_order(name):
    """distributed.py:99-104 split and the LIFO / window-of-5 dispatch (:108-111)."""
    g = load_golden(name)
    m = int(g["m"])
    ranges = ref_cpu.split_batches(g["X"].shape[0], m)
    order = ref_cpu.dispatch_order(m)
    expect = np.array([ranges[i] for i in order])
    np.testing.assert_array_equal(g["request_ranges"], expect)
    np.testing.assert_array_equal(g["ranges"], expect)  # FIFO broker: arrival == dispatch
    assert set(g["request_ranks"].tolist()) == {int(g["k"])}
    # remainder rows are dropped
    assert g["ranges"].max() == (g["X"].shape[0] // m) * m


def test_dispatch_window_needs_five():
    with pytest.raises(IndexError):
        ref_cpu.dispatch_order(4)


def test_notebook_online_matches_reference():
    g = load_golden("notebook_online_d64")
    batches = ref_cpu.make_batches(g["X"], int(g["batch_size"]))
    assert len(batches) == int(g["n_batches"])
    assert batches[-1].shape[0] < int(g["batch_size"])  # last batch partial (NB:149-153)
    mw, w, se = ref_cpu.online_notebook(batches, int(g["m"]), int(g["T"]), int(g["k"]))
    np.testing.assert_allclose(se, g["segma_e"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(w, g["final_evals"], rtol=1e-12)
    np.testing.assert_allclose(ref_cpu.align_signs(mw, g["matrix_w"]), g["matrix_w"], rtol=0,
                               atol=1e-10)


def test_figure_schedule_reduces_to_one_shot_when_data_is_static():
    """Parity unpinned (figure only); sanity: static data -> every V_bar(t) equal."""
    g = load_golden("spiked_d64_k4_m8")
    X, k = g["X"], int(g["k"])
    m = 4
    step = X.shape[0] // m
    fn = lambda t, l: X[(l - 1) * step:l * step]  # noqa: E731
    w, v, vbars = ref_cpu.online_figure(fn, m, 3, k)
    _, _, sw, sv = ref_cpu.one_shot(X, k, m)
    assert ref_cpu.projector_distance(v, sv) < 1e-6
    np.testing.assert_allclose(w, np.ones(k), rtol=1e-9)  # (1/T) sum of T equal projectors


def test_projector_distance_exact():
    rng = np.random.default_rng(0)
    A, B = rng.standard_normal((40, 3)), rng.standard_normal((40, 3))
    assert abs(ref_cpu.projector_distance(A, B) - np.linalg.norm(A @ A.T - B @ B.T)) < 1e-9
    Q, _ = np.linalg.qr(A)
    assert ref_cpu.projector_distance(Q, Q @ np.diag([1, -1, 1])) < 1e-12


def test_my_threading_fixture():
    info = json.load(open(os.path.join(GOLDEN, "my_threading.json")))
    assert info["calls"] == [[3, "x"]] and info["is_thread"]
