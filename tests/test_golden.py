"""Committed golden fixtures (tests/golden/*.npz, made by make_golden.py from
the numpy restatement): the CPU oracle must reproduce them at 1e-9 (CPU
test), libfddp_hip within the north_star bar — exact iteration counts and
statuses, xs/us/cost within 1e-6 relative (GPU test)."""
import glob
import os

import numpy as np
import pytest

import helpers
import oracle_lib
from crocoddyl_amd import _abi

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))


def _load(path):
    z = np.load(path, allow_pickle=False)
    d = {k: z[k] for k in z.files}
    dims = _abi.Dims(*[int(v) for v in d["dims"]])
    knots = [tuple(int(v) for v in k) for k in d["knots"]]
    return d, dims, knots


def _check(h, d, dims, rtol):
    r = helpers.results_dict(h.solve(maxiter=100))
    np.testing.assert_array_equal(r["iter"], d["iter"])
    np.testing.assert_array_equal(r["status"], d["status"])
    np.testing.assert_allclose(r["cost"], d["cost"], rtol=rtol, atol=1e-12)
    assert helpers.rel_err(h.xs(), d["xs"]) < rtol
    assert helpers.rel_err(h.us(), d["us"]) < rtol


def _check_direction(h, d, dims, tol):
    if "K" not in d:
        return
    n, m, T = dims.ndx, dims.nu_max, dims.T
    h.set_candidate(d["dir_xs"], d["dir_us"], False)
    h.set_solver_state(0, 1e-9, 1e-9, 0)
    assert not h.compute_direction(True).any()
    h.update_expected_improvement()
    K = h.quantity(_abi.Q_K, T, m * n).reshape(dims.B, T, n, m).transpose(0, 1, 3, 2)
    k = h.quantity(_abi.Q_KV, T, m)
    np.testing.assert_allclose(K, d["K"], rtol=tol, atol=tol)
    np.testing.assert_allclose(k, d["k"], rtol=tol, atol=tol)
    dV, st = h.try_step(1.0)
    assert not st.any()
    np.testing.assert_allclose(dV, d["dV1"], rtol=tol, atol=tol)
    np.testing.assert_allclose(h.expected_improvement(), d["d1"], rtol=tol, atol=tol)


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_oracle_reproduces_golden(path):
    d, dims, knots = _load(path)
    o = oracle_lib.Oracle(dims, knots, d["pool"], d["x0s"])
    o.set_candidate(None, None, False)
    _check(o, d, dims, 1e-9)
    _check_direction(o, d, dims, 1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_gpu_reproduces_golden(path):
    d, dims, knots = _load(path)
    g = helpers.Gpu(dims, knots, d["pool"], d["x0s"])
    g.set_candidate(None, None, False)
    _check(g, d, dims, 1e-6)
    _check_direction(g, d, dims, 1e-8)
