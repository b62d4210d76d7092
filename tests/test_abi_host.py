"""CPU-only checks of the boundary: the C-ABI library loads and exports every
symbol include/fddp_hip.h declares, the host-side packing matches the
documented parameter-block layouts, and the facade validates like the
reference (no GPU needed, no compute calls)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import crocoddyl_amd as croc
from crocoddyl_amd import _abi
from crocoddyl_amd._lib import LIB_PATH
from crocoddyl_amd.problem import pack_problem
from oracle import fddp_np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fddp_hip.h")


def _declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(fddp_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB_PATH), "libfddp_hip.so not built (run __graft_entry__.build())"
    L = C.CDLL(LIB_PATH)
    names = _declared()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_ctypes_prototypes_cover_header():
    bound = set("fddp_" + k for k in list(_abi.PROTOS) + list(_abi.PROTOS_GPU))
    assert set(_declared()) <= bound | {"fddp_create"}


def test_struct_layouts():
    assert C.sizeof(_abi.Dims) == 20
    assert C.sizeof(_abi.KnotDesc) == 24
    assert C.sizeof(_abi.Params) == 9 * 8 + 8 + 16 * 8
    assert C.sizeof(_abi.Result) == 16 + 9 * 8


def test_no_device_fails_loudly():
    """Without a GPU the product raises; there is no CPU fallback."""
    m = croc.ActionModelLQR(4, 2)
    p = croc.ShootingProblem(np.zeros(4), [m] * 3, m)
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present")
    with pytest.raises(croc.FDDPError):
        croc.SolverFDDP(p)


def test_lqr_block_layout_matches_header():
    m = croc.ActionModelLQR(3, 2, driftFree=False)
    rng = np.random.default_rng(0)
    for a, shape in [("Fx", (3, 3)), ("Fu", (3, 2)), ("f0", (3,)), ("Lxx", (3, 3)), ("Lxu", (3, 2)),
                     ("Luu", (2, 2)), ("lx", (3,)), ("lu", (2,))]:
        setattr(m, a, rng.standard_normal(shape))
    kind, nu, blk = m.pack()
    assert kind == _abi.KNOT_LQR and nu == 2 and blk.shape == (1, fddp_np.block_size(kind, 3, 2))
    k = fddp_np.Knot(kind, 3, 2, blk[0])
    for a in ("Fx", "Fu", "f0", "Lxx", "Lxu", "Luu", "lx", "lu"):
        np.testing.assert_array_equal(getattr(k, a), getattr(m, a))
    assert blk[0, 0] == 0.0  # drift_free flag


def test_euler_block_layout_and_batching():
    d = croc.DifferentialActionModelLQR(2, 1)
    B = 3
    d.Fq = np.random.default_rng(1).standard_normal((B, 2, 2))
    e = croc.IntegratedActionModelEuler(d, 0.01)
    kind, nu, blk = e.pack()
    assert blk.shape == (B, fddp_np.block_size(kind, 4, 1))
    for b in range(B):
        k = fddp_np.Knot(kind, 4, 1, blk[b])
        np.testing.assert_array_equal(k.Fq, d.Fq[b])
        np.testing.assert_array_equal(k.Fv, np.eye(2))
        assert k.dt == 0.01
    knots, pool = pack_problem([e] * 5, croc.IntegratedActionModelEuler(d, 0.0), B)
    assert len(knots) == 6
    assert knots[0] == knots[4]  # one shared block set for the 5 running knots
    assert knots[0][3] == blk.shape[1]  # per-element stride
    assert knots[5][2] != knots[0][2]


def test_problem_validation():
    m = croc.ActionModelLQR(4, 2)
    with pytest.raises(ValueError):
        croc.ShootingProblem(np.zeros(3), [m] * 3, m)
    with pytest.raises(ValueError):
        m.Fx = np.zeros((3, 3))
    with pytest.raises(NotImplementedError):
        croc.IntegratedActionModelEuler(object())
    p = croc.ShootingProblem(np.zeros((5, 4)), [m] * 3, m)
    assert p.B == 5 and p.batched and p.T == 3 and p.nu_max == 2
