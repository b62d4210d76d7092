"""The knot calcDiff's lane plan at every workgroup size the device launches.

libfddp_hip runs the multibody calcDiff (multibody.hpp knot_calc_diff_x) in workgroups of
128 threads (small trees: mb_knot_kernel_x2), 256 (mb_knot_kernel) or 512
(mb_knot_kernel_x8, one-per-CU LDS plans). The phases hand work to lanes and waves by
the workgroup size (wave-split sums, spare lanes for the cost table, the wide cost
records' lane base), so the same knot must give the same blocks at every size. The
host build of the device code (tests/cpp/mb_host.cpp, sequential-lane executor;
MB_HOST_NT = the emulated size) is run on gait and arm knots of C3-C5 at 128 and 512
threads against 256: equal up to the reassociation of the wave-split sums (1e-11).
"""
import os

import numpy as np
import pytest

from crocoddyl_amd import synthetic
from test_multibody_host import _p, lib  # noqa: F401  (the host build of the device code)

CASES = [("C3_arm_multibody", (0, 7, 250)), ("C3_arm_contact", (0, 11, 250)),
         ("C4_solo12_trot", (0, 9, 14, 60)), ("C5_talos_walk", (0, 20, 51, 100))]
QS = ["Fx", "Fu", "Lxx", "Lxu", "Luu", "Lx", "Lu"]


def _knot_blocks(lib, em, x, u, nt, m):  # noqa: F811
    kind, nu, blk = em.pack()
    blk = np.ascontiguousarray(blk[0])
    n = em.state.ndx
    nx = em.state.nx
    mm = max(m, 1)
    out = {q: np.zeros(s) for q, s in [("Fx", n * n), ("Fu", n * mm), ("Lxx", n * n), ("Lxu", n * mm),
                                       ("Luu", mm * mm), ("Lx", n), ("Lu", mm)]}
    xn, c = np.zeros(nx), np.zeros(1)
    os.environ["MB_HOST_NT"] = str(nt)
    try:
        lib.mb_host_calc_diff(_p(blk), nx, mm, _p(x), _p(u), 1 if nu > 0 else 0,
                              *[_p(out[q]) for q in QS], _p(xn), _p(c))
    finally:
        os.environ.pop("MB_HOST_NT", None)
    out["xnext"], out["cost"] = xn, c
    return out


@pytest.mark.parametrize("cfg,knots", CASES)
def test_calc_diff_same_at_every_workgroup_size(lib, cfg, knots):  # noqa: F811
    x0s, running, terminal = synthetic.build(cfg, B=1)
    m = max(r.nu for r in running)
    rng = np.random.default_rng(7)
    for t in knots:
        em = running[t] if t < len(running) else terminal
        x = x0s[0].copy()
        nv = em.state.nv
        x[em.state.nq:] += rng.uniform(-0.3, 0.3, nv)  # a moving state (velocity-product terms)
        u = np.zeros(max(m, 1))
        if em.nu and hasattr(em, "quasiStatic"):
            u[:em.nu] = em.quasiStatic(None, x0s[0]) + rng.uniform(-1, 1, em.nu)
        ref = _knot_blocks(lib, em, x, u, 256, m)
        for nt in (128, 512):
            got = _knot_blocks(lib, em, x, u, nt, m)
            for q, want in ref.items():
                scale = max(1.0, float(np.max(np.abs(want))))
                err = float(np.max(np.abs(got[q] - want)))
                assert err / scale < 1e-11, (cfg, t, nt, q, err)
