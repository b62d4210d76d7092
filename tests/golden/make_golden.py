"""Generate the committed golden fixtures (tests/golden/*.npz).

Outputs come from the independent numpy restatement oracle/fddp_np.py (which
is itself pinned to the reference's own test designs in tests/test_oracle.py:
KKT equivalence, closed-form Riccati, numdiff). The reference cannot be run
here, so these fixtures are the repository's frozen vectors:
the C++ oracle and the GPU path are checked against them.

Each fixture holds arrays only (numpy.load(allow_pickle=False) works):
  dims [nx, ndx, nu_max, T, B], knots (T+1, 4) int64 [kind, nu, offset, stride],
  pool, x0s, and per case the outputs (xs, us, cost, iter, status, ...).

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from crocoddyl_amd import synthetic  # noqa: E402
from crocoddyl_amd.models import ActionModelLQR  # noqa: E402
from crocoddyl_amd.problem import pack_problem  # noqa: E402
from oracle import fddp_np  # noqa: E402

MAXITER = 100


def _inputs(x0s, running, terminal):
    B = x0s.shape[0]
    knots, pool = pack_problem(running, terminal, B)
    nx = running[0].state.nx
    nu_max = max(m.nu for m in running)
    dims = np.array([nx, nx, nu_max, len(running), B], dtype=np.int64)
    return dims, np.array(knots, dtype=np.int64), pool, np.asarray(x0s, float)


def _solve_case(dims, knots, pool, x0s, warm=None, maxiter=MAXITER):
    nx, _, nu_max, T, B = [int(v) for v in dims]
    xs = np.zeros((B, T + 1, nx))
    us = np.zeros((B, T, nu_max))
    out = {k: np.zeros(B) for k in ("cost", "stop", "xreg", "steplength")}
    it = np.zeros(B, dtype=np.int64)
    st = np.zeros(B, dtype=np.int64)
    for b in range(B):
        s = fddp_np.FDDP(x0s[b], fddp_np.bind_problem([tuple(k) for k in knots], pool, b, nx))
        wx, wu = (None, None) if warm is None else (list(warm[0][b]), list(warm[1][b]))
        s.solve(wx, wu, maxiter=maxiter)
        xs[b] = np.array(s.xs)
        us[b] = np.array(s.us)
        out["cost"][b], out["stop"][b], out["xreg"][b], out["steplength"][b] = s.cost, s.stop, s.xreg, s.steplength
        it[b], st[b] = s.iter, s.status
    return dict(xs=xs, us=us, iter=it, status=st, **out)


def _direction_case(dims, knots, pool, x0s, seed):
    nx, _, nu_max, T, B = [int(v) for v in dims]
    rng = np.random.default_rng(seed)
    xs = rng.uniform(-1, 1, (B, T + 1, nx))
    us = rng.uniform(-1, 1, (B, T, nu_max))
    K = np.zeros((B, T, nu_max, nx))
    k = np.zeros((B, T, nu_max))
    Vxx = np.zeros((B, T + 1, nx, nx))
    Vx = np.zeros((B, T + 1, nx))
    dV1 = np.zeros(B)
    d1 = np.zeros((B, 2))
    for b in range(B):
        s = fddp_np.FDDP(x0s[b], fddp_np.bind_problem([tuple(kk) for kk in knots], pool, b, nx))
        s.set_candidate(list(xs[b]), list(us[b]), False)
        s.xreg = s.ureg = 1e-9
        assert s.compute_direction(True)
        s.update_expected_improvement()
        K[b], k[b] = np.array(s.K), np.array(s.k)
        Vxx[b], Vx[b] = np.array(s.Vxx), np.array(s.Vx)
        dV1[b] = s.try_step(1.0)
        d1[b] = s.expected_improvement()
    return dict(dir_xs=xs, dir_us=us, K=K, k=k, Vxx=Vxx, Vx=Vx, dV1=dV1, d1=d1)


def main():
    cases = {}
    # C1: unicycle towards the origin (x0 = (-1,-1,1) + seeded draws), T=30
    cases["unicycle_T30_B4"] = synthetic.build("C1_unicycle", T=30, B=4)
    # C2 dims, per-element matrices, with and without drift
    cases["lqr24x12_T10_B2"] = synthetic.build("C2_lqr", T=10, B=2)
    cases["lqr24x12_drift_T10_B2"] = synthetic.build("C2_lqr", T=10, B=2, drift_free=False)
    # C3 / C5 dims with Euler(DiffLQR) knots
    cases["euler14x7_T5_B2"] = synthetic.build("C3_talos_arm", T=5, B=2)
    cases["euler76x32_T3_B1"] = synthetic.build("C5_talos_full", T=3, B=1)
    # the reference factory's LQR(80, 40) with default matrices (unittest/factory/action.cpp:42-59)
    m = ActionModelLQR(80, 40, False)
    cases["lqr80x40_default_T10"] = (np.zeros((1, 80)), [m] * 10, m)
    for name, (x0s, running, terminal) in cases.items():
        dims, knots, pool, x0s = _inputs(x0s, running, terminal)
        out = _solve_case(dims, knots, pool, x0s)
        if name in ("lqr24x12_T10_B2", "euler14x7_T5_B2"):
            out.update(_direction_case(dims, knots, pool, x0s, seed=99))
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, dims=dims, knots=knots, pool=pool, x0s=x0s, **out)
        print(f"{path}: iters {out['iter'].tolist()} status {out['status'].tolist()} cost {out['cost'].tolist()}")


if __name__ == "__main__":
    main()
