"""Phase-by-phase GPU vs C++ oracle comparison on the smoke problem (C5 Talos walk,
T=8, B=3 by default), each quantity next to the oracle's own spread under one-ulp
parameter noise (helpers.ulp_floor), so the phase whose error leaves its floor stands
out: iteration-0 calc, the calcDiff blocks, the backward blocks, tryStep at each alpha,
then whole solves at maxiter 1..N. Errors are helpers.elem_err (each coordinate at its
own scale), as in smoke() and the parity tests.

  python tools/parity_trace.py [config] [T] [B] [maxiter] [reps]
Test tooling: loads the oracle as the checker only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import bench  # noqa: E402
import helpers  # noqa: E402
import oracle_lib  # noqa: E402
from crocoddyl_amd import _abi  # noqa: E402


def trace(h, S, xs, us, maxit, fresh):
    """Every phase's outputs of one implementation (h: a fresh handle per call of fresh())."""
    d = S["dims"]
    n, m = d.ndx, d.nu_max
    out = {}
    h.set_candidate(xs, us, False)
    out["calc.cost"] = h.calc()
    out["calc.xnext"] = h.quantity(_abi.Q_XNEXT, d.T, d.nx)
    h.set_solver_state(it=0, xreg=1e-9, ureg=1e-9)
    h.compute_direction(True)
    for name, q, nk, per in [("Fx", _abi.Q_FX, d.T + 1, n * n), ("Fu", _abi.Q_FU, d.T + 1, n * m),
                             ("Lxx", _abi.Q_LXX, d.T + 1, n * n), ("Lxu", _abi.Q_LXU, d.T + 1, n * m),
                             ("Luu", _abi.Q_LUU, d.T + 1, m * m), ("Lx", _abi.Q_LX, d.T + 1, n),
                             ("Lu", _abi.Q_LU, d.T + 1, m), ("fs", _abi.Q_FS, d.T + 1, n),
                             ("Quu", _abi.Q_QUU, d.T, m * m), ("Qu", _abi.Q_QU, d.T, m), ("K", _abi.Q_K, d.T, m * n),
                             ("k", _abi.Q_KV, d.T, m), ("Vxx", _abi.Q_VXX, d.T + 1, n * n), ("Vx", _abi.Q_VX, d.T + 1, n)]:
        out["dir." + name] = h.quantity(q, nk, per)
    h.update_expected_improvement()
    for a in (1.0, 0.25):
        dV, _ = h.try_step(a)
        out[f"try{a}.dV"] = dV
        out[f"try{a}.xs"] = h.xs(trial=True)
        out[f"try{a}.us"] = h.us(trial=True)
    for it in range(1, maxit + 1):
        f = fresh()
        f.set_candidate(xs, us, False)
        r = helpers.results_dict(f.solve(maxiter=it))
        out[f"solve{it}.xs"] = f.xs()
        out[f"solve{it}.us"] = f.us()
        out[f"solve{it}.cost"] = r["cost"]
        out[f"solve{it}.steplength"] = r["steplength"]
    return out


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C5_talos_walk"
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    maxit = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    S = helpers.setup(cfg, T=T, B=B)
    d = S["dims"]
    print(f"{cfg} T={d.T} B={d.B} nx={d.nx} ndx={d.ndx} nu={d.nu_max}", flush=True)
    xs, us = bench.warm_start_arrays(cfg, S["running"], S["x0s"], d)

    def gpu():
        g = helpers.Gpu(d, S["knots"], S["pool"], S["x0s"], device=0)
        g.set_debug(True)  # the Q / V blocks are stored only in debug mode
        return g

    def oracle(pool):
        def fresh():
            return oracle_lib.Oracle(d, S["knots"], pool, S["x0s"], threads=4)
        return trace(fresh(), S, xs, us, maxit, fresh)

    G = trace(gpu(), S, xs, us, maxit, gpu)
    keys = list(G)
    O, floors = helpers.ulp_floor(lambda p: tuple(oracle(p)[k] for k in keys), S["pool"], reps=reps)
    print(f"{'quantity':<16s} {'gpu-oracle':>11s} {'floor':>10s} {'ratio':>7s}", flush=True)
    for k, o, fl in zip(keys, O, floors):
        e = helpers.elem_err(G[k], o)
        print(f"{k:<16s} {e:11.3e} {fl:10.3e} {e / fl if fl > 0 else float('inf'):7.2f}", flush=True)


if __name__ == "__main__":
    main()
