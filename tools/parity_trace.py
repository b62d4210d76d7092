"""Phase-by-phase GPU vs C++ oracle comparison on the smoke problem (C5 Talos walk,
T=8, B=3 by default): iteration-0 calc, the calcDiff blocks, the backward blocks,
tryStep at each alpha, then whole solves at maxiter 1..N. Prints, per quantity, the
normwise relative error (max |g - o| / max(1, max |o|)) and the worst element-wise
relative error over entries with |o| >= 1e-6 max|o| (so small components are seen).

  python tools/parity_trace.py [config] [T] [B] [maxiter]
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


def errs(g, o):
    g = np.asarray(g, float)
    o = np.asarray(o, float)
    scale = float(np.max(np.abs(o))) if o.size else 0.0
    nw = float(np.max(np.abs(g - o))) / max(1.0, scale) if o.size else 0.0
    mask = np.abs(o) >= 1e-6 * max(scale, 1e-300)
    ew = float(np.max(np.abs(g - o)[mask] / np.abs(o)[mask])) if mask.any() else 0.0
    return nw, ew


def row(name, g, o, extra=""):
    nw, ew = errs(g, o)
    print(f"  {name:<10s} normwise {nw:9.2e}  elementwise {ew:9.2e} {extra}", flush=True)
    return nw, ew


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C5_talos_walk"
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    maxit = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    S = helpers.setup(cfg, T=T, B=B)
    d = S["dims"]
    n, m = d.ndx, d.nu_max
    print(f"{cfg} T={d.T} B={d.B} nx={d.nx} ndx={n} nu={m}; knot kinds "
          f"{[k[0] for k in S['knots']]} nu {[k[1] for k in S['knots']]}", flush=True)
    xs, us = bench.warm_start_arrays(cfg, S["running"], S["x0s"], d)

    def fresh():
        g = helpers.Gpu(d, S["knots"], S["pool"], S["x0s"], device=0)
        g.set_debug(True)  # the Q / V blocks are stored only in debug mode
        o = oracle_lib.Oracle(d, S["knots"], S["pool"], S["x0s"], threads=4)
        for h in (g, o):
            h.set_candidate(xs, us, False)
        return g, o

    g, o = fresh()
    print("phase 1: iteration-0 calc at the warm start", flush=True)
    row("cost", g.calc(), o.calc())
    row("xnext", g.quantity(_abi.Q_XNEXT, d.T, d.nx), o.quantity(_abi.Q_XNEXT, d.T, d.nx))
    row("knotcost", g.quantity(_abi.Q_COST, d.T + 1, 1), o.quantity(_abi.Q_COST, d.T + 1, 1))

    print("phase 2: computeDirection (calcDiff + gaps + backward), xreg = ureg = 1e-9", flush=True)
    for h in (g, o):
        h.set_solver_state(it=0, xreg=1e-9, ureg=1e-9)
    sg, so = g.compute_direction(True), o.compute_direction(True)
    print(f"  status gpu {sg.tolist()} oracle {so.tolist()}")
    blocks = [("Fx", _abi.Q_FX, d.T + 1, n * n), ("Fu", _abi.Q_FU, d.T + 1, n * m), ("Lxx", _abi.Q_LXX, d.T + 1, n * n),
              ("Lxu", _abi.Q_LXU, d.T + 1, n * m), ("Luu", _abi.Q_LUU, d.T + 1, m * m), ("Lx", _abi.Q_LX, d.T + 1, n),
              ("Lu", _abi.Q_LU, d.T + 1, m), ("fs", _abi.Q_FS, d.T + 1, n)]
    for name, q, nk, per in blocks:
        G, O = g.quantity(q, nk, per), o.quantity(q, nk, per)
        row(name, G, O)
        if name in ("Fx", "Fu"):
            for t in range(nk):
                nw, ew = errs(G[:, t], O[:, t])
                print(f"      t={t} kind={S['knots'][t][0]} normwise {nw:9.2e} elementwise {ew:9.2e}")
    for name, q, nk, per in [("Quu", _abi.Q_QUU, d.T, m * m), ("Qxu", _abi.Q_QXU, d.T, n * m),
                             ("Qxx", _abi.Q_QXX, d.T, n * n), ("Qu", _abi.Q_QU, d.T, m), ("Qx", _abi.Q_QX, d.T, n),
                             ("K", _abi.Q_K, d.T, m * n), ("k", _abi.Q_KV, d.T, m),
                             ("Vxx", _abi.Q_VXX, d.T + 1, n * n), ("Vx", _abi.Q_VX, d.T + 1, n)]:
        G, O = g.quantity(q, nk, per), o.quantity(q, nk, per)
        row(name, G, O)
        if name in ("k", "K"):
            for t in range(nk):
                nw, ew = errs(G[:, t], O[:, t])
                print(f"      t={t} normwise {nw:9.2e} elementwise {ew:9.2e}")
    # cond of Quu per knot (from the oracle's blocks)
    Quu = o.quantity(_abi.Q_QUU, d.T, m * m)
    conds = [np.linalg.cond(Quu[0, t].reshape(m, m)[:S["knots"][t][1], :S["knots"][t][1]])
             if S["knots"][t][1] else 0 for t in range(d.T)]
    print("  cond(Quu) elem 0 per knot:", " ".join(f"{c:.1e}" for c in conds))

    print("phase 3: expected improvement and tryStep", flush=True)
    g.update_expected_improvement()
    o.update_expected_improvement()
    for a in (1.0, 0.5, 0.25):
        dg, stg = g.try_step(a)
        do, sto = o.try_step(a)
        print(f" alpha {a}: status gpu {stg.tolist()} oracle {sto.tolist()}")
        row("dV", dg, do)
        row("xs_try", g.xs(trial=True), o.xs(trial=True))
        row("us_try", g.us(trial=True), o.us(trial=True))
        row("d(EI)", g.expected_improvement(), o.expected_improvement())

    print("phase 4: whole solves from the warm start", flush=True)
    for it in range(1, maxit + 1):
        g, o = fresh()
        rg = helpers.results_dict(g.solve(maxiter=it))
        ro = helpers.results_dict(o.solve(maxiter=it))
        print(f" maxiter={it}: steplength gpu {rg['steplength'].tolist()} oracle {ro['steplength'].tolist()} "
              f"iter {rg['iter'].tolist()} / {ro['iter'].tolist()}")
        row("xs", g.xs(), o.xs())
        row("us", g.us(), o.us())
        row("cost", rg["cost"], ro["cost"])
        row("stop", rg["stop"], ro["stop"])
        row("xreg", rg["xreg"], ro["xreg"])


if __name__ == "__main__":
    main()
