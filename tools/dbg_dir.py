"""Diagnostic: after solve(maxiter=1), compute_direction at the same candidate on the GPU
and in the oracle; per-knot max rel err of the derivative blocks and of K, k."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import helpers
from crocoddyl_amd import _abi, synthetic
from crocoddyl_amd.problem import pack_problem
from oracle import fddp_np
name = "C5_talos_walk"
T, B = 6, 1
x0s, running, terminal = synthetic.build(name, T=T, B=B)
st = running[0].state
knots, pool = pack_problem(running, terminal, B)
d = _abi.Dims(st.nx, st.ndx, max(r.nu for r in running), T, B)
xs, us = synthetic.gait_warm_start(name, running, x0s[0])
ua = np.zeros((T, d.nu_max))
for t, u in enumerate(us):
    ua[t, :len(u)] = u
xs = np.array(xs)
o = fddp_np.FDDP(x0s[0], fddp_np.bind_problem(knots, pool, 0, d.nx))
o.solve(list(xs), [ua[t, :running[t].nu] for t in range(T)], maxiter=1, is_feasible=False, reg_init=1e-9)
X = np.array(o.xs)
U = np.zeros((T, d.nu_max))
for t in range(T):
    U[t, :running[t].nu] = np.asarray(o.us[t])[:running[t].nu]
g = helpers.Gpu(d, knots, pool, x0s)
g.set_candidate(X[None], U[None], is_feasible=True)
g.set_solver_state(it=int(os.environ.get("DBG_IT", "1")), xreg=1e-9, ureg=1e-9, was_feasible=1)
print("status", g.compute_direction(True))
o2 = fddp_np.FDDP(x0s[0], fddp_np.bind_problem(knots, pool, 0, d.nx))
o2.set_candidate(list(X), [U[t, :running[t].nu] for t in range(T)], is_feasible=True)
o2.iter, o2.xreg, o2.ureg = 0, 1e-9, 1e-9
o2.compute_direction(True)
n, m = d.ndx, d.nu_max
Q = {k: g.quantity(q, T + 1, s) for k, q, s in [("Fx", _abi.Q_FX, n * n), ("Fu", _abi.Q_FU, n * m),
      ("Lxx", _abi.Q_LXX, n * n), ("Lxu", _abi.Q_LXU, n * m), ("Luu", _abi.Q_LUU, m * m), ("Lx", _abi.Q_LX, n),
      ("Lu", _abi.Q_LU, m)]}
for t in range(T + 1):
    ref = o2.data[t]
    errs = {}
    for name2, shape in [("Fx", (n, n)), ("Fu", (n, m)), ("Lxx", (n, n)), ("Lxu", (n, m)), ("Luu", (m, m)),
                         ("Lx", (n,)), ("Lu", (m,))]:
        got = Q[name2][0, t].reshape(shape[::-1]).T if len(shape) == 2 else Q[name2][0, t]
        want = ref[name2]
        if name2 in ("Fu", "Lxu"):
            got = got[:, :want.shape[1]]
        elif name2 == "Luu":
            got = got[:want.shape[0], :want.shape[0]]
        elif name2 == "Lu":
            got = got[:want.shape[0]]
        if want.size:
            errs[name2] = helpers.rel_err(got, want)
    print(t, {k: f"{v:.1e}" for k, v in errs.items()}, flush=True)
print("Lx0 gpu", Q["Lx"][0, 0][:8])
print("Lx0 ora", o2.data[0]["Lx"][:8])
print("Lu0 gpu", Q["Lu"][0, 0][:6])
print("Lu0 ora", o2.data[0]["Lu"][:6])
Kg = g.quantity(_abi.Q_K, T, m * n)
kg = g.quantity(_abi.Q_KV, T, m) if hasattr(_abi, "Q_KV") else None
for t in range(T):
    nu = running[t].nu
    if nu:
        Kt = Kg[0, t].reshape(n, m).T[:nu]
        print("K", t, helpers.rel_err(Kt, np.asarray(o2.K[t])[:nu]))
