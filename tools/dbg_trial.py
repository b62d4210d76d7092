"""Diagnostic: Talos walk T=6 try_step(alpha) cost / xs vs the oracle, per knot."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import helpers
from crocoddyl_amd import _abi, synthetic
from crocoddyl_amd.problem import pack_problem
from oracle import fddp_np
name = sys.argv[1] if len(sys.argv) > 1 else "C5_talos_walk"
T, B = 6, 1
x0s, running, terminal = synthetic.build(name, T=T, B=B)
st = running[0].state
knots, pool = pack_problem(running, terminal, B)
d = _abi.Dims(st.nx, st.ndx, max(r.nu for r in running), T, B)
g = helpers.Gpu(d, knots, pool, x0s)
xs, us = synthetic.gait_warm_start(name, running, x0s[0])
ua = np.zeros((T, d.nu_max))
for t, u in enumerate(us):
    ua[t, :len(u)] = u
xs = np.array(xs)
g.set_candidate(xs[None], ua[None], is_feasible=False)
g.set_solver_state(it=0, xreg=1e-6, ureg=1e-6)
print("dir status", g.compute_direction(True))
g.update_expected_improvement()
o = fddp_np.FDDP(x0s[0], fddp_np.bind_problem(knots, pool, 0, d.nx))
o.set_candidate(list(xs), [ua[t, :running[t].nu] for t in range(T)], is_feasible=False)
o.iter, o.xreg, o.ureg = 0, 1e-6, 1e-6
o.compute_direction(True)
o.update_expected_improvement()
for alpha in (1.0, 0.5):
    dV, stt = g.try_step(alpha)
    dvo = o.try_step(alpha)
    xt = g.xs(trial=True)[0]
    kc = g.quantity(_abi.Q_KCOST, T + 1, 1)[0, :, 0] if hasattr(_abi, "Q_KCOST") else None
    print("alpha", alpha, "dV gpu", dV[0], "oracle", dvo, "status", stt)
    for t in range(T + 1):
        print(t, helpers.rel_err(xt[t], np.array(o.xs_try[t])))
