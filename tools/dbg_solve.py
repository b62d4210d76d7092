"""Diagnostic: Talos walk T=6 solve(maxiter=k) GPU vs oracle: iter, cost, steplength, xreg."""
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
for mi in (1, 2, 3, 4):
    g = helpers.Gpu(d, knots, pool, x0s)
    g.set_candidate(xs[None], ua[None])
    r = helpers.results_dict(g.solve(maxiter=mi, is_feasible=False, reg_init=1e-9))
    o = fddp_np.FDDP(x0s[0], fddp_np.bind_problem(knots, pool, 0, d.nx))
    o.solve(list(xs), [ua[t, :running[t].nu] for t in range(T)], maxiter=mi, is_feasible=False, reg_init=1e-9)
    print(mi, "gpu", r["iter"][0], r["cost"][0], r["steplength"][0], r["xreg"][0], "| oracle", o.iter, o.cost,
          o.steplength, o.xreg, flush=True)
