"""Diagnostics: statuses / costs of the contact bench problem over a few solves."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import crocoddyl_amd as crocoddyl
from crocoddyl_amd import synthetic

for T, B in [(20, 4), (250, 8)]:
    x0s, running, terminal = synthetic.build("C3_arm_contact", T=T, B=B)
    problem = crocoddyl.ShootingProblem(x0s, running, terminal)
    solver = crocoddyl.SolverFDDP(problem)
    for it in range(6):
        solver.solve(np.repeat(x0s[:, None, :], T + 1, axis=1), [], 5) if it == 0 else solver.solve_from_candidate(maxiter=1, isFeasible=False, regInit=0.1)
        print(T, it, "status", np.array(solver.status).tolist(), "iter", list(solver.n_iter_run),
              "cost", np.round(np.array(solver.cost), 4).tolist(), "step", np.array(solver.stepLength).tolist(),
              "xreg", np.array(solver.x_reg).tolist(), flush=True)
