"""Diagnostics: one rollout (tryStep) / calc / calcDiff time, free vs contact arm."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import crocoddyl_amd as crocoddyl
from crocoddyl_amd import synthetic

for cfg in ["C3_arm_multibody", "C3_arm_contact"]:
    x0s, running, terminal = synthetic.build(cfg)
    T = len(running)
    problem = crocoddyl.ShootingProblem(x0s, running, terminal)
    solver = crocoddyl.SolverFDDP(problem)
    solver.solve(np.repeat(x0s[:, None, :], T + 1, axis=1), [], 3)
    solver.computeDirection(True)
    for a in (1.0, 1.0, 0.5):
        solver.synchronize()
        t0 = time.perf_counter()
        solver.tryStep(a)
        solver.synchronize()
        print(cfg, "tryStep", a, round((time.perf_counter() - t0) * 1e3, 2), "ms", flush=True)
    for _ in range(2):
        t0 = time.perf_counter()
        problem.calc(solver.xs, solver.us) if hasattr(problem, "calc") else None
        solver.synchronize()
        print(cfg, "problem.calc", round((time.perf_counter() - t0) * 1e3, 2), "ms", flush=True)
