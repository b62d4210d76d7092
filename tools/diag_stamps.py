"""Diagnostic (not a test): per-phase cycle breakdown of the MFMA Riccati sweep."""
import os
import sys
import time

os.environ["FDDP_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crocoddyl_amd import ShootingProblem, SolverFDDP, synthetic  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C5_talos_full"
x0s, running, terminal = synthetic.build(cfg)
p = ShootingProblem(x0s, running, terminal)
s = SolverFDDP(p)
s.solve(maxiter=1)
s.set_timing(True)
t0 = time.time()
s.solve_from_candidate(maxiter=1)
s.synchronize()
print(cfg, "solve ms", (time.time() - t0) * 1e3, s.get_timing(), flush=True)
del s, p
