"""Diagnostic: C3 fixed-protocol steps: per-step backward time and the per-element state."""
import os
import sys
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT", ".")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import helpers  # noqa: E402

s = bench.make_shard_solver(os.environ.get("CFG", "C3_arm_multibody"), 512, 0, 0, presolve=False)
step = bench.FixedWarmStart(s, 0)
for k in range(6):
    s.get_timing()
    s.set_timing(True)
    t0 = time.perf_counter()
    step(1)
    s.synchronize()
    t = s.get_timing()
    s.set_timing(False)
    r = helpers.results_dict(s._res())
    print(k, "wall %.2f" % ((time.perf_counter() - t0) * 1e3), "bwd %.3f" % t["backward"][0],
          "xreg", np.unique(np.round(r["xreg"], 12)).tolist()[:6], "cost %.15g" % float(np.sum(r["cost"])), flush=True)
