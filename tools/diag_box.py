"""Diagnostic (not a test): phase stamps of SolverBoxFDDP's backward sweep on one bench
step (--solver boxfddp protocol: restart from a feasible presolved iterate). Stamps
build: CROCODDYL_AMD_LIB=.../libfddp_hip_stamps.so (FDDP_STAMPS=1 is set here).
  python tools/diag_box.py [config] [B]"""
import os
import sys

os.environ["FDDP_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from crocoddyl_amd import synthetic  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C5_talos_walk"
B = int(sys.argv[2]) if len(sys.argv) > 2 else synthetic.CONFIGS[cfg][4]
s = bench.make_shard_solver(cfg, B, 0, 0, box=True, presolve=False)
fr = bench.FeasibleRestart(s, 0)
s.set_timing(True)
fr(1)
s.synchronize()
print(cfg, "B", B, "box step", s.get_timing(), flush=True)
del fr
del s
