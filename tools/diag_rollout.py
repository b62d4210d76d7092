"""Diagnostic (not a test): per-phase cycles of the rollout kernels on one bench step of a
config (stamps build: CROCODDYL_AMD_LIB=.../libfddp_hip_stamps.so; FDDP_STAMPS=1 is set
here). Prints the kernel times of the step; the handle's destructor prints the stamps.
  python tools/diag_rollout.py [config] [B] [steps]"""
import os
import sys

os.environ["FDDP_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C5_talos_walk"
B = int(sys.argv[2]) if len(sys.argv) > 2 else None
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
from crocoddyl_amd import synthetic  # noqa: E402
B = B or synthetic.CONFIGS[cfg][4]
s = bench.make_shard_solver(cfg, B, 0, 0, presolve=False)
fw = bench.FixedWarmStart(s, 0)
s.set_timing(True)
for _ in range(steps):
    fw(1)
s.synchronize()
print(cfg, "B", B, "steps", steps, s.get_timing(), "trials", bench.trials_summary(bench.line_search_trials(s)), flush=True)
del fw
del s
