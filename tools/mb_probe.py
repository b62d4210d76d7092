"""Diagnostic (not a test): writes one knot of a config (block, x, u) for
tools/mb_probe and runs it. Usage: python tools/mb_probe.py <config> <knot> <nwg>
(PROBE_BIN: another probe build; PROBE_COSTS=a,b keeps only those cost records active; PROBE_COSTS= none; a 4th
argument "layout" prints the LDS plan only, no GPU needed).
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from crocoddyl_amd import synthetic  # noqa: E402

cfg, t, nwg = sys.argv[1], int(sys.argv[2]), sys.argv[3]
x0s, running, terminal = synthetic.build(cfg, B=1)
m = running[t] if t < len(running) else terminal
keep = os.environ.get("PROBE_COSTS")  # comma-separated cost names to keep active ("" = none)
if keep is not None:
    dam = getattr(m, "differential", m)
    for name, it in dam.costs.costs.items():
        it.active = name in keep.split(",")
    print("costs kept:", [n for n, it in dam.costs.costs.items() if it.active])
kind, nu, blk = m.pack()
blk = np.ascontiguousarray(blk[0], np.float64)
mm = max(r.nu for r in running)
x = x0s[0]
u = np.zeros(max(mm, 1))
if nu and hasattr(m, "quasiStatic"):
    u[:nu] = m.quasiStatic(None, x)
path = os.path.join(ROOT, "gpurun_out", f"probe_{cfg}_{t}.bin")
os.makedirs(os.path.dirname(path), exist_ok=True)
with open(path, "wb") as f:
    np.array([x.size, nu, mm, blk.size], np.int32).tofile(f)
    blk.tofile(f)
    x.astype(np.float64).tofile(f)
    u.astype(np.float64).tofile(f)
sys.exit(subprocess.call([os.environ.get("PROBE_BIN", os.path.join(ROOT, "tools", "mb_probe")), path, nwg] + sys.argv[4:]))
