"""Diagnostic (not a test): where the host time of one bench step goes (config's fixed
protocol): the Python facade calls, the C ABI solve, and the device time between the
step's first and last kernel (HIP events on the solver stream).
  python tools/diag_host.py [config] [steps]"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
from crocoddyl_amd import _abi, synthetic  # noqa: E402
from crocoddyl_amd._lib import lib  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2_lqr"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
B = synthetic.CONFIGS[cfg][4]
s = bench.make_shard_solver(cfg, B, 0, 0, presolve=False)
fw = bench.FixedWarmStart(s, 0)
for _ in range(5):
    fw(1)
s.synchronize()
L = lib()
acc = {"refresh": 0., "set_candidate_device": 0., "set_params": 0., "fddp_solve": 0., "n_iter_run": 0., "step": 0.}
ptr0 = s._ptr
r = (_abi.Result * B)()
for _ in range(steps):
    t0 = time.perf_counter()
    ptr = s._ptr
    t1 = time.perf_counter()
    L.fddp_set_candidate_device(ptr, None if fw.xs is None else C.cast(C.c_void_p(fw.xs.data_ptr()), _abi.D),
                                None if fw.us is None else C.cast(C.c_void_p(fw.us.data_ptr()), _abi.D), 0)
    t2 = time.perf_counter()
    L.fddp_set_params(ptr, C.byref(s._prm))
    t3 = time.perf_counter()
    L.fddp_solve(ptr, 1, 0, 0.1, r)
    t4 = time.perf_counter()
    s._results = r
    int(np.sum(s.n_iter_run))
    t5 = time.perf_counter()
    for k, v in (("refresh", t1 - t0), ("set_candidate_device", t2 - t1), ("set_params", t3 - t2),
                 ("fddp_solve", t4 - t3), ("n_iter_run", t5 - t4), ("step", t5 - t0)):
        acc[k] += v
print(cfg, {k: round(v / steps * 1e3, 4) for k, v in acc.items()}, "ms per step", flush=True)
# the facade's own step
t0 = time.perf_counter()
for _ in range(steps):
    fw(1)
    int(np.sum(s.n_iter_run))
s.synchronize()
print(cfg, "facade step", round((time.perf_counter() - t0) / steps * 1e3, 4), "ms", flush=True)
s.set_timing(True)
t0 = time.perf_counter()
for _ in range(steps):
    fw(1)
    int(np.sum(s.n_iter_run))
s.synchronize()
print(cfg, "facade step (timing on)", round((time.perf_counter() - t0) / steps * 1e3, 4), "ms", s.get_timing(), flush=True)
