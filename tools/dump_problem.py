"""Write a config's packed problem + bench warm start for oracle/cpu_driver (test
infrastructure: the CPU oracle's standalone driver).

usage: python tools/dump_problem.py CONFIG B OUT_FILE"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import bench  # noqa: E402
import helpers  # noqa: E402
from crocoddyl_amd import synthetic  # noqa: E402


def main():
    cfg, B, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    S = helpers.setup(cfg, B=B, seed=synthetic.seed_of(cfg))
    d = S["dims"]
    xs, us = bench.warm_start_arrays(cfg, S["running"], S["x0s"], d)
    kd = np.zeros(len(S["knots"]), dtype=[("kind", "<i4"), ("nu", "<i4"), ("off", "<i8"), ("stride", "<i8")])
    for i, k in enumerate(S["knots"]):
        kd[i] = k
    with open(out, "wb") as f:
        np.array([d.nx, d.ndx, d.nu_max, d.T, d.B], "<i4").tofile(f)
        np.array([len(kd)], "<i8").tofile(f)
        kd.tofile(f)
        np.array([S["pool"].size], "<i8").tofile(f)
        S["pool"].astype("<f8").tofile(f)
        np.ascontiguousarray(S["x0s"], "<f8").tofile(f)
        for a in (xs, us):
            np.array([0 if a is None else 1], "<i4").tofile(f)
            if a is not None:
                np.ascontiguousarray(a, "<f8").tofile(f)
    print(f"wrote {out}: {cfg} nx={d.nx} ndx={d.ndx} nu={d.nu_max} T={d.T} B={d.B}")


if __name__ == "__main__":
    main()
