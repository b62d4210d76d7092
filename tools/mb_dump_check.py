"""Parity diagnosis of one multibody calcDiff (test tooling): compares the LDS
matrices tools/mb_probe dumps from the device calcDiff (multibody.hpp MB_DUMP: M, nle,
Jc^T, a0, M^-1, the KKT inverse's top-left block, a, Y, S^-1, H) and its Fu block with
the numpy oracle's (oracle/multibody_np.py: local-frame CRBA / RNEA, frame Jacobians),
reporting the normwise and element-wise relative errors.

  python tools/mb_probe.py C5_talos_walk <knot> 1 dump     (GPU: writes the .dump)
  python tools/mb_dump_check.py C5_talos_walk <knot>        (CPU)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from crocoddyl_amd import synthetic  # noqa: E402
from oracle import multibody_np as onp  # noqa: E402

SLOTS, CAP = 12, 4096
NAMES = ["M", "nle", "JcT", "a0", "Minv", "Kinv_tl", "a", "Y", "Sinv", "H"]


def errs(g, o):
    scale = float(np.max(np.abs(o)))
    d = np.abs(g - o)
    mask = np.abs(o) >= 1e-6 * max(scale, 1e-300)
    return float(d.max()) / max(scale, 1e-300), float(np.max(d[mask] / np.abs(o[mask]))) if mask.any() else 0.0


def host_run(blk, nx, nu, mm, x, u):
    """The device code compiled for the host (tests/cpp/mb_host.cpp): its MB_DUMP slots
    and output blocks, in the probe's layout."""
    import ctypes as C
    import subprocess
    src = os.path.join(ROOT, "tests", "cpp", "mb_host.cpp")
    out = os.path.join(ROOT, "tests", "_build", "libmb_host.so")
    hdr = os.path.join(ROOT, "crocoddyl_amd", "csrc", "multibody.hpp")
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "-O2", "-std=c++17",
                               "-shared", "-fPIC", "-o", out, src])
    Dp = C.POINTER(C.c_double)
    L = C.CDLL(out)
    L.mb_host_calc_diff.argtypes = [Dp, C.c_int, C.c_int, Dp, Dp, C.c_int] + [Dp] * 9
    n = 2 * int(blk[1])
    so = 2 * n * n + 2 * n * mm + mm * mm + n + mm + nx + 2
    ob = np.zeros(so)
    offs = np.cumsum([0, n * n, n * mm, n * n, n * mm, mm * mm, n, mm, nx])
    ptrs = [ob[o:].ctypes.data_as(Dp) for o in offs]
    uu = np.ascontiguousarray(u)
    L.mb_host_calc_diff(blk.ctypes.data_as(Dp), int(nx), int(mm), np.ascontiguousarray(x).ctypes.data_as(Dp),
                        uu.ctypes.data_as(Dp), 1 if nu else 0, *ptrs)
    sh = np.zeros(2 * SLOTS, np.int32)
    dm = np.zeros(SLOTS * CAP)
    L.mb_host_dump(sh.ctypes.data_as(C.POINTER(C.c_int)), dm.ctypes.data_as(Dp))
    return sh.reshape(SLOTS, 2), dm.reshape(SLOTS, CAP), ob


def main():
    host = "--host" in sys.argv
    args = [a for a in sys.argv[1:] if a != "--host"]
    cfg, t = args[0], int(args[1])
    path = os.path.join(ROOT, "gpurun_out", f"probe_{cfg}_{t}.bin")
    if host and not os.path.exists(path):  # write the probe input as tools/mb_probe.py does
        x0s, running, terminal = synthetic.build(cfg, B=1)
        mdl = running[t] if t < len(running) else terminal
        kind, nu_, blk_ = mdl.pack()
        blk_ = np.ascontiguousarray(blk_[0], np.float64)
        mm_ = max(r.nu for r in running)
        uu = np.zeros(max(mm_, 1))
        if nu_ and hasattr(mdl, "quasiStatic"):
            uu[:nu_] = mdl.quasiStatic(None, x0s[0])
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "wb") as f:
            np.array([x0s.shape[1], nu_, mm_, blk_.size], np.int32).tofile(f)
            blk_.tofile(f)
            x0s[0].astype(np.float64).tofile(f)
            uu.tofile(f)
    with open(path, "rb") as f:
        nx, nu, mm, psz = np.fromfile(f, np.int32, 4)
        blk = np.fromfile(f, np.float64, psz)
        x = np.fromfile(f, np.float64, nx)
        u = np.fromfile(f, np.float64, max(mm, 1))
    if host:
        sh, dm, ob = host_run(blk, nx, nu, mm, x, u)
    else:
        with open(path + ".dump", "rb") as f:
            sh = np.fromfile(f, np.int32, 2 * SLOTS).reshape(SLOTS, 2)
            dm = np.fromfile(f, np.float64, SLOTS * CAP).reshape(SLOTS, CAP)
            so = int(np.fromfile(f, np.int64, 1)[0])
            ob = np.fromfile(f, np.float64, so)
    dev = {}
    for s, name in enumerate(NAMES):
        r, c = sh[s]
        if r > 0:
            dev[name] = dm[s, :r * c].reshape(c, r).T  # column-major
    k = onp.ContactFwdKnot(blk, nx, nu)
    rb = k.robot
    q, v = x[:k.nq], x[k.nq:]
    M = rb.crba(q) + np.diag(rb.armature)
    nle = rb.rnea(q, v, np.zeros(k.nv))
    Jc, a0 = k.contact_terms(x)
    Minv = np.linalg.inv(M)
    Y = Minv @ Jc.T
    S = Jc @ Y + k.damping * np.eye(Jc.shape[0])
    Sinv = np.linalg.inv(S)
    H = Y @ Sinv
    G = Minv - H @ Y.T
    a, lam = k.accel_force(x, u[:nu])
    ref = {"M": M, "nle": nle[:, None], "JcT": Jc.T, "a0": a0[:, None], "Minv": Minv, "Kinv_tl": G, "a": a[:, None],
           "Y": Y, "Sinv": Sinv, "H": H}
    print(("host build" if host else "device") + f" {cfg} knot {t}: nv={k.nv} nc={Jc.shape[0]} cond(M)={np.linalg.cond(M):.2e} cond(S)={np.linalg.cond(S):.2e}")
    for name in NAMES:
        if name in dev:
            g, o = dev[name], ref[name]
            if g.shape != o.shape:
                print(f"  {name:8s} shape {g.shape} vs {o.shape}")
                continue
            nw, ew = errs(g, o)
            print(f"  {name:8s} normwise {nw:9.2e} elementwise {ew:9.2e}")
    n = 2 * k.nv
    m = mm
    Fu_dev = ob[n * n:n * n + n * m].reshape(m, n).T[:, :nu]
    Fx_dev = ob[:n * n].reshape(n, n).T
    d = k.calc_diff(x, u[:nu])
    for name, g in (("Fx", Fx_dev), ("Fu", Fu_dev)):
        nw, ew = errs(g, d[name])
        print(f"  {name:8s} normwise {nw:9.2e} elementwise {ew:9.2e}  (vs the numpy oracle's complex-step derivative)")


if __name__ == "__main__":
    main()
