"""The reference's DDP-phase timing harness (benchmark/arm-kinova-codegen.cpp:258-285)
ported onto the C++ facade (tests/cpp/arm_phases.cpp): calcDiff, then backwardPass and
forwardPass(0.005) called one at a time through crocoddyl_amd::SolverFDDP.
  * CPU: it compiles against include/, links libfddp_hip and packs its problem;
  * GPU: its calcDiff cost, gains K / k after backwardPass and cost_try / xs_try / us_try
    after forwardPass(0.005) match the C++ oracle's same phases on the packed problem,
    and an invalid step length throws (fddp.cpp:150-153)."""
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
N = 100


def _build(tmp_path):
    exe = str(tmp_path / "arm_phases")
    lib = os.path.join(ROOT, "crocoddyl_amd", "lib")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-I", os.path.join(ROOT, "include"),
                    os.path.join(HERE, "cpp", "arm_phases.cpp"), "-L", lib, "-lfddp_hip", f"-Wl,-rpath,{lib}",
                    "-o", exe], check=True)
    return exe


def _read_pack(path):
    with open(path, "rb") as f:
        dims = np.frombuffer(f.read(16), "<i4")
        nk = int(np.frombuffer(f.read(8), "<i8")[0])
        kd = np.frombuffer(f.read(24 * nk), dtype=[("kind", "<i4"), ("nu", "<i4"), ("off", "<i8"), ("stride", "<i8")])
        n = int(np.frombuffer(f.read(8), "<i8")[0])
        pool = np.frombuffer(f.read(8 * n), "<f8").copy()
    return dims, [tuple(int(v) for v in k) for k in kd], pool


def test_cpp_phases_compiles_and_packs(tmp_path):
    exe = _build(tmp_path)
    out = str(tmp_path / "pack.bin")
    r = subprocess.run([exe, "pack", out], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    dims, knots, pool = _read_pack(out)
    assert list(dims) == [12, 12, 6, N]
    # one shared running block (std::vector(N, model)) + the terminal block
    assert len(knots) == N + 1 and len({k[2] for k in knots[:N]}) == 1 and knots[N][2] != knots[0][2]
    assert all(k[0] == 4 for k in knots)  # Euler over FreeFwdDynamics


@pytest.mark.gpu
def test_cpp_phases_match_the_oracle(tmp_path):
    import helpers
    import oracle_lib
    from crocoddyl_amd import _abi
    exe = _build(tmp_path)
    pk, res = str(tmp_path / "pack.bin"), str(tmp_path / "phases.bin")
    assert subprocess.run([exe, "pack", pk], capture_output=True, timeout=60).returncode == 0
    r = subprocess.run([exe, "phases", res, "20"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    print(r.stdout)
    assert "backwardPass [us]" in r.stdout and "forwardPass [us]" in r.stdout
    assert "invalid_step_throws=1" in r.stdout
    dims, knots, pool = _read_pack(pk)
    nx, ndx, nu, T = (int(v) for v in dims)
    flat = np.frombuffer(open(res, "rb").read(), "<f8")
    sizes = [("cost", 1), ("K", T * nu * ndx), ("k", T * nu), ("cost_try", 1), ("xs_try", (T + 1) * nx),
             ("us_try", T * nu), ("x0", nx)]
    g, o = {}, 0
    for name, s in sizes:
        g[name] = flat[o:o + s]
        o += s
    assert o == flat.size
    x0 = g["x0"]
    orc = oracle_lib.Oracle(_abi.Dims(nx, ndx, nu, T, 1), knots, pool, x0[None])
    orc.set_candidate(np.repeat(x0[None, None], T + 1, axis=1), np.zeros((1, T, nu)), False)
    orc.set_solver_state(it=0)
    cost = orc.ddp_calc_diff()
    assert orc.backward_pass()[0] == 0
    rc, ct, st = orc.forward_pass(0.005)
    assert rc == 0 and st[0] == 0
    helpers.parity("arm cost", g["cost"], cost, 1e-8)
    helpers.parity("arm K", g["K"].reshape(T, nu * ndx), orc.quantity(_abi.Q_K, T, nu * ndx)[0], 1e-8)
    helpers.parity("arm k", g["k"].reshape(T, nu), orc.quantity(_abi.Q_KV, T, nu)[0], 1e-8)
    helpers.parity("arm cost_try", g["cost_try"], ct, 1e-8)
    helpers.parity("arm xs_try", g["xs_try"].reshape(T + 1, nx), orc.xs(trial=True)[0], 1e-8)
    helpers.parity("arm us_try", g["us_try"].reshape(T, nu), orc.us(trial=True)[0], 1e-8)
