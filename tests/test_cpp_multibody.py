"""The C++ drop-in for the legged-robot path (include/crocoddyl_amd/multibody.hpp).

tests/cpp/trot_example.cpp builds the C4 Solo12 trotting problem the way a C++ user
of the reference does (robot model, SimpleQuadrupedGaitProblem's trotting phases:
Euler ∘ ContactFwdDynamics knots with 3D contacts, friction cones, CoM / foot
tracking, state bounds, impulse foot switches) on the C++ facade, and
  * CPU: packs it; the knot descriptors and the parameter pool must equal, double
    for double, what the Python facade packs for the same gait (crocoddyl_amd.gaits);
  * GPU: solves it with the facade's SolverFDDP through the C ABI; the result must
    match the C++ oracle run on the same packed problem from the same warm start
    (identical status / iterations / step length, xs / us / cost within 1e-6)."""
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
T = 60


def _build(tmp_path):
    exe = str(tmp_path / "trot_example")
    lib = os.path.join(ROOT, "crocoddyl_amd", "lib")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-I", os.path.join(ROOT, "include"),
                    os.path.join(HERE, "cpp", "trot_example.cpp"), "-L", lib, "-lfddp_hip", f"-Wl,-rpath,{lib}",
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


def test_cpp_trot_packs_as_the_python_facade(tmp_path):
    from crocoddyl_amd import synthetic
    from crocoddyl_amd.problem import pack_problem
    exe = _build(tmp_path)
    out = str(tmp_path / "pack.bin")
    r = subprocess.run([exe, "pack", out], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    dims, knots, pool = _read_pack(out)
    _, running, terminal = synthetic.gait_models("C4_solo12_trot", T)
    knots_py, pool_py = pack_problem(running, terminal, 1)
    assert list(dims) == [37, 36, 12, T]
    assert knots == [tuple(k) for k in knots_py]
    assert pool.size == pool_py.size
    same = (pool == pool_py) | (np.isnan(pool) & np.isnan(pool_py))
    assert same.all(), np.where(~same)[0][:10]
    kinds = [k[0] for k in knots]
    # two impulse foot switches (the second is also the terminal knot), the rest contact knots
    assert kinds.count(6) == 3 and kinds.count(5) == T + 1 - 3


@pytest.mark.gpu
def test_cpp_trot_solves_on_gpu_as_the_oracle(tmp_path):
    import oracle_lib
    from crocoddyl_amd import _abi
    exe = _build(tmp_path)
    pk, res = str(tmp_path / "pack.bin"), str(tmp_path / "solve.bin")
    assert subprocess.run([exe, "pack", pk], capture_output=True, timeout=60).returncode == 0
    r = subprocess.run([exe, "solve", res, "3"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    dims, knots, pool = _read_pack(pk)
    nx, ndx, nu, _ = (int(v) for v in dims)
    with open(res, "rb") as f:
        rg = _abi.Result.from_buffer_copy(f.read(C_SIZE := __import__("ctypes").sizeof(_abi.Result)))
        flat = np.frombuffer(f.read(), "<f8")
    xs_g = flat[:(T + 1) * nx].reshape(T + 1, nx)
    us_g = flat[(T + 1) * nx:].reshape(T, nu)
    assert C_SIZE == 88
    from crocoddyl_amd import synthetic
    g, _, _ = synthetic.gait_models("C4_solo12_trot", T)
    x0 = g.rmodel.defaultState
    o = oracle_lib.Oracle(_abi.Dims(nx, ndx, nu, T, 1), knots, pool, x0[None])
    o.set_candidate(np.repeat(x0[None, None], T + 1, axis=1), None, False)
    ro = o.solve(maxiter=3, is_feasible=False, reg_init=1e-9)[0]
    assert (rg.status, rg.iter, rg.steplength) == (ro.status, ro.iter, ro.steplength), r.stdout
    assert abs(rg.cost - ro.cost) <= 1e-6 * abs(ro.cost)
    xo, uo = o.xs()[0], o.us()[0]
    assert np.max(np.abs(xs_g - xo)) / max(1.0, np.max(np.abs(xo))) < 1e-6
    assert np.max(np.abs(us_g - uo)) / max(1.0, np.max(np.abs(uo))) < 1e-6
