"""The C++ facade (include/crocoddyl_amd/solver_fddp_hip.hpp) compiles against
the C ABI and links libfddp_hip (CPU); on the GPU the example solves an
LQR(24,12) T=100 and the unicycle-towards-origin problem and matches the
oracle's cost (GPU)."""
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _build(tmp_path):
    exe = str(tmp_path / "facade_example")
    lib = os.path.join(ROOT, "crocoddyl_amd", "lib")
    subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"),
                    os.path.join(HERE, "cpp", "facade_example.cpp"), "-L", lib, "-lfddp_hip",
                    f"-Wl,-rpath,{lib}", "-o", exe], check=True)
    return exe


def test_facade_compiles_and_links(tmp_path):
    exe = _build(tmp_path)
    assert os.path.exists(exe)


@pytest.mark.gpu
def test_facade_solves_on_gpu(tmp_path):
    exe = _build(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = dict(l.split(" ", 1) for l in r.stdout.strip().splitlines() if " " in l)
    assert "converged=1" in lines["lqr"] and "converged=1" in lines["unicycle"]
    assert "setter" in r.stdout and "validation ok" in r.stdout
    # cost parity with the CPU oracle on the same problems
    import oracle_lib
    from crocoddyl_amd import _abi
    from crocoddyl_amd.models import ActionModelLQR, ActionModelUnicycle
    from crocoddyl_amd.problem import pack_problem
    for key, model, T, x0 in [("lqr", ActionModelLQR(24, 12, False), 100, np.zeros(24)),
                              ("unicycle", ActionModelUnicycle(), 30, np.array([-1.0, -1.0, 1.0]))]:
        knots, pool = pack_problem([model] * T, model, 1)
        o = oracle_lib.Oracle(_abi.Dims(len(x0), len(x0), model.nu, T, 1), knots, pool, x0[None])
        o.set_candidate(None, None, False)
        r0 = o.solve(100)[0]
        cost = float(lines[key].split("cost=")[1].split()[0])
        assert abs(cost - r0.cost) <= 1e-6 * max(1, abs(r0.cost))
        assert f"iter={r0.iter}" in lines[key]
    # per-iteration callbacks: the logger's rows == the oracle's per-iteration trace of
    # the unicycle solve (cost, stop, steplength, xreg, grad = -d[1]), CallbackVerbose on stderr
    model = ActionModelUnicycle()
    knots, pool = pack_problem([model] * 30, model, 1)
    o = oracle_lib.Oracle(_abi.Dims(3, 3, 2, 30, 1), knots, pool, np.array([[-1.0, -1.0, 1.0]]))
    o.set_candidate(None, None, False)
    o.solve(100)
    tr = o.trace(0)
    rows = [lines[f"trace{i}"] for i in range(len(tr))]
    assert f"trace{len(tr)}" not in lines
    for rec, row in zip(tr, rows):
        got = {kv.split("=")[0]: float(kv.split("=")[1]) for kv in row.split()}
        for key, want in (("cost", rec[0]), ("stop", rec[1]), ("step", rec[6]), ("xreg", rec[4]), ("grad", -rec[3])):
            assert abs(got[key] - want) <= 1e-9 * max(1.0, abs(want)), (key, got[key], want)
    assert r.stderr.count("iter") >= 1 and "dV-exp" in r.stderr
    # SolverBoxFDDP on the limited LQR
    assert "converged=1" in lines["box"] and "th_stop=5.0e-05" in lines["box"]
    model = ActionModelLQR(24, 12, False)
    knots, pool = pack_problem([model] * 100, model, 1)
    o = oracle_lib.Oracle(_abi.Dims(24, 24, 12, 100, 1), knots, pool, np.zeros((1, 24)))
    o.set_solver_kind(_abi.SOLVER_BOXFDDP)
    o.set_control_limits(np.full((1, 100, 12), -0.05), np.full((1, 100, 12), 0.05))
    p = oracle_lib.default_params()
    p.th_stop = 5e-5
    o.set_params(p)
    o.set_candidate(None, None, False)
    r0 = o.solve(100)[0]
    cost = float(lines["box"].split("cost=")[1].split()[0])
    assert abs(cost - r0.cost) <= 1e-6 * max(1, abs(r0.cost)) and f"iter={r0.iter}" in lines["box"]
