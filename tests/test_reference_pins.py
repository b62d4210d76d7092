"""Parity pinned by output the reference itself produced.

`examples/notebooks/unicycle_towards_origin.ipynb` (in /root/reference) stores the
printed result of a real Crocoddyl run:
  * ActionModelUnicycle with costWeights = (3, 1)            (ipynb line 94)
  * x0 = (-4, -4, 0), T = 20, ShootingProblem(x0, [model] * T, model)  (lines 121-122)
  * SolverDDP(problem).solve() with the defaults             (lines 201-202)
  * print(ddp.xs[-1]) -> (0.03379973, -0.30646301, 0.02773356)  (lines 256-258)
The model is core/actions/unicycle.hxx:13-40 (dt = 0.1, r = (w0 x, w1 u)). SolverDDP and
SolverFDDP stop at the same stationary point of this problem (the final step is a
Newton step from a point with ||Qu||^2 < th_stop), so the printed digits pin the
converged trajectory of every solver here: the numpy restatement, the C++ oracle
and the HIP path (-m gpu). The bar is the print's resolution: 5e-9 absolute.

The vector is copied here as data (three numbers); nothing reads /root/reference at
run time.
"""
import numpy as np
import pytest

import oracle_lib
from crocoddyl_amd import _abi
from crocoddyl_amd.models import ActionModelUnicycle
from crocoddyl_amd.problem import pack_problem
from oracle import fddp_np

NOTEBOOK_X0 = np.array([-4.0, -4.0, 0.0])
NOTEBOOK_T = 20
NOTEBOOK_WEIGHTS = (3.0, 1.0)
NOTEBOOK_XS_LAST = np.array([0.03379973, -0.30646301, 0.02773356])
PRINT_TOL = 5e-9  # half a unit in the 8th printed decimal


def _model():
    m = ActionModelUnicycle()
    m.costWeights = list(NOTEBOOK_WEIGHTS)
    return m


def _packed():
    m = _model()
    return pack_problem([m] * NOTEBOOK_T, m, 1)


def test_notebook_unicycle_numpy_restatement():
    knots, pool = _packed()
    s = fddp_np.FDDP(NOTEBOOK_X0, fddp_np.bind_problem(knots, pool, 0, 3))
    assert s.solve(maxiter=100)
    np.testing.assert_allclose(np.asarray(s.xs[-1]), NOTEBOOK_XS_LAST, atol=PRINT_TOL, rtol=0)


def test_notebook_unicycle_cpp_oracle():
    knots, pool = _packed()
    o = oracle_lib.Oracle(_abi.Dims(3, 3, 2, NOTEBOOK_T, 1), knots, pool, NOTEBOOK_X0[None])
    o.set_candidate(None, None, False)
    r = o.solve(maxiter=100)
    assert r[0].status == _abi.STATUS_CONVERGED
    np.testing.assert_allclose(o.xs()[0, -1], NOTEBOOK_XS_LAST, atol=PRINT_TOL, rtol=0)


@pytest.mark.gpu
def test_notebook_unicycle_gpu():
    """The notebook's own script, through the drop-in Python API, on the HIP path."""
    import crocoddyl_amd as crocoddyl
    model = crocoddyl.ActionModelUnicycle()
    model.costWeights = np.array(NOTEBOOK_WEIGHTS)
    problem = crocoddyl.ShootingProblem(NOTEBOOK_X0, [model] * NOTEBOOK_T, model)
    solver = crocoddyl.SolverFDDP(problem)
    done = solver.solve()
    assert done
    np.testing.assert_allclose(np.asarray(solver.xs[-1]), NOTEBOOK_XS_LAST, atol=PRINT_TOL, rtol=0)


@pytest.mark.gpu
def test_notebook_unicycle_gpu_batched():
    """The same problem replicated over a batch (one x0 per element): every element
    lands on the notebook's final state."""
    import crocoddyl_amd as crocoddyl
    model = crocoddyl.ActionModelUnicycle()
    model.costWeights = np.array(NOTEBOOK_WEIGHTS)
    B = 64
    problem = crocoddyl.ShootingProblem(np.repeat(NOTEBOOK_X0[None], B, axis=0), [model] * NOTEBOOK_T, model)
    solver = crocoddyl.SolverFDDP(problem)
    solver.solve()
    xs = np.asarray(solver.xs)
    assert xs.shape == (B, NOTEBOOK_T + 1, 3)
    np.testing.assert_allclose(xs[:, -1], np.repeat(NOTEBOOK_XS_LAST[None], B, axis=0), atol=PRINT_TOL, rtol=0)
