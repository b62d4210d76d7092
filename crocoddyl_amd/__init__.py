"""crocoddyl_amd — MI355X-native batched FDDP behind Crocoddyl's Python API.

The hot path of the reference (ShootingProblem::calc/calcDiff + SolverFDDP,
/root/reference) runs in libfddp_hip (hand-written HIP for gfx950, C ABI in
include/fddp_hip.h). This package mirrors the reference's Python names so a
problem written for ``crocoddyl`` drops in:

    import crocoddyl_amd as crocoddyl
    model = crocoddyl.ActionModelLQR(24, 12)
    problem = crocoddyl.ShootingProblem(x0, [model] * T, model)   # x0: (nx,) or (B, nx)
    solver = crocoddyl.SolverFDDP(problem)
    solver.solve()
"""
from ._lib import FDDPError, LIB_PATH  # noqa: F401
from .models import (ActionData, ActionDataAbstract, ActionModelAbstract, ActionModelLQR, ActionModelUnicycle,  # noqa: F401
                     DifferentialActionData, DifferentialActionDataAbstract, DifferentialActionModelAbstract,
                     DifferentialActionModelLQR, DifferentialActionModelNumDiff, IntegratedActionModelEuler,
                     StateVector)
from .problem import ShootingProblem, SolverBoxFDDP, SolverFDDP, pack_problem  # noqa: F401
from .boxqp import BoxQP, BoxQPSolution  # noqa: F401
from .callbacks import CallbackAbstract, CallbackLogger, CallbackVerbose, VerboseLevel  # noqa: F401

__version__ = "0.1.0"
