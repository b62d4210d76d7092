"""Solver callbacks with the reference's names.

CallbackAbstract (include/crocoddyl/core/solver-base.hpp:284-298), CallbackVerbose
(src/core/utils/callbacks.cpp:13-67) and CallbackLogger
(bindings/python/crocoddyl/__init__.py:356-381). SolverFDDP.solve calls each callback
once per iteration, after the regularisation update and stoppingCriteria
(fddp.cpp:92-98); the solver's getters then read that iteration's state (through
fddp_set_callback, the C ABI's per-iteration hook). Batched solvers pass the whole
batch: the getters return arrays and ``solver.callbackMask`` marks the elements that
ran the iteration.
"""
import copy
import sys

import numpy as np


class CallbackAbstract:
    """Base class: override __call__(self, solver)."""

    def __call__(self, solver):
        raise NotImplementedError


class VerboseLevel:
    _1 = 1
    _2 = 2


class CallbackVerbose(CallbackAbstract):
    """One table row per iteration (iter, cost, stop, grad = -d[1], xreg, ureg, step,
    feas; level 2 adds dV-exp and dV), a header every 10 iterations. Batched solvers
    print the row of the first element that ran the iteration (``solver.callbackMask``),
    so a finished element 0 does not repeat its last row under later iterations."""

    def __init__(self, level=VerboseLevel._1, stream=None):
        self.level = level
        self.stream = stream

    def __call__(self, solver):
        out = self.stream or sys.stdout
        mask = getattr(solver, "callbackMask", None)
        e = 0
        if mask is not None and np.size(mask) > 1:
            ran = np.flatnonzero(np.asarray(mask))
            if ran.size == 0:
                return
            e = int(ran[0])
        first = (lambda v: np.asarray(v).reshape(-1)[e] if np.size(v) > e else np.asarray(v).reshape(-1)[0])
        it = int(first(solver.iter))
        if it % 10 == 0:
            out.write("iter \t cost \t      stop \t    grad \t  xreg \t      ureg \t step \t feas"
                      + (" \tdV-exp \t      dV" if self.level == VerboseLevel._2 else "") + "\n")
        d = np.asarray(solver.d).reshape(-1, 2)
        d = d[e] if d.shape[0] > e else d[0]
        row = (f"{it:4d}  {first(solver.cost):.5e}  {first(solver.stop):.5e}  {-d[1]:.5e}  "
               f"{first(solver.x_reg):.5e}  {first(solver.u_reg):.5e}   {first(solver.stepLength):.4f}     "
               f"{int(bool(first(solver.isFeasible)))}")
        if self.level == VerboseLevel._2:
            row += f"  {first(solver.dVexp):.5e}  {first(solver.dV):.5e}"
        out.write(row + "\n")


class CallbackLogger(CallbackAbstract):
    """Records the iteration trace: xs / us (last), fs, steps, iters, costs, u_regs,
    x_regs, stops, grads (= -expectedImprovement()[1])."""

    def __init__(self):
        self.xs = []
        self.us = []
        self.fs = []
        self.steps = []
        self.iters = []
        self.costs = []
        self.u_regs = []
        self.x_regs = []
        self.stops = []
        self.grads = []

    def __call__(self, solver):
        self.xs = copy.copy(solver.xs)
        self.us = copy.copy(solver.us)
        self.fs.append(copy.copy(solver.fs))
        self.steps.append(solver.stepLength)
        self.iters.append(solver.iter)
        self.costs.append(solver.cost)
        self.u_regs.append(solver.u_reg)
        self.x_regs.append(solver.x_reg)
        self.stops.append(solver.stoppingCriteria())
        d = np.asarray(solver.expectedImprovement())
        self.grads.append(-d[..., 1] if d.ndim > 1 else -float(d[1]))
