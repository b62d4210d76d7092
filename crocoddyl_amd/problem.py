"""ShootingProblem and SolverFDDP with the reference's Python API, batched.

Reference API mirrored:
  ShootingProblem(x0, runningModels, terminalModel)
      bindings/python/crocoddyl/core/optctrl/shooting.cpp:18-120,
      include/crocoddyl/core/optctrl/shooting.hxx:17-223
  SolverFDDP(problem).solve(init_xs=[], init_us=[], maxiter=100, isFeasible=False, regInit=1e-9)
      bindings/python/crocoddyl/core/solvers/fddp.cpp:18-70, core/solver-base.cpp:100-126,
      core/solvers/ddp.cpp:84-125

Batching: x0 of shape (B, nx) (or models with batched parameters) makes the
problem a batch of B independent problems sharing the knot sequence. Then
xs/us are arrays (B, T+1, nx) / (B, T, nu_max) and scalars become (B,)
arrays; with a 1-D x0 everything has the reference's single-problem shapes.

All computation runs in libfddp_hip on the GPU; nothing here computes.
"""
import ctypes as C
import math
import warnings

import numpy as np

from . import _abi
from ._lib import FDDPError, check, default_params, lib
from .host import HostProblem, HostSolverFDDP, is_host_model
from .models import ActionData, ActionModelAbstract


def pack_problem(running, terminal, B, cache=None):
    """Knot descriptors + parameter pool for T running knots and the terminal.

    Models shared by several knots get one block (or one block per batch
    element if their parameters are batched). `cache` (dict, optional) keeps each
    model's packed block by (id, version), so a re-pack after circularAppend /
    updateNode only packs the models that changed."""
    models = list(running) + [terminal]
    for m in models:
        if not isinstance(m, ActionModelAbstract) or m.kind is None:
            raise NotImplementedError(f"crocoddyl_amd: knot model {type(m).__name__} has no device implementation")
    offsets = {}
    pool = []
    pos = 0
    knots = []
    for m in models:
        key = id(m)
        if key not in offsets:
            if cache is not None:
                ver = m._version
                hit = cache.get(key)
                if hit is None or hit[0] != ver or hit[1] is not m:
                    hit = (ver, m, m.pack())
                    cache[key] = hit
                kind, nu, blocks = hit[2]
            else:
                kind, nu, blocks = m.pack()
            if blocks.shape[0] not in (1, B):
                raise ValueError(f"Invalid argument: model parameters are batched over {blocks.shape[0]} "
                                 f"elements but the problem has B={B}")
            stride = blocks.shape[1] if blocks.shape[0] == B and B > 1 else 0
            offsets[key] = (kind, nu, pos, stride)
            pool.append(blocks[0:1] if stride == 0 else blocks)
            pos += blocks.size if stride else blocks.shape[1]
        kind, nu, off, stride = offsets[key]
        knots.append((kind, nu, off, stride))
    flat = np.concatenate([p.reshape(-1) for p in pool]) if pool else np.zeros(1)
    return knots, np.ascontiguousarray(flat, dtype=np.float64)


def batch_size_of(x0, models):
    x0 = np.asarray(x0, float)
    B = x0.shape[0] if x0.ndim == 2 else 1
    for m in models:
        _, _, blocks = m.pack()
        if blocks.shape[0] > 1:
            if B == 1 and x0.ndim == 1:
                B = blocks.shape[0]
            elif blocks.shape[0] != B:
                raise ValueError("Invalid argument: batched model parameters and x0 disagree on B")
    return B


class _Handle:
    """Owns one fddp_handle (device memory for one batched problem+solver)."""

    def __init__(self, problem, device):
        self.problem = problem
        self.device = device
        self.ptr = C.c_void_p()
        knots, pool = problem._packed(fresh=True)
        self.n_params = pool.size
        self._knots = knots
        self._sig = problem._signature()
        dims = problem._dims()
        kd = (_abi.KnotDesc * len(knots))(*[_abi.KnotDesc(*k) for k in knots])
        check(lib().fddp_create(C.byref(dims), kd, _abi.dptr(pool), pool.size, device, C.byref(self.ptr)))
        self.set_x0(problem._x0b)
        self._lsig = None
        self._push_limits()

    def _push_limits(self):
        lsig = self.problem._limits_signature()
        if lsig != self._lsig:
            lb, ub = self.problem._limits()
            check(lib().fddp_set_control_limits(self.ptr, _abi.dptr(lb), _abi.dptr(ub)))
            self._lsig = lsig

    def refresh(self):
        """Push model changes: parameter setters (same layout) or a new knot
        sequence (circularAppend / updateNode / updateModel -> fddp_set_knots)."""
        sig = self.problem._signature()
        if sig != self._sig:
            knots, pool = self.problem._packed()
            if pool.size == self.n_params and knots == self._knots:
                check(lib().fddp_set_model_params(self.ptr, _abi.dptr(pool), pool.size))
            else:
                kd = (_abi.KnotDesc * len(knots))(*[_abi.KnotDesc(*k) for k in knots])
                check(lib().fddp_set_knots(self.ptr, kd, _abi.dptr(pool), pool.size))
                self._knots, self.n_params = knots, pool.size
            self._sig = sig
        self._push_limits()
        return self.ptr

    def set_x0(self, x0b):
        check(lib().fddp_set_x0(self.ptr, _abi.dptr(np.ascontiguousarray(x0b, dtype=np.float64))))

    def __del__(self):
        try:
            if self.ptr:
                lib().fddp_destroy(self.ptr)
                self.ptr = C.c_void_p()
        except Exception:
            pass


class ShootingProblem:
    """ShootingProblem (shooting.hxx:17-59): x0, T running models, terminal model."""

    def __init__(self, x0, runningModels, terminalModel, device=0):
        runningModels = list(runningModels)
        if len(runningModels) < 1:
            raise ValueError("Invalid argument: at least one running model is needed")
        x0 = np.array(x0, dtype=np.float64)
        self._models = runningModels
        self._terminal = terminalModel
        self.nx = runningModels[0].state.nx
        self.ndx = runningModels[0].state.ndx
        self.nu_max = max(m.nu for m in runningModels)
        for i, m in enumerate(runningModels):  # shooting.hxx:39-49
            if m.state.nx != self.nx:
                raise ValueError(f"Invalid argument: nx in {i} node is not consistent with the other nodes")
            if m.state.ndx != self.ndx:
                raise ValueError(f"Invalid argument: ndx in {i} node is not consistent with the other nodes")
        if terminalModel.state.nx != self.nx:
            raise ValueError("Invalid argument: nx in terminal node is not consistent with the other nodes")
        if x0.shape[-1] != self.nx or x0.ndim not in (1, 2):
            raise ValueError(f"Invalid argument: x0 has wrong dimension (it should be {self.nx})")
        # a Python-defined model anywhere: the whole problem runs on the host (host.py)
        self.host_mode = any(is_host_model(m) for m in runningModels + [terminalModel])
        if self.host_mode:
            if x0.ndim != 1 or any(m.pack()[2].shape[0] > 1 for m in set(runningModels + [terminalModel])
                                   if not is_host_model(m)):
                raise ValueError("Invalid argument: problems with Python-defined action models are single problems "
                                 "(one x0, unbatched model parameters)")
            self.batched, self.B = False, 1
        else:
            self.batched = x0.ndim == 2 or any(m.pack()[2].shape[0] > 1 for m in set(runningModels + [terminalModel]))
            self.B = batch_size_of(x0, set(runningModels + [terminalModel]))
        self._x0b = np.broadcast_to(x0, (self.B, self.nx)).copy() if x0.ndim == 1 else x0.copy()
        self.device = device
        self._calc_h = None
        self._solver_handles = []
        self.runningDatas = [m.createData() for m in runningModels]
        self.terminalData = terminalModel.createData()
        self.cost = 0.0

    # -- reference accessors -------------------------------------------------
    @property
    def T(self):
        return len(self._models)

    @property
    def runningModels(self):
        return list(self._models)

    @property
    def terminalModel(self):
        return self._terminal

    @property
    def x0(self):
        return self._x0b.copy() if self.batched else self._x0b[0].copy()

    @x0.setter
    def x0(self, x0):
        """ShootingProblem::set_x0 (shooting.hxx:391-397)."""
        x0 = np.asarray(x0, dtype=np.float64)
        if x0.shape[-1] != self.nx:
            raise ValueError(f"Invalid argument: x0 has wrong dimension (it should be {self.nx})")
        self._x0b = np.broadcast_to(x0, (self.B, self.nx)).copy()
        for h in self._handles():
            h.set_x0(self._x0b)

    # -- packing ---------------------------------------------------------------
    def _dims(self):
        return _abi.Dims(self.nx, self.ndx, self.nu_max, self.T, self.B)

    def _packed(self, fresh=False):
        cache = self.__dict__.setdefault("_pack_cache", {})
        if fresh:  # a new handle packs every model again (in-place array edits included)
            cache.clear()
        live = {id(m) for m in self._models + [self._terminal]}
        for k in [k for k in cache if k not in live]:  # models no longer in the horizon
            del cache[k]
        return pack_problem(self._models, self._terminal, self.B, cache)

    def _signature(self):
        return tuple((id(m), m._version) for m in self._models + [self._terminal])

    # -- MPC plumbing (shooting.hxx:235-346) -------------------------------------
    def _check_node(self, model, data=None):
        if model.state.nx != self.nx:
            raise ValueError("Invalid argument: nx is not consistent with the other nodes")
        if model.state.ndx != self.ndx:
            raise ValueError("Invalid argument: ndx node is not consistent with the other nodes")
        if model.nu > self.nu_max:
            raise ValueError("Invalid argument: nu node is not bigger than the maximun nu")
        if data is not None and (not isinstance(data, ActionData) or data.Fu.shape[1] != model.nu):
            raise ValueError("Invalid argument: action data is not consistent with the action model")
        if is_host_model(model) and not self.host_mode:
            raise ValueError("Invalid argument: a Python-defined model cannot join a device problem; build a new "
                             "ShootingProblem")
        if not is_host_model(model) and model.pack()[2].shape[0] not in (1, self.B):
            raise ValueError(f"Invalid argument: model parameters are batched over {model.pack()[2].shape[0]} "
                             f"elements but the problem has B={self.B}")

    def circularAppend(self, model, data=None):
        """ShootingProblem::circularAppend (shooting.hxx:235-281): drop the
        first running node, append (model, data) at the end. The device handles
        get the rotated knot sequence on their next use (fddp_set_knots)."""
        self._check_node(model, data)
        self._models = self._models[1:] + [model]
        self.runningDatas = self.runningDatas[1:] + [data if data is not None else model.createData()]

    def updateNode(self, i, model, data):
        """ShootingProblem::updateNode (shooting.hxx:283-315): node i < T is a
        running node, i == T the terminal one. (The reference accepts i == T+1
        and then writes past its running models; that is an error here.)"""
        if not 0 <= i <= self.T:
            raise ValueError(f"Invalid argument: i is bigger than the allocated horizon (it should be less than "
                             f"or equal to {self.T})")
        self._check_node(model, data)
        if i == self.T:
            self._terminal, self.terminalData = model, data
        else:
            self._models[i] = model
            self.runningDatas[i] = data

    def updateModel(self, i, model):
        """ShootingProblem::updateModel (shooting.hxx:317-346): i < T running,
        i == T+1 terminal, with a fresh data. (The reference's i == T indexes
        past its running models; that is an error here.)"""
        if not (0 <= i < self.T or i == self.T + 1):
            raise ValueError(f"Invalid argument: i is bigger than the allocated horizon (it should be lower than "
                             f"{self.T} or equal to {self.T + 1})")
        self._check_node(model)
        if i == self.T + 1:
            self._terminal, self.terminalData = model, model.createData()
        else:
            self._models[i] = model
            self.runningDatas[i] = model.createData()

    def _limits_signature(self):
        return tuple((id(m), m._lim_version) for m in self._models)

    def _limits(self):
        """Control limits of the running models as (B, T, nu_max) arrays
        (fddp_set_control_limits), or (None, None) when no model has any."""
        B, T, m = self.B, self.T, self.nu_max
        if not any(np.isfinite(md._u_lb).any() or np.isfinite(md._u_ub).any() for md in self._models):
            return None, None
        lb = np.full((B, T, max(m, 1)), -np.inf)
        ub = np.full((B, T, max(m, 1)), np.inf)
        for t, md in enumerate(self._models):
            lb[:, t, :md.nu] = np.broadcast_to(md._u_lb, (B, md.nu))
            ub[:, t, :md.nu] = np.broadcast_to(md._u_ub, (B, md.nu))
        return np.ascontiguousarray(lb[..., :m]), np.ascontiguousarray(ub[..., :m])

    def _handles(self):
        hs = []
        if self._calc_h is not None:
            hs.append(self._calc_h)
        hs.extend(self._solver_handles)
        return hs

    def _new_handle(self):
        return _Handle(self, self.device)

    def _calc_handle(self):
        if self._calc_h is None:
            self._calc_h = _Handle(self, self.device)
        return self._calc_h.refresh()

    # -- trajectories in/out ---------------------------------------------------
    def _xs_array(self, xs):
        T, nx, B = self.T, self.nx, self.B
        if xs is None or (isinstance(xs, (list, tuple)) and len(xs) == 0):
            return None
        a = np.asarray(xs, dtype=np.float64) if not isinstance(xs, (list, tuple)) else np.stack(
            [np.asarray(x, float) for x in xs], axis=-2)
        if a.shape[-2:] != (T + 1, nx):
            raise ValueError(f"Invalid argument: xs has wrong dimension (it should be {T + 1})")
        return np.ascontiguousarray(np.broadcast_to(a, (B, T + 1, nx)))

    def _us_array(self, us):
        T, m, B = self.T, self.nu_max, self.B
        if us is None or (isinstance(us, (list, tuple)) and len(us) == 0):
            return None
        if isinstance(us, (list, tuple)):
            rows = []
            for u in us:
                u = np.asarray(u, float)
                if u.shape[-1] != m:
                    pad = np.zeros(u.shape[:-1] + (m,))
                    pad[..., :u.shape[-1]] = u
                    u = pad
                rows.append(u)
            a = np.stack(rows, axis=-2)
        else:
            a = np.asarray(us, dtype=np.float64)
        if a.shape[-2:] != (T, m):
            raise ValueError(f"Invalid argument: us has wrong dimension (it should be {T})")
        return np.ascontiguousarray(np.broadcast_to(a, (B, T, m)))

    def _out_x(self, a):
        return a if self.batched else [a[0, t].copy() for t in range(a.shape[1])]

    def _out_u(self, a):
        if self.batched:
            return a
        return [a[0, t, :self._models[t].nu].copy() for t in range(a.shape[1])]

    def _fill_datas(self, h, diff):
        L = lib()
        B, T, n, m = self.B, self.T, self.ndx, self.nu_max

        def q(which, nk, per):
            out = np.zeros((B, nk, per))
            check(L.fddp_get_quantity(h, which, _abi.dptr(out)))
            return out

        xn = q(_abi.Q_XNEXT, T, self.nx)
        if diff:
            Fx = q(_abi.Q_FX, T + 1, n * n)
            Fu = q(_abi.Q_FU, T + 1, n * m)
            Lxx = q(_abi.Q_LXX, T + 1, n * n)
            Lxu = q(_abi.Q_LXU, T + 1, n * m)
            Luu = q(_abi.Q_LUU, T + 1, m * m)
            Lx = q(_abi.Q_LX, T + 1, n)
            Lu = q(_abi.Q_LU, T + 1, max(m, 0))
        datas = self.runningDatas + [self.terminalData]
        models = self._models + [self._terminal]
        sel = (slice(None),) if self.batched else (0,)
        for t, (d, mdl) in enumerate(zip(datas, models)):
            if t < T:
                d.xnext = xn[sel + (t,)].copy()
            if diff:
                d.Fx = _cm(Fx[:, t], n, n)[sel]
                d.Fu = _cm(Fu[:, t], n, m)[sel][..., :mdl.nu]
                d.Lxx = _cm(Lxx[:, t], n, n)[sel]
                d.Lxu = _cm(Lxu[:, t], n, m)[sel][..., :mdl.nu]
                d.Luu = _cm(Luu[:, t], m, m)[sel][..., :mdl.nu, :mdl.nu]
                d.Lx = Lx[:, t][sel].copy()
                d.Lu = Lu[:, t][sel][..., :mdl.nu].copy()

    # -- ShootingProblem::calc / calcDiff / rollout ----------------------------
    def _host(self):
        if getattr(self, "_hostp", None) is None:
            self._hostp = HostProblem(self)
        return self._hostp

    def calc(self, xs, us):
        """shooting.hxx:133-161; returns the total cost (per element if batched)."""
        if self.host_mode:
            self.cost = self._host().calc(list(xs), list(us))
            return self.cost
        h = self._calc_handle()
        xa, ua = self._xs_array(xs), self._us_array(us)
        if xa is None or (ua is None and self.nu_max > 0):
            raise ValueError("Invalid argument: xs/us have wrong dimension")
        check(lib().fddp_set_candidate(h, _abi.dptr(xa), _abi.dptr(ua), 0))
        cost = np.zeros(self.B)
        check(lib().fddp_problem_calc(h, _abi.dptr(cost)))
        self._fill_datas(h, diff=False)
        self.cost = cost if self.batched else float(cost[0])
        return self.cost

    def calcDiff(self, xs, us):
        """shooting.hxx:164-195 (calc first, as the reference's datas carry the costs)."""
        self.calc(xs, us)
        if self.host_mode:
            self.cost = self._host().calc(list(xs), list(us), diff=True)
            return self.cost
        h = self._calc_handle()
        cost = np.zeros(self.B)
        check(lib().fddp_problem_calc_diff(h, _abi.dptr(cost)))
        self._fill_datas(h, diff=True)
        self.cost = cost if self.batched else float(cost[0])
        return self.cost

    def rollout(self, us):
        """shooting.hxx:198-223: xs[0] = x0, xs[t+1] = f(xs[t], us[t]).

        Runs as the device forward pass with zero feedback gains (this
        handle never computes a backward pass, so K = k = 0), alpha = 1."""
        if self.host_mode:
            return self._host().rollout(list(us))
        h = self._calc_handle()
        ua = self._us_array(us)
        check(lib().fddp_set_candidate(h, None, _abi.dptr(ua), 1))
        st = np.zeros(self.B, dtype=np.int32)
        check(lib().fddp_try_step(h, 1.0, None, st.ctypes.data_as(_abi.I32)))
        xs = np.zeros((self.B, self.T + 1, self.nx))
        check(lib().fddp_get_xs_try(h, _abi.dptr(xs)))
        return self._out_x(xs)

    def rollout_us(self, us):
        return self.rollout(us)


def _cm(flat, r, c):
    """(B, r*c) column-major rows -> (B, r, c)."""
    return np.ascontiguousarray(flat.reshape(flat.shape[0], c, r).transpose(0, 2, 1))


class SolverFDDP:
    """SolverFDDP (src/core/solvers/fddp.cpp) on the device, batched. A problem with
    Python-defined action models gets the host solver (host.HostSolverFDDP)."""

    def __new__(cls, problem):
        if getattr(problem, "host_mode", False):
            if cls is not SolverFDDP:
                raise NotImplementedError(f"crocoddyl_amd: {cls.__name__} needs device models (Python-defined "
                                          "action models run with SolverFDDP)")
            return HostSolverFDDP(problem)
        return super().__new__(cls)

    def __init__(self, problem):
        self.problem = problem
        self._h = problem._new_handle()
        problem._solver_handles.append(self._h)
        self._prm = default_params()
        self._results = None
        self.callbacks = []
        self.callbackMask = None
        self._cb_error = None
        self._cb_snap = None

    # -- helpers -----------------------------------------------------------
    @property
    def _ptr(self):
        return self._h.refresh()

    def _push_params(self):
        check(lib().fddp_set_params(self._ptr, C.byref(self._prm)))

    def _scalar(self, arr):
        return arr if self.problem.batched else arr[0]

    def _res(self):
        if self._cb_snap is not None:  # inside a per-iteration callback: that iteration's state
            return self._cb_snap
        if self._results is None:
            r = (_abi.Result * self.problem.B)()
            check(lib().fddp_get_results(self._ptr, r))
            self._results = r
        return self._results

    def _field(self, name, conv=float):
        arr = _abi.result_array(self._res())[name].astype(conv)
        return arr if self.problem.batched else arr[0]

    # -- SolverAbstract::setCandidate / solve --------------------------------
    def setCandidate(self, xs=[], us=[], isFeasible=False):
        p = self.problem
        xa, ua = p._xs_array(xs), p._us_array(us)
        check(lib().fddp_set_candidate(self._ptr, _abi.dptr(xa), _abi.dptr(ua), 1 if isFeasible else 0))
        self._results = None

    def setCandidate_device(self, xs_ptr, us_ptr, isFeasible=False):
        """setCandidate from device-resident (B, T+1, nx) / (B, T, nu_max) fp64 arrays
        (integer device addresses on the solver's GPU, or None); enqueued on the
        handle's stream without a host synchronisation."""
        cast = (lambda p: None if p is None else C.cast(C.c_void_p(int(p)), _abi.D))
        check(lib().fddp_set_candidate_device(self._ptr, cast(xs_ptr), cast(us_ptr), 1 if isFeasible else 0))
        self._results = None

    def solve(self, init_xs=[], init_us=[], maxiter=100, isFeasible=False, regInit=1e-9):
        """fddp.cpp:19-105 for every batch element; returns solve()'s bool
        (an array of bools when batched)."""
        self._push_params()
        self.setCandidate(init_xs, init_us, isFeasible)
        return self.solve_from_candidate(maxiter, isFeasible, regInit)

    def solve_from_candidate(self, maxiter=100, isFeasible=False, regInit=1e-9):
        """solve() without re-uploading a warm start (device-resident MPC loops)."""
        ptr = self._ptr
        check(lib().fddp_set_params(ptr, C.byref(self._prm)))
        reg = float("nan") if regInit is None else float(regInit)
        r = (_abi.Result * self.problem.B)()
        if self.callbacks:
            # every callback once per iteration of the loop (fddp.cpp:92-98), with the
            # solver's getters reading that iteration's state
            B = self.problem.B

            def on_iter(_user, it, res, reported, _B):
                snap = (_abi.Result * B)()
                C.memmove(snap, res, C.sizeof(snap))
                self._cb_snap = snap
                self.callbackMask = np.ctypeslib.as_array(reported, (B,)).astype(bool)
                if not self.problem.batched and not self.callbackMask[0]:
                    return 0
                try:
                    for cb in self.callbacks:
                        cb(self)
                except BaseException as e:  # stops fddp_solve after this iteration; re-raised below
                    self._cb_error = e
                    return 1
                return 0

            self._cb_error = None
            cfn = _abi.IterationCallback(on_iter)
            check(lib().fddp_set_callback(ptr, cfn, None))
            try:
                rc = lib().fddp_solve(ptr, int(maxiter), 1 if isFeasible else 0, reg, r)
            finally:
                check(lib().fddp_set_callback(ptr, _abi.IterationCallback(), None))
                self.callbackMask = None
                self._cb_snap = None
            if rc == _abi.FDDP_ERR_CALLBACK_ABORT and self._cb_error is not None:
                # the reference's exception leaves solve() in that iteration (fddp.cpp:92-98):
                # iter / xs / us / regularisation stay there
                self._results = r
                raise self._cb_error
            check(rc)
        else:
            check(lib().fddp_solve(ptr, int(maxiter), 1 if isFeasible else 0, reg, r))
        self._results = r
        ok = _abi.result_array(r)["status"] == _abi.STATUS_CONVERGED
        return ok if self.problem.batched else bool(ok[0])

    def setCallbacks(self, callbacks):
        """SolverAbstract::setCallbacks (solver-base.cpp:69-73): each callback is called
        as cb(solver) once per iteration of solve(), after the regularisation update and
        stoppingCriteria (fddp.cpp:92-98). When batched, the getters return the whole
        batch and ``solver.callbackMask`` marks the elements that ran that iteration."""
        self.callbacks = list(callbacks)

    def getCallbacks(self):
        return list(self.callbacks)

    # -- step API (SolverDDP methods) ----------------------------------------
    def computeDirection(self, recalc=True):
        """ddp.cpp:120-125. Raises on backward_error (single problem); returns
        the per-element failure flags when batched."""
        self._push_params()
        st = np.zeros(self.problem.B, dtype=np.int32)
        check(lib().fddp_compute_direction(self._ptr, 1 if recalc else 0, st.ctypes.data_as(_abi.I32)))
        self._results = None
        if not self.problem.batched and st[0]:
            raise FDDPError("backward_error")
        return st.astype(bool) if self.problem.batched else None

    def calcDiff(self):
        """SolverDDP::calcDiff (ddp.cpp:157-178): problem.calc at iter 0, problem.calcDiff,
        the gaps. Returns the cost (an array when batched)."""
        c = np.zeros(self.problem.B)
        check(lib().fddp_calc_diff(self._ptr, _abi.dptr(c)))
        self._results = None
        return self._scalar(c)

    def backwardPass(self):
        """SolverDDP::backwardPass (ddp.cpp:180-253) on the last calcDiff's derivatives.
        Raises on backward_error (single problem); returns the per-element failure flags
        when batched."""
        self._push_params()
        st = np.zeros(self.problem.B, dtype=np.int32)
        check(lib().fddp_backward_pass(self._ptr, st.ctypes.data_as(_abi.I32)))
        self._results = None
        if not self.problem.batched and st[0]:
            raise FDDPError("backward_error")
        return st.astype(bool) if self.problem.batched else None

    def forwardPass(self, stepLength=1.0):
        """SolverFDDP::forwardPass (fddp.cpp:149-225): rolls the policy out into
        xs_try / us_try (properties xs_try, us_try) and cost_try. Raises on
        forward_error (single problem); the per-element flags when batched."""
        ct = np.zeros(self.problem.B)
        st = np.zeros(self.problem.B, dtype=np.int32)
        check(lib().fddp_forward_pass(self._ptr, float(stepLength), _abi.dptr(ct), st.ctypes.data_as(_abi.I32)))
        self._results = None
        self._cost_try = ct
        if not self.problem.batched and st[0]:
            raise FDDPError("forward_error")
        return st.astype(bool) if self.problem.batched else None

    @property
    def cost_try(self):
        """cost_try_ of the last forwardPass / tryStep."""
        return self._scalar(self._cost_try) if getattr(self, "_cost_try", None) is not None else None

    @property
    def xs_try(self):
        p = self.problem
        a = np.zeros((p.B, p.T + 1, p.nx))
        check(lib().fddp_get_xs_try(self._ptr, _abi.dptr(a)))
        return p._out_x(a)

    @property
    def us_try(self):
        p = self.problem
        a = np.zeros((p.B, p.T, p.nu_max))
        check(lib().fddp_get_us_try(self._ptr, _abi.dptr(a)))
        return p._out_u(a)

    def tryStep(self, stepLength=1.0):
        """ddp.cpp:127-130; returns cost - cost_try."""
        dV = np.zeros(self.problem.B)
        st = np.zeros(self.problem.B, dtype=np.int32)
        check(lib().fddp_try_step(self._ptr, float(stepLength), _abi.dptr(dV), st.ctypes.data_as(_abi.I32)))
        self._results = None
        if not self.problem.batched and st[0]:
            raise FDDPError("forward_error")
        return self._scalar(dV)

    def stoppingCriteria(self):
        s = np.zeros(self.problem.B)
        check(lib().fddp_stopping_criteria(self._ptr, _abi.dptr(s)))
        return self._scalar(s)

    def expectedImprovement(self):
        d = np.zeros((self.problem.B, 2))
        check(lib().fddp_expected_improvement(self._ptr, _abi.dptr(d)))
        self._results = None
        return d if self.problem.batched else d[0]

    def updateExpectedImprovement(self):
        check(lib().fddp_update_expected_improvement(self._ptr))

    def setSolverState(self, iter=0, xreg=float("nan"), ureg=float("nan"), wasFeasible=False):
        check(lib().fddp_set_solver_state(self._ptr, int(iter), float(xreg), float(ureg), int(wasFeasible)))
        self._results = None

    # -- trajectories -----------------------------------------------------------
    @property
    def xs(self):
        p = self.problem
        a = np.zeros((p.B, p.T + 1, p.nx))
        check(lib().fddp_get_xs(self._ptr, _abi.dptr(a), 0))
        return p._out_x(a)

    @xs.setter
    def xs(self, v):
        self.setCandidate(v, self.us, bool(np.all(self._field("is_feasible", int))))

    @property
    def us(self):
        p = self.problem
        a = np.zeros((p.B, p.T, p.nu_max))
        check(lib().fddp_get_us(self._ptr, _abi.dptr(a), 0))
        return p._out_u(a)

    @us.setter
    def us(self, v):
        self.setCandidate(self.xs, v, bool(np.all(self._field("is_feasible", int))))

    def xs_device(self, out_ptr):
        """Copy xs (B, T+1, nx) into a device buffer on the solver's GPU."""
        check(lib().fddp_get_xs(self._ptr, C.cast(out_ptr, _abi.D), 1))

    def us_device(self, out_ptr):
        check(lib().fddp_get_us(self._ptr, C.cast(out_ptr, _abi.D), 1))

    def _quantity(self, which, nk, r, c=None, nu_slice=None):
        p = self.problem
        per = r * (c or 1)
        a = np.zeros((p.B, nk, per))
        check(lib().fddp_get_quantity(self._ptr, which, _abi.dptr(a)))
        if c is not None:
            a = a.reshape(p.B, nk, c, r).transpose(0, 1, 3, 2)
        if p.batched:
            return a
        out = []
        models = p._models + [p._terminal]
        for t in range(nk):
            v = a[0, t]
            if nu_slice == "rows":
                v = v[:models[t].nu]
            elif nu_slice == "cols":
                v = v[..., :models[t].nu]
            elif nu_slice == "both":
                v = v[:models[t].nu, :models[t].nu]
            out.append(np.array(v))
        return out

    def _debug(self, on=True):
        check(lib().fddp_set_debug(self._ptr, 1 if on else 0))

    # SolverDDP getters (ddp.hpp:60-271)
    K = property(lambda s: s._quantity(_abi.Q_K, s.problem.T, s.problem.nu_max, s.problem.ndx, "rows"))
    k = property(lambda s: s._quantity(_abi.Q_KV, s.problem.T, s.problem.nu_max, None, "rows"))
    fs = property(lambda s: s._quantity(_abi.Q_FS, s.problem.T + 1, s.problem.ndx))
    Vxx = property(lambda s: s._quantity(_abi.Q_VXX, s.problem.T + 1, s.problem.ndx, s.problem.ndx))
    Vx = property(lambda s: s._quantity(_abi.Q_VX, s.problem.T + 1, s.problem.ndx))
    Qxx = property(lambda s: s._quantity(_abi.Q_QXX, s.problem.T, s.problem.ndx, s.problem.ndx))
    Qxu = property(lambda s: s._quantity(_abi.Q_QXU, s.problem.T, s.problem.ndx, s.problem.nu_max, "cols"))
    Quu = property(lambda s: s._quantity(_abi.Q_QUU, s.problem.T, s.problem.nu_max, s.problem.nu_max, "both"))
    Qx = property(lambda s: s._quantity(_abi.Q_QX, s.problem.T, s.problem.ndx))
    Qu = property(lambda s: s._quantity(_abi.Q_QU, s.problem.T, s.problem.nu_max, None, "rows"))

    # SolverAbstract getters (solver-base.cpp:100-126)
    cost = property(lambda s: s._field("cost"))
    stop = property(lambda s: s._field("stop"))
    iter = property(lambda s: s._field("iter", int))
    x_reg = property(lambda s: s._field("xreg"))
    u_reg = property(lambda s: s._field("ureg"))
    stepLength = property(lambda s: s._field("steplength"))
    isFeasible = property(lambda s: s._field("is_feasible", bool))
    dV = property(lambda s: s._field("dV"))
    dVexp = property(lambda s: s._field("dVexp"))
    status = property(lambda s: s._field("status", int))
    n_iter_run = property(lambda s: s._field("n_iter_run", int))

    @property
    def d(self):
        r = _abi.result_array(self._res())
        a = np.stack([r["d0"], r["d1"]], axis=1)
        return a if self.problem.batched else a[0]

    # thresholds with the reference setter validation (via fddp_set_params)
    def _prm_prop(name, alias=None):
        def get(self):
            return getattr(self._prm, name)

        def set_(self, v):
            old = getattr(self._prm, name)
            setattr(self._prm, name, float(v))
            try:
                self._push_params()
            except FDDPError:
                setattr(self._prm, name, old)
                raise

        return property(get, set_)

    th_acceptStep = _prm_prop("th_acceptstep")
    th_stop = _prm_prop("th_stop")
    th_grad = _prm_prop("th_grad")
    th_stepDec = _prm_prop("th_stepdec")
    th_stepInc = _prm_prop("th_stepinc")
    th_acceptNegStep = _prm_prop("th_acceptnegstep")
    regFactor = _prm_prop("regfactor")
    regMin = _prm_prop("regmin")
    regMax = _prm_prop("regmax")

    @property
    def alphas(self):
        return [self._prm.alphas[i] for i in range(self._prm.n_alphas)]

    @alphas.setter
    def alphas(self, a):
        a = [float(x) for x in a]
        if not a or len(a) > 16:
            raise ValueError("Invalid argument: between 1 and 16 alphas")
        if a[0] != 1.0:
            warnings.warn("alpha[0] should be 1")  # ddp.cpp:446-448
        old = (self._prm.n_alphas, list(self._prm.alphas))
        self._prm.n_alphas = len(a)
        for i in range(16):
            self._prm.alphas[i] = a[i] if i < len(a) else 0.0
        try:
            self._push_params()
        except FDDPError:
            self._prm.n_alphas = old[0]
            for i in range(16):
                self._prm.alphas[i] = old[1][i]
            raise

    # -- MPC plumbing ---------------------------------------------------------
    def mpcShift(self):
        """x0 <- xs[1]; shift xs/us one knot (on device)."""
        check(lib().fddp_mpc_shift(self._ptr))
        x0 = np.zeros((self.problem.B, self.problem.nx))
        check(lib().fddp_get_x0(self._ptr, _abi.dptr(x0)))
        self.problem._x0b = x0
        for h in self.problem._handles():
            if h is not self._h:
                h.set_x0(x0)

    # -- timing (HIP events on the handle's stream) ----------------------------
    def set_timing(self, on=True):
        check(lib().fddp_set_timing(self._ptr, 1 if on else 0))

    def get_timing(self):
        ms = np.zeros(4)
        cnt = np.zeros(4, dtype=np.int64)
        check(lib().fddp_get_timing(self._ptr, _abi.dptr(ms), cnt.ctypes.data_as(C.POINTER(C.c_int64))))
        names = ["calc", "calcDiff", "backward", "forward"]
        return {n: (float(ms[i]), int(cnt[i])) for i, n in enumerate(names)}

    def synchronize(self):
        check(lib().fddp_synchronize(self._ptr))

    def line_search_info(self):
        """(trial-group size, rollout dispatches) of the last line search
        (fddp_get_line_search_info; diagnostics)."""
        g, n = C.c_int32(), C.c_int32()
        check(lib().fddp_get_line_search_info(self._ptr, C.byref(g), C.byref(n)))
        return g.value, n.value


class SolverBoxFDDP(SolverFDDP):
    """SolverBoxFDDP (src/core/solvers/box-fddp.cpp:15-164) on the device:
    control-limited FDDP. Once an element is feasible, knots whose model has
    control limits get their gains from a box QP on (Quu, Qu) with bounds
    u_lb - us, u_ub - us; the forward pass clamps the controls. th_stop
    defaults to 5e-5 (box-fddp.cpp:28)."""

    def __init__(self, problem):
        super().__init__(problem)
        check(lib().fddp_set_solver_kind(self._h.ptr, _abi.SOLVER_BOXFDDP))
        self._prm.th_stop = 5e-5
        self._push_params()

    @property
    def Quu_inv(self):
        """SolverBoxFDDP::get_Quu_inv (box-fddp.cpp:162); needs _debug(True)
        before the backward pass (device-side store)."""
        p = self.problem
        return self._quantity(_abi.Q_QUU_INV, p.T, p.nu_max, p.nu_max, "both")
