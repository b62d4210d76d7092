"""ORACLE — TEST INFRASTRUCTURE ONLY (numpy restatement of the reference path).

Second, independent CPU restatement of the reference hot path, written with
numpy linear algebra instead of the loop-level C++ of oracle/fddp_oracle.cpp,
so the two cross-check each other (the reference's own design: C++ solver vs
numpy ``*Derived`` restatement at 1e-9, unittest/bindings/test_solvers.py).
Only tests/ and the golden-fixture generator import this module.

It follows the C++ files (not the Python ``FDDPDerived``, which differs —
SURVEY.md §8a "Restatement traps"):
  * SolverFDDP::solve                  src/core/solvers/fddp.cpp:19-105
  * SolverDDP::calcDiff / backwardPass ddp.cpp:157-253, computeGains :298-310
  * SolverFDDP::forwardPass            fddp.cpp:149-225
  * (update)ExpectedImprovement        fddp.cpp:107-147
  * ShootingProblem::calc/calcDiff     include/crocoddyl/core/optctrl/shooting.hxx:133-195
  * ActionModelLQR                     core/actions/lqr.hxx:30-70
  * ActionModelUnicycle                core/actions/unicycle.hxx:22-73
  * IntegratedActionModelEuler∘DifferentialActionModelLQR
                                       core/integrator/euler.hxx:41-131, core/actions/diff-lqr.hxx:34-79
  * Euler∘DifferentialActionModelFreeFwdDynamics (multibody knots)
                                       oracle/multibody_np.py
  * BoxQP::solve                       src/core/solvers/box-qp.cpp:51-182
  * SolverBoxFDDP computeGains / forwardPass  src/core/solvers/box-fddp.cpp:48-160
It also restates SolverKKT (src/core/solvers/kkt.cpp:34-227), the dense
Newton/KKT solver the reference uses as the oracle of its DDP/FDDP tests
(unittest/test_solvers.cpp:65-110).
"""
import math

import numpy as np

LQR, UNICYCLE, EULER_DIFFLQR, EULER_FREEFWD, EULER_CONTACTFWD, IMPULSEFWD = 1, 2, 3, 4, 5, 6
HDR = 4


def default_params():
    """ddp.cpp:15-37, fddp.cpp:14-15, solver-base.cpp:24-25."""
    return dict(th_acceptstep=0.1, th_stop=1e-9, th_grad=1e-12, th_stepdec=0.5, th_stepinc=0.01,
                th_acceptnegstep=2.0, regfactor=10.0, regmin=1e-9, regmax=1e9,
                alphas=[2.0 ** (-k) for k in range(10)])


def raise_if_nan(v):
    """solver-base.cpp:175-181."""
    return math.isnan(v) or math.isinf(v) or v >= 1e30


class Knot:
    """One knot model bound to one element's parameter block."""

    def __init__(self, kind, nx, nu, block):
        self.kind, self.nx, self.nu = kind, nx, nu
        self.ndx = nx
        p = np.asarray(block, dtype=np.float64)
        q = p[HDR:]
        if kind == LQR:
            self.drift_free = p[0] != 0
            o = 0

            def take(r, c=None):
                nonlocal o
                size = r * (c if c is not None else 1)
                a = q[o:o + size]
                o += size
                return a.reshape(c, r).T if c is not None else a

            self.Fx = take(nx, nx)
            self.Fu = take(nx, nu)
            self.f0 = take(nx)
            self.Lxx = take(nx, nx)
            self.Lxu = take(nx, nu)
            self.Luu = take(nu, nu)
            self.lx = take(nx)
            self.lu = take(nu)
        elif kind == UNICYCLE:
            self.dt, self.wx, self.wu = p[0], p[1], p[2]
        elif kind == EULER_DIFFLQR:
            self.dt = p[0]
            self.drift_free = p[1] != 0
            nq = nx // 2
            o = 0

            def take(r, c=None):
                nonlocal o
                size = r * (c if c is not None else 1)
                a = q[o:o + size]
                o += size
                return a.reshape(c, r).T if c is not None else a

            self.Fq = take(nq, nq)
            self.Fv = take(nq, nq)
            self.Fuc = take(nq, nu)
            self.f0 = take(nq)
            self.Lxx = take(nx, nx)
            self.Lxu = take(nx, nu)
            self.Luu = take(nu, nu)
            self.lx = take(nx)
            self.lu = take(nu)
        else:
            raise ValueError(kind)

    # StateVector (core/states/euclidean.hxx:28-61)
    def state_diff(self, x0, x1):
        return x1 - x0

    def state_integrate(self, x, dx):
        return x + dx

    def state_zero(self):
        return np.zeros(self.nx)

    # -- calc: returns (xnext, cost) -------------------------------------
    def calc(self, x, u=None):
        if u is None:
            u = np.zeros(self.nu)
        if self.kind == LQR:
            xn = self.Fx @ x + self.Fu @ u
            if not self.drift_free:
                xn = xn + self.f0
            c = 0.5 * x @ (self.Lxx @ x) + 0.5 * u @ (self.Luu @ u) + x @ (self.Lxu @ u) + self.lx @ x + self.lu @ u
            return xn, c
        if self.kind == UNICYCLE:
            c, s = math.cos(x[2]), math.sin(x[2])
            xn = np.array([x[0] + c * u[0] * self.dt, x[1] + s * u[0] * self.dt, x[2] + u[1] * self.dt])
            r = np.concatenate([self.wx * x, self.wu * u])
            return xn, 0.5 * r @ r
        nq = self.nx // 2
        q, v = x[:nq], x[nq:]
        a = self.Fq @ q + self.Fv @ v + self.Fuc @ u
        if not self.drift_free:
            a = a + self.f0
        cc = 0.5 * x @ (self.Lxx @ x) + 0.5 * u @ (self.Luu @ u) + x @ (self.Lxu @ u) + self.lx @ x + self.lu @ u
        if self.dt != 0:
            dx = np.concatenate([v * self.dt + a * self.dt ** 2, a * self.dt])
            return x + dx, self.dt * cc
        return x.copy(), cc

    # -- calcDiff: returns dict of Fx, Fu, Lx, Lu, Lxx, Lxu, Luu ----------
    def calc_diff(self, x, u=None):
        if u is None:
            u = np.zeros(self.nu)
        n, m = self.nx, self.nu
        if self.kind == LQR:
            return dict(Fx=self.Fx.copy(), Fu=self.Fu.copy(), Lx=self.lx + self.Lxx @ x + self.Lxu @ u,
                        Lu=self.lu + self.Lxu.T @ x + self.Luu @ u, Lxx=self.Lxx.copy(), Lxu=self.Lxu.copy(),
                        Luu=self.Luu.copy())
        if self.kind == UNICYCLE:
            c, s = math.cos(x[2]), math.sin(x[2])
            wx2, wu2 = self.wx ** 2, self.wu ** 2
            Fx = np.eye(3)
            Fx[0, 2] = -s * u[0] * self.dt
            Fx[1, 2] = c * u[0] * self.dt
            Fu = np.zeros((3, 2))
            Fu[0, 0], Fu[1, 0], Fu[2, 1] = c * self.dt, s * self.dt, self.dt
            return dict(Fx=Fx, Fu=Fu, Lx=wx2 * x, Lu=wu2 * u, Lxx=wx2 * np.eye(3), Lxu=np.zeros((3, 2)),
                        Luu=wu2 * np.eye(2))
        nq = n // 2
        da_dx = np.hstack([self.Fq, self.Fv])
        Lx = self.lx + self.Lxx @ x + self.Lxu @ u
        Lu = self.lu + self.Lxu.T @ x + self.Luu @ u
        dt = self.dt
        if dt != 0:
            Fx = np.vstack([da_dx * dt * dt, da_dx * dt])
            Fx[:nq, nq:] += dt * np.eye(nq)
            Fx += np.eye(n)
            Fu = np.vstack([self.Fuc * dt * dt, self.Fuc * dt])
            return dict(Fx=Fx, Fu=Fu, Lx=dt * Lx, Lu=dt * Lu, Lxx=dt * self.Lxx, Lxu=dt * self.Lxu, Luu=dt * self.Luu)
        return dict(Fx=np.eye(n), Fu=np.zeros((n, m)), Lx=Lx, Lu=Lu, Lxx=self.Lxx.copy(), Lxu=self.Lxu.copy(),
                    Luu=self.Luu.copy())


def bind_problem(knot_descs, pool, b, nx):
    """Knot models of element b; knot_descs: list of (kind, nu, offset, stride)."""
    out = []
    for kind, nu, off, stride in knot_descs:
        o = off + b * stride
        if kind == EULER_FREEFWD:  # variable-size multibody block (oracle/multibody_np.py)
            from oracle.multibody_np import FreeFwdKnot
            out.append(FreeFwdKnot(pool[o:o + int(pool[o + 3])], nx, nu))
            continue
        if kind == EULER_CONTACTFWD:
            from oracle.multibody_np import ContactFwdKnot
            out.append(ContactFwdKnot(pool[o:o + int(pool[o + 3])], nx, nu))
            continue
        if kind == IMPULSEFWD:
            from oracle.multibody_np import ImpulseFwdKnot
            out.append(ImpulseFwdKnot(pool[o:o + int(pool[o + 3])], nx, nu))
            continue
        size = block_size(kind, nx, nu)
        out.append(Knot(kind, nx, nu, pool[o:o + size]))
    return out


def block_size(kind, nx, nu):
    if kind == LQR:
        return HDR + 2 * nx * nx + 2 * nx * nu + nu * nu + 2 * nx + nu
    if kind == UNICYCLE:
        return HDR
    nq = nx // 2
    return HDR + 2 * nq * nq + nq * nu + nq + nx * nx + nx * nu + nu * nu + nx + nu


def box_qp(H, q, lb, ub, xinit, maxiter=100, th_acceptstep=0.1, th_grad=1e-9, reg=1e-9, alphas=None):
    """BoxQP::solve (box-qp.cpp:51-182), numpy linear algebra.

    Returns dict(x, free_idx, clamped_idx, Hff_inv (compact), inv_idx (the
    free set Hff_inv was factorised on), iters) or None where the reference
    throws "backward_error" (LLT failure)."""
    alphas = alphas if alphas is not None else [2.0 ** (-k) for k in range(10)]
    H = np.asarray(H, float)
    q = np.asarray(q, float)
    n = q.size
    x = np.maximum(np.minimum(np.asarray(xinit, float), ub), lb)
    Hff_inv, inv_idx = np.zeros((0, 0)), []
    free, clamped = [], []
    iters = 0

    def chol_inv(idx):
        Hff = H[np.ix_(idx, idx)] + (reg * np.eye(len(idx)) if reg != 0.0 else 0.0)
        try:
            L = np.linalg.cholesky(Hff)
        except np.linalg.LinAlgError:
            return None, None
        if len(idx) and not np.all(np.diag(L) > 0):
            return None, None
        I = np.eye(len(idx))
        return L, np.linalg.solve(L.T, np.linalg.solve(L, I))

    for k in range(maxiter):
        g = q + H @ x
        clamped = [j for j in range(n) if (x[j] == lb[j] and g[j] > 0.0) or (x[j] == ub[j] and g[j] < 0.0)]
        free = [j for j in range(n) if j not in clamped]
        if np.max(np.abs(g)) <= th_grad or len(free) == 0:
            if k == 0:
                L, Hi = chol_inv(free)
                if Hi is None:
                    return None
                Hff_inv, inv_idx = Hi, list(free)
            return dict(x=x, free_idx=free, clamped_idx=clamped, Hff_inv=Hff_inv, inv_idx=inv_idx, iters=iters)
        iters += 1
        L, Hi = chol_inv(free)
        if Hi is None:
            return None
        Hff_inv, inv_idx = Hi, list(free)
        rhs = -q[free]
        if clamped:
            rhs = rhs - H[np.ix_(free, clamped)] @ x[clamped]
        dxf = np.linalg.solve(L.T, np.linalg.solve(L, rhs)) - x[free]
        dx = np.zeros(n)
        dx[free] = dxf
        fold = 0.5 * x @ (H @ x) + q @ x
        for a in alphas:
            xnew = np.maximum(np.minimum(x + a * dx, ub), lb)
            fnew = 0.5 * xnew @ (H @ xnew) + q @ xnew
            if fold - fnew > th_acceptstep * (g @ (x - xnew)):
                x = xnew
                break
    return dict(x=x, free_idx=free, clamped_idx=clamped, Hff_inv=Hff_inv, inv_idx=inv_idx, iters=iters)


class FDDP:
    """SolverFDDP over one problem (x0, models[0..T-1], models[T])."""

    def __init__(self, x0, models, params=None, box=False, u_lb=None, u_ub=None):
        """box=True: SolverBoxFDDP (box-fddp.cpp) with per-knot limits u_lb/u_ub
        (lists of T arrays of the knot's nu; None = no limits)."""
        self.x0 = np.array(x0, dtype=np.float64)
        self.models = models
        self.box = box
        T0 = len(models) - 1
        self.u_lb = u_lb if u_lb is not None else [np.full(m.nu, -np.inf) for m in models[:-1]]
        self.u_ub = u_ub if u_ub is not None else [np.full(m.nu, np.inf) for m in models[:-1]]
        self.haslim = [bool(np.isfinite(self.u_lb[t]).any() and np.isfinite(self.u_ub[t]).any()) for t in range(T0)]
        self.kprev = [np.zeros(m.nu) for m in models[:-1]]  # k_ persists across sweeps (warm start)
        self.Quu_inv = [np.zeros((m.nu, m.nu)) for m in models[:-1]]
        self.T = len(models) - 1
        self.nx = models[0].nx
        self.ndx = models[0].ndx
        self.st = models[0]  # the problem's state: diff / integrate / zero (StateAbstract)
        self.nu_max = max(m.nu for m in models[:-1])
        self.p = params or default_params()
        T, n = self.T, self.ndx
        self.xs = [np.zeros(self.nx) for _ in range(T + 1)]
        self.us = [np.zeros(self.nu_max) for _ in range(T)]
        self.is_feasible = False
        self.was_feasible = False
        self.cost = 0.0
        self.stop = 0.0
        self.xreg = self.ureg = float("nan")
        self.steplength = 1.0
        self.iter = 0
        self.fs = [np.zeros(n) for _ in range(T + 1)]
        self.xnext = [np.zeros(self.nx) for _ in range(T)]
        self.trace = []
        self.status = 0

    # ShootingProblem::calc / calcDiff
    def problem_calc(self, xs, us):
        T = self.T
        costs = []
        for t in range(T):
            m = self.models[t]
            xn, c = m.calc(xs[t], us[t][:m.nu] if m.nu else None)
            self.xnext[t] = xn
            costs.append(c)
        _, cT = self.models[T].calc(xs[T])
        total = 0.0
        for c in costs:
            total += c
        total += cT
        self.knot_costs = costs + [cT]
        return total

    def problem_calc_diff(self, xs, us):
        self.data = []
        for t in range(self.T):
            m = self.models[t]
            self.data.append(m.calc_diff(xs[t], us[t][:m.nu] if m.nu else None))
        self.data.append(self.models[self.T].calc_diff(xs[self.T]))
        total = 0.0
        for c in self.knot_costs:
            total += c
        return total

    def calc_diff(self):
        """ddp.cpp:157-178."""
        if self.iter == 0:
            self.problem_calc(self.xs, self.us)
        self.cost = self.problem_calc_diff(self.xs, self.us)
        if not self.is_feasible:  # fs[0] = diff(xs[0], x0), fs[t+1] = diff(xs[t+1], xnext[t])
            self.fs[0] = self.st.state_diff(self.xs[0], self.x0)
            for t in range(self.T):
                self.fs[t + 1] = self.st.state_diff(self.xs[t + 1], self.xnext[t])
        elif not self.was_feasible:
            self.fs = [np.zeros(self.ndx) for _ in range(self.T + 1)]
        return self.cost

    def backward_pass(self):
        """ddp.cpp:180-253; returns False on backward_error."""
        T, n = self.T, self.ndx
        dT = self.data[T]
        self.Vxx = [None] * (T + 1)
        self.Vx = [None] * (T + 1)
        self.Qxx, self.Qxu, self.Quu = [None] * T, [None] * T, [None] * T
        self.Qx, self.Qu, self.K, self.k, self.Quuk = [None] * T, [None] * T, [None] * T, [None] * T, [None] * T
        Vxx = dT["Lxx"].copy()
        Vx = dT["Lx"].copy()
        if not math.isnan(self.xreg):
            Vxx += self.xreg * np.eye(n)
        if not self.is_feasible:
            Vx = Vx + Vxx @ self.fs[T]
        self.Vxx[T], self.Vx[T] = Vxx, Vx
        for t in range(T - 1, -1, -1):
            d = self.data[t]
            nu = self.models[t].nu
            Vxx_p, Vx_p = self.Vxx[t + 1], self.Vx[t + 1]
            FxTV = d["Fx"].T @ Vxx_p
            Qxx = d["Lxx"] + FxTV @ d["Fx"]
            Qx = d["Lx"] + d["Fx"].T @ Vx_p
            self.Qxx[t], self.Qx[t] = Qxx, Qx
            Vx = Qx.copy()
            Vxx = Qxx.copy()
            if nu != 0:
                Qxu = d["Lxu"] + FxTV @ d["Fu"]
                Quu = d["Luu"] + (d["Fu"].T @ Vxx_p) @ d["Fu"]
                Qu = d["Lu"] + d["Fu"].T @ Vx_p
                if not math.isnan(self.ureg):
                    Quu = Quu + self.ureg * np.eye(nu)
                if self.box and self.haslim[t] and self.is_feasible:
                    # SolverBoxFDDP::computeGains (box-fddp.cpp:48-79)
                    if nu != self.models[0].nu:
                        return False  # qp_ has runningModels[0]->nu variables
                    u = self.us[t][:nu]
                    sol = box_qp(Quu, Qu, self.u_lb[t] - u, self.u_ub[t] - u, self.kprev[t], 100, 0.1, 1e-5, 0.0)
                    if sol is None:
                        return False
                    Qi = np.zeros((nu, nu))
                    Hi, f = sol["Hff_inv"], sol["free_idx"]
                    ni = Hi.shape[0]
                    for i, fi in enumerate(f):
                        for j, fj in enumerate(f):
                            Qi[fi, fj] = Hi[i, j] if (i < ni and j < ni) else 0.0
                    self.Quu_inv[t] = Qi
                    K = Qi @ Qxu.T
                    k = -sol["x"]
                    Qu = Qu.copy()
                    Qu[sol["clamped_idx"]] = 0.0
                else:
                    try:
                        L = np.linalg.cholesky(Quu)
                    except np.linalg.LinAlgError:
                        return False
                    if not np.all(np.diag(L) > 0):
                        return False
                    K = np.linalg.solve(L.T, np.linalg.solve(L, Qxu.T))
                    k = np.linalg.solve(L.T, np.linalg.solve(L, Qu))
                self.kprev[t] = k
                self.Qxu[t], self.Quu[t], self.Qu[t], self.K[t], self.k[t] = Qxu, Quu, Qu, K, k
                if math.isnan(self.ureg):
                    Vx = Vx - K.T @ Qu
                else:
                    Quuk = Quu @ k
                    self.Quuk[t] = Quuk
                    Vx = Vx + K.T @ Quuk - 2 * (K.T @ Qu)
                Vxx = Vxx - Qxu @ K
            else:
                self.Qxu[t], self.Quu[t], self.Qu[t] = np.zeros((n, 0)), np.zeros((0, 0)), np.zeros(0)
                self.K[t], self.k[t], self.Quuk[t] = np.zeros((0, n)), np.zeros(0), np.zeros(0)
            Vxx = 0.5 * (Vxx + Vxx.T)
            if not math.isnan(self.xreg):
                Vxx = Vxx + self.xreg * np.eye(n)
            if not self.is_feasible:
                Vx = Vx + Vxx @ self.fs[t]
            self.Vxx[t], self.Vx[t] = Vxx, Vx
            if raise_if_nan(np.max(np.abs(Vx))) or raise_if_nan(np.max(np.abs(Vxx))):
                return False
            if np.any(np.isnan(Vx)) or np.any(np.isnan(Vxx)):
                return False
        return True

    def compute_direction(self, recalc=True):
        if recalc:
            self.calc_diff()
        return self.backward_pass()

    def forward_pass(self, alpha):
        """fddp.cpp:149-225; returns False on forward_error."""
        T = self.T
        self.cost_try = 0.0
        xnext = self.x0.copy()
        self.xs_try = [None] * (T + 1)
        self.us_try = [np.zeros(self.nu_max) for _ in range(T)]
        xnexts = [None] * T
        costs = [None] * (T + 1)
        for t in range(T):
            m = self.models[t]
            if self.is_feasible or alpha == 1:
                xt = xnext.copy()
            else:
                xt = self.st.state_integrate(xnext, self.fs[t] * (alpha - 1))
            self.xs_try[t] = xt
            dx = self.st.state_diff(self.xs[t], xt)
            if m.nu != 0:
                u = (self.us[t][:m.nu] - self.k[t] * alpha) - self.K[t] @ dx
                if self.box and self.haslim[t]:  # box-fddp.cpp:100-102
                    u = np.minimum(np.maximum(u, self.u_lb[t]), self.u_ub[t])
                self.us_try[t][:m.nu] = u
                xnext, c = m.calc(xt, u)
            else:
                xnext, c = m.calc(xt)
            xnexts[t] = xnext
            costs[t] = c
            self.cost_try += c
            if raise_if_nan(self.cost_try) or raise_if_nan(np.max(np.abs(xnext))) or np.any(np.isnan(xnext)):
                return False
        if self.is_feasible or alpha == 1:
            xT = xnext.copy()
        else:
            xT = self.st.state_integrate(xnext, self.fs[T] * (alpha - 1))
        self.xs_try[T] = xT
        _, cT = self.models[T].calc(xT)
        costs[T] = cT
        self.cost_try += cT
        if raise_if_nan(self.cost_try):
            return False
        self.try_xnext = xnexts
        self.try_costs = costs
        return True

    def try_step(self, alpha=1.0):
        if not self.forward_pass(alpha):
            return None
        return self.cost - self.cost_try

    def update_expected_improvement(self):
        """fddp.cpp:126-147."""
        self.dg = 0.0
        self.dq = 0.0
        T = self.T
        if not self.is_feasible:
            self.dg -= self.Vx[T] @ self.fs[T]
            self.dq += self.fs[T] @ (self.Vxx[T] @ self.fs[T])
        for t in range(T):
            if self.models[t].nu != 0:
                self.dg += self.Qu[t] @ self.k[t]
                self.dq -= self.k[t] @ self.Quuk[t]
            if not self.is_feasible:
                self.dg -= self.Vx[t] @ self.fs[t]
                self.dq += self.fs[t] @ (self.Vxx[t] @ self.fs[t])

    def expected_improvement(self):
        """fddp.cpp:107-124."""
        dv = 0.0
        T = self.T
        if not self.is_feasible:  # dx = diff(xs_try, xs)
            dx = self.st.state_diff(self.xs_try[T], self.xs[T])
            dv -= self.fs[T] @ (self.Vxx[T] @ dx)
            for t in range(T):
                dx = self.st.state_diff(self.xs_try[t], self.xs[t])
                dv -= self.fs[t] @ (self.Vxx[t] @ dx)
        self.d = np.array([self.dg + dv, self.dq - 2 * dv])
        return self.d

    def stopping_criteria(self):
        self.stop = 0.0
        for t in range(self.T):
            if self.models[t].nu != 0:
                self.stop += self.Qu[t] @ self.Qu[t]
        return self.stop

    def _inc(self):
        self.xreg = min(self.xreg * self.p["regfactor"], self.p["regmax"])
        self.ureg = self.xreg

    def _dec(self):
        self.xreg = max(self.xreg / self.p["regfactor"], self.p["regmin"])
        self.ureg = self.xreg

    def set_candidate(self, xs=None, us=None, is_feasible=False):
        T = self.T
        self.xs = [self.st.state_zero() for _ in range(T + 1)] if xs is None else [np.array(x, float) for x in xs]
        self.us = [np.zeros(self.nu_max) for _ in range(T)] if us is None else [np.array(u, float) for u in us]
        self.is_feasible = is_feasible

    def _accept(self):
        self.was_feasible = self.is_feasible
        self.xs = [x.copy() for x in self.xs_try]
        self.us = [u.copy() for u in self.us_try]
        self.xnext = [x.copy() for x in self.try_xnext]
        self.knot_costs = list(self.try_costs)
        self.is_feasible = self.was_feasible or self.steplength == 1
        self.cost = self.cost_try

    def solve(self, xs=None, us=None, maxiter=100, is_feasible=False, reg_init=1e-9):
        """fddp.cpp:19-105."""
        p = self.p
        self.set_candidate(xs, us, is_feasible)
        if reg_init is None or math.isnan(reg_init):
            self.xreg = self.ureg = p["regmin"]
        else:
            self.xreg = self.ureg = reg_init
        self.was_feasible = False
        self.trace = []
        self.status = 0
        self.n_iter_run = 0
        recalc = True
        self.iter = 0
        while self.iter < maxiter:
            self.n_iter_run += 1
            while True:
                if not self.compute_direction(recalc):
                    recalc = False
                    self._inc()
                    if self.xreg == p["regmax"]:
                        self.status = 2
                        return False
                    continue
                break
            self.update_expected_improvement()
            recalc = False
            for a in p["alphas"]:
                self.steplength = a
                dV = self.try_step(a)
                if dV is None:
                    continue
                self.dV = dV
                d = self.expected_improvement()
                self.dVexp = a * (d[0] + 0.5 * a * d[1])
                if self.dVexp >= 0:
                    if d[0] < p["th_grad"] or dV > p["th_acceptstep"] * self.dVexp:
                        self._accept()
                        recalc = True
                        break
                else:
                    if dV > p["th_acceptnegstep"] * self.dVexp:
                        self._accept()
                        recalc = True
                        break
            if self.steplength > p["th_stepdec"]:
                self._dec()
            if self.steplength <= p["th_stepinc"]:
                self._inc()
                if self.xreg == p["regmax"]:
                    self.status = 2
                    return False
            self.stopping_criteria()
            self.trace.append((self.cost, self.stop, self.d[0], self.d[1], self.xreg, self.ureg, self.steplength,
                               float(self.is_feasible)))
            if self.was_feasible and self.stop < p["th_stop"]:
                self.status = 1
                return True
            self.iter += 1
        return False


class KKT:
    """SolverKKT restatement (src/core/solvers/kkt.cpp:34-227): dense Newton
    on the full-horizon KKT system, line search on the true cost. The
    reference's own oracle for DDP/FDDP (unittest/test_solvers.cpp:65-110)."""

    def __init__(self, x0, models):
        self.x0 = np.array(x0, float)
        self.models = models
        self.T = len(models) - 1
        self.nx = models[0].nx
        T, n = self.T, self.nx
        self.nus = [m.nu for m in models[:-1]]
        self.NX = n * (T + 1)
        self.NU = sum(self.nus)
        self.alphas = [2.0 ** (-k) for k in range(10)]
        self.th_acceptstep, self.th_stop, self.th_grad = 0.1, 1e-9, 1e-12

    def _problem_calc(self, xs, us):
        cost = 0.0
        xn = []
        for t in range(self.T):
            m = self.models[t]
            x1, c = m.calc(xs[t], us[t] if m.nu else None)
            xn.append(x1)
            cost += c
        _, cT = self.models[self.T].calc(xs[self.T])
        return cost + cT, xn

    def _calc(self):
        """kkt.cpp:177-221."""
        T, n = self.T, self.nx
        NX, NU = self.NX, self.NU
        self.cost, xnext = self._problem_calc(self.xs, self.us)
        N = NX + NU + NX
        kkt = np.zeros((N, N))
        ref = np.zeros(N)
        kkt[NX + NU:NX + NU + n, 0:n] = np.eye(n)  # block(ndx+nu, 0, ndx, ndx) = I (partial)
        ref[NX + NU:NX + NU + n] = self.xs[0] - self.x0
        ix = iu = 0
        self.data = []
        for t in range(T):
            m = self.models[t]
            d = m.calc_diff(self.xs[t], self.us[t] if m.nu else None)
            self.data.append(d)
            nu = m.nu
            kkt[ix:ix + n, ix:ix + n] = d["Lxx"]
            kkt[ix:ix + n, NX + iu:NX + iu + nu] = d["Lxu"]
            kkt[NX + iu:NX + iu + nu, ix:ix + n] = d["Lxu"].T
            kkt[NX + iu:NX + iu + nu, NX + iu:NX + iu + nu] = d["Luu"]
            r0 = NX + NU + n + ix
            kkt[r0:r0 + n, ix:ix + n] = -d["Fx"]
            kkt[r0:r0 + n, NX + iu:NX + iu + nu] = -d["Fu"]
            kkt[r0:r0 + n, ix + n:ix + 2 * n] = np.eye(n)
            ref[ix:ix + n] = d["Lx"]
            ref[NX + iu:NX + iu + nu] = d["Lu"]
            ref[r0:r0 + n] = self.xs[t + 1] - xnext[t]
            ix += n
            iu += nu
        dT = self.models[T].calc_diff(self.xs[T])
        kkt[ix:ix + n, ix:ix + n] = dT["Lxx"]
        ref[ix:ix + n] = dT["Lx"]
        kkt[0:NX + NU, NX + NU:] = kkt[NX + NU:, 0:NX + NU].T
        self.kkt, self.kktref = kkt, ref

    def _direction(self):
        pd = np.linalg.solve(self.kkt, -self.kktref)
        NX, NU = self.NX, self.NU
        self.primal = pd[:NX + NU]
        px, pu = pd[:NX], pd[NX:NX + NU]
        self.dual = pd[NX + NU:]
        n = self.nx
        self.dxs = [px[t * n:(t + 1) * n] for t in range(self.T + 1)]
        self.dus = []
        iu = 0
        for nu in self.nus:
            self.dus.append(pu[iu:iu + nu])
            iu += nu

    def solve(self, xs, us, maxiter=100):
        self.xs = [np.array(x, float) for x in xs]
        self.us = [np.array(u, float) for u in us]
        is_feasible = False
        was_feasible = False
        for self.iter in range(maxiter):
            self._calc()
            self._direction()
            d0 = -self.kktref[:self.NX + self.NU] @ self.primal
            d1 = -(self.kkt[:self.NX + self.NU, :self.NX + self.NU] @ self.primal) @ self.primal
            for a in self.alphas:
                xs_try = [x + a * dx for x, dx in zip(self.xs, self.dxs)]
                us_try = [u + a * du for u, du in zip(self.us, self.dus)]
                cost_try, _ = self._problem_calc(xs_try, us_try)
                dV = self.cost - cost_try
                dVexp = a * d0 + 0.5 * a * a * d1
                if d0 < self.th_grad or not is_feasible or dV > self.th_acceptstep * dVexp:
                    was_feasible = is_feasible
                    self.xs, self.us = xs_try, us_try
                    is_feasible = True
                    break
            # stoppingCriteria (kkt.cpp:133-157): kktref and Fx/Fu of the
            # pre-step point (computeDirection), duals of this iteration
            n = self.nx
            lam = [self.dual[t * n:(t + 1) * n] for t in range(self.T + 1)]
            dF = np.zeros(self.NX + self.NU)
            ix = iu = 0
            for t in range(self.T):
                d = self.data[t]
                nu = self.nus[t]
                dF[ix:ix + n] = lam[t] - d["Fx"].T @ lam[t + 1]
                dF[self.NX + iu:self.NX + iu + nu] = -(lam[t + 1] @ d["Fu"])
                ix += n
                iu += nu
            dF[ix:ix + n] = lam[self.T]
            stop = np.sum((self.kktref[:self.NX + self.NU] + dF) ** 2) + np.sum(self.kktref[self.NX + self.NU:] ** 2)
            if was_feasible and stop < self.th_stop:
                return True
        return False
