"""ORACLE — TEST INFRASTRUCTURE ONLY (numpy restatement of the multibody knot).

CPU restatement of the knot the reference builds in
benchmark/factory/arm.hpp:31-96 and the Talos-arm config (C3):

  IntegratedActionModelEuler          include/crocoddyl/core/integrator/euler.hxx:41-131
   ∘ DifferentialActionModelFreeFwdDynamics
                                      include/crocoddyl/multibody/actions/free-fwddyn.hxx:44-118
     actuation ActuationModelFull     (tau = u)
     costs CostModelSum               multibody/costs/cost-sum.hxx:89-160
       CostModelState                 multibody/costs/state.hxx:130-169
       CostModelControl               multibody/costs/control.hxx:56-87
       CostModelFramePlacement        multibody/costs/frame-placement.hxx:45-80
       CostModelFrameTranslation      multibody/costs/frame-translation.hxx:50-81
     activations Quad / WeightedQuad  core/activations/{quadratic,weighted-quadratic}.hpp
   on a fixed-base kinematic tree of revolute joints (StateMultibody over a
   Pinocchio model whose q and v spaces coincide, so integrate / diff are
   Euclidean and Jintegrate / Jdiff are identities).

The rigid-body algorithms of Pinocchio (>= 2.4.7, third-party, absent here)
are restated from their published form (Featherstone, "Rigid Body Dynamics
Algorithms", 2008): ABA (Table 7.1) for the forward dynamics the reference
gets from pinocchio::aba (free-fwddyn.hxx:64), RNEA (Table 5.1) and CRBA
(Table 6.2) for the consistency checks, SE(3) log (Pinocchio's log6) for
the frame-placement residual. The derivatives (Fx, Fu, the residual
Jacobians Rx / Ru that the cost Hessians are built from) come from
complex-step differentiation of those functions, exact to rounding and
independent of the analytic linearisation the device uses.

Pinocchio itself is not available offline, so the multibody arithmetic is
"parity unpinned" against the reference's own binary; it is pinned here by
closed-form pendulum dynamics, ABA == CRBA^-1 (tau - RNEA(q, v, 0)),
RNEA(q, v, ABA(q, v, tau)) == tau and finite differences at the reference's
numdiff tolerance (tests/test_multibody_oracle.py).

Parameter-block layout: include/fddp_hip.h (FDDP_KNOT_EULER_FREEFWD).
"""
import numpy as np

HDR = 4
JOINT_REC = 26
COST_HDR = 4
STATE, CONTROL, FRAME_PLACEMENT, FRAME_TRANSLATION = 1, 2, 3, 4
CONTACT_3D, CONTACT_6D = 5, 6  # contact records (FDDP_KNOT_EULER_CONTACTFWD)
CONTACT_FORCE = 7  # CostModelContactForce: r = lambda[row0:row0+nr] - fref (contact-force.hxx:33-50)
H_CS = 1e-30  # complex-step size


# ---------------------------------------------------------------------------
# small SO(3)/SE(3) helpers (dtype-generic: float or complex for complex step)
# ---------------------------------------------------------------------------
def skew(w):
    return np.array([[0 * w[0], -w[2], w[1]], [w[2], 0 * w[0], -w[0]], [-w[1], w[0], 0 * w[0]]])


def rot_axis(axis, q):
    """exp(q [axis]x), Rodrigues (axis unit)."""
    K = skew(np.asarray(axis, float))
    return np.eye(3) + np.sin(q) * K + (1 - np.cos(q)) * (K @ K)


def motion_X(R, p):
    """6x6 motion transform child <- parent for liMi = (R, p), (lin, ang) order:
    SE3::actInv on a motion: lin' = R^T (v - p x w), ang' = R^T w."""
    Rt = R.T
    X = np.zeros((6, 6), dtype=np.result_type(R, p))
    X[:3, :3] = Rt
    X[:3, 3:] = -Rt @ skew(p)
    X[3:, 3:] = Rt
    return X


def spatial_inertia(m, c, Ic):
    """6x6 spatial inertia about the joint origin, (lin, ang) order."""
    C = skew(c)
    I6 = np.zeros((6, 6))
    I6[:3, :3] = m * np.eye(3)
    I6[:3, 3:] = -m * C
    I6[3:, :3] = m * C
    I6[3:, 3:] = Ic - m * C @ C
    return I6


def crm(m):
    """motion cross product matrix, m = (v, w): m x_m n."""
    v, w = m[:3], m[3:]
    X = np.zeros((6, 6), dtype=m.dtype)
    X[:3, :3] = skew(w)
    X[:3, 3:] = skew(v)
    X[3:, 3:] = skew(w)
    return X


def crf(m):
    return -crm(m).T


def log3(R):
    """SO(3) log. Branches on real parts only (complex-step safe)."""
    tr = R[0, 0] + R[1, 1] + R[2, 2]
    c = (tr - 1) / 2
    w = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    s2 = (w[0] * w[0] + w[1] * w[1] + w[2] * w[2]) / 4  # sin^2(theta)
    if np.real(s2) < 1e-8 and np.real(c) > 0:
        # theta / (2 sin theta) as a series in sin^2 (asin(s)/s)
        k = 0.5 * (1 + s2 / 6 + 3 * s2 * s2 / 40 + 5 * s2 ** 3 / 112)
        return k * w
    if np.real(s2) < 1e-8:  # theta near pi: axis from the symmetric part
        theta = np.arccos(np.clip(np.real(c), -1, 1)) + 0 * c
        d = np.array([R[0, 0], R[1, 1], R[2, 2]])
        ax = np.sqrt(np.maximum(np.real((d - c) / (1 - c)), 0)) + 0 * c
        i0 = int(np.argmax(np.real(ax)))
        sgn = np.ones(3)
        for j in range(3):
            if j != i0:
                sgn[j] = 1.0 if np.real(R[i0, j] + R[j, i0]) >= 0 else -1.0
        if np.real(w[i0]) < 0:
            sgn = -sgn
        return theta * sgn * ax
    s = np.sqrt(s2)
    # the better-conditioned inverse on each range of theta
    if np.real(c) > 0.5:
        theta = np.arcsin(s)
    elif np.real(c) < -0.5:
        theta = np.pi - np.arcsin(s)
    else:
        theta = np.arccos(c)
    return theta / (2 * s) * w


def log6(R, p):
    """SE(3) log as (lin, ang): w = log3(R), v = V^-1(w) p."""
    w = log3(R)
    t2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2]
    if np.real(t2) < 1e-2:  # 1/t^2 - (1 + cos t) / (2 t sin t), series of (t/2) cot(t/2)
        beta = 1.0 / 12 + t2 / 720 + t2 * t2 / 30240 + t2 ** 3 / 1209600
    else:
        t = np.sqrt(t2)
        beta = 1 / t2 - np.sin(t) / (2 * t * (1 - np.cos(t)))
    W = skew(w)
    Vinv = np.eye(3) - 0.5 * W + beta * (W @ W)
    return np.concatenate([Vinv @ p, w])


def exp6(nu):
    """SE(3) exp of (lin, ang) — tests only."""
    v, w = np.asarray(nu[:3], float), np.asarray(nu[3:], float)
    t = np.linalg.norm(w)
    W = skew(w)
    if t < 1e-12:
        return np.eye(3) + W, v + 0.5 * W @ v
    R = np.eye(3) + np.sin(t) / t * W + (1 - np.cos(t)) / t ** 2 * W @ W
    V = np.eye(3) + (1 - np.cos(t)) / t ** 2 * W + (t - np.sin(t)) / t ** 3 * W @ W
    return R, V @ v


# ---------------------------------------------------------------------------
# model block
# ---------------------------------------------------------------------------
class Robot:
    """Kinematic tree parsed from the block's robot section."""

    def __init__(self, nj, gravity, armature, joints):
        self.nj = nj
        self.gravity = np.asarray(gravity, float)
        self.armature = np.asarray(armature, float)
        self.parent = [int(j[0]) for j in joints]
        self.axis = [np.asarray(j[1:4], float) for j in joints]
        self.Rpl = [np.asarray(j[4:13], float).reshape(3, 3).T for j in joints]  # column-major
        self.ppl = [np.asarray(j[13:16], float) for j in joints]
        self.mass = [float(j[16]) for j in joints]
        self.com = [np.asarray(j[17:20], float) for j in joints]
        self.Ic = []
        for j in joints:
            xx, yy, zz, xy, xz, yz = j[20:26]
            self.Ic.append(np.array([[xx, xy, xz], [xy, yy, yz], [xz, yz, zz]], float))
        self.I6 = [spatial_inertia(self.mass[i], self.com[i], self.Ic[i]) for i in range(nj)]

    def S(self, i):
        return np.concatenate([np.zeros(3), self.axis[i]])

    def liMi(self, q, i):
        return self.Rpl[i] @ rot_axis(self.axis[i], q[i]), self.ppl[i] + 0 * q[i]

    def placements(self, q):
        """oMi of every joint."""
        out = []
        for i in range(self.nj):
            R, p = self.liMi(q, i)
            lam = self.parent[i]
            if lam >= 0:
                R0, p0 = out[lam]
                out.append((R0 @ R, p0 + R0 @ p))
            else:
                out.append((R, p))
        return out

    # Featherstone Table 5.1 (Pinocchio rnea)
    def rnea(self, q, v, a, gravity=None):
        dt = np.result_type(q, v, a)
        nj = self.nj
        X = [motion_X(*self.liMi(q, i)) for i in range(nj)]
        vs, as_, fs = [None] * nj, [None] * nj, [None] * nj
        g = self.gravity if gravity is None else np.asarray(gravity, float)
        a0 = np.concatenate([-g, np.zeros(3)]).astype(dt)
        for i in range(nj):
            lam = self.parent[i]
            S = self.S(i)
            vp = vs[lam] if lam >= 0 else np.zeros(6, dt)
            ap = as_[lam] if lam >= 0 else a0
            vs[i] = X[i] @ vp + S * v[i]
            as_[i] = X[i] @ ap + S * a[i] + crm(vs[i]) @ (S * v[i])
            fs[i] = self.I6[i] @ as_[i] + crf(vs[i]) @ (self.I6[i] @ vs[i])
        tau = np.zeros(nj, dt)
        for i in reversed(range(nj)):
            tau[i] = self.S(i) @ fs[i]
            lam = self.parent[i]
            if lam >= 0:
                fs[lam] = fs[lam] + X[i].T @ fs[i]
        return tau

    # Featherstone Table 6.2 (Pinocchio crba)
    def crba(self, q):
        nj = self.nj
        X = [motion_X(*self.liMi(q, i)) for i in range(nj)]
        Ic = [I.copy() for I in self.I6]
        for i in reversed(range(nj)):
            lam = self.parent[i]
            if lam >= 0:
                Ic[lam] = Ic[lam] + X[i].T @ Ic[i] @ X[i]
        M = np.zeros((nj, nj), dtype=np.result_type(q, float))
        for i in range(nj):
            F = Ic[i] @ self.S(i)
            M[i, i] = self.S(i) @ F
            j = i
            while self.parent[j] >= 0:
                F = X[j].T @ F
                j = self.parent[j]
                M[i, j] = M[j, i] = self.S(j) @ F
        return M

    # Featherstone Table 7.1 (Pinocchio aba), armature added to D (rotor inertia)
    def aba(self, q, v, tau):
        dt = np.result_type(q, v, tau)
        nj = self.nj
        X = [motion_X(*self.liMi(q, i)) for i in range(nj)]
        vs, cs, IA, pA = [None] * nj, [None] * nj, [None] * nj, [None] * nj
        for i in range(nj):
            lam = self.parent[i]
            S = self.S(i)
            vp = vs[lam] if lam >= 0 else np.zeros(6, dt)
            vs[i] = X[i] @ vp + S * v[i]
            cs[i] = crm(vs[i]) @ (S * v[i])
            IA[i] = self.I6[i].astype(dt)
            pA[i] = crf(vs[i]) @ (self.I6[i] @ vs[i])
        U, D, u = [None] * nj, [None] * nj, [None] * nj
        for i in reversed(range(nj)):
            S = self.S(i)
            U[i] = IA[i] @ S
            D[i] = S @ U[i] + self.armature[i]
            u[i] = tau[i] - S @ pA[i]
            lam = self.parent[i]
            if lam >= 0:
                Ia = IA[i] - np.outer(U[i], U[i]) / D[i]
                pa = pA[i] + Ia @ cs[i] + U[i] * (u[i] / D[i])
                IA[lam] = IA[lam] + X[i].T @ Ia @ X[i]
                pA[lam] = pA[lam] + X[i].T @ pa
        a = [None] * nj
        qdd = np.zeros(nj, dt)
        a0 = np.concatenate([-self.gravity, np.zeros(3)]).astype(dt)
        for i in range(nj):
            lam = self.parent[i]
            ap = a[lam] if lam >= 0 else a0
            ai = X[i] @ ap + cs[i]
            qdd[i] = (u[i] - U[i] @ ai) / D[i]
            a[i] = ai + self.S(i) * qdd[i]
        return qdd


def parse_robot(body, nj):
    g = body[0:3]
    arm = body[3:3 + nj]
    o = 3 + nj
    joints = [body[o + JOINT_REC * i:o + JOINT_REC * (i + 1)] for i in range(nj)]
    return Robot(nj, g, arm, joints), o + JOINT_REC * nj


class Cost:
    def __init__(self, rec, nx, nu):
        self.type = int(rec[0])
        self.weight = float(rec[1])
        weighted = rec[2] != 0
        d = rec[COST_HDR:]
        if self.type == STATE:
            self.xref, w, nr = d[:nx], d[nx:2 * nx], nx
        elif self.type == CONTROL:
            self.uref, w, nr = d[:nu], d[nu:2 * nu], nu
        elif self.type in (FRAME_PLACEMENT, FRAME_TRANSLATION):
            self.joint = int(d[0])
            self.Rf = d[1:10].reshape(3, 3).T
            self.pf = d[10:13]
            if self.type == FRAME_PLACEMENT:
                self.Rri = d[13:22].reshape(3, 3).T  # Mref^-1
                self.pri = d[22:25]
                w, nr = d[25:31], 6
            else:
                self.pref = d[13:16]
                w, nr = d[16:19], 3
        elif self.type == CONTACT_FORCE:
            self.row0, nr = int(d[0]), int(d[1])
            self.fref = d[2:2 + nr]
            w = d[8:8 + nr]
            self.force_fn = None  # set by ContactFwdKnot: (x, u) -> lambda
            self.zero_jac = False  # reference: Rx = Ru = 0 unless enable_force
        else:
            raise ValueError(f"unknown cost type {self.type}")
        self.w = np.asarray(w, float) if weighted else np.ones(nr)

    def residual(self, robot, x, u, oM=None):
        nj = robot.nj
        if self.type == STATE:
            return x - self.xref  # diff(xref, x), state.hxx:136
        if self.type == CONTROL:
            return u - self.uref  # control.hxx:67
        if self.type == CONTACT_FORCE:
            return self.force_fn(x, u)[self.row0:self.row0 + len(self.fref)] - self.fref
        if oM is None:
            oM = robot.placements(x[:nj])
        R0, p0 = oM[self.joint]
        Rf, pf = R0 @ self.Rf, p0 + R0 @ self.pf  # oMf = oMi[parent] * placement
        if self.type == FRAME_TRANSLATION:
            return pf - self.pref  # frame-translation.hxx:57
        return log6(self.Rri @ Rf, self.pri + self.Rri @ pf)  # log6(Mref^-1 oMf), frame-placement.hxx:48-50


class FreeFwdKnot:
    """Euler(dt) ∘ DifferentialActionModelFreeFwdDynamics, parsed from a block."""

    def __init__(self, block, nx, nu, _contact=False):
        p = np.asarray(block, float)
        self.dt = float(p[0])
        nj = int(p[1])
        ncost = int(p[2])
        self.size = int(p[3])
        assert nx == 2 * nj and (_contact or nu == nj), "free-fwddyn knots: nx = 2 nv, nu = nv (full actuation)"
        self.nx, self.nu, self.nj = nx, nu, nj
        self.ndx = nx
        self.kind = 4
        body = p[HDR:]
        self.robot, o = parse_robot(body, nj)
        self.costs = []
        for _ in range(ncost):
            rs = int(body[o + 3])
            self.costs.append(Cost(body[o:o + rs], nx, nu))
            o += rs

    # DAM calc: a and the differential cost
    def accel(self, x, u):
        nj = self.nj
        return self.robot.aba(x[:nj], x[nj:], u)

    def cost_c(self, x, u):
        oM = self.robot.placements(x[:self.nj])
        c = 0.0
        for k in self.costs:
            r = k.residual(self.robot, x, u, oM)
            c = c + k.weight * (0.5 * np.sum(k.w * r * r))
        return c

    def calc(self, x, u=None):
        """IntegratedActionModelEuler::calc (euler.hxx:41-80) -> (xnext, cost)."""
        if u is None:
            u = np.zeros(self.nu)
        nj, dt = self.nj, self.dt
        a = self.accel(x, u)
        cc = self.cost_c(x, u)
        if dt != 0:
            v = x[nj:]
            xn = np.concatenate([x[:nj] + v * dt + a * dt * dt, x[nj:] + a * dt])
            return xn, dt * cc
        return np.array(x, copy=True), cc

    def _cs_jac(self, f, z, n_out):
        J = np.zeros((n_out, z.size))
        for j in range(z.size):
            zc = z.astype(complex)
            zc[j] += 1j * H_CS
            J[:, j] = np.imag(f(zc)) / H_CS
        return J

    def calc_diff(self, x, u=None):
        """IntegratedActionModelEuler::calcDiff (euler.hxx:83-131) with the
        DAM's derivatives; Gauss-Newton cost Hessians (cost-sum.hxx:122-160)."""
        if u is None:
            u = np.zeros(self.nu)
        n, m, nj, dt = self.nx, self.nu, self.nj, self.dt
        z = np.concatenate([x, u])
        if dt != 0:
            Fz = self._cs_jac(lambda zz: self.calc(zz[:n], zz[n:])[0], z, n)
            Fx, Fu = Fz[:, :n], Fz[:, n:]
        else:
            Fx, Fu = np.eye(n), np.zeros((n, m))
        Lz = np.zeros(n + m)
        Lzz = np.zeros((n + m, n + m))
        for k in self.costs:
            r = k.residual(self.robot, x, u)
            Rz = self._cs_jac(lambda zz: k.residual(self.robot, zz[:n], zz[n:]), z, r.size)
            if getattr(k, "zero_jac", False):
                Rz[:] = 0.0
            Lz += k.weight * Rz.T @ (k.w * r)
            Lzz += k.weight * Rz.T @ (k.w[:, None] * Rz)
        s = dt if dt != 0 else 1.0
        return dict(Fx=Fx, Fu=Fu, Lx=s * Lz[:n], Lu=s * Lz[n:], Lxx=s * Lzz[:n, :n], Lxu=s * Lzz[:n, n:],
                    Luu=s * Lzz[n:, n:])


class Contact:
    """One active contact record (ContactModel3D / ContactModel6D, LOCAL frame)."""

    def __init__(self, rec):
        self.type = int(rec[0])
        self.gains = (float(rec[1]), float(rec[2]))
        d = rec[COST_HDR:]
        self.joint = int(d[0])
        self.Rf = d[1:10].reshape(3, 3).T  # frame placement in its joint
        self.pf = d[10:13]
        if self.type == CONTACT_3D:
            self.pref = d[13:16]  # (empty for an impulse record)
            self.nc = 3
        elif self.type == CONTACT_6D:
            if d.size >= 25:
                self.Rri = d[13:22].reshape(3, 3).T  # Mref^-1
                self.pri = d[22:25]
            self.nc = 6
        else:
            raise ValueError(f"unknown contact type {self.type}")


def local_motions(robot, q, v, qdd):
    """Featherstone's forward recursion in joint frames WITHOUT gravity: spatial
    velocity and acceleration of every joint (Pinocchio data.v / data.a after
    computeAllTerms (qdd = 0) or forwardKinematics(q, v, qdd))."""
    dt = np.result_type(q, v, qdd)
    vs, as_ = [], []
    for i in range(robot.nj):
        X = motion_X(*robot.liMi(q, i))
        lam = robot.parent[i]
        S = robot.S(i)
        vp = vs[lam] if lam >= 0 else np.zeros(6, dt)
        ap = as_[lam] if lam >= 0 else np.zeros(6, dt)
        vi = X @ vp + S * v[i]
        vs.append(vi)
        as_.append(X @ ap + S * qdd[i] + crm(vi) @ (S * v[i]))
    return vs, as_


class ContactFwdKnot(FreeFwdKnot):
    """Euler(dt) ∘ DifferentialActionModelContactFwdDynamics
    (multibody/actions/contact-fwddyn.hxx:59-160) with ActuationModelFloatingBase
    (tau = [0_{nun}; u], actuations/floating-base.hpp:29-40) and a
    ContactModelMultiple of ContactModel3D / ContactModel6D in name order
    (contacts/{contact-3d,contact-6d,multiple-contacts}.hxx).

    The constrained dynamics are solved as ONE KKT system
        [M  Jc^T ; Jc  -damping I] [a ; -lambda] = [tau - nle ; -a0]
    (pinocchio::forwardDynamics, contact-fwddyn.hxx:94-96, restated), where Jc
    stacks the LOCAL frame Jacobians (3 linear rows for a 3D contact) and a0 the
    frame drift accelerations with the Baumgarte terms (contact-3d.hxx:27-43,
    contact-6d.hxx:27-45). Fx / Fu come from complex-step differentiation of
    this calc: the reference's analytic KKT-inverse formula
    (contact-fwddyn.hxx:127-140) is the implicit-function derivative of the
    same map, so the two agree to rounding."""

    def __init__(self, block, nx, nu):
        p = np.asarray(block, float)
        nj = int(p[1])
        ncost = int(p[2])
        body = p[HDR:]
        o = 3 + nj + JOINT_REC * nj
        for _ in range(ncost):
            o += int(body[o + 3])
        self.nun = int(body[o])
        self.damping = float(body[o + 1])
        ncon = int(body[o + 2])
        self.enable_force = int(body[o + 3]) == 2
        o += 4
        self.contacts = []
        for _ in range(ncon):
            rs = int(body[o + 3])
            self.contacts.append(Contact(body[o:o + rs]))
            o += rs
        assert nu == nj - self.nun, "contact-fwddyn knots: nu = nv - (unactuated root dofs)"
        super().__init__(block, nx, nu, _contact=True)
        self.kind = 5
        self.nc = sum(c.nc for c in self.contacts)
        for c in self.costs:
            if c.type == CONTACT_FORCE:
                c.force_fn = lambda xx, uu: self.accel_force(xx, uu)[1]
                c.zero_jac = not self.enable_force

    def contact_terms(self, x):
        """(Jc (nc x nv), a0 (nc)) at ddq = 0 (ContactModelMultiple::calc)."""
        nj = self.nj
        q, v = x[:nj], x[nj:]
        dt = np.result_type(x, float)
        vs, as_ = local_motions(self.robot, q, v, np.zeros(nj, dt))
        oM = self.robot.placements(q)
        Js, a0s = [], []
        for c in self.contacts:
            Xf = motion_X(c.Rf, c.pf)  # joint -> frame (SE3::actInv by jMf)
            vf = Xf @ vs[c.joint]
            af = Xf @ as_[c.joint]
            # LOCAL frame Jacobian: frame velocity per unit joint velocity
            J = np.zeros((6, nj), dt)
            for k in range(nj):
                e = np.zeros(nj, dt)
                e[k] = 1.0
                J[:, k] = Xf @ local_motions(self.robot, q, e, np.zeros(nj, dt))[0][c.joint]
            R0, p0 = oM[c.joint]
            Rw, pw = R0 @ c.Rf, p0 + R0 @ c.pf  # oMf
            kp, kd = c.gains
            if c.type == CONTACT_3D:
                a0 = af[:3] + np.cross(vf[3:], vf[:3])  # classical acceleration, contact-3d.hxx:37
                if kp != 0.0:
                    a0 = a0 + kp * (pw - c.pref)
                if kd != 0.0:
                    a0 = a0 + kd * vf[:3]
                Js.append(J[:3])
            else:
                a0 = af.copy()
                if kp != 0.0:
                    a0 = a0 + kp * log6(c.Rri @ Rw, c.pri + c.Rri @ pw)
                if kd != 0.0:
                    a0 = a0 + kd * vf
                Js.append(J)
            a0s.append(a0)
        if not Js:
            return np.zeros((0, nj), dt), np.zeros(0, dt)
        return np.vstack(Js), np.concatenate(a0s)

    def accel_force(self, x, u):
        nj, nc = self.nj, self.nc
        q, v = x[:nj], x[nj:]
        M = self.robot.crba(q) + np.diag(self.robot.armature)
        nle = self.robot.rnea(q, v, np.zeros(nj, np.result_type(x, float)))
        tau = np.concatenate([np.zeros(self.nun, np.result_type(u, float)), u])
        Jc, a0 = self.contact_terms(x)
        K = np.zeros((nj + nc, nj + nc), dtype=np.result_type(M, Jc))
        K[:nj, :nj] = M
        K[:nj, nj:] = Jc.T
        K[nj:, :nj] = Jc
        K[nj:, nj:] = -self.damping * np.eye(nc)
        sol = np.linalg.solve(K, np.concatenate([tau - nle, -a0]))
        return sol[:nj], -sol[nj:]

    def accel(self, x, u):
        return self.accel_force(x, u)[0]


class ImpulseFwdKnot(FreeFwdKnot):
    """ActionModelImpulseFwdDynamics (multibody/actions/impulse-fwddyn.hxx:53-127)
    with an ImpulseModelMultiple of ImpulseModel3D / 6D (impulses/impulse-{3d,6d}.hxx,
    LOCAL frame), nu = 0:
        [M  Jc^T ; Jc  -damping I] [v+ ; -Lambda] = [M v ; -r Jc v]
    (pinocchio::impulseDynamics restated), xnext = (q, v+), cost = costs(x).
    calcDiff restates the reference's formula (impulse-fwddyn.hxx:111-119):
    Fx = [[I, 0], [-G dtau_dq - H dv0_dq, G M]] with G, H the KKT-inverse blocks,
    dtau_dq = d/dq [RNEA(q, 0, v+ - v) - Jc^T Lambda] without gravity (fext fixed
    in their frames) and dv0_dq = d/dq (Jc v+), each by complex step of that
    sub-function. For r = 0 this is the exact derivative of calc (tested); for
    r > 0 the reference drops the restitution terms, and so does this."""

    def __init__(self, block, nx, nu):
        p = np.asarray(block, float)
        nj = int(p[1])
        ncost = int(p[2])
        body = p[HDR:]
        o = 3 + nj + JOINT_REC * nj
        for _ in range(ncost):
            o += int(body[o + 3])
        self.r_coeff = float(body[o])
        self.damping = float(body[o + 1])
        nimp = int(body[o + 2])
        assert int(body[o + 3]) == 1, "impulse section flag"
        o += 4
        self.contacts = []
        for _ in range(nimp):
            rs = int(body[o + 3])
            self.contacts.append(Contact(body[o:o + rs]))
            o += rs
        assert nu == 0, "impulse knots have no controls"
        super().__init__(block, nx, nu, _contact=True)
        self.kind = 6
        self.nun = nj
        self.nc = sum(c.nc for c in self.contacts)

    def jac(self, q):
        nj = self.nj
        dt = np.result_type(q, float)
        Js = []
        for c in self.contacts:
            Xf = motion_X(c.Rf, c.pf)
            J = np.zeros((6, nj), dt)
            for k in range(nj):
                e = np.zeros(nj, dt)
                e[k] = 1.0
                J[:, k] = Xf @ local_motions(self.robot, q, e, np.zeros(nj, dt))[0][c.joint]
            Js.append(J[:3] if c.type == CONTACT_3D else J)
        return np.vstack(Js) if Js else np.zeros((0, nj), dt)

    def kkt(self, q):
        nj, nc = self.nj, self.nc
        M = self.robot.crba(q) + np.diag(self.robot.armature)
        J = self.jac(q)
        K = np.zeros((nj + nc, nj + nc), dtype=np.result_type(M, J))
        K[:nj, :nj] = M
        K[:nj, nj:] = J.T
        K[nj:, :nj] = J
        K[nj:, nj:] = -self.damping * np.eye(nc)
        return M, J, K

    def impulse(self, x):
        nj = self.nj
        q, v = x[:nj], x[nj:]
        M, J, K = self.kkt(q)
        sol = np.linalg.solve(K, np.concatenate([M @ v, -self.r_coeff * (J @ v)]))
        return sol[:nj], -sol[nj:]

    def calc(self, x, u=None):
        nj = self.nj
        vp, _ = self.impulse(x)
        xn = np.concatenate([x[:nj] + 0 * vp, vp])
        return xn, self.cost_c(x, np.zeros(0))

    def calc_diff(self, x, u=None):
        n, nj = self.nx, self.nj
        x = np.asarray(x, float)
        q, v = x[:nj], x[nj:]
        vp, lam = self.impulse(x)
        M, J, _ = self.kkt(q)
        Minv = np.linalg.inv(M)
        Y = Minv @ J.T
        S = J @ Y + self.damping * np.eye(self.nc)
        H = Y @ np.linalg.inv(S)
        G = Minv - H @ Y.T
        dv = vp - v

        def tau(qq):  # RNEA(q, 0, dv) - Jc^T lambda, no gravity, lambda fixed in the frames
            return self.robot.rnea(qq, np.zeros(nj), dv, gravity=np.zeros(3)) - self.jac(qq).T @ lam

        dtau = self._cs_jac(tau, q, nj)
        dv0 = self._cs_jac(lambda qq: self.jac(qq) @ vp, q, self.nc)
        Fx = np.zeros((n, n))
        Fx[:nj, :nj] = np.eye(nj)
        Fx[nj:, :nj] = -G @ dtau - H @ dv0
        Fx[nj:, nj:] = G @ M
        Lx = np.zeros(n)
        Lxx = np.zeros((n, n))
        u0 = np.zeros(0)
        for k in self.costs:
            r = k.residual(self.robot, x, u0)
            Rx = self._cs_jac(lambda xx: k.residual(self.robot, xx, u0), x, r.size)
            Lx += k.weight * Rx.T @ (k.w * r)
            Lxx += k.weight * Rx.T @ (k.w[:, None] * Rx)
        return dict(Fx=Fx, Fu=np.zeros((n, 0)), Lx=Lx, Lu=np.zeros(0), Lxx=Lxx, Lxu=np.zeros((n, 0)),
                    Luu=np.zeros((0, 0)))


def block_size(block):
    return int(block[3])
