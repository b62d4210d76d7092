"""ORACLE — TEST INFRASTRUCTURE ONLY (numpy restatement of the multibody knots).

CPU restatement of the knots the reference builds in
benchmark/factory/arm.hpp:31-96 (C3), benchmark/bipedal-timings.cpp:52-140 (C5)
and bindings/python/crocoddyl/utils/{quadruped,biped}.py (C4 / C5 gaits):

  IntegratedActionModelEuler          include/crocoddyl/core/integrator/euler.hxx:41-131
   ∘ DifferentialActionModelFreeFwdDynamics
                                      include/crocoddyl/multibody/actions/free-fwddyn.hxx:44-118
   ∘ DifferentialActionModelContactFwdDynamics
                                      multibody/actions/contact-fwddyn.hxx:59-160
  ActionModelImpulseFwdDynamics       multibody/actions/impulse-fwddyn.hxx:53-127
     costs CostModelSum               multibody/costs/cost-sum.hxx:89-160
       CostModelState                 multibody/costs/state.hxx:130-169
       CostModelControl               multibody/costs/control.hxx:56-87
       CostModelFramePlacement        multibody/costs/frame-placement.hxx:45-80
       CostModelFrameTranslation      multibody/costs/frame-translation.hxx:50-81
       CostModelContactForce          multibody/costs/contact-force.hxx:33-74
       CostModelContactFrictionCone   multibody/costs/contact-friction-cone.hxx:51-91
       CostModelCoMPosition           multibody/costs/com-position.hxx:49-75
       CostModelFrameVelocity         multibody/costs/frame-velocity.hxx:53-84
     activations Quad / WeightedQuad / QuadraticBarrier / WeightedQuadraticBarrier
                                      core/activations/{quadratic,weighted-quadratic,
                                      quadratic-barrier,weighted-quadratic-barrier}.hpp
  StateMultibody                      multibody/states/multibody.hxx:54-240

over a kinematic tree whose root joint is either fixed (a revolute joint on the
universe) or a free-flyer (pinocchio JointModelFreeFlyer: q = (p, quat xyzw),
v = body twist (linear, angular) in the base frame), with revolute joints below.

The state is a manifold: x = (q, v) with nq = nv + 1 for a free-flyer root, and
the reference's diff / integrate are pinocchio::difference / integrate
(multibody.hxx:54-91): for the free-flyer, M0^-1 M1 -> log6 and M exp6(dq) with
the quaternion re-extracted from the rotation (Eigen's algorithm), kept in the
input's hemisphere and first-order normalised (pinocchio
SpecialEuclideanOperationTpl<3>::integrate). Every derivative the oracle returns
is in tangent coordinates, as the reference's: Fx = d diff(xnext, calc(x [+] dx)) / d dx.

The rigid-body algorithms of Pinocchio (>= 2.4.7, third-party, absent here)
are restated from their published form (Featherstone, "Rigid Body Dynamics
Algorithms", 2008): ABA (Table 7.1) with multi-dof joints for the forward
dynamics the reference gets from pinocchio::aba (free-fwddyn.hxx:64), RNEA
(Table 5.1) and CRBA (Table 6.2), SE(3) exp / log (Pinocchio's exp6 / log6).
The derivatives (Fx, Fu, the residual Jacobians Rx / Ru that the cost Hessians
are built from) come from complex-step differentiation of those functions in
tangent coordinates (x [+] i h e_j), exact to rounding and independent of the
analytic world-frame linearisation the device uses.

Pinocchio itself is not available offline, so the multibody arithmetic is
"parity unpinned" against the reference's own binary; it is pinned here by
closed-form pendulum dynamics, ABA == CRBA^-1 (tau - RNEA(q, v, 0)),
RNEA(q, v, ABA(q, v, tau)) == tau, free-body Newton-Euler in closed form, the
exp / log identities and finite differences at the reference's numdiff
tolerance (tests/test_multibody_oracle.py).

Parameter-block layout: include/fddp_hip.h (FDDP_KNOT_EULER_FREEFWD).
"""
import numpy as np

HDR = 4
JOINT_REC = 27
REVOLUTE, FREEFLYER = 0, 1
COST_HDR = 4
STATE, CONTROL, FRAME_PLACEMENT, FRAME_TRANSLATION = 1, 2, 3, 4
CONTACT_3D, CONTACT_6D = 5, 6  # contact records (FDDP_KNOT_EULER_CONTACTFWD)
CONTACT_FORCE = 7  # CostModelContactForce: r = lambda[row0:row0+nr] - fref (contact-force.hxx:33-50)
COM_POSITION = 8  # CostModelCoMPosition: r = com(q) - cref (com-position.hxx:49-75)
FRICTION_CONE = 9  # CostModelContactFrictionCone: r = A lambda_lin (contact-friction-cone.hxx:51-91)
FRAME_VELOCITY = 10  # CostModelFrameVelocity: r = v_frame (LOCAL) - vref (frame-velocity.hxx:53-84)
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
    """SE(3) exp of (lin, ang) (pinocchio exp6): R = cos t I + (1 - cos t)/t^2 w w^T
    + sin t / t [w]x, p = V(w) v. Taylor branch for t^2 < 1e-8 (polynomial in t^2,
    so complex steps through it are exact)."""
    v, w = nu[:3], nu[3:]
    t2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2]
    if np.real(t2) < 1e-8:
        ct = 1 - t2 / 2 + t2 * t2 / 24
        st_t = 1 - t2 / 6 + t2 * t2 / 120
        a_wxv = 0.5 - t2 / 24 + t2 * t2 / 720
        a_w = 1.0 / 6 - t2 / 120 + t2 * t2 / 5040
    else:
        t = np.sqrt(t2)
        ct = np.cos(t)
        st_t = np.sin(t) / t
        a_wxv = (1 - ct) / t2
        a_w = (1 - st_t) / t2
    R = ct * np.eye(3) + a_wxv * np.outer(w, w) + st_t * skew(w)
    wv = w[0] * v[0] + w[1] * v[1] + w[2] * v[2]
    p = st_t * v + a_w * wv * w + a_wxv * np.cross(w, v)
    return R, p


def quat_to_R(qv):
    """Eigen QuaternionBase::toRotationMatrix, coefficients (x, y, z, w)."""
    x, y, z, w = qv
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return np.array([[1 - (tyy + tzz), txy - twz, txz + twy],
                     [txy + twz, 1 - (txx + tzz), tyz - twx],
                     [txz - twy, tyz + twx, 1 - (txx + tyy)]])


def R_to_quat(R):
    """Eigen's quaternion-from-rotation (quaternionbase_assign_impl), branches on
    real parts. Returns (x, y, z, w)."""
    t = R[0, 0] + R[1, 1] + R[2, 2]
    q = [None] * 4
    if np.real(t) > 0:
        t = np.sqrt(t + 1.0)
        q[3] = 0.5 * t
        t = 0.5 / t
        q[0] = (R[2, 1] - R[1, 2]) * t
        q[1] = (R[0, 2] - R[2, 0]) * t
        q[2] = (R[1, 0] - R[0, 1]) * t
    else:
        i = 0
        if np.real(R[1, 1]) > np.real(R[0, 0]):
            i = 1
        if np.real(R[2, 2]) > np.real(R[i, i]):
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = np.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0)
        q[i] = 0.5 * t
        t = 0.5 / t
        q[3] = (R[k, j] - R[j, k]) * t
        q[j] = (R[j, i] + R[i, j]) * t
        q[k] = (R[k, i] + R[i, k]) * t
    return np.array(q)


def se3_integrate(q7, dq6):
    """pinocchio SpecialEuclideanOperationTpl<3>::integrate: M1 = M0 exp6(dq);
    quaternion from M1's rotation, flipped into q0's hemisphere, first-order
    normalised."""
    R0 = quat_to_R(q7[3:7])
    Re, pe = exp6(dq6)
    R1 = R0 @ Re
    p1 = q7[:3] + R0 @ pe
    qn = R_to_quat(R1)
    if np.real(np.dot(qn, q7[3:7])) < 0:
        qn = -qn
    n2 = np.dot(qn, qn)
    qn = qn * ((3 - n2) / 2)
    return np.concatenate([p1, qn])


def se3_difference(q0, q1):
    """pinocchio SpecialEuclideanOperationTpl<3>::difference: log6(M0^-1 M1)."""
    R0, R1 = quat_to_R(q0[3:7]), quat_to_R(q1[3:7])
    return log6(R0.T @ R1, R0.T @ (q1[:3] - q0[:3]))


# ---------------------------------------------------------------------------
# model block
# ---------------------------------------------------------------------------
class Robot:
    """Kinematic tree parsed from the block's robot section: one record per
    pinocchio joint (a free-flyer may only be the root)."""

    def __init__(self, nv, gravity, armature, joints):
        self.gravity = np.asarray(gravity, float)
        self.armature = np.asarray(armature, float)
        self.kind = [int(j[0]) for j in joints]
        self.parent = [int(j[1]) for j in joints]
        self.axis = [np.asarray(j[2:5], float) for j in joints]
        self.Rpl = [np.asarray(j[5:14], float).reshape(3, 3).T for j in joints]  # column-major
        self.ppl = [np.asarray(j[14:17], float) for j in joints]
        self.mass = [float(j[17]) for j in joints]
        self.com = [np.asarray(j[18:21], float) for j in joints]
        self.Ic = []
        for j in joints:
            xx, yy, zz, xy, xz, yz = j[21:27]
            self.Ic.append(np.array([[xx, xy, xz], [xy, yy, yz], [xz, yz, zz]], float))
        self.nb = len(joints)
        self.I6 = [spatial_inertia(self.mass[i], self.com[i], self.Ic[i]) for i in range(self.nb)]
        self.nvj = [6 if k == FREEFLYER else 1 for k in self.kind]
        self.nqj = [7 if k == FREEFLYER else 1 for k in self.kind]
        self.iv = np.concatenate([[0], np.cumsum(self.nvj)[:-1]]).astype(int)
        self.iq = np.concatenate([[0], np.cumsum(self.nqj)[:-1]]).astype(int)
        self.nv, self.nq = int(sum(self.nvj)), int(sum(self.nqj))
        self.ff = self.kind[0] == FREEFLYER
        assert self.nv == nv, "record count does not match nv"
        assert all(k != FREEFLYER for k in self.kind[1:]), "a free-flyer may only be the root"
        self.nj = self.nv  # legacy name: dofs

    def S(self, i):
        if self.kind[i] == FREEFLYER:
            return np.eye(6)
        return np.concatenate([np.zeros(3), self.axis[i]]).reshape(6, 1)

    def vseg(self, v, i):
        return v[self.iv[i]:self.iv[i] + self.nvj[i]]

    def liMi(self, q, i):
        if self.kind[i] == FREEFLYER:
            qq = q[self.iq[i]:self.iq[i] + 7]
            Rj, pj = quat_to_R(qq[3:7]), qq[:3]
        else:
            qi = q[self.iq[i]]
            Rj, pj = rot_axis(self.axis[i], qi), np.zeros(3) + 0 * qi
        return self.Rpl[i] @ Rj, self.ppl[i] + self.Rpl[i] @ pj

    def placements(self, q):
        """oMi of every joint."""
        out = []
        for i in range(self.nb):
            R, p = self.liMi(q, i)
            lam = self.parent[i]
            if lam >= 0:
                R0, p0 = out[lam]
                out.append((R0 @ R, p0 + R0 @ p))
            else:
                out.append((R, p))
        return out

    # Featherstone Table 5.1 (Pinocchio rnea); fext: forces in the joint frames
    # (pinocchio's fext convention), may be None
    def rnea(self, q, v, a, gravity=None, fext=None):
        dt = np.result_type(q, v, a)
        nb = self.nb
        X = [motion_X(*self.liMi(q, i)) for i in range(nb)]
        vs, as_, fs = [None] * nb, [None] * nb, [None] * nb
        g = self.gravity if gravity is None else np.asarray(gravity, float)
        a0 = np.concatenate([-g, np.zeros(3)]).astype(dt)
        for i in range(nb):
            lam = self.parent[i]
            S = self.S(i)
            vp = vs[lam] if lam >= 0 else np.zeros(6, dt)
            ap = as_[lam] if lam >= 0 else a0
            vJ = S @ self.vseg(v, i)
            vs[i] = X[i] @ vp + vJ
            as_[i] = X[i] @ ap + S @ self.vseg(a, i) + crm(vs[i]) @ vJ
            fs[i] = self.I6[i] @ as_[i] + crf(vs[i]) @ (self.I6[i] @ vs[i])
            if fext is not None:
                fs[i] = fs[i] - fext[i]
        tau = np.zeros(self.nv, dt)
        for i in reversed(range(nb)):
            tau[self.iv[i]:self.iv[i] + self.nvj[i]] = self.S(i).T @ fs[i]
            lam = self.parent[i]
            if lam >= 0:
                fs[lam] = fs[lam] + X[i].T @ fs[i]
        return tau

    # Featherstone Table 6.2 (Pinocchio crba)
    def crba(self, q):
        nb = self.nb
        X = [motion_X(*self.liMi(q, i)) for i in range(nb)]
        Ic = [I.astype(np.result_type(q, float)) for I in self.I6]
        for i in reversed(range(nb)):
            lam = self.parent[i]
            if lam >= 0:
                Ic[lam] = Ic[lam] + X[i].T @ Ic[i] @ X[i]
        M = np.zeros((self.nv, self.nv), dtype=np.result_type(q, float))
        for i in range(nb):
            Si = self.S(i)
            si = slice(self.iv[i], self.iv[i] + self.nvj[i])
            F = Ic[i] @ Si
            M[si, si] = Si.T @ F
            j = i
            while self.parent[j] >= 0:
                F = X[j].T @ F
                j = self.parent[j]
                sj = slice(self.iv[j], self.iv[j] + self.nvj[j])
                M[sj, si] = self.S(j).T @ F
                M[si, sj] = M[sj, si].T
        return M

    # Featherstone Table 7.1 (Pinocchio aba) with multi-dof joints, armature added to D
    def aba(self, q, v, tau):
        dt = np.result_type(q, v, tau)
        nb = self.nb
        X = [motion_X(*self.liMi(q, i)) for i in range(nb)]
        vs, cs, IA, pA = [None] * nb, [None] * nb, [None] * nb, [None] * nb
        for i in range(nb):
            lam = self.parent[i]
            S = self.S(i)
            vp = vs[lam] if lam >= 0 else np.zeros(6, dt)
            vJ = S @ self.vseg(v, i)
            vs[i] = X[i] @ vp + vJ
            cs[i] = crm(vs[i]) @ vJ
            IA[i] = self.I6[i].astype(dt)
            pA[i] = crf(vs[i]) @ (self.I6[i] @ vs[i])
        U, Dinv, u = [None] * nb, [None] * nb, [None] * nb
        for i in reversed(range(nb)):
            S = self.S(i)
            sl = slice(self.iv[i], self.iv[i] + self.nvj[i])
            U[i] = IA[i] @ S
            D = S.T @ U[i] + np.diag(self.armature[sl])
            Dinv[i] = np.linalg.inv(D)
            u[i] = tau[sl] - S.T @ pA[i]
            lam = self.parent[i]
            if lam >= 0:
                Ia = IA[i] - U[i] @ Dinv[i] @ U[i].T
                pa = pA[i] + Ia @ cs[i] + U[i] @ (Dinv[i] @ u[i])
                IA[lam] = IA[lam] + X[i].T @ Ia @ X[i]
                pA[lam] = pA[lam] + X[i].T @ pa
        a = [None] * nb
        qdd = np.zeros(self.nv, dt)
        a0 = np.concatenate([-self.gravity, np.zeros(3)]).astype(dt)
        for i in range(nb):
            lam = self.parent[i]
            ap = a[lam] if lam >= 0 else a0
            ai = X[i] @ ap + cs[i]
            sl = slice(self.iv[i], self.iv[i] + self.nvj[i])
            qdd[sl] = Dinv[i] @ (u[i] - U[i].T @ ai)
            a[i] = ai + self.S(i) @ qdd[sl]
        return qdd

    def center_of_mass(self, q):
        """Centre of mass (pinocchio::centerOfMass)."""
        oM = self.placements(q)
        mt = sum(self.mass)
        c = 0
        for i in range(self.nb):
            R, p = oM[i]
            c = c + self.mass[i] * (p + R @ self.com[i])
        return c / mt

    # -- StateMultibody restated (multibody.hxx:54-91) -------------------------
    def neutral(self):
        q = np.zeros(self.nq)
        if self.ff:
            q[6] = 1.0
        return q

    def integrate_q(self, q, dq):
        if self.ff:
            return np.concatenate([se3_integrate(q[:7], dq[:6]), q[7:] + dq[6:]])
        return q + dq

    def difference_q(self, q0, q1):
        if self.ff:
            return np.concatenate([se3_difference(q0[:7], q1[:7]), q1[7:] - q0[7:]])
        return q1 - q0

    def state_integrate(self, x, dx):
        nq, nv = self.nq, self.nv
        return np.concatenate([self.integrate_q(x[:nq], dx[:nv]), x[nq:] + dx[nv:]])

    def state_diff(self, x0, x1):
        nq, nv = self.nq, self.nv
        return np.concatenate([self.difference_q(x0[:nq], x1[:nq]), x1[nq:] - x0[nq:]])


def parse_robot(body, nv):
    g = body[0:3]
    arm = body[3:3 + nv]
    o = 3 + nv
    nb = nv - 5 if int(body[o]) == FREEFLYER else nv
    joints = [body[o + JOINT_REC * i:o + JOINT_REC * (i + 1)] for i in range(nb)]
    return Robot(nv, g, arm, joints), o + JOINT_REC * nb


class Cost:
    def __init__(self, rec, nx, ndx, nu):
        self.type = int(rec[0])
        self.weight = float(rec[1])
        self.act = int(rec[2])  # 0 Quad, 1 WeightedQuad, 2 QuadraticBarrier, 3 WeightedQuadraticBarrier
        d = rec[COST_HDR:]
        self.size = int(rec[3])
        if self.type == STATE:
            self.xref, o, nr = d[:nx], nx, ndx
        elif self.type == CONTROL:
            self.uref, o, nr = d[:nu], nu, nu
        elif self.type in (FRAME_PLACEMENT, FRAME_TRANSLATION, FRAME_VELOCITY):
            self.joint = int(d[0])
            self.Rf = d[1:10].reshape(3, 3).T
            self.pf = d[10:13]
            if self.type == FRAME_PLACEMENT:
                self.Rri = d[13:22].reshape(3, 3).T  # Mref^-1
                self.pri = d[22:25]
                o, nr = 25, 6
            elif self.type == FRAME_VELOCITY:
                self.vref = d[13:19]
                o, nr = 19, 6
            else:
                self.pref = d[13:16]
                o, nr = 16, 3
        elif self.type == COM_POSITION:
            self.cref = d[0:3]
            o, nr = 3, 3
        elif self.type == CONTACT_FORCE:
            self.row0, nr = int(d[0]), int(d[1])
            self.fref = d[2:2 + nr]
            o = 8
            self.force_fn = None  # set by ContactFwdKnot: (x, u) -> lambda
            self.zero_jac = False  # reference: Rx = Ru = 0 unless enable_force
        elif self.type == FRICTION_CONE:
            self.row0, nr = int(d[0]), int(d[2])
            self.A = d[3:3 + 3 * nr].reshape(nr, 3)
            o = 3 + 3 * nr
            self.force_fn = None
            self.zero_jac = False
        else:
            raise ValueError(f"unknown cost type {self.type}")
        self.nr = nr
        prm = np.asarray(d[o:], float)
        if self.act in (0, 1):
            self.w = prm[:nr] if self.act == 1 else np.ones(nr)
        elif self.act in (2, 3):
            self.lb, self.ub = prm[:nr], prm[nr:2 * nr]
            self.w = prm[2 * nr:3 * nr] if self.act == 3 else None
        else:
            raise ValueError(f"unknown activation kind {self.act}")

    # activations (core/activations/*.hpp): value, Ar, diag(Arr) of a real residual
    def a_value(self, r):
        if self.act in (0, 1):
            return 0.5 * np.sum(self.w * r * r)
        rl, ru = np.minimum(r - self.lb, 0.0), np.maximum(r - self.ub, 0.0)
        if self.act == 3:  # weighted-quadratic-barrier.hpp:42-46: w scales before squaring
            rl, ru = self.w * rl, self.w * ru
        return 0.5 * np.sum(rl * rl) + 0.5 * np.sum(ru * ru)

    def a_grad(self, r):
        if self.act in (0, 1):
            return self.w * r
        g = np.minimum(r - self.lb, 0.0) + np.maximum(r - self.ub, 0.0)
        return self.w * self.w * g if self.act == 3 else g

    def a_hess(self, r):
        if self.act in (0, 1):
            return self.w
        h = np.where(r - self.lb <= 0.0, 1.0, np.where(r - self.ub >= 0.0, 1.0, 0.0))
        return self.w * h if self.act == 3 else h

    def residual(self, robot, x, u, oM=None):
        nq = robot.nq
        if self.type == STATE:
            return robot.state_diff(self.xref, x)  # diff(xref, x), state.hxx:136
        if self.type == CONTROL:
            return u - self.uref  # control.hxx:67
        if self.type == CONTACT_FORCE:  # an inactive contact has lambda = 0 (row0 = -2)
            if self.row0 < 0:
                return -self.fref + 0 * x[0]
            return self.force_fn(x, u)[self.row0:self.row0 + len(self.fref)] - self.fref
        if self.type == FRICTION_CONE:  # r = A lambda_lin (contact-friction-cone.hxx:58)
            if self.row0 < 0:
                return np.zeros(self.nr) + 0 * x[0]
            return self.A @ self.force_fn(x, u)[self.row0:self.row0 + 3]
        if self.type == COM_POSITION:
            return robot.center_of_mass(x[:nq]) - self.cref
        if self.type == FRAME_VELOCITY:  # LOCAL frame velocity - vref (frame-velocity.hxx:57-59)
            vs, _ = local_motions(robot, x[:nq], x[nq:], np.zeros(robot.nv))
            return motion_X(self.Rf, self.pf) @ vs[self.joint] - self.vref
        if oM is None:
            oM = robot.placements(x[:nq])
        R0, p0 = oM[self.joint]
        Rf, pf = R0 @ self.Rf, p0 + R0 @ self.pf  # oMf = oMi[parent] * placement
        if self.type == FRAME_TRANSLATION:
            return pf - self.pref  # frame-translation.hxx:57
        return log6(self.Rri @ Rf, self.pri + self.Rri @ pf)  # log6(Mref^-1 oMf), frame-placement.hxx:48-50


def _cs_jac(f, n_in, n_out):
    """Complex-step Jacobian of f(dz) (dz complex, n_in) at dz = 0."""
    J = np.zeros((n_out, n_in))
    for j in range(n_in):
        dz = np.zeros(n_in, complex)
        dz[j] = 1j * H_CS
        J[:, j] = np.imag(f(dz)) / H_CS
    return J


class FreeFwdKnot:
    """Euler(dt) ∘ DifferentialActionModelFreeFwdDynamics, parsed from a block."""

    def __init__(self, block, nx, nu, _contact=False):
        p = np.asarray(block, float)
        self.dt = float(p[0])
        nv = int(p[1])
        ncost = int(p[2])
        self.size = int(p[3])
        body = p[HDR:]
        self.robot, o = parse_robot(body, nv)
        nq = self.robot.nq
        assert nx == nq + nv, "multibody knots: nx = nq + nv"
        assert _contact or nu == nv, "free-fwddyn knots: nu = nv (full actuation)"
        self.nx, self.nu, self.nj, self.nv, self.nq = nx, nu, nv, nv, nq
        self.ndx = 2 * nv
        self.kind = 4
        self.costs = []
        for _ in range(ncost):
            rs = int(body[o + 3])
            self.costs.append(Cost(body[o:o + rs], nx, self.ndx, nu))
            o += rs
        self._sec = o  # offset (in body) of the contact / impulse section

    # StateMultibody (multibody.hxx:54-91)
    def state_diff(self, x0, x1):
        return self.robot.state_diff(x0, x1)

    def state_integrate(self, x, dx):
        return self.robot.state_integrate(x, dx)

    def state_zero(self):
        return np.concatenate([self.robot.neutral(), np.zeros(self.nv)])

    # DAM calc: a and the differential cost
    def accel(self, x, u):
        nq = self.nq
        return self.robot.aba(x[:nq], x[nq:], u)

    def cost_c(self, x, u):
        oM = self.robot.placements(x[:self.nq])
        c = 0.0
        for k in self.costs:
            r = k.residual(self.robot, x, u, oM)
            c = c + k.weight * k.a_value(r)
        return c

    def calc(self, x, u=None):
        """IntegratedActionModelEuler::calc (euler.hxx:41-80) -> (xnext, cost)."""
        if u is None:
            u = np.zeros(self.nu)
        nq, dt = self.nq, self.dt
        a = self.accel(x, u)
        cc = self.cost_c(x, u)
        if dt != 0:
            v = x[nq:]
            dx = np.concatenate([v * dt + a * dt * dt, a * dt])
            return self.state_integrate(x, dx), dt * cc
        return np.array(x, copy=True), cc

    def _calc_res(self, x, u):
        """(xnext, residuals of every cost) from one evaluation of the dynamics."""
        nq, dt = self.nq, self.dt
        a, lam = self.accel_force(x, u)
        oM = self.robot.placements(x[:nq])
        res = []
        for k in self.costs:
            if k.type == CONTACT_FORCE:
                res.append(lam[k.row0:k.row0 + len(k.fref)] - k.fref if k.row0 >= 0 else 0 * lam[:0].sum() - k.fref)
            elif k.type == FRICTION_CONE:
                res.append(k.A @ lam[k.row0:k.row0 + 3] if k.row0 >= 0 else np.zeros(k.nr) + 0 * lam[:0].sum())
            else:
                res.append(k.residual(self.robot, x, u, oM))
        if dt != 0:
            v = x[nq:]
            xn = self.state_integrate(x, np.concatenate([v * dt + a * dt * dt, a * dt]))
        else:
            xn = x
        return xn, res

    def accel_force(self, x, u):
        return self.accel(x, u), np.zeros(0)

    def calc_diff(self, x, u=None):
        """IntegratedActionModelEuler::calcDiff (euler.hxx:83-131) with the
        DAM's derivatives; Gauss-Newton cost Hessians (cost-sum.hxx:122-160).
        Tangent coordinates: Fx = d diff(xnext, calc(x [+] dx)) / d dx; one complex
        step per direction drives the dynamics and every residual."""
        if u is None:
            u = np.zeros(self.nu)
        n, m, dt = self.ndx, self.nu, self.dt
        x = np.asarray(x, float)
        u = np.asarray(u, float)
        xn0, r0 = self._calc_res(x, u)
        Fz = np.zeros((n, n + m))
        Rz = [np.zeros((np.size(r), n + m)) for r in r0]
        for j in range(n + m):
            dz = np.zeros(n + m, complex)
            dz[j] = 1j * H_CS
            xn, res = self._calc_res(self.state_integrate(x, dz[:n]), u + dz[n:])
            if dt != 0:
                Fz[:, j] = np.imag(self.state_diff(xn0, xn)) / H_CS
            for R, r in zip(Rz, res):
                R[:, j] = np.imag(r) / H_CS
        if dt != 0:
            Fx, Fu = Fz[:, :n], Fz[:, n:]
        else:
            Fx, Fu = np.eye(n), np.zeros((n, m))
        Lz = np.zeros(n + m)
        Lzz = np.zeros((n + m, n + m))
        for k, r, R in zip(self.costs, r0, Rz):
            if getattr(k, "zero_jac", False):
                R = np.zeros_like(R)
            Lz += k.weight * R.T @ k.a_grad(r)
            Lzz += k.weight * R.T @ (k.a_hess(r)[:, None] * R)
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
    for i in range(robot.nb):
        X = motion_X(*robot.liMi(q, i))
        lam = robot.parent[i]
        S = robot.S(i)
        vp = vs[lam] if lam >= 0 else np.zeros(6, dt)
        ap = as_[lam] if lam >= 0 else np.zeros(6, dt)
        vJ = S @ robot.vseg(v, i)
        vi = X @ vp + vJ
        vs.append(vi)
        as_.append(X @ ap + S @ robot.vseg(qdd, i) + crm(vi) @ vJ)
    return vs, as_


def joint_jacobians(robot, q):
    """LOCAL joint Jacobians J_i (6 x nv): joint i's spatial velocity (joint frame)
    per unit generalised velocity, by the forward recursion J_i = X_i J_parent + S_i."""
    dt = np.result_type(q, float)
    out = []
    for i in range(robot.nb):
        X = motion_X(*robot.liMi(q, i))
        lam = robot.parent[i]
        J = X @ out[lam] if lam >= 0 else np.zeros((6, robot.nv), dt)
        J[:, robot.iv[i]:robot.iv[i] + robot.nvj[i]] += robot.S(i)
        out.append(J)
    return out


def frame_jacobian(robot, q, joint, Rf, pf, Js=None):
    """LOCAL frame Jacobian (6 x nv): frame velocity per unit joint velocity."""
    Js = joint_jacobians(robot, q) if Js is None else Js
    return motion_X(Rf, pf) @ Js[joint]


def _section(body, nv, ncost):
    """Offset (in body) of the contact / impulse section."""
    o = 3 + nv
    nb = nv - 5 if int(body[o]) == FREEFLYER else nv
    o += JOINT_REC * nb
    for _ in range(ncost):
        o += int(body[o + 3])
    return o


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
    this calc in tangent coordinates: the reference's analytic KKT-inverse formula
    (contact-fwddyn.hxx:127-140) is the implicit-function derivative of the
    same map, so the two agree to rounding."""

    def __init__(self, block, nx, nu):
        p = np.asarray(block, float)
        nv = int(p[1])
        ncost = int(p[2])
        body = p[HDR:]
        o = _section(body, nv, ncost)
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
        assert nu == nv - self.nun, "contact-fwddyn knots: nu = nv - (unactuated root dofs)"
        super().__init__(block, nx, nu, _contact=True)
        self.kind = 5
        self.nc = sum(c.nc for c in self.contacts)
        for c in self.costs:
            if c.type in (CONTACT_FORCE, FRICTION_CONE):
                c.force_fn = lambda xx, uu: self.accel_force(xx, uu)[1]
                c.zero_jac = not self.enable_force

    def contact_terms(self, x):
        """(Jc (nc x nv), a0 (nc)) at ddq = 0 (ContactModelMultiple::calc)."""
        nq, nv = self.nq, self.nv
        q, v = x[:nq], x[nq:]
        dt = np.result_type(x, float)
        vs, as_ = local_motions(self.robot, q, v, np.zeros(nv, dt))
        oM = self.robot.placements(q)
        JJ = joint_jacobians(self.robot, q)
        Js, a0s = [], []
        for c in self.contacts:
            Xf = motion_X(c.Rf, c.pf)  # joint -> frame (SE3::actInv by jMf)
            vf = Xf @ vs[c.joint]
            af = Xf @ as_[c.joint]
            J = frame_jacobian(self.robot, q, c.joint, c.Rf, c.pf, JJ)
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
            return np.zeros((0, nv), dt), np.zeros(0, dt)
        return np.vstack(Js), np.concatenate(a0s)

    def accel_force(self, x, u):
        nq, nv, nc = self.nq, self.nv, self.nc
        q, v = x[:nq], x[nq:]
        M = self.robot.crba(q) + np.diag(self.robot.armature)
        nle = self.robot.rnea(q, v, np.zeros(nv, np.result_type(x, float)))
        tau = np.concatenate([np.zeros(self.nun, np.result_type(u, float)), u])
        Jc, a0 = self.contact_terms(x)
        K = np.zeros((nv + nc, nv + nc), dtype=np.result_type(M, Jc))
        K[:nv, :nv] = M
        K[:nv, nv:] = Jc.T
        K[nv:, :nv] = Jc
        K[nv:, nv:] = -self.damping * np.eye(nc)
        sol = np.linalg.solve(K, np.concatenate([tau - nle, -a0]))
        return sol[:nv], -sol[nv:]

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
    sub-function in tangent coordinates. For r = 0 this is the exact derivative of
    calc (tested); for r > 0 the reference drops the restitution terms, and so does this."""

    def __init__(self, block, nx, nu):
        p = np.asarray(block, float)
        nv = int(p[1])
        ncost = int(p[2])
        body = p[HDR:]
        o = _section(body, nv, ncost)
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
        self.nun = nv
        self.nc = sum(c.nc for c in self.contacts)

    def jac(self, q):
        Js = []
        JJ = joint_jacobians(self.robot, q)
        for c in self.contacts:
            J = frame_jacobian(self.robot, q, c.joint, c.Rf, c.pf, JJ)
            Js.append(J[:3] if c.type == CONTACT_3D else J)
        return np.vstack(Js) if Js else np.zeros((0, self.nv), np.result_type(q, float))

    def kkt(self, q):
        nv, nc = self.nv, self.nc
        M = self.robot.crba(q) + np.diag(self.robot.armature)
        J = self.jac(q)
        K = np.zeros((nv + nc, nv + nc), dtype=np.result_type(M, J))
        K[:nv, :nv] = M
        K[:nv, nv:] = J.T
        K[nv:, :nv] = J
        K[nv:, nv:] = -self.damping * np.eye(nc)
        return M, J, K

    def impulse(self, x):
        nq, nv = self.nq, self.nv
        q, v = x[:nq], x[nq:]
        M, J, K = self.kkt(q)
        sol = np.linalg.solve(K, np.concatenate([M @ v, -self.r_coeff * (J @ v)]))
        return sol[:nv], -sol[nv:]

    def calc(self, x, u=None):
        nq = self.nq
        vp, _ = self.impulse(x)
        xn = np.concatenate([x[:nq] + 0 * vp[0], vp])
        return xn, self.cost_c(x, np.zeros(0))

    def calc_diff(self, x, u=None):
        n, nq, nv = self.ndx, self.nq, self.nv
        x = np.asarray(x, float)
        q, v = x[:nq], x[nq:]
        vp, lam = self.impulse(x)
        M, J, _ = self.kkt(q)
        Minv = np.linalg.inv(M)
        Y = Minv @ J.T
        S = J @ Y + self.damping * np.eye(self.nc)
        H = Y @ np.linalg.inv(S)
        G = Minv - H @ Y.T
        dv = vp - v
        rob = self.robot

        def tau(dq):  # RNEA(q, 0, dv) - Jc^T lambda, no gravity, lambda fixed in the frames
            qq = rob.integrate_q(q, dq)
            return rob.rnea(qq, np.zeros(nv), dv, gravity=np.zeros(3)) - self.jac(qq).T @ lam

        dtau = _cs_jac(tau, nv, nv)
        dv0 = _cs_jac(lambda dq: self.jac(rob.integrate_q(q, dq)) @ vp, nv, self.nc)
        Fx = np.zeros((n, n))
        Fx[:nv, :nv] = np.eye(nv)
        Fx[nv:, :nv] = -G @ dtau - H @ dv0
        Fx[nv:, nv:] = G @ M
        Lx = np.zeros(n)
        Lxx = np.zeros((n, n))
        u0 = np.zeros(0)
        for k in self.costs:
            r = k.residual(rob, x, u0)
            Rx = _cs_jac(lambda dz: k.residual(rob, self.state_integrate(x, dz), u0), n, r.size)
            Lx += k.weight * Rx.T @ k.a_grad(r)
            Lxx += k.weight * Rx.T @ (k.a_hess(r)[:, None] * Rx)
        return dict(Fx=Fx, Fu=np.zeros((n, 0)), Lx=Lx, Lu=np.zeros(0), Lxx=Lxx, Lxu=np.zeros((n, 0)),
                    Luu=np.zeros((0, 0)))


def block_size(block):
    return int(block[3])
