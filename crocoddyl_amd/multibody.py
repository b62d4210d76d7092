"""Multibody knot models with the reference's Python API, as parameter carriers.

The device computes these knots (crocoddyl_amd/csrc/multibody.hpp); the
classes here hold the parameters, validate them like the reference, and pack
the multibody parameter blocks declared in include/fddp_hip.h.

Reference API mirrored:
  StateMultibody(model)                         multibody/states/multibody.hxx
  ActuationModelFull(state)                     multibody/actuations/full.hpp
  ActuationModelFloatingBase(state)             multibody/actuations/floating-base.hpp
  ActivationModelQuad(nr), ActivationModelWeightedQuad(weights)
                                                core/activations/{quadratic,weighted-quadratic}.hpp
  CostModelSum(state, nu).addCost(name, cost, weight)   multibody/costs/cost-sum.hxx:18-85
  CostModelState / CostModelControl / CostModelFramePlacement / CostModelFrameTranslation
  / CostModelCoMPosition / CostModelContactForce / CostModelContactFrictionCone
                                                multibody/costs/*.hxx
  FramePlacement(id, SE3), FrameTranslation(id, p)      multibody/frames.hpp
  DifferentialActionModelFreeFwdDynamics(state, actuation, costs)  .armature
                                                multibody/actions/free-fwddyn.hxx:24-160
Pinocchio is not available offline, so ``RobotModel`` stands in for
``pinocchio.Model`` over the subset the device covers: a kinematic tree of
revolute joints (any unit axis) below either the universe or a free-flyer root
(JointModelFreeFlyer: q = (p, quat xyzw), v = base twist), with joint
placements, body inertias, operational frames and gravity. Joint and frame
indices follow Pinocchio's (joint 0 / frame 0 = universe).
"""
import numpy as np

from . import _abi

JOINT_REC = 27
JOINT_REVOLUTE, JOINT_FREEFLYER = 0, 1
COST_HDR = 4
COST_STATE, COST_CONTROL, COST_FRAME_PLACEMENT, COST_FRAME_TRANSLATION = 1, 2, 3, 4
CONTACT_3D, CONTACT_6D = 5, 6
COST_CONTACT_FORCE = 7
COST_COM_POSITION = 8
COST_FRICTION_CONE = 9
MAX_CONTACT_ROWS = 24
MAX_DOFS = 64  # nv of the device path (one lane per tangent direction of a wave pair)


class SE3:
    """pinocchio.SE3 subset: rotation (3x3), translation (3)."""

    def __init__(self, rotation=None, translation=None):
        self.rotation = np.eye(3) if rotation is None else np.array(rotation, dtype=np.float64).reshape(3, 3)
        self.translation = np.zeros(3) if translation is None else np.array(translation, np.float64).reshape(3)

    @staticmethod
    def Identity():
        return SE3()

    def inverse(self):
        Rt = self.rotation.T
        return SE3(Rt, -Rt @ self.translation)

    def __mul__(self, o):
        return SE3(self.rotation @ o.rotation, self.translation + self.rotation @ o.translation)

    def __repr__(self):
        return f"SE3(R={self.rotation.tolist()}, p={self.translation.tolist()})"


class Inertia:
    """pinocchio.Inertia: mass, lever (CoM in the joint frame), rotational
    inertia about the CoM (3x3 symmetric)."""

    def __init__(self, mass, lever, inertia):
        self.mass = float(mass)
        self.lever = np.array(lever, np.float64).reshape(3)
        I = np.array(inertia, np.float64).reshape(3, 3)
        if not np.allclose(I, I.T):
            raise ValueError("Invalid argument: the rotational inertia must be symmetric")
        self.inertia = I

    @staticmethod
    def Zero():
        return Inertia(0.0, np.zeros(3), np.zeros((3, 3)))

    def se3Action(self, M):
        """Inertia expressed in the frame M maps to (pinocchio Inertia::se3Action)."""
        return Inertia(self.mass, M.rotation @ self.lever + M.translation,
                       M.rotation @ self.inertia @ M.rotation.T)

    def __add__(self, o):
        """Sum of two inertias in the same frame (pinocchio Inertia::operator+)."""
        m = self.mass + o.mass
        if m == 0:
            return Inertia.Zero()
        c = (self.mass * self.lever + o.mass * o.lever) / m
        def shift(I, mi, ci):
            d = ci - c
            return I + mi * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
        return Inertia(m, c, shift(self.inertia, self.mass, self.lever) + shift(o.inertia, o.mass, o.lever))


class JointModelFreeFlyer:
    """pinocchio::JointModelFreeFlyer: 6 dofs, q = (p, quaternion x y z w)."""
    nq, nv = 7, 6


class JointModelRevoluteUnaligned:
    """pinocchio::JointModelRevoluteUnaligned(axis)."""
    nq, nv = 1, 1

    def __init__(self, *axis):
        ax = np.array(axis[0] if len(axis) == 1 else axis, np.float64).reshape(3)
        n = np.linalg.norm(ax)
        if n == 0:
            raise ValueError("Invalid argument: zero joint axis")
        self.axis = ax / n


def JointModelRX():
    return JointModelRevoluteUnaligned((1.0, 0.0, 0.0))


def JointModelRY():
    return JointModelRevoluteUnaligned((0.0, 1.0, 0.0))


def JointModelRZ():
    return JointModelRevoluteUnaligned((0.0, 0.0, 1.0))


class RobotModel:
    """Stand-in for pinocchio.Model: revolute trees, optionally below a
    free-flyer root (the only joint allowed to be a JointModelFreeFlyer)."""

    def __init__(self, root_joint=None):
        self.names = ["universe"]
        self.parents = [0]
        self.kinds = [JOINT_REVOLUTE]
        self.axes = [np.zeros(3)]
        self.jointPlacements = [SE3()]
        self.inertias = [Inertia.Zero()]
        self.frames = [("universe", 0, SE3())]
        self.gravity = np.array([0.0, 0.0, -9.81])  # pinocchio Model::gravity981
        self.referenceConfigurations = {}
        self._version = 0
        if root_joint is not None:  # pinocchio::buildModel(urdf, JointModelFreeFlyer(), model)
            self.addJoint(0, root_joint, SE3(), "root_joint")

    @property
    def njoints(self):
        return len(self.names)

    @property
    def nq(self):
        return sum(7 if k == JOINT_FREEFLYER else 1 for k in self.kinds[1:])

    @property
    def nv(self):
        return sum(6 if k == JOINT_FREEFLYER else 1 for k in self.kinds[1:])

    @property
    def has_freeflyer(self):
        return self.njoints > 1 and self.kinds[1] == JOINT_FREEFLYER

    def idx_q(self, j):
        """Model::idx_qs[j]: first configuration index of joint j."""
        return sum(7 if k == JOINT_FREEFLYER else 1 for k in self.kinds[1:j])

    def idx_v(self, j):
        """Model::idx_vs[j]: first velocity index of joint j."""
        return sum(6 if k == JOINT_FREEFLYER else 1 for k in self.kinds[1:j])

    def addJoint(self, parent_id, joint, placement, name):
        """pinocchio Model::addJoint(parent, joint_model, placement, name):
        ``joint`` is a JointModelFreeFlyer / JointModelRevoluteUnaligned (or a
        bare axis, a revolute joint about it), placed at ``placement`` in the
        parent joint's frame. Returns its index."""
        parent_id = int(parent_id)
        if not 0 <= parent_id < self.njoints:
            raise ValueError("Invalid argument: unknown parent joint")
        if isinstance(joint, JointModelFreeFlyer) or joint is JointModelFreeFlyer:
            if self.njoints != 1 or parent_id != 0:
                raise ValueError("Invalid argument: the device path takes a free-flyer as the root joint only")
            kind, ax, nvj = JOINT_FREEFLYER, np.zeros(3), 6
        else:
            if not isinstance(joint, JointModelRevoluteUnaligned):
                joint = JointModelRevoluteUnaligned(joint)
            kind, ax, nvj = JOINT_REVOLUTE, joint.axis, 1
        if self.nv + nvj > MAX_DOFS:
            raise ValueError(f"Invalid argument: the device path holds at most {MAX_DOFS} dofs")
        self.names.append(str(name))
        self.parents.append(parent_id)
        self.kinds.append(kind)
        self.axes.append(ax)
        self.jointPlacements.append(placement if placement is not None else SE3())
        self.inertias.append(Inertia.Zero())
        self._version += 1
        return self.njoints - 1

    def getJointId(self, name):
        if name in self.names:
            return self.names.index(name)
        return self.njoints

    def appendBodyToJoint(self, joint_id, inertia, placement=None):
        """pinocchio Model::appendBodyToJoint: add a body (inertia given in
        the body frame ``placement`` relative to the joint)."""
        M = placement if placement is not None else SE3()
        self.inertias[joint_id] = self.inertias[joint_id] + inertia.se3Action(M)
        self._version += 1

    def addFrame(self, name, parent_joint, placement=None):
        self.frames.append((str(name), int(parent_joint), placement if placement is not None else SE3()))
        self._version += 1
        return len(self.frames) - 1

    def getFrameId(self, name):
        for i, f in enumerate(self.frames):
            if f[0] == name:
                return i
        raise ValueError(f"Invalid argument: unknown frame {name}")

    def existFrame(self, name):
        return any(f[0] == name for f in self.frames)

    def neutral(self):
        """pinocchio::neutral: identity quaternion for the free-flyer, zeros else."""
        q = np.zeros(self.nq)
        if self.has_freeflyer:
            q[6] = 1.0
        return q

    def placements(self, q):
        """oMi of every joint (pinocchio::forwardKinematics, host side)."""
        q = np.asarray(q, float)
        out = [SE3()]
        for j in range(1, self.njoints):
            iq = self.idx_q(j)
            if self.kinds[j] == JOINT_FREEFLYER:
                Mj = SE3(_quat_to_R(q[iq + 3:iq + 7]), q[iq:iq + 3])
            else:
                Mj = SE3(_rot_axis(self.axes[j], q[iq]))
            out.append(out[self.parents[j]] * (self.jointPlacements[j] * Mj))
        return out

    def framePlacement(self, q, frame_id):
        name, pj, pl = self.frames[frame_id]
        return self.placements(q)[pj] * pl

    def centerOfMass(self, q):
        oM = self.placements(q)
        mt = sum(I.mass for I in self.inertias)
        c = sum(I.mass * (oM[j].translation + oM[j].rotation @ I.lever) for j, I in enumerate(self.inertias))
        return c / mt

    def pack_robot(self, armature):
        """gravity(3) armature(nv) then one 27-double record per joint:
        [type, parent record (-1 universe), axis(3), placement R(9) p(3), mass, CoM(3), I(6)]."""
        nv = self.nv
        rows = [self.gravity, np.asarray(armature, float).reshape(nv)]
        for j in range(1, self.njoints):
            P = self.jointPlacements[j]
            I = self.inertias[j]
            Ic = I.inertia
            rows.append(np.concatenate([[self.kinds[j], self.parents[j] - 1], self.axes[j],
                                        P.rotation.T.reshape(-1), P.translation, [I.mass], I.lever,
                                        [Ic[0, 0], Ic[1, 1], Ic[2, 2], Ic[0, 1], Ic[0, 2], Ic[1, 2]]]))
        return np.concatenate(rows)


def _skew(w):
    return np.array([[0.0, -w[2], w[1]], [w[2], 0.0, -w[0]], [-w[1], w[0], 0.0]])


def _rot_axis(ax, q):
    K = _skew(ax)
    return np.eye(3) + np.sin(q) * K + (1 - np.cos(q)) * (K @ K)


def _quat_to_R(qv):
    x, y, z, w = qv
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def _R_to_quat(R):
    t = np.trace(R)
    if t > 0:
        s = np.sqrt(t + 1.0)
        w = 0.5 * s
        s = 0.5 / s
        return np.array([(R[2, 1] - R[1, 2]) * s, (R[0, 2] - R[2, 0]) * s, (R[1, 0] - R[0, 1]) * s, w])
    i = int(np.argmax([R[0, 0], R[1, 1], R[2, 2]]))
    j, k = (i + 1) % 3, (i + 2) % 3
    s = np.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0)
    q = np.zeros(4)
    q[i] = 0.5 * s
    s = 0.5 / s
    q[3] = (R[k, j] - R[j, k]) * s
    q[j] = (R[j, i] + R[i, j]) * s
    q[k] = (R[k, i] + R[i, k]) * s
    return q


def _exp6(nu):
    v, w = np.asarray(nu[:3], float), np.asarray(nu[3:], float)
    t2 = w @ w
    if t2 < 1e-8:
        ct, st_t = 1 - t2 / 2 + t2 * t2 / 24, 1 - t2 / 6 + t2 * t2 / 120
        a_wxv, a_w = 0.5 - t2 / 24 + t2 * t2 / 720, 1.0 / 6 - t2 / 120 + t2 * t2 / 5040
    else:
        t = np.sqrt(t2)
        ct, st_t = np.cos(t), np.sin(t) / t
        a_wxv, a_w = (1 - ct) / t2, (1 - st_t) / t2
    R = ct * np.eye(3) + a_wxv * np.outer(w, w) + st_t * _skew(w)
    return R, st_t * v + a_w * (w @ v) * w + a_wxv * np.cross(w, v)


def _log6(R, p):
    c = 0.5 * (np.trace(R) - 1)
    wv = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    s = 0.5 * np.linalg.norm(wv)
    th = np.arctan2(s, c)
    if s < 1e-8 and c > 0:
        w = 0.5 * (1 + s * s / 6) * wv
    elif s < 1e-8:
        th = np.arccos(max(-1.0, min(1.0, c)))
        ax = np.sqrt(np.maximum((np.diag(R) - c) / (1 - c), 0))
        i0 = int(np.argmax(ax))
        sg = np.array([1.0 if j == i0 else (1.0 if R[i0, j] + R[j, i0] >= 0 else -1.0) for j in range(3)])
        w = (th if wv[i0] >= 0 else -th) * sg * ax
    else:
        w = th / (2 * s) * wv
    t2 = w @ w
    if t2 < 1e-2:
        beta = 1.0 / 12 + t2 / 720 + t2 * t2 / 30240
    else:
        t = np.sqrt(t2)
        beta = 1 / t2 - np.sin(t) / (2 * t * (1 - np.cos(t)))
    W = _skew(w)
    return np.concatenate([(np.eye(3) - 0.5 * W + beta * W @ W) @ p, w])


def sample_talos_arm():
    """A 7-DoF arm with the kinematic layout and mass distribution of a
    humanoid (Talos-class) left arm: shoulder yaw/roll/pitch, elbow, forearm
    twist, wrist pitch/roll, and a ``gripper_left_joint`` frame 0.1 m past
    the wrist. Synthetic stand-in: example-robot-data's URDF is absent
    offline (benchmark/factory/arm.hpp:47-56 loads talos_left_arm.urdf)."""
    m = RobotModel()
    specs = [  # (axis, placement translation, mass, lever, diag inertia)
        ((0, 0, 1), (0.0, 0.157, 0.232), 2.71, (-0.002, 0.04, 0.0), (0.012, 0.004, 0.011)),
        ((1, 0, 0), (0.0, 0.0, 0.0), 1.51, (0.01, 0.0, -0.06), (0.008, 0.008, 0.002)),
        ((0, 0, 1), (0.0, 0.0, -0.0), 1.43, (0.0, 0.0, -0.15), (0.012, 0.012, 0.002)),
        ((0, 1, 0), (0.02, 0.0, -0.273), 1.02, (-0.01, 0.0, -0.05), (0.004, 0.004, 0.001)),
        ((0, 0, 1), (-0.02, 0.0, -0.1), 1.12, (0.0, 0.0, -0.08), (0.006, 0.006, 0.001)),
        ((1, 0, 0), (0.0, 0.0, -0.164), 0.52, (0.0, 0.0, -0.01), (0.0005, 0.0005, 0.0003)),
        ((0, 1, 0), (0.0, 0.0, 0.0), 0.40, (0.0, 0.0, -0.05), (0.0004, 0.0004, 0.0002)),
    ]
    parent = 0
    for k, (ax, p, mass, c, d) in enumerate(specs):
        j = m.addJoint(parent, ax, SE3(np.eye(3), p), f"arm_left_{k + 1}_joint")
        m.appendBodyToJoint(j, Inertia(mass, c, np.diag(d)))
        parent = j
    m.addFrame("gripper_left_joint", parent, SE3(np.eye(3), (0.0, 0.0, -0.1)))
    return m


def sample_tree(nj, seed=0, branching=True, freeflyer=False):
    """Random kinematic tree (tests): random axes, placements and inertias; with
    ``freeflyer`` the nj revolute joints hang below a free-flyer base (joint 1)."""
    rng = np.random.default_rng(seed)
    m = RobotModel(JointModelFreeFlyer() if freeflyer else None)
    if freeflyer:
        A = rng.normal(size=(3, 3)) * 0.1
        m.appendBodyToJoint(1, Inertia(rng.uniform(2.0, 6.0), rng.uniform(-0.05, 0.05, 3), A @ A.T + 0.05 * np.eye(3)))
    first = m.njoints
    for j in range(first, first + nj):
        lo = 1 if freeflyer else 0
        parent = int(rng.integers(lo, j)) if branching else j - 1
        ax = rng.normal(size=3)
        ang = rng.normal(size=3) * 0.5
        t = np.linalg.norm(ang)
        K = np.array([[0, -ang[2], ang[1]], [ang[2], 0, -ang[0]], [-ang[1], ang[0], 0]])
        R = np.eye(3) + np.sin(t) / t * K + (1 - np.cos(t)) / t ** 2 * K @ K
        jid = m.addJoint(parent, ax, SE3(R, rng.uniform(-0.3, 0.3, 3)), f"j{j}")
        A = rng.normal(size=(3, 3)) * 0.05
        m.appendBodyToJoint(jid, Inertia(rng.uniform(0.3, 3.0), rng.uniform(-0.1, 0.1, 3),
                                         A @ A.T + 0.01 * np.eye(3)))
    m.addFrame("tip", m.njoints - 1, SE3(np.eye(3), (0.0, 0.0, -0.1)))
    return m


class StateMultibody:
    """StateMultibody (multibody.hxx:14-240): x = (q, v), nx = nq + nv,
    ndx = 2 nv; diff / integrate are pinocchio::difference / integrate
    (multibody.hxx:54-91): Euclidean on revolute joints, SE(3) (M0^-1 M1 ->
    log6, M exp6(dq)) on a free-flyer root."""

    def __init__(self, model):
        if not isinstance(model, RobotModel):
            raise TypeError("StateMultibody needs a crocoddyl_amd.multibody.RobotModel")
        self.pinocchio = model
        self.nq = model.nq
        self.nv = model.nv
        self.nx = self.nq + self.nv
        self.ndx = 2 * self.nv

    def zero(self):
        return np.concatenate([self.pinocchio.neutral(), np.zeros(self.nv)])

    def rand(self):
        q = np.random.uniform(-np.pi, np.pi, self.nq)
        if self.pinocchio.has_freeflyer:
            q[:3] = np.random.uniform(-1, 1, 3)
            qq = np.random.normal(size=4)
            q[3:7] = qq / np.linalg.norm(qq)
        return np.concatenate([q, np.random.uniform(-1, 1, self.nv)])

    def diff(self, x0, x1):
        x0, x1 = np.asarray(x0, float), np.asarray(x1, float)
        nq = self.nq
        dq = x1[:nq] - x0[:nq]
        if self.pinocchio.has_freeflyer:
            R0, R1 = _quat_to_R(x0[3:7]), _quat_to_R(x1[3:7])
            dq = np.concatenate([_log6(R0.T @ R1, R0.T @ (x1[:3] - x0[:3])), dq[7:]])
        return np.concatenate([dq, x1[nq:] - x0[nq:]])

    def integrate(self, x, dx):
        x, dx = np.asarray(x, float), np.asarray(dx, float)
        nq, nv = self.nq, self.nv
        if self.pinocchio.has_freeflyer:
            R0 = _quat_to_R(x[3:7])
            Re, pe = _exp6(dx[:6])
            qn = _R_to_quat(R0 @ Re)
            if qn @ x[3:7] < 0:
                qn = -qn
            qn *= (3 - qn @ qn) / 2
            q = np.concatenate([x[:3] + R0 @ pe, qn, x[7:nq] + dx[6:nv]])
        else:
            q = x[:nq] + dx[:nv]
        return np.concatenate([q, x[nq:] + dx[nv:]])


class ActuationModelFull:
    """ActuationModelFull: tau = u, nu = nv."""

    def __init__(self, state):
        if state.pinocchio.has_freeflyer:
            raise ValueError("Invalid argument: the first joint cannot be a free-flyer")
        self.state = state
        self.nu = state.nv


class ActuationModelFloatingBase:
    """ActuationModelFloatingBase (actuations/floating-base.hpp:29-61): the
    root joint's dofs are unactuated, tau = [0; u], nu = nv - nv(joint 1)
    (6 for a free-flyer root, 1 for a revolute one)."""

    def __init__(self, state):
        self.state = state
        model = state.pinocchio
        self.nun = 6 if model.has_freeflyer else 1
        self.nu = state.nv - self.nun


class ActivationModelQuad:
    """a = 0.5 ||r||^2, Ar = r, Arr = I (core/activations/quadratic.hpp)."""

    def __init__(self, nr):
        self.nr = int(nr)
        self.weights = None


class ActivationModelWeightedQuad:
    """a = 0.5 r^T diag(w) r, Ar = w r, Arr = diag(w) (weighted-quadratic.hpp:42-71)."""

    def __init__(self, weights):
        self.weights = np.array(weights, np.float64).reshape(-1)
        self.nr = self.weights.size


class FramePlacement:
    def __init__(self, id, placement):
        self.id = int(id)
        self.placement = placement


class FrameTranslation:
    def __init__(self, id, translation):
        self.id = int(id)
        self.translation = np.array(translation, np.float64)


class _Cost:
    """CostModelAbstract (multibody/cost-base.hxx): state, activation, nu."""

    type = 0

    def __init__(self, state, activation, nr, nu):
        self.state = state
        self.nu = state.nv if nu is None else int(nu)
        self.activation = activation if activation is not None else ActivationModelQuad(nr)
        if self.activation.nr != nr:
            raise ValueError(f"Invalid argument: nr is equals to {nr}")

    def _payload(self):
        raise NotImplementedError

    def pack(self):
        """(Bm, size) record: [type, weight=0 (set by the sum), weighted, size] + payload."""
        parts = self._payload()
        w = self.activation.weights
        parts.append(np.ones((1, self.activation.nr)) if w is None else w.reshape(1, -1))
        Bm = max(p.shape[0] for p in parts)
        size = COST_HDR + sum(p.shape[1] for p in parts)
        hdr = np.array([[self.type, 0.0, 0.0 if w is None else 1.0, size]])
        return np.concatenate([np.broadcast_to(p, (Bm, p.shape[1])) for p in [hdr] + parts], axis=1)


def _rows(a, n):
    a = np.asarray(a, np.float64)
    return a.reshape(1, n) if a.ndim == 1 else a.reshape(a.shape[0], n)


def _cost_args(args, kw):
    """Sort the reference's overloads: (activation?, reference?, nu?)."""
    act = ref = nu = None
    for a in args:
        if isinstance(a, (ActivationModelQuad, ActivationModelWeightedQuad)):
            act = a
        elif isinstance(a, (int, np.integer)) and not isinstance(a, bool):
            nu = int(a)
        else:
            ref = a
    act = kw.get("activation", act)
    nu = kw.get("nu", nu)
    return act, ref, nu


class CostModelState(_Cost):
    """r = diff(xref, x) = x - xref (state.hxx:130-169); xref defaults to state.zero()."""

    type = COST_STATE

    def __init__(self, state, *args, **kw):
        act, ref, nu = _cost_args(args, kw)
        ref = kw.get("xref", ref)
        super().__init__(state, act, state.ndx, nu)
        self.xref = state.zero() if ref is None else np.array(ref, np.float64)
        if self.xref.shape[-1] != state.nx:
            raise ValueError(f"Invalid argument: xref has wrong dimension (it should be {state.nx})")

    def _payload(self):
        return [_rows(self.xref, self.state.nx)]


class CostModelControl(_Cost):
    """r = u - uref (control.hxx:56-87); uref defaults to zeros(nu)."""

    type = COST_CONTROL

    def __init__(self, state, *args, **kw):
        act, ref, nu = _cost_args(args, kw)
        ref = kw.get("uref", ref)
        if ref is not None:
            nu = np.asarray(ref).shape[-1]
        elif act is not None and nu is None:
            nu = act.nr
        nu = state.nv if nu is None else nu
        super().__init__(state, act, nu, nu)
        self.uref = np.zeros(nu) if ref is None else np.array(ref, np.float64)

    def _payload(self):
        return [_rows(self.uref, self.nu)]


class CostModelFramePlacement(_Cost):
    """r = log6(Mref^-1 oMf) (frame-placement.hxx:45-80)."""

    type = COST_FRAME_PLACEMENT

    def __init__(self, state, *args, **kw):
        act, ref, nu = _cost_args(args, kw)
        ref = kw.get("Mref", ref)
        if not isinstance(ref, FramePlacement):
            raise TypeError("CostModelFramePlacement needs a FramePlacement reference")
        super().__init__(state, act, 6, nu)
        self.Mref = ref

    def _payload(self):
        model = self.state.pinocchio
        name, pj, pl = model.frames[self.Mref.id]
        if pj == 0:
            raise ValueError("Invalid argument: frames attached to the universe are not supported")
        Pinv = self.Mref.placement.inverse()
        frame = np.concatenate([[pj - 1], pl.rotation.T.reshape(-1), pl.translation]).reshape(1, -1)
        return [frame, np.concatenate([Pinv.rotation.T.reshape(-1), Pinv.translation]).reshape(1, -1)]


class CostModelFrameTranslation(_Cost):
    """r = oMf.translation - pref (frame-translation.hxx:50-81). ``xref.translation``
    may carry a leading batch axis (B, 3): one target per batch element."""

    type = COST_FRAME_TRANSLATION

    def __init__(self, state, *args, **kw):
        act, ref, nu = _cost_args(args, kw)
        ref = kw.get("xref", ref)
        if not isinstance(ref, FrameTranslation):
            raise TypeError("CostModelFrameTranslation needs a FrameTranslation reference")
        super().__init__(state, act, 3, nu)
        self.xref = ref

    def _payload(self):
        model = self.state.pinocchio
        name, pj, pl = model.frames[self.xref.id]
        if pj == 0:
            raise ValueError("Invalid argument: frames attached to the universe are not supported")
        frame = np.concatenate([[pj - 1], pl.rotation.T.reshape(-1), pl.translation]).reshape(1, -1)
        return [frame, _rows(self.xref.translation, 3)]


class CostModelCoMPosition(_Cost):
    """r = com(q) - cref (com-position.hxx:49-75): Rx = [Jcom, 0]."""

    type = COST_COM_POSITION

    def __init__(self, state, *args, **kw):
        act, ref, nu = _cost_args(args, kw)
        ref = kw.get("cref", ref)
        if ref is None:
            raise TypeError("CostModelCoMPosition needs a reference position cref")
        super().__init__(state, act, 3, nu)
        self.cref = np.array(ref, np.float64)
        if self.cref.shape[-1] != 3:
            raise ValueError("Invalid argument: cref has wrong dimension (it should be 3)")

    def _payload(self):
        return [_rows(self.cref, 3)]


class FrameForce:
    """FrameForce (multibody/frames.hpp): frame id and a spatial force (linear, angular)."""

    def __init__(self, id, force):
        self.id = int(id)
        self.force = np.array(force, np.float64).reshape(6)


class CostModelContactForce(_Cost):
    """r = jMf.actInv(f) - fref = lambda_contact - fref (contact-force.hxx:33-74): the
    force of the contact defined on frame fref.id (3 linear rows for a 3D contact, 6
    for a 6D one). Its derivatives are the force Jacobians of the contact dynamics,
    which the DAM computes only with enable_force=True (otherwise Rx = Ru = 0, as in
    the reference)."""

    type = COST_CONTACT_FORCE

    def __init__(self, state, *args, **kw):
        act = None
        fref = None
        ints = []
        for a in args:
            if isinstance(a, (ActivationModelQuad, ActivationModelWeightedQuad)):
                act = a
            elif isinstance(a, FrameForce):
                fref = a
            elif isinstance(a, (int, np.integer)) and not isinstance(a, bool):
                ints.append(int(a))
        act = kw.get("activation", act)
        fref = kw.get("fref", fref)
        if not isinstance(fref, FrameForce):
            raise TypeError("CostModelContactForce needs a FrameForce reference")
        if act is not None:  # (state, activation, fref[, nu])
            nr, nu = act.nr, (ints[0] if ints else None)
        else:  # (state, fref[, nc[, nu]]): ActivationModelQuad(6) by default (contact-force.hxx:57-59)
            nr = ints[0] if ints else 6
            nu = ints[1] if len(ints) > 1 else None
        nu = kw.get("nu", nu)
        if nr not in (3, 6):
            raise ValueError("Invalid argument: nr has to be 3 or 6 (the contact's force)")
        super().__init__(state, act, nr, nu)
        self.fref = fref

    @property
    def frame_id(self):
        return self.fref.id

    def _payload(self):  # the contact row offset is resolved by the DAM (pack_body)
        return [np.concatenate([[-1.0, self.activation.nr], self.fref.force]).reshape(1, -1)]


class CostItem:
    def __init__(self, name, cost, weight, active=True):
        self.name, self.cost, self.weight, self.active = name, cost, float(weight), bool(active)


class CostModelSum:
    """CostModelSum (cost-sum.hxx:18-85): named costs in a std::map, so they
    are evaluated and summed in name order."""

    def __init__(self, state, nu=None):
        self.state = state
        self.nu = state.nv if nu is None else int(nu)
        self.costs = {}
        self._version = 0

    def addCost(self, name, cost, weight, active=True):
        if cost.nu != self.nu:
            raise ValueError(f"Invalid argument: {name} cost item doesn't have the same control dimension "
                             f"(it should be {self.nu})")
        if name in self.costs:
            raise ValueError(f"Invalid argument: {name} cost item already existed")
        self.costs[name] = CostItem(name, cost, weight, active)
        self._version += 1

    def removeCost(self, name):
        if name not in self.costs:
            raise ValueError(f"Invalid argument: {name} cost item doesn't exist")
        del self.costs[name]
        self._version += 1

    def changeCostStatus(self, name, active):
        if name not in self.costs:
            raise ValueError(f"Invalid argument: {name} cost item doesn't exist")
        self.costs[name].active = bool(active)
        self._version += 1

    @property
    def nr(self):
        return sum(c.cost.activation.nr for c in self.costs.values() if c.active)

    def pack(self):
        recs = []
        for name in sorted(self.costs):  # std::map<std::string, ...> order
            it = self.costs[name]
            if not it.active:
                continue
            r = np.array(it.cost.pack())
            r[:, 1] = it.weight
            recs.append(r)
        return recs


class DifferentialActionModelFreeFwdDynamics:
    """free-fwddyn.hxx:24-160: a = ABA(q, v, tau(u)) (or (M + diag(armature))^-1
    (tau - nle) once an armature is set), cost = costs.calc(x, u)."""

    def __init__(self, state, actuation, costs):
        if not isinstance(actuation, (ActuationModelFull, ActuationModelFloatingBase)):
            raise NotImplementedError("crocoddyl_amd: the device path covers ActuationModelFull and "
                                      "ActuationModelFloatingBase only")
        self._init_dam(state, actuation, costs)

    @property
    def knot_kind(self):
        """Device knot kind of Euler(this DAM): free dynamics with a floating-base
        actuation is the contact knot with an empty ContactModelMultiple."""
        return _abi.KNOT_EULER_FREEFWD if isinstance(self.actuation, ActuationModelFull) else \
            _abi.KNOT_EULER_CONTACTFWD

    def _init_dam(self, state, actuation, costs):
        if costs.nu != actuation.nu:
            raise ValueError(f"Invalid argument: Costs doesn't have the same control dimension "
                             f"(it should be {actuation.nu})")
        self.state = state
        self.actuation = actuation
        self.costs = costs
        self.nu = actuation.nu
        self.nr = costs.nr
        self._armature = np.zeros(state.nv)
        self._arm_version = 0
        self._u_lb = np.full(self.nu, -np.inf)
        self._u_ub = np.full(self.nu, np.inf)

    u_lb = property(lambda s: s._u_lb)
    u_ub = property(lambda s: s._u_ub)

    @property
    def armature(self):
        return self._armature.copy()

    @armature.setter
    def armature(self, a):
        a = np.array(a, np.float64).reshape(-1)
        if a.size != self.state.nv:
            raise ValueError(f"Invalid argument: The armature dimension is wrong (it should be {self.state.nv})")
        self._armature = a
        self._arm_version += 1

    def version(self):
        return (self.state.pinocchio._version, self.costs._version, self._arm_version,
                tuple(getattr(c.cost, "_version", 0) for c in self.costs.costs.values()))

    def pack_body(self, dt):
        """(Bm, size) rows of the FDDP_KNOT_EULER_FREEFWD block for step dt (with a
        floating-base actuation: the FDDP_KNOT_EULER_CONTACTFWD block, no contacts)."""
        if isinstance(self.actuation, ActuationModelFloatingBase):
            return _pack_mb(self.state, self._armature, self.costs, dt, [self.actuation.nun, 0.0, 0.0, 0.0])
        return _pack_mb(self.state, self._armature, self.costs, dt)


def _pack_mb(state, armature, costs, dt, section=None):
    """(Bm, size) rows of a multibody block: header [dt, nv, ncost, size], robot,
    cost records, then the optional contact / impulse section."""
    model = state.pinocchio
    robot = model.pack_robot(armature).reshape(1, -1)
    recs = costs.pack()
    parts = [robot] + recs + ([np.asarray(section, float).reshape(1, -1)] if section is not None else [])
    Bm = max(p.shape[0] for p in parts)
    size = _abi.PARAM_HEADER + sum(p.shape[1] for p in parts)
    hdr = np.array([[dt, model.nv, len(recs), size]])
    return np.ascontiguousarray(
        np.concatenate([np.broadcast_to(p, (Bm, p.shape[1])) for p in [hdr] + parts], axis=1))


class _Contact:
    """ContactModelAbstract (contact-base.hxx): state, nc, nu, gains (Baumgarte
    position / velocity gains, default zero)."""

    type = 0
    nc = 0

    def __init__(self, state, ref, args, kw):
        nu = None
        gains = None
        for a in args:
            if isinstance(a, (int, np.integer)) and not isinstance(a, bool) and nu is None and gains is None:
                nu = int(a)
            else:
                gains = a
        nu = kw.get("nu", nu)
        gains = kw.get("gains", gains)
        self.state = state
        self.nu = state.nv if nu is None else int(nu)
        g = np.zeros(2) if gains is None else np.array(gains, np.float64).reshape(-1)
        if g.size != 2:
            raise ValueError("Invalid argument: gains has wrong dimension (it should be 2)")
        self.gains = g
        self._ref = ref

    def _frame(self, fid):
        model = self.state.pinocchio
        name, pj, pl = model.frames[fid]
        if pj == 0:
            raise ValueError("Invalid argument: frames attached to the universe are not supported")
        return np.concatenate([[pj - 1], pl.rotation.T.reshape(-1), pl.translation])

    def pack(self):
        body = np.concatenate([self._frame(self._ref.id), self._ref_payload()])
        return np.concatenate([[self.type, self.gains[0], self.gains[1], COST_HDR + body.size], body])


class ContactModel3D(_Contact):
    """ContactModel3D(state, xref, nu=nv, gains=[0, 0]) (contact-3d.hxx:12-43):
    point contact on frame xref.id; a0 = classical acceleration of the frame
    origin (LOCAL) + gains[0] (oMf.translation - xref.translation) + gains[1] v."""

    type = CONTACT_3D
    nc = 3

    def __init__(self, state, xref, *args, **kw):
        if not isinstance(xref, FrameTranslation):
            raise TypeError("ContactModel3D needs a FrameTranslation reference")
        super().__init__(state, xref, args, kw)
        self.xref = xref

    def _ref_payload(self):
        t = np.asarray(self.xref.translation, np.float64).reshape(-1)
        if t.size != 3:
            raise ValueError("Invalid argument: contact references cannot vary over the batch")
        return t


class ContactModel6D(_Contact):
    """ContactModel6D(state, Mref, nu=nv, gains=[0, 0]) (contact-6d.hxx:12-45):
    rigid contact on frame Mref.id; a0 = frame spatial acceleration (LOCAL)
    + gains[0] log6(Mref^-1 oMf) + gains[1] v."""

    type = CONTACT_6D
    nc = 6

    def __init__(self, state, Mref, *args, **kw):
        if not isinstance(Mref, FramePlacement):
            raise TypeError("ContactModel6D needs a FramePlacement reference")
        super().__init__(state, Mref, args, kw)
        self.Mref = Mref

    def _ref_payload(self):
        Pinv = self.Mref.placement.inverse()
        return np.concatenate([Pinv.rotation.T.reshape(-1), Pinv.translation])


class ContactItem:
    def __init__(self, name, contact, active=True):
        self.name, self.contact, self.active = name, contact, bool(active)


class ContactModelMultiple:
    """ContactModelMultiple (multiple-contacts.hxx:14-88): named contacts in a
    std::map; the active ones stack their rows (Jc, a0, lambda) in name order."""

    def __init__(self, state, nu=None):
        self.state = state
        self.nu = state.nv if nu is None else int(nu)
        self.contacts = {}
        self._version = 0

    def addContact(self, name, contact, active=True):
        if contact.nu != self.nu:
            raise ValueError(f"Invalid argument: {name} contact item doesn't have the same control dimension "
                             f"({self.nu})")
        if name in self.contacts:  # the reference prints a warning and keeps the old item
            return
        self.contacts[name] = ContactItem(name, contact, active)
        self._version += 1

    def removeContact(self, name):
        if name in self.contacts:
            del self.contacts[name]
            self._version += 1

    def changeContactStatus(self, name, active):
        if name in self.contacts:
            self.contacts[name].active = bool(active)
            self._version += 1

    @property
    def nc(self):
        return sum(c.contact.nc for c in self.contacts.values() if c.active)

    @property
    def nc_total(self):
        return sum(c.contact.nc for c in self.contacts.values())

    @property
    def active(self):
        return sorted(n for n, c in self.contacts.items() if c.active)

    @property
    def inactive(self):
        return sorted(n for n, c in self.contacts.items() if not c.active)

    def pack(self):
        return [self.contacts[n].contact.pack() for n in self.active]


class DifferentialActionModelContactFwdDynamics(DifferentialActionModelFreeFwdDynamics):
    """contact-fwddyn.hxx:24-160: the KKT dynamics
        [M  Jc^T ; Jc  0] [a ; -lambda] = [tau(u) - nle ; -a0]
    (Schur complement with JMinvJt + inv_damping I), costs.calc(x, u).
    ``enable_force`` only selects the force Jacobians, which no device-covered
    cost reads."""

    def __init__(self, state, actuation, contacts, costs, inv_damping=0.0, enable_force=False):
        if not isinstance(actuation, ActuationModelFloatingBase):
            raise TypeError("DifferentialActionModelContactFwdDynamics needs an ActuationModelFloatingBase")
        if not isinstance(contacts, ContactModelMultiple):
            raise TypeError("DifferentialActionModelContactFwdDynamics needs a ContactModelMultiple")
        if contacts.nu != actuation.nu:
            raise ValueError(f"Invalid argument: Contacts doesn't have the same control dimension "
                             f"(it should be {actuation.nu})")
        self._init_dam(state, actuation, costs)
        self.contacts = contacts
        self.JMinvJt_damping = abs(float(inv_damping))
        self.enable_force = bool(enable_force)

    def version(self):
        return super().version() + (self.contacts._version, self.JMinvJt_damping,
                                    tuple(c.contact.gains.tobytes() for c in self.contacts.contacts.values()))

    knot_kind = _abi.KNOT_EULER_CONTACTFWD

    def pack_body(self, dt):
        """(Bm, size) rows of the FDDP_KNOT_EULER_CONTACTFWD block: the
        FDDP_KNOT_EULER_FREEFWD layout, then [nun, damping, ncontact, flag] and the
        active contact records in name order."""
        recs = self.contacts.pack()
        if self.contacts.nc > MAX_CONTACT_ROWS:
            raise ValueError(f"Invalid argument: the device path holds at most {MAX_CONTACT_ROWS} contact rows")
        sec = np.concatenate([[self.actuation.nun, self.JMinvJt_damping, len(recs), 2.0 if self.enable_force else 0.0]]
                             + recs)
        out = _pack_mb(self.state, self._armature, self.costs, dt, sec)
        # costs on a contact's force: the row offset of the contact on fref.id among the
        # active contacts; a contact that exists but is inactive has f = 0 and zero force
        # Jacobians (contact-force.hxx createData looks the frame up among all contacts,
        # the first match in name order; updateForce / setZeroForceDiff)
        rows, r0 = {}, 0
        for n in self.contacts.active:
            c = self.contacts.contacts[n].contact
            rows.setdefault(c._ref.id, (r0, c.nc))
            r0 += c.nc
        for n in self.contacts.inactive:
            c = self.contacts.contacts[n].contact
            rows.setdefault(c._ref.id, (INACTIVE_FORCE_ROW, c.nc))
        o = _abi.PARAM_HEADER + 3 + self.state.nv + JOINT_REC * (self.state.pinocchio.njoints - 1)
        for name in sorted(self.costs.costs):
            it = self.costs.costs[name]
            if not it.active:
                continue
            size = int(out[0, o + 3])
            if it.cost.type in (COST_CONTACT_FORCE, COST_FRICTION_CONE):
                fid = it.cost.frame_id
                if fid not in rows:
                    raise ValueError(f"Invalid argument: there is not contact defined for frame {fid}")
                row0, nci = rows[fid]
                if it.cost.type == COST_CONTACT_FORCE and nci != it.cost.activation.nr:
                    raise ValueError("Invalid argument: the contact-force cost and its contact differ in size")
                out[:, o + COST_HDR] = row0
                if it.cost.type == COST_FRICTION_CONE:
                    out[:, o + COST_HDR + 1] = nci
            o += size
        return out


INACTIVE_FORCE_ROW = -2  # contact exists but is inactive: lambda = 0, zero force Jacobians


class _Impulse:
    """ImpulseModelAbstract (impulse-base.hxx): an impulse on a frame (LOCAL)."""

    type = 0
    ni = 0

    def __init__(self, state, frame):
        self.state = state
        self.frame = int(frame)
        model = state.pinocchio
        if not 0 <= self.frame < len(model.frames):
            raise ValueError("Invalid argument: unknown frame")

    def pack(self):
        name, pj, pl = self.state.pinocchio.frames[self.frame]
        if pj == 0:
            raise ValueError("Invalid argument: frames attached to the universe are not supported")
        body = np.concatenate([[pj - 1], pl.rotation.T.reshape(-1), pl.translation])
        return np.concatenate([[self.type, 0.0, 0.0, COST_HDR + body.size], body])


class ImpulseModel3D(_Impulse):
    """ImpulseModel3D(state, frame) (impulses/impulse-3d.hxx): point impulse,
    Jc = the 3 linear rows of the LOCAL frame Jacobian."""

    type = CONTACT_3D
    ni = 3


class ImpulseModel6D(_Impulse):
    """ImpulseModel6D(state, frame) (impulses/impulse-6d.hxx): rigid impulse,
    Jc = the LOCAL frame Jacobian."""

    type = CONTACT_6D
    ni = 6


class ImpulseItem:
    def __init__(self, name, impulse, active=True):
        self.name, self.impulse, self.active = name, impulse, bool(active)


class ImpulseModelMultiple:
    """ImpulseModelMultiple (impulses/multiple-impulses.hxx): named impulses in a
    std::map; the active ones stack their rows in name order."""

    def __init__(self, state):
        self.state = state
        self.impulses = {}
        self._version = 0

    def addImpulse(self, name, impulse, active=True):
        if name in self.impulses:  # the reference prints a warning and keeps the old item
            return
        self.impulses[name] = ImpulseItem(name, impulse, active)
        self._version += 1

    def removeImpulse(self, name):
        if name in self.impulses:
            del self.impulses[name]
            self._version += 1

    def changeImpulseStatus(self, name, active):
        if name in self.impulses:
            self.impulses[name].active = bool(active)
            self._version += 1

    @property
    def ni(self):
        return sum(c.impulse.ni for c in self.impulses.values() if c.active)

    @property
    def ni_total(self):
        return sum(c.impulse.ni for c in self.impulses.values())

    @property
    def active(self):
        return sorted(n for n, c in self.impulses.items() if c.active)

    @property
    def inactive(self):
        return sorted(n for n, c in self.impulses.items() if not c.active)

    def pack(self):
        return [self.impulses[n].impulse.pack() for n in self.active]


def _impulse_model_base():
    from .models import ActionModelAbstract
    return ActionModelAbstract


class ActionModelImpulseFwdDynamics(_impulse_model_base()):
    """ActionModelImpulseFwdDynamics(state, impulses, costs, r_coeff=0.,
    inv_damping=0., enable_force=False) (multibody/actions/impulse-fwddyn.hxx:15-127):
    nu = 0, xnext = (q, v+) with
        [M  Jc^T ; Jc  0] [v+ ; -Lambda] = [M v ; -r_coeff Jc v]
    (Schur complement with JMinvJt + inv_damping I), cost = costs.calc(x).
    An action model itself (no integrator): a running knot of the ShootingProblem."""

    kind = _abi.KNOT_IMPULSEFWD

    def __init__(self, state, impulses, costs, r_coeff=0.0, inv_damping=0.0, enable_force=False):
        if not isinstance(impulses, ImpulseModelMultiple):
            raise TypeError("ActionModelImpulseFwdDynamics needs an ImpulseModelMultiple")
        if r_coeff < 0.0:
            raise ValueError("Invalid argument: The restitution coefficient has to be positive, set to 0")
        if inv_damping < 0.0:
            raise ValueError("Invalid argument: The damping factor has to be positive, set to 0")
        if costs.nu != 0:
            raise ValueError("Invalid argument: impulse knots have no controls (CostModelSum(state, 0))")
        super().__init__(state, 0, costs.nr)
        self.impulses = impulses
        self.costs = costs
        self.r_coeff = float(r_coeff)
        self.JMinvJt_damping = float(inv_damping)
        self.enable_force = bool(enable_force)
        self._armature = np.zeros(state.nv)
        self._arm_version = 0

    @property
    def armature(self):
        return self._armature.copy()

    @armature.setter
    def armature(self, a):
        a = np.array(a, np.float64).reshape(-1)
        if a.size != self.state.nv:
            raise ValueError(f"Invalid argument: The armature dimension is wrong (it should be {self.state.nv})")
        self._armature = a
        self._arm_version += 1

    @property
    def _version(self):
        return (self.__dict__.get("_own_version", 0), self.state.pinocchio._version, self.costs._version,
                self.impulses._version, self._arm_version, self.r_coeff, self.JMinvJt_damping,
                tuple(getattr(c.cost, "_version", 0) for c in self.costs.costs.values()))

    @_version.setter
    def _version(self, v):
        self.__dict__["_own_version"] = v if not isinstance(v, tuple) else v[0]

    def _touch(self):
        self.__dict__["_own_version"] = self.__dict__.get("_own_version", 0) + 1

    def pack(self):
        recs = self.impulses.pack()
        if self.impulses.ni > MAX_CONTACT_ROWS:
            raise ValueError(f"Invalid argument: the device path holds at most {MAX_CONTACT_ROWS} impulse rows")
        sec = np.concatenate([[self.r_coeff, self.JMinvJt_damping, len(recs), 1.0]] + recs)
        return self.kind, 0, _pack_mb(self.state, self._armature, self.costs, 0.0, sec)
