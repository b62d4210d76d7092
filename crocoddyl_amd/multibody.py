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
from .models import _ControlLimits

JOINT_REC = 27
JOINT_REVOLUTE, JOINT_FREEFLYER = 0, 1
COST_HDR = 4
COST_STATE, COST_CONTROL, COST_FRAME_PLACEMENT, COST_FRAME_TRANSLATION = 1, 2, 3, 4
CONTACT_3D, CONTACT_6D = 5, 6
COST_CONTACT_FORCE = 7
COST_COM_POSITION = 8
COST_FRICTION_CONE = 9
COST_FRAME_VELOCITY = 10
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
        self._limits = {}  # joint id -> (lower, upper, velocity) (pinocchio Model limits; +-inf by default)
        self._effort = {}  # joint id -> effort limit (pinocchio Model::effortLimit; +inf by default)
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

    def setJointLimits(self, joint_id, lower, upper, velocity):
        """Position / velocity limits of a revolute joint (the URDF <limit> that
        pinocchio stores in lower/upperPositionLimit, velocityLimit)."""
        self._limits[int(joint_id)] = (float(lower), float(upper), float(velocity))

    @property
    def lowerPositionLimit(self):
        return self._qlim(0, -np.inf)

    @property
    def upperPositionLimit(self):
        return self._qlim(1, np.inf)

    @property
    def velocityLimit(self):
        out = np.full(self.nv, np.inf)
        for j in range(1, self.njoints):
            if self.kinds[j] != JOINT_FREEFLYER and j in self._limits:
                out[self.idx_v(j)] = self._limits[j][2]
        return out

    def setEffortLimit(self, joint_id, effort):
        """Torque limit of a revolute joint (the URDF <limit effort> that pinocchio
        stores in Model::effortLimit)."""
        self._effort[int(joint_id)] = float(effort)

    @property
    def effortLimit(self):
        """Model::effortLimit (nv; +inf where unset, as on the free-flyer's dofs). A copy,
        as pinocchio's Python binding returns; write it back with the setter
        (examples/bipedal_walk_ubound.py:16-18: lims = model.effortLimit; lims *= 0.5;
        model.effortLimit = lims)."""
        out = np.full(self.nv, np.inf)
        for j, e in self._effort.items():
            if self.kinds[j] != JOINT_FREEFLYER:
                out[self.idx_v(j)] = e
        return out

    @effortLimit.setter
    def effortLimit(self, lims):
        lims = np.array(lims, np.float64).reshape(-1)
        if lims.size != self.nv:
            raise ValueError(f"Invalid argument: effortLimit has wrong dimension (it should be {self.nv})")
        for j in range(1, self.njoints):
            if self.kinds[j] != JOINT_FREEFLYER:
                self._effort[j] = float(lims[self.idx_v(j)])
        self._version += 1

    def _qlim(self, k, default):
        out = np.full(self.nq, default)
        for j in range(1, self.njoints):
            if self.kinds[j] != JOINT_FREEFLYER and j in self._limits:
                out[self.idx_q(j)] = self._limits[j][k]
        return out

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

    def _world_motions(self, q, oM):
        """(nv, 6) world motion subspace of every dof at the world origin (linear,
        angular) and the joint owning it; free-flyer dofs are the base twist axes in
        the base frame (pinocchio's local free-flyer velocity)."""
        S, owner = [], []
        for j in range(1, self.njoints):
            R, p = oM[j].rotation, oM[j].translation
            if self.kinds[j] == JOINT_FREEFLYER:
                for k in range(6):
                    ax = R[:, k % 3]
                    S.append(np.concatenate([ax, np.zeros(3)]) if k < 3 else np.concatenate([np.cross(p, ax), ax]))
                    owner.append(j)
            else:
                w = R @ self.axes[j]
                S.append(np.concatenate([np.cross(p, w), w]))
                owner.append(j)
        return np.array(S), owner

    def _ancestors(self, j):
        out = set()
        while j > 0:
            out.add(j)
            j = self.parents[j]
        return out

    def getFrameJacobian(self, q, frame_id):
        """pinocchio::getFrameJacobian(LOCAL) after computeJointJacobians (6 x nv)."""
        oM = self.placements(q)
        S, owner = self._world_motions(q, oM)
        name, pj, pl = self.frames[frame_id]
        oMf = oM[pj] * pl
        anc = self._ancestors(pj)
        Rt, pf = oMf.rotation.T, oMf.translation
        J = np.zeros((6, self.nv))
        for d in range(self.nv):
            if owner[d] in anc:
                J[:3, d] = Rt @ (S[d, :3] - np.cross(pf, S[d, 3:]))
                J[3:, d] = Rt @ S[d, 3:]
        return J

    def computeGeneralizedGravity(self, q):
        """pinocchio::computeGeneralizedGravity = rnea(q, 0, 0): tau_d = S_d . F_d with F
        the gravity wrenches (-m g at the CoM, about the world origin) of d's subtree."""
        oM = self.placements(q)
        S, owner = self._world_motions(q, oM)
        wrench = np.zeros((self.njoints, 6))
        for j in range(1, self.njoints):
            I = self.inertias[j]
            f = -I.mass * self.gravity
            c = oM[j].translation + oM[j].rotation @ I.lever
            wrench[j] = np.concatenate([f, np.cross(c, f)])
        tau = np.zeros(self.nv)
        for d in range(self.nv):
            F = sum(wrench[b] for b in range(1, self.njoints) if owner[d] in self._ancestors(b))
            tau[d] = S[d] @ F
        return tau

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
        # limits (multibody.hxx:23-34): the first joint unbounded, then the model's
        nq0 = 7 if model.has_freeflyer else 1
        lb = np.concatenate([model.lowerPositionLimit, -model.velocityLimit])
        ub = np.concatenate([model.upperPositionLimit, model.velocityLimit])
        lb[:nq0], ub[:nq0] = -np.inf, np.inf
        self.lb, self.ub = lb, ub

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


ACT_QUAD, ACT_WEIGHTED_QUAD, ACT_QUAD_BARRIER, ACT_WEIGHTED_QUAD_BARRIER = 0, 1, 2, 3
DBL_MAX = np.finfo(np.float64).max


class ActivationModelQuad:
    """a = 0.5 ||r||^2, Ar = r, Arr = I (core/activations/quadratic.hpp)."""

    kind = ACT_QUAD

    def __init__(self, nr):
        self.nr = int(nr)
        self.weights = None

    def params(self):
        return np.ones((1, self.nr))


class ActivationModelWeightedQuad:
    """a = 0.5 r^T diag(w) r, Ar = w r, Arr = diag(w) (weighted-quadratic.hpp:42-71)."""

    kind = ACT_WEIGHTED_QUAD

    def __init__(self, weights):
        self.weights = np.array(weights, np.float64).reshape(-1)
        self.nr = self.weights.size

    def params(self):
        return self.weights.reshape(1, -1)


class ActivationBounds:
    """ActivationBounds(lb, ub, beta=1) (quadratic-barrier.hpp:24-68): the bounds
    are stored shrunk around their midpoint, m -+ beta d with m = (lb + ub) / 2,
    d = (ub - lb) / 2 (so infinite bounds give NaN, as in the reference)."""

    def __init__(self, lb, ub, beta=1.0):
        lb = np.array(lb, np.float64).reshape(-1)
        ub = np.array(ub, np.float64).reshape(-1)
        if lb.size != ub.size:
            raise ValueError("Invalid argument: The lower and upper bounds don't have the same dimension "
                             f"(lb,ub dimensions equal to {lb.size},{ub.size}, respectively)")
        if beta < 0.0 or beta > 1.0:
            raise ValueError("Invalid argument: The range of beta is between 0 and 1")
        fin = np.isfinite(lb) & np.isfinite(ub)
        if np.any(lb[fin] > ub[fin]):
            raise ValueError("Invalid argument: The lower and upper bounds are badly defined; ub has to be "
                             "bigger / equals to lb")
        with np.errstate(invalid="ignore", over="ignore"):
            m = 0.5 * (lb + ub)
            d = 0.5 * (ub - lb)
            self.lb = m - beta * d
            self.ub = m + beta * d
        self.beta = float(beta)


class ActivationModelQuadraticBarrier:
    """a = 0.5 ||min(r - lb, 0)||^2 + 0.5 ||max(r - ub, 0)||^2, Ar = min(r - lb, 0) +
    max(r - ub, 0), Arr = diag(r <= lb or r >= ub) (quadratic-barrier.hpp:88-117)."""

    kind = ACT_QUAD_BARRIER

    def __init__(self, bounds):
        if not isinstance(bounds, ActivationBounds):
            raise TypeError("ActivationModelQuadraticBarrier needs an ActivationBounds")
        self.bounds = bounds
        self.nr = bounds.lb.size
        self.weights = None

    def params(self):
        return np.concatenate([self.bounds.lb, self.bounds.ub]).reshape(1, -1)


class ActivationModelWeightedQuadraticBarrier:
    """ActivationModelWeightedQuadraticBarrier(bounds, weights)
    (weighted-quadratic-barrier.hpp:35-70): the barrier residuals scaled by w before
    squaring, a = 0.5 sum w^2 (rl^2 + ru^2), Ar = w^2 (rl + ru), and — as the
    reference has it — Arr = w (r <= lb or r >= ub)."""

    kind = ACT_WEIGHTED_QUAD_BARRIER

    def __init__(self, bounds, weights):
        if not isinstance(bounds, ActivationBounds):
            raise TypeError("ActivationModelWeightedQuadraticBarrier needs an ActivationBounds")
        self.bounds = bounds
        self.weights = np.array(weights, np.float64).reshape(-1)
        self.nr = bounds.lb.size
        if self.weights.size != self.nr:
            raise ValueError(f"Invalid argument: weight vector has wrong dimension (it should be {self.nr})")

    def params(self):
        return np.concatenate([self.bounds.lb, self.bounds.ub, self.weights]).reshape(1, -1)


_ACTIVATIONS = (ActivationModelQuad, ActivationModelWeightedQuad, ActivationModelQuadraticBarrier,
                ActivationModelWeightedQuadraticBarrier)


def _quat_from_two_vectors(a, b):
    """Eigen Quaternion::setFromTwoVectors(a, b) as a rotation matrix (the rotation
    taking a onto b)."""
    v0 = np.asarray(a, float) / np.linalg.norm(a)
    v1 = np.asarray(b, float) / np.linalg.norm(b)
    c = float(v1 @ v0)
    if c < -1.0 + np.finfo(float).eps:  # antiparallel: the axis from the null space of [v0; v1]
        c = max(c, -1.0)
        _, _, vt = np.linalg.svd(np.vstack([v0, v1]))
        axis = vt[2]
        w2 = (1.0 + c) * 0.5
        q = np.concatenate([axis * np.sqrt(1.0 - w2), [np.sqrt(w2)]])
    else:
        axis = np.cross(v0, v1)
        s = np.sqrt((1.0 + c) * 2.0)
        q = np.concatenate([axis / s, [0.5 * s]])
    return _quat_to_R(q)


class FrictionCone:
    """FrictionCone(normal, mu, nf=4, inner_appr=True, min_nforce=0, max_nforce=DBL_MAX)
    (multibody/friction-cone.hxx:24-96): lb <= A f <= ub with nf facets
    A_{2i} = (-mu z + t_i)^T cRo, A_{2i+1} = (-mu z - t_i)^T cRo (t_i at angle 2 pi i / nf,
    mu scaled by cos(pi / nf) for the inner approximation) and the normal row
    nsurf^T in [min_nforce, max_nforce]."""

    def __init__(self, normal=(0.0, 0.0, 1.0), mu=0.7, nf=4, inner_appr=True, min_nforce=0.0, max_nforce=DBL_MAX):
        nf = int(nf)
        if nf % 2 != 0:
            nf = 4  # the reference warns and uses 4
        self.nf = nf
        self.update(normal, mu, inner_appr, min_nforce, max_nforce)

    def update(self, normal, mu, inner_appr=True, min_nforce=0.0, max_nforce=DBL_MAX):
        n = np.array(normal, np.float64).reshape(3)
        if abs(np.linalg.norm(n) - 1.0) > 1e-12:
            n = n / np.linalg.norm(n)
        self.nsurf = n
        self.mu = float(mu)
        self.inner_appr = bool(inner_appr)
        self.min_nforce = float(min_nforce) if min_nforce >= 0 else 0.0
        self.max_nforce = float(max_nforce) if max_nforce >= 0 else DBL_MAX
        theta = 2.0 * np.pi / self.nf
        if self.inner_appr:
            self.mu *= np.cos(theta / 2.0)
        cRo = _quat_from_two_vectors(n, (0.0, 0.0, 1.0))
        A = np.zeros((self.nf + 1, 3))
        lb = np.zeros(self.nf + 1)
        ub = np.zeros(self.nf + 1)
        z = np.array([0.0, 0.0, 1.0])
        for i in range(self.nf // 2):
            ti = np.array([np.cos(theta * i), np.sin(theta * i), 0.0])
            A[2 * i] = (-self.mu * z + ti) @ cRo
            A[2 * i + 1] = (-self.mu * z - ti) @ cRo
            lb[2 * i] = lb[2 * i + 1] = -DBL_MAX
        A[self.nf] = n
        lb[self.nf] = self.min_nforce
        ub[self.nf] = self.max_nforce
        self.A, self.lb, self.ub = A, lb, ub


class FrameFrictionCone:
    """FrameFrictionCone(id, cone) (multibody/frames.hpp:139-152)."""

    def __init__(self, id, cone):
        self.id = int(id)
        self.cone = cone


class Motion:
    """pinocchio.Motion subset: linear, angular."""

    def __init__(self, linear=None, angular=None):
        self.linear = np.zeros(3) if linear is None else np.array(linear, np.float64).reshape(3)
        self.angular = np.zeros(3) if angular is None else np.array(angular, np.float64).reshape(3)

    @staticmethod
    def Zero():
        return Motion()

    @property
    def vector(self):
        return np.concatenate([self.linear, self.angular])


LOCAL = 0  # pinocchio::ReferenceFrame (the device covers LOCAL frame velocities)


class FrameMotion:
    """FrameMotion(id, motion, reference=LOCAL) (multibody/frames.hpp:86-116)."""

    def __init__(self, id, motion, reference=LOCAL):
        if reference != LOCAL:
            raise NotImplementedError("crocoddyl_amd: frame velocities are covered in the LOCAL frame only")
        self.id = int(id)
        self.motion = motion if isinstance(motion, Motion) else Motion(np.asarray(motion)[:3], np.asarray(motion)[3:])
        self.reference = reference


class FramePlacement:
    def __init__(self, id, placement):
        self.id = int(id)
        self.placement = placement

    # deprecated aliases the reference's bindings keep (bindings/python/crocoddyl/multibody/frames.cpp:77-86)
    frame = property(lambda s: s.id)
    oMf = property(lambda s: s.placement)


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
        """(Bm, size) record: [type, weight=0 (set by the sum), activation kind, size]
        + payload + activation parameters (w | lb, ub | lb, ub, w)."""
        parts = self._payload()
        parts.append(self.activation.params())
        Bm = max(p.shape[0] for p in parts)
        size = COST_HDR + sum(p.shape[1] for p in parts)
        hdr = np.array([[self.type, 0.0, float(self.activation.kind), size]])
        return np.concatenate([np.broadcast_to(p, (Bm, p.shape[1])) for p in [hdr] + parts], axis=1)


def _rows(a, n):
    a = np.asarray(a, np.float64)
    return a.reshape(1, n) if a.ndim == 1 else a.reshape(a.shape[0], n)


def _cost_args(args, kw):
    """Sort the reference's overloads: (activation?, reference?, nu?)."""
    act = ref = nu = None
    for a in args:
        if isinstance(a, _ACTIVATIONS):
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
            if isinstance(a, _ACTIVATIONS):
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


class CostModelContactFrictionCone(_Cost):
    """r = A lambda_lin (contact-friction-cone.hxx:51-91): the cone matrix times the
    linear part of the force of the contact on frame fref.id, in the contact frame.
    Overloads (state, activation, fref[, nu]) and (state, fref[, nu]) with
    ActivationModelQuad(nf + 1) by default; the activation must have nf + 1 rows.
    Its derivatives are A d lambda_lin / dx (du), which the DAM computes only with
    enable_force=True (zero otherwise, as in the reference)."""

    type = COST_FRICTION_CONE

    def __init__(self, state, *args, **kw):
        act = fref = nu = None
        for a in args:
            if isinstance(a, _ACTIVATIONS):
                act = a
            elif isinstance(a, FrameFrictionCone):
                fref = a
            elif isinstance(a, (int, np.integer)) and not isinstance(a, bool):
                nu = int(a)
        act = kw.get("activation", act)
        fref = kw.get("fref", fref)
        nu = kw.get("nu", nu)
        if not isinstance(fref, FrameFrictionCone):
            raise TypeError("CostModelContactFrictionCone needs a FrameFrictionCone reference")
        nr = fref.cone.nf + 1
        if act is not None and act.nr != nr:
            raise ValueError(f"Invalid argument: nr is equals to {nr}")
        super().__init__(state, act, nr, nu)
        self.fref = fref

    @property
    def frame_id(self):
        return self.fref.id

    def _payload(self):  # [row0 (resolved by the DAM), contact rows, nr, A (nr x 3, row-major)]
        A = self.fref.cone.A
        return [np.concatenate([[-1.0, 0.0, A.shape[0]], A.reshape(-1)]).reshape(1, -1)]


class CostModelFrameVelocity(_Cost):
    """r = v_f - vref (frame-velocity.hxx:53-84): the LOCAL spatial velocity of frame
    vref.id (pinocchio::getFrameVelocity) minus the reference motion; Rx =
    getFrameVelocityDerivatives (dv/dq, dv/dv), Ru = 0."""

    type = COST_FRAME_VELOCITY

    def __init__(self, state, *args, **kw):
        act, ref, nu = _cost_args(args, kw)
        ref = kw.get("vref", ref)
        if not isinstance(ref, FrameMotion):
            raise TypeError("CostModelFrameVelocity needs a FrameMotion reference")
        super().__init__(state, act, 6, nu)
        self.vref = ref

    def _payload(self):
        model = self.state.pinocchio
        name, pj, pl = model.frames[self.vref.id]
        if pj == 0:
            raise ValueError("Invalid argument: frames attached to the universe are not supported")
        frame = np.concatenate([[pj - 1], pl.rotation.T.reshape(-1), pl.translation]).reshape(1, -1)
        return [frame, self.vref.motion.vector.reshape(1, -1)]


class CostItem:
    """CostItem (cost-sum.hpp): name, cost, weight, active; changing the weight
    marks the owning CostModelSum as modified (its blocks are re-packed)."""

    def __init__(self, name, cost, weight, active=True, owner=None):
        self.name, self.cost, self._weight, self.active = name, cost, float(weight), bool(active)
        self._owner = owner

    @property
    def weight(self):
        return self._weight

    @weight.setter
    def weight(self, w):
        self._weight = float(w)
        if self._owner is not None:
            self._owner._version += 1


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
        self.costs[name] = CostItem(name, cost, weight, active, self)
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


class DifferentialActionModelFreeFwdDynamics(_ControlLimits):
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
        self._init_limits()

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

    def quasiStatic(self, x, maxiter=100, tol=1e-9):
        """u holding x = (q, 0) still (free-fwddyn.hxx:137-160): pinv(dtau/du) g(q),
        i.e. g(q) on the actuated dofs. Host-side setup (warm starts), not the device path."""
        x = np.asarray(x, float)
        g = self.state.pinocchio.computeGeneralizedGravity(x[:self.state.nq])
        return g[self.state.nv - self.nu:].copy()

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
    ``enable_force`` selects the force Jacobians d lambda / d(x, u)
    (contact-fwddyn.hxx:141-156) that CostModelContactForce / ContactFrictionCone
    read; without it their residual Jacobians are zero, as in the reference."""

    def __init__(self, state, actuation, contacts, costs, inv_damping=0.0, enable_force=False):
        if not isinstance(actuation, ActuationModelFloatingBase):
            raise TypeError("DifferentialActionModelContactFwdDynamics needs an ActuationModelFloatingBase")
        if not isinstance(contacts, ContactModelMultiple):
            raise TypeError("DifferentialActionModelContactFwdDynamics needs a ContactModelMultiple")
        if contacts.nu != actuation.nu:
            raise ValueError(f"Invalid argument: Contacts doesn't have the same control dimension "
                             f"(it should be {actuation.nu})")
        self._init_dam(state, actuation, costs)
        # the control limits start at the robot's torque limits on the actuated dofs
        # (contact-fwddyn.hxx:51-52: set_u_lb(-effortLimit.tail(nu)), set_u_ub(+...))
        lim = state.pinocchio.effortLimit[state.nv - self.nu:]
        self.u_lb, self.u_ub = -lim, lim.copy()
        self.contacts = contacts
        self.JMinvJt_damping = abs(float(inv_damping))
        self.enable_force = bool(enable_force)

    def version(self):
        return super().version() + (self.contacts._version, self.JMinvJt_damping,
                                    tuple(c.contact.gains.tobytes() for c in self.contacts.contacts.values()))

    knot_kind = _abi.KNOT_EULER_CONTACTFWD

    def quasiStatic(self, x, maxiter=100, tol=1e-9):
        """u = (pinv([dtau/du | Jc^T]) g(q))[:nu] (contact-fwddyn.hxx:169-207): the
        controls (with the contact forces) that hold x = (q, 0) still. Host-side setup."""
        x = np.asarray(x, float)
        model, nv, nu = self.state.pinocchio, self.state.nv, self.nu
        q = x[:self.state.nq]
        g = model.computeGeneralizedGravity(q)
        cols = [np.vstack([np.zeros((nv - nu, nu)), np.eye(nu)])]
        for n in self.contacts.active:
            c = self.contacts.contacts[n].contact
            J = model.getFrameJacobian(q, c._ref.id)
            cols.append((J[:3] if c.nc == 3 else J).T)
        return (np.linalg.pinv(np.hstack(cols)) @ g)[:nu]

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
        if any(it.active and it.cost.type in (COST_FRAME_VELOCITY, COST_CONTACT_FORCE, COST_FRICTION_CONE)
               for it in self.costs.costs.values()):
            raise NotImplementedError("crocoddyl_amd: frame-velocity / force costs on impulse knots are not covered")
        if self.impulses.ni > MAX_CONTACT_ROWS:
            raise ValueError(f"Invalid argument: the device path holds at most {MAX_CONTACT_ROWS} impulse rows")
        sec = np.concatenate([[self.r_coeff, self.JMinvJt_damping, len(recs), 1.0]] + recs)
        return self.kind, 0, _pack_mb(self.state, self._armature, self.costs, 0.0, sec)
