"""Code-built legged robots in the role of example-robot-data (absent offline).

The reference's legged benchmarks load URDFs through Pinocchio
(benchmark/bipedal-timings.cpp:50 talos_reduced.urdf + JointModelFreeFlyer;
benchmark/quadrupedal-gaits-optctrl.cpp:26 hyq; bindings/python/crocoddyl/utils/
{biped,quadruped}.py with example_robot_data's talos / solo). Neither Pinocchio
nor the robot files exist here, so these builders construct trees of the same
kinematic structure, joint ordering, dimensions and mass distribution
(approximate link lengths / inertias; same nq, nv, joint names, frames and
reference configurations), as ``crocoddyl_amd.multibody.RobotModel`` objects.

  sample_talos():  free-flyer + 32 revolute joints (talos_reduced: legs 2 x 6, torso 2,
                   arms 2 x 7 + grippers 2, head 2): nq = 39, nv = 38 (C5)
  sample_solo12(): free-flyer + 4 legs x 3 (HAA, HFE, KFE): nq = 19, nv = 18 (C4)
"""
import numpy as np

from .multibody import (SE3, Inertia, JointModelFreeFlyer, JointModelRevoluteUnaligned, RobotModel)

_X, _Y, _Z = (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0)


def _body(m, joint, mass, com, diag):
    m.appendBodyToJoint(joint, Inertia(mass, com, np.diag(diag)))


def _chain(m, parent, specs, prefix):
    """specs: (name suffix, axis, placement translation, mass, CoM, inertia diag)."""
    j = parent
    ids = []
    for suffix, ax, p, mass, c, d in specs:
        j = m.addJoint(j, JointModelRevoluteUnaligned(ax), SE3(np.eye(3), p), f"{prefix}{suffix}")
        _body(m, j, mass, c, d)
        m.addFrame(f"{prefix}{suffix}", j)  # pinocchio adds a JOINT frame per joint
        ids.append(j)
    return ids


def sample_talos():
    """Talos full body (talos_reduced layout, Pinocchio's depth-first joint order):
    root_joint (free-flyer), leg_left_1..6, leg_right_1..6, torso_1..2,
    arm_left_1..7, gripper_left_joint, arm_right_1..7, gripper_right_joint,
    head_1..2. Frames: one per joint (its name), ``left_sole_link`` /
    ``right_sole_link`` 0.107 m below the ankles, ``gripper_*_tip``.
    referenceConfigurations["half_sitting"]."""
    m = RobotModel(JointModelFreeFlyer())
    _body(m, 1, 13.53, (-0.051, 0.0, 0.044), (0.068, 0.053, 0.073))  # pelvis / base_link
    m.addFrame("root_joint", 1)
    for side, s in (("left", 1.0), ("right", -1.0)):
        _chain(m, 1, [
            ("_1_joint", _Z, (-0.02, 0.085 * s, -0.27105), 1.85, (0.02, 0.0, 0.05), (0.004, 0.004, 0.002)),
            ("_2_joint", _X, (0.0, 0.0, 0.0), 1.49, (0.0, 0.0, -0.04), (0.003, 0.003, 0.002)),
            ("_3_joint", _Y, (0.0, 0.0, 0.0), 6.24, (0.02, 0.0, -0.22), (0.11, 0.11, 0.02)),
            ("_4_joint", _Y, (0.0, 0.0, -0.38), 3.63, (0.01, 0.0, -0.17), (0.05, 0.05, 0.008)),
            ("_5_joint", _Y, (0.0, 0.0, -0.325), 1.49, (0.0, 0.0, 0.0), (0.002, 0.002, 0.002)),
            ("_6_joint", _X, (0.0, 0.0, 0.0), 1.48, (0.02, 0.0, -0.07), (0.004, 0.006, 0.007)),
        ], f"leg_{side}")
        m.addFrame(f"{side}_sole_link", m.getJointId(f"leg_{side}_6_joint"), SE3(np.eye(3), (0.0, 0.0, -0.107)))
    t1, t2 = _chain(m, 1, [
        ("_1_joint", _Z, (0.0, 0.0, 0.0722), 3.02, (0.0, 0.0, 0.0), (0.01, 0.01, 0.01)),
        ("_2_joint", _Y, (0.0, 0.0, 0.0), 17.55, (-0.05, 0.0, 0.18), (0.32, 0.26, 0.2)),
    ], "torso")
    for side, s in (("left", 1.0), ("right", -1.0)):
        arm = _chain(m, t2, [
            ("_1_joint", _Z, (0.0, 0.157 * s, 0.232), 2.71, (-0.002, 0.04 * s, 0.0), (0.012, 0.004, 0.011)),
            ("_2_joint", _X, (0.0, 0.0, 0.0), 1.51, (0.01, 0.0, -0.06), (0.008, 0.008, 0.002)),
            ("_3_joint", _Z, (0.0, 0.0, 0.0), 1.43, (0.0, 0.0, -0.15), (0.012, 0.012, 0.002)),
            ("_4_joint", _Y, (0.02, 0.0, -0.273), 1.02, (-0.01, 0.0, -0.05), (0.004, 0.004, 0.001)),
            ("_5_joint", _Z, (-0.02, 0.0, -0.1), 1.12, (0.0, 0.0, -0.08), (0.006, 0.006, 0.001)),
            ("_6_joint", _X, (0.0, 0.0, -0.164), 0.52, (0.0, 0.0, -0.01), (0.0005, 0.0005, 0.0003)),
            ("_7_joint", _Y, (0.0, 0.0, 0.0), 0.40, (0.0, 0.0, -0.05), (0.0004, 0.0004, 0.0002)),
        ], f"arm_{side}")
        _chain(m, arm[-1], [("_joint", _Z, (0.0, 0.0, -0.12), 0.28, (0.0, 0.0, -0.03), (0.0002, 0.0002, 0.0001))],
               f"gripper_{side}")
        m.addFrame(f"gripper_{side}_tip", m.getJointId(f"gripper_{side}_joint"), SE3(np.eye(3), (0.0, 0.0, -0.06)))
    _chain(m, t2, [
        ("_1_joint", _Y, (0.0, 0.0, 0.4), 0.66, (0.0, 0.0, 0.02), (0.001, 0.001, 0.001)),
        ("_2_joint", _Z, (0.0, 0.0, 0.0), 1.16, (0.02, 0.0, 0.09), (0.006, 0.006, 0.005)),
    ], "head")
    # effort limits (N m) of the Talos actuator classes, standing in for the talos URDF's
    # <limit effort> (approximate and PARITY UNPINNED: the URDF is not in this image, so
    # box-limited workloads on these limits are not bipedal_walk_ubound.py parity);
    # hips / knee / ankles, torso, shoulder / elbow / wrist, gripper, neck
    effort = {"leg_%s_1_joint": 100.0, "leg_%s_2_joint": 160.0, "leg_%s_3_joint": 160.0, "leg_%s_4_joint": 300.0,
              "leg_%s_5_joint": 160.0, "leg_%s_6_joint": 100.0, "arm_%s_1_joint": 44.64, "arm_%s_2_joint": 22.32,
              "arm_%s_3_joint": 22.32, "arm_%s_4_joint": 22.32, "arm_%s_5_joint": 3.0, "arm_%s_6_joint": 3.0,
              "arm_%s_7_joint": 3.0, "gripper_%s_joint": 1.0}
    for side in ("left", "right"):
        for name, e in effort.items():
            m.setEffortLimit(m.getJointId(name % side), e)
    for name, e in (("torso_1_joint", 200.0), ("torso_2_joint", 200.0), ("head_1_joint", 6.0), ("head_2_joint", 6.0)):
        m.setEffortLimit(m.getJointId(name), e)
    leg = [0.0, 0.0, -0.411354, 0.859395, -0.448041, -0.001708]
    q = np.concatenate([[0.0, 0.0, 1.0192720229567027, 0.0, 0.0, 0.0, 1.0], leg, leg, [0.0, 0.006761],
                        [0.25847, 0.173046, -0.0002, -0.525366, 0.0, 0.0, 0.1, -0.005],
                        [-0.25847, -0.173046, 0.0002, -0.525366, 0.0, 0.0, 0.1, -0.005], [0.0, 0.0]])
    assert q.size == m.nq == 39 and m.nv == 38
    m.referenceConfigurations["half_sitting"] = q
    return m


def sample_solo12():
    """Solo12 (example-robot-data solo12): root_joint (free-flyer), then FL, FR, HL,
    HR legs with HAA (x), HFE (y), KFE (y) joints; foot frames ``FL_FOOT`` ...
    referenceConfigurations["standing"]."""
    m = RobotModel(JointModelFreeFlyer())
    _body(m, 1, 1.43, (0.0, 0.0, 0.0), (0.0025, 0.0108, 0.0126))
    m.addFrame("root_joint", 1)
    for leg, sx, sy in (("FL", 1.0, 1.0), ("FR", 1.0, -1.0), ("HL", -1.0, 1.0), ("HR", -1.0, -1.0)):
        ids = _chain(m, 1, [
            ("_HAA", _X, (0.1946 * sx, 0.0875 * sy, 0.0), 0.148, (-0.078 * sx, 0.015 * sy, 0.0),
             (0.00002, 0.0001, 0.0001)),
            ("_HFE", _Y, (0.0, 0.014 * sy, 0.0), 0.148, (0.0, 0.016 * sy, -0.078), (0.0004, 0.0004, 0.00002)),
            ("_KFE", _Y, (0.0, 0.03745 * sy, -0.16), 0.033, (0.0, 0.007 * sy, -0.078), (0.0001, 0.0001, 0.000003)),
        ], leg)
        m.addFrame(f"{leg}_FOOT", ids[-1], SE3(np.eye(3), (0.0, 0.008 * sy, -0.16)))
        for j, (lo, hi) in zip(ids, ((-0.9, 0.9), (-1.9, 1.9), (-3.0, 3.0))):  # URDF-style limits, 20 rad/s
            m.setJointLimits(j, lo, hi, 20.0)
    front, hind = [0.0, 0.8, -1.6], [0.0, -0.8, 1.6]
    q = np.concatenate([[0.0, 0.0, 0.235, 0.0, 0.0, 0.0, 1.0], front, front, hind, hind])
    assert q.size == m.nq == 19 and m.nv == 18
    m.referenceConfigurations["standing"] = q
    return m
