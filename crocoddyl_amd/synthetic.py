"""Seeded synthetic problems for the BASELINE.json configs.

The robot configs run on real multibody knots over code-built robots
(crocoddyl_amd.robots: URDFs and Pinocchio are absent offline):
  C3_arm_multibody / C3_arm_contact   the 7-DoF Talos-class arm (free / contact dynamics)
  C4_solo12_trot                      Solo12 trotting gait (utils/quadruped.py), T = 60
  C5_talos_walk                       Talos walking gait (utils/biped.py), T = 100
The gait configs give every batch element its own x0 (the reference posture
perturbed on the manifold) over one shared knot sequence.

C3_talos_arm / C4_solo12 / C5_talos_full are the Euler(dt) ∘
DifferentialActionModelLQR stand-ins with the robots' (n, m, T, B): the solver core
alone at those shapes; every batch element gets its own seeded perturbation of the
model matrices (shared over t), so every (b, t) derivative block is distinct data.
"""
import numpy as np

from .models import (ActionModelLQR, ActionModelUnicycle, DifferentialActionModelLQR,
                     IntegratedActionModelEuler)

# name -> (kind, nx or nq, nu, T, B, dt)
CONFIGS = {
    "C1_unicycle": ("unicycle", 3, 2, 30, 1, 0.1),
    "C2_lqr": ("lqr", 24, 12, 100, 256, None),
    "C3_talos_arm": ("euler", 7, 7, 250, 512, 1e-3),
    "C4_solo12": ("euler", 18, 12, 60, 1024, 1e-2),
    "C5_talos_full": ("euler", 38, 32, 100, 1024, 1e-3),
    # C3 on real multibody knots: Euler ∘ FreeFwdDynamics of the 7-DoF arm (build_arm)
    "C3_arm_multibody": ("multibody", 7, 7, 250, 512, 1e-3),
    # the same arm on contact dynamics: Euler ∘ ContactFwdDynamics, gripper 6D
    # contact, floating-base actuation (nu = 6), build_arm_contact
    "C3_arm_contact": ("multibody_contact", 7, 6, 250, 512, 1e-3),
    # legged robots on their gaits (contact dynamics, free-flyer root): nq, nu
    "C4_solo12_trot": ("gait_quadruped", 19, 12, 60, 1024, 1e-2),
    "C5_talos_walk": ("gait_biped", 39, 32, 100, 1024, 0.0375),
}


def gait_models(name, T=None):
    """(gait builder, running models, terminal model) of a gait config. The knot
    counts are the reference benchmark's gait parameters stretched to the config's
    T: Talos walking (benchmark/bipedal_walk_optctrl.py:82-90: step 0.6 m / 0.1 m,
    dt 0.0375, 1 support knot) with 48 step knots -> T = 100; Solo12 trotting
    (benchmark/quadrupedal_gaits_optctrl.py:134-142: step 0.15 m / 0.1 m, dt 1e-2,
    2 support knots) with 27 step knots -> T = 60. A smaller T shortens the steps
    (for parity tests)."""
    from . import gaits, robots
    kind, _, _, T0, _, dt = CONFIGS[name]
    T = T0 if T is None else T
    if kind == "gait_biped":
        g = gaits.SimpleBipedGaitProblem(robots.sample_talos(), "right_sole_link", "left_sole_link")
        sk = max(1, T // 2 - 2)
        models = g.createWalkingModels(g.rmodel.defaultState, 0.6, 0.1, dt, sk, 1)
    else:
        g = gaits.SimpleQuadrupedalGaitProblem(robots.sample_solo12(), "FL_FOOT", "FR_FOOT", "HL_FOOT", "HR_FOOT")
        sk = max(1, T // 2 - 3)
        models = g.createTrottingModels(g.rmodel.defaultState, 0.15, 0.1, dt, sk, 2)
    models = models[:T]
    return g, models, models[-1]


def build_gait(name, T=None, B=None, seed=None, spread=0.02, v_spread=0.1):
    """(x0s, running, terminal) of a gait config: x0_b = the reference posture
    integrated along a seeded tangent perturbation (q +- spread, v +- v_spread)."""
    _, _, _, T0, B0, _ = CONFIGS[name]
    B = B0 if B is None else B
    g, running, terminal = gait_models(name, T)
    rng = np.random.default_rng(seed_of(name) + 1 if seed is None else seed)
    x0 = g.rmodel.defaultState
    nv = g.state.nv
    x0s = np.stack([g.state.integrate(x0, np.concatenate([rng.uniform(-spread, spread, nv),
                                                          rng.uniform(-v_spread, v_spread, nv)]))
                    for _ in range(B)])
    if B:
        x0s[0] = x0
    return x0s, running, terminal


def gait_warm_start(name, running, x0):
    """The reference benchmark's warm start (bipedal_walk_optctrl.py:29-32): xs =
    the default state at every knot, us = each knot's quasiStatic controls."""
    xs = [x0] * (len(running) + 1)
    us = [m.quasiStatic(None, x0) if m.nu else np.zeros(0) for m in running]
    return xs, us


def seed_of(name):
    """Seed = 0x5EED + cfg_id."""
    return 0x5EED + int(name[1])


def _spd(rng, B, n, scale):
    A = rng.standard_normal((B, n, n))
    return np.einsum("bki,bkj->bij", A, A) / (n * scale) + np.eye(n)


def lqr_models(nx, nu, B, rng, drift_free=True):
    """ActionModelLQR(nx, nu) with per-element matrices (§8d C2 recipe)."""
    m = ActionModelLQR(nx, nu, drift_free)
    Fx = np.eye(nx) + 0.01 * rng.standard_normal((B, nx, nx))
    rho = np.max(np.abs(np.linalg.eigvals(Fx)), axis=1)
    Fx = np.where((rho > 1.05)[:, None, None], Fx * (1.05 / rho)[:, None, None], Fx)
    m.Fx = Fx
    m.Fu = np.eye(nx, nu) + 0.01 * rng.standard_normal((B, nx, nu))
    m.Lxx = _spd(rng, B, nx, 1.0)
    m.Luu = _spd(rng, B, nu, 1.0)
    m.Lxu = 0.01 * rng.standard_normal((B, nx, nu))
    m.lx = rng.uniform(-1, 1, (B, nx))
    m.lu = rng.uniform(-1, 1, (B, nu))
    if not drift_free:
        m.f0 = rng.uniform(-1, 1, (B, nx))
    return m


def difflqr_model(nq, nu, B, rng, drift_free=True):
    d = DifferentialActionModelLQR(nq, nu, drift_free)
    nx = 2 * nq
    d.Fq = -np.eye(nq) + 0.1 * rng.standard_normal((B, nq, nq)) / np.sqrt(nq)
    d.Fv = -0.1 * np.eye(nq) + 0.1 * rng.standard_normal((B, nq, nq)) / np.sqrt(nq)
    d.Fu = np.eye(nq, nu) + 0.1 * rng.standard_normal((B, nq, nu))
    d.Lxx = _spd(rng, B, nx, 1.0)
    d.Luu = _spd(rng, B, nu, 1.0)
    d.Lxu = 0.01 * rng.standard_normal((B, nx, nu))
    d.lx = rng.uniform(-1, 1, (B, nx))
    d.lu = rng.uniform(-1, 1, (B, nu))
    if not drift_free:
        d.f0 = rng.uniform(-1, 1, (B, nq))
    return d


def build(name, T=None, B=None, seed=None, drift_free=True):
    """(x0s (B, nx), running models [T], terminal model) for a config.
    T/B override the config's sizes (parity tests use small ones)."""
    kind, d1, nu, T0, B0, dt = CONFIGS[name]
    T = T0 if T is None else T
    B = B0 if B is None else B
    if kind == "multibody":
        return build_arm(T=T, B=B, seed=seed)
    if kind in ("gait_biped", "gait_quadruped"):
        return build_gait(name, T=T, B=B, seed=seed)
    if kind == "multibody_contact":
        return build_arm_contact(T=T, B=B, seed=seed_of(name) + 1 if seed is None else seed, dt=dt, contact="6d",
                                 q_nominal=ARM_BENT, spread=0.3)
    rng = np.random.default_rng(seed_of(name) if seed is None else seed)
    if kind == "unicycle":
        model = ActionModelUnicycle()
        x0s = np.vstack([[-1.0, -1.0, 1.0], rng.uniform(-1, 1, (max(B - 1, 0), 3))])[:B]
        return x0s, [model] * T, model
    if kind == "lqr":
        model = lqr_models(d1, nu, B, rng, drift_free)
        x0s = rng.uniform(-1, 1, (B, d1))
        return x0s, [model] * T, model
    dm = difflqr_model(d1, nu, B, rng, drift_free)
    running = IntegratedActionModelEuler(dm, dt)
    terminal = IntegratedActionModelEuler(dm, 0.0)
    x0s = rng.uniform(-1, 1, (B, 2 * d1))
    return x0s, [running] * T, terminal


def build_hetero(name, T=None, B=None, seed=None, phase=10, impulse_every=7):
    """Heterogeneous knot sequence at a config's dims (optional
    variant; §8f #4): two parameter sets alternating every `phase` knots
    (contact phases) and a control-free knot (nu = 0, impulse-like) at every
    `impulse_every`-th running knot. Returns (x0s, running, terminal)."""
    kind, d1, nu, T0, B0, dt = CONFIGS[name]
    T = T0 if T is None else T
    B = B0 if B is None else B
    rng = np.random.default_rng(seed_of(name) + 77 if seed is None else seed)
    if kind == "lqr":
        A = lqr_models(d1, nu, B, rng)
        Bm = lqr_models(d1, nu, B, rng)
        Z = lqr_models(d1, 0, B, rng)
        terminal = A
        nx = d1
    elif kind == "euler":
        A = IntegratedActionModelEuler(difflqr_model(d1, nu, B, rng), dt)
        Bm = IntegratedActionModelEuler(difflqr_model(d1, nu, B, rng), dt)
        Z = IntegratedActionModelEuler(difflqr_model(d1, 0, B, rng), dt)
        terminal = IntegratedActionModelEuler(A.differential, 0.0)
        nx = 2 * d1
    else:
        raise ValueError("heterogeneous sequences are built for the LQR / Euler configs")
    running = []
    for t in range(T):
        if impulse_every and t % impulse_every == impulse_every - 1:
            running.append(Z)
        else:
            running.append(A if (t // phase) % 2 == 0 else Bm)
    x0s = rng.uniform(-1, 1, (B, nx))
    return x0s, running, terminal


def build_arm_contact(T=4, B=2, seed=0, robot=None, dt=1e-2, contact="6d", gains=(2.0, 1.5), damping=0.0,
                      weighted=False, armature=None, inactive=False, q_nominal=None, spread=1.0, force_costs=False,
                      enable_force=None):
    """Contact-dynamics knots on the arm: Euler(dt) ∘ DifferentialActionModelContactFwdDynamics
    (contact-fwddyn.hxx) with ActuationModelFloatingBase (first joint unactuated)
    and a ContactModelMultiple on the gripper frame ("6d": ContactModel6D, "3d":
    ContactModel3D) and, for "6d+3d" / "3d+3d", a second 3D contact on a frame of
    joint 4; costs xReg + uReg (+ a weighted xReg and an elbow FrameTranslation
    when ``weighted``). ``inactive`` adds a contact item that is switched off
    (ContactModelMultiple::changeContactStatus). The terminal model is the same
    DAM with dt = 0. x0_b ~ U[-1,1]^(2 nv) per element (off the contact
    manifold: the Baumgarte gains pull the frames back); with ``q_nominal``,
    q0_b ~ q_nominal + U[-spread, spread]^nq and v0_b ~ U[-spread, spread]^nv.
    ``force_costs`` adds a CostModelContactForce per contact (a weighted one on the
    elbow); ``enable_force`` defaults to ``force_costs``."""
    from . import multibody as mb
    rng = np.random.default_rng(seed)
    model = mb.sample_talos_arm() if robot is None else robot
    if not model.existFrame("elbow_site"):
        model.addFrame("elbow_site", min(4, model.nv), mb.SE3(np.eye(3), (0.0, 0.05, -0.1)))
    state = mb.StateMultibody(model)
    act = mb.ActuationModelFloatingBase(state)
    nu = act.nu
    fid = model.getFrameId("gripper_left_joint") if model.existFrame("gripper_left_joint") else model.getFrameId("tip")
    eid = model.getFrameId("elbow_site")
    contacts = mb.ContactModelMultiple(state, nu)
    kinds = contact.split("+")
    if kinds[0] == "6d":
        contacts.addContact("gripper", mb.ContactModel6D(
            state, mb.FramePlacement(fid, mb.SE3(np.eye(3), (0.1, 0.2, 0.3))), nu, gains))
    else:
        contacts.addContact("gripper", mb.ContactModel3D(state, mb.FrameTranslation(fid, (0.1, 0.2, 0.3)), nu, gains))
    if len(kinds) > 1:
        contacts.addContact("elbow", mb.ContactModel3D(state, mb.FrameTranslation(eid, (0.0, 0.1, 0.2)), nu,
                                                       (gains[0] * 0.5, gains[1])))
    if inactive:
        contacts.addContact("aux", mb.ContactModel3D(state, mb.FrameTranslation(eid, (0.0, 0.0, 0.0)), nu, gains),
                            active=False)
    costs = mb.CostModelSum(state, nu)
    if weighted:
        costs.addCost("xReg", mb.CostModelState(state, mb.ActivationModelWeightedQuad(
            np.linspace(0.5, 2.0, state.ndx)), nu), 1e-2)
        costs.addCost("elbowTrans", mb.CostModelFrameTranslation(state, mb.FrameTranslation(eid, (0.1, 0.0, 0.2)),
                                                                 nu), 0.3)
    else:
        costs.addCost("xReg", mb.CostModelState(state, nu), 1e-2)
    costs.addCost("uReg", mb.CostModelControl(state, nu), 1e-3)
    if force_costs:
        costs.addCost("gripperForce", mb.CostModelContactForce(
            state, mb.FrameForce(fid, (1.0, 2.0, 3.0, 0.1, 0.2, 0.3)), 6 if kinds[0] == "6d" else 3, nu), 1e-3)
        if len(kinds) > 1:
            costs.addCost("elbowForce", mb.CostModelContactForce(
                state, mb.ActivationModelWeightedQuad(np.array([1.0, 2.0, 3.0])), mb.FrameForce(eid, np.zeros(6)), nu),
                1e-2)
    dam = mb.DifferentialActionModelContactFwdDynamics(state, act, contacts, costs, damping,
                                                       force_costs if enable_force is None else enable_force)
    if armature is not None:
        dam.armature = armature
    running = IntegratedActionModelEuler(dam, dt)
    terminal = IntegratedActionModelEuler(dam, 0.0)
    if q_nominal is None:
        x0s = np.hstack([rng.uniform(-1, 1, (B, state.nq)), rng.uniform(-1, 1, (B, state.nv))])
    else:
        x0s = np.hstack([np.asarray(q_nominal, float) + rng.uniform(-spread, spread, (B, state.nq)),
                         rng.uniform(-spread, spread, (B, state.nv))])
    return x0s, [running] * T, terminal


def impulse_model(robot=None, kind="6d", r_coeff=0.0, damping=0.0, weighted=False, armature=None, inactive=False):
    """ActionModelImpulseFwdDynamics on the arm's gripper ("6d": ImpulseModel6D,
    "3d": ImpulseModel3D, "6d+3d": plus a 3D impulse on the elbow frame),
    costs xReg (+ an elbow FrameTranslation when ``weighted``)."""
    from . import multibody as mb
    model = mb.sample_talos_arm() if robot is None else robot
    if not model.existFrame("elbow_site"):
        model.addFrame("elbow_site", min(4, model.nv), mb.SE3(np.eye(3), (0.0, 0.05, -0.1)))
    state = mb.StateMultibody(model)
    fid = model.getFrameId("gripper_left_joint") if model.existFrame("gripper_left_joint") else model.getFrameId("tip")
    eid = model.getFrameId("elbow_site")
    imps = mb.ImpulseModelMultiple(state)
    kinds = kind.split("+")
    imps.addImpulse("gripper", mb.ImpulseModel6D(state, fid) if kinds[0] == "6d" else mb.ImpulseModel3D(state, fid))
    if len(kinds) > 1:
        imps.addImpulse("elbow", mb.ImpulseModel3D(state, eid))
    if inactive:
        imps.addImpulse("aux", mb.ImpulseModel3D(state, eid), active=False)
    costs = mb.CostModelSum(state, 0)
    costs.addCost("xReg", mb.CostModelState(state, 0), 1e-2)
    if weighted:
        costs.addCost("elbowTrans", mb.CostModelFrameTranslation(state, mb.FrameTranslation(eid, (0.1, 0.0, 0.2)),
                                                                 0), 0.3)
    am = mb.ActionModelImpulseFwdDynamics(state, imps, costs, r_coeff, damping)
    if armature is not None:
        am.armature = armature
    return am


def build_arm_impact(T=8, B=2, seed=0, dt=1e-2, r_coeff=0.0):
    """A contact-switch horizon (the pattern of the reference's gait / jumping
    problems): free-flight knots (Euler ∘ FreeFwdDynamics, nu = 7) up to T/2,
    an impulse knot (ActionModelImpulseFwdDynamics, nu = 0) on the gripper at
    T/2, then gripper-contact knots (Euler ∘ ContactFwdDynamics, nu = 6)."""
    x0s, run_c, term_c = build_arm_contact(T=T, B=B, seed=seed, dt=dt, contact="6d", q_nominal=ARM_BENT, spread=0.3)
    _, run_f, _ = build_arm(T=T, B=B, dt=dt, w_x=1e-2, w_u=1e-2)
    imp = impulse_model(robot=run_c[0].differential.state.pinocchio, kind="6d", r_coeff=r_coeff)
    h = T // 2
    return x0s, run_f[:h] + [imp] + run_c[h + 1:], term_c


# a bent arm posture (elbow flexed, wrist pitched), away from the stretched
# contact singularity: the contact bench's nominal configuration
ARM_BENT = (0.3, 0.4, -0.2, -1.3, 0.1, 0.6, 0.0)


def build_arm(T=None, B=None, seed=None, robot=None, dt=1e-3, weighted=False, armature=None, w_x=1e-4, w_u=1e-4):
    """The reference's arm-manipulation problem (benchmark/factory/arm.hpp:31-96,
    benchmark/arm-manipulation-optctrl.cpp:20-40) on real multibody knots:
    Euler(dt) ∘ DifferentialActionModelFreeFwdDynamics with costs
    gripperPose (FramePlacement to (I, (0, 0, 0.4)), weight 1), xReg (1e-4),
    uReg (1e-4); the terminal model is Euler(runningDAM, 0) as in the factory.
    x0_b = (q0 ~ U[-1,1]^nq, v0 ~ U[-1,1]^nv) per element. ``robot``: a
    multibody.RobotModel (default: the 7-DoF Talos-class arm, C3's robot).
    ``weighted`` adds a weighted xReg activation and a FrameTranslation cost
    (parity coverage of the remaining cost / activation kinds). w_x / w_u: the
    xReg / uReg weights (the factory's 1e-4 by default)."""
    from . import multibody as mb
    _, _, _, T0, B0, _ = CONFIGS["C3_talos_arm"]
    T = T0 if T is None else T
    B = B0 if B is None else B
    rng = np.random.default_rng(seed_of("C3_talos_arm") + 1 if seed is None else seed)
    model = mb.sample_talos_arm() if robot is None else robot
    state = mb.StateMultibody(model)
    act = mb.ActuationModelFull(state)
    fid = model.getFrameId("gripper_left_joint") if model.existFrame("gripper_left_joint") else len(model.frames) - 1
    Mref = mb.FramePlacement(fid, mb.SE3(np.eye(3), (0.0, 0.0, 0.4)))
    costs = mb.CostModelSum(state)
    costs.addCost("gripperPose", mb.CostModelFramePlacement(state, Mref), 1.0)
    if weighted:
        w = np.linspace(0.5, 2.0, state.ndx)
        costs.addCost("xReg", mb.CostModelState(state, mb.ActivationModelWeightedQuad(w)), w_x)
        costs.addCost("gripperTrans", mb.CostModelFrameTranslation(
            state, mb.FrameTranslation(fid, (0.1, 0.2, 0.3))), 0.3)
    else:
        costs.addCost("xReg", mb.CostModelState(state), w_x)
    costs.addCost("uReg", mb.CostModelControl(state), w_u)
    dam = mb.DifferentialActionModelFreeFwdDynamics(state, act, costs)
    if armature is not None:
        dam.armature = armature
    running = IntegratedActionModelEuler(dam, dt)
    terminal = IntegratedActionModelEuler(dam, 0.0)
    x0s = np.hstack([rng.uniform(-1, 1, (B, state.nq)), rng.uniform(-1, 1, (B, state.nv))])
    return x0s, [running] * T, terminal


def random_floating_state(model, rng, B, spread=0.3, v_spread=0.5):
    """(B, nq + nv) states around the neutral configuration: the free-flyer pose
    integrated along a random twist (unit quaternion), joint angles and velocities
    uniform in [-spread, spread] / [-v_spread, v_spread]."""
    from . import multibody as mb
    state = mb.StateMultibody(model)
    x0 = state.zero()
    out = np.zeros((B, state.nx))
    for b in range(B):
        dx = np.concatenate([rng.uniform(-spread, spread, state.nv), rng.uniform(-v_spread, v_spread, state.nv)])
        out[b] = state.integrate(x0, dx)
    return out


def build_floating(T=4, B=2, seed=0, robot=None, dt=1e-2, contacts=(), gains=(2.0, 1.5), damping=0.0,
                   weighted=False, com=False, force_costs=False, enable_force=None, armature=None, spread=0.3,
                   friction=False, fvel=False, barrier=False):
    """Floating-base knots (the reference's legged-robot models, on a tree below a
    free-flyer root): Euler(dt) ∘ DifferentialAction{Free,Contact}FwdDynamics with
    ActuationModelFloatingBase (nu = nv - 6). ``contacts``: ("6d" | "3d", frame
    name) pairs -> ContactModel6D / 3D; none: free dynamics. Costs: xReg (to a
    non-neutral reference state, weighted with ``weighted``), uReg, a tip
    FramePlacement (+ a FrameTranslation when ``weighted``), CoMPosition with
    ``com``, a CostModelContactForce per contact with ``force_costs``. The
    terminal model is the same DAM with dt = 0. ``friction``: a
    CostModelContactFrictionCone per contact (QuadraticBarrier on the cone bounds, a
    tilted surface normal); ``fvel``: a CostModelFrameVelocity on the tip;
    ``barrier``: a WeightedQuadraticBarrier state-bounds cost and a QuadraticBarrier
    control-bounds cost (finite bounds the random states cross)."""
    from . import multibody as mb
    rng = np.random.default_rng(seed)
    model = mb.sample_tree(5, seed=3, freeflyer=True) if robot is None else robot
    if not model.existFrame("mid_site"):
        model.addFrame("mid_site", min(3, model.njoints - 1), mb.SE3(np.eye(3), (0.0, 0.05, -0.1)))
    state = mb.StateMultibody(model)
    act = mb.ActuationModelFloatingBase(state)
    nu = act.nu
    tip = model.getFrameId("tip")
    xref = random_floating_state(model, rng, 1, spread=0.5, v_spread=0.2)[0]
    costs = mb.CostModelSum(state, nu)
    if weighted:
        costs.addCost("xReg", mb.CostModelState(state, mb.ActivationModelWeightedQuad(
            np.linspace(0.5, 2.0, state.ndx)), xref, nu), 1e-2)
        costs.addCost("midTrans", mb.CostModelFrameTranslation(state, mb.FrameTranslation(
            model.getFrameId("mid_site"), (0.1, 0.0, 0.2)), nu), 0.3)
    else:
        costs.addCost("xReg", mb.CostModelState(state, xref, nu), 1e-2)
    costs.addCost("uReg", mb.CostModelControl(state, nu), 1e-3)
    costs.addCost("tipPose", mb.CostModelFramePlacement(state, mb.FramePlacement(
        tip, mb.SE3(mb._rot_axis(np.array([0.0, 0.6, 0.8]), 0.4), (0.2, -0.1, 0.3))), nu), 0.5)
    if com:
        costs.addCost("comTrack", mb.CostModelCoMPosition(state, (0.05, -0.02, 0.1), nu), 2.0)
    if fvel:
        costs.addCost("tipVel", mb.CostModelFrameVelocity(state, mb.FrameMotion(
            tip, mb.Motion((0.1, -0.2, 0.05), (0.3, 0.0, -0.1))), nu), 0.2)
    if barrier:
        nd = state.ndx
        bounds = mb.ActivationBounds(np.full(nd, -0.2), np.full(nd, 0.25), 0.9)
        costs.addCost("xBounds", mb.CostModelState(state, mb.ActivationModelWeightedQuadraticBarrier(
            bounds, np.linspace(1.0, 3.0, nd)), state.zero(), nu), 5.0)
        costs.addCost("uBounds", mb.CostModelControl(state, mb.ActivationModelQuadraticBarrier(
            mb.ActivationBounds(np.full(nu, -0.5), np.full(nu, 0.5))), nu), 3.0)
    if contacts:
        cm = mb.ContactModelMultiple(state, nu)
        for i, (kind, fname) in enumerate(contacts):
            fid = model.getFrameId(fname)
            if kind == "6d":
                c = mb.ContactModel6D(state, mb.FramePlacement(fid, mb.SE3(np.eye(3), (0.1, 0.2, 0.3))), nu, gains)
            else:
                c = mb.ContactModel3D(state, mb.FrameTranslation(fid, (0.1, 0.2, 0.3)), nu, gains)
            cm.addContact(f"c{i}_{fname}", c)
            if force_costs:
                nr = 6 if kind == "6d" else 3
                costs.addCost(f"force{i}", mb.CostModelContactForce(
                    state, mb.FrameForce(fid, rng.uniform(-1, 1, 6)), nr, nu), 1e-3)
            if friction:
                cone = mb.FrictionCone(np.array([0.1, -0.2, 1.0]), 0.7, 4, False, 0.5)
                costs.addCost(f"cone{i}", mb.CostModelContactFrictionCone(
                    state, mb.ActivationModelQuadraticBarrier(mb.ActivationBounds(cone.lb, cone.ub)),
                    mb.FrameFrictionCone(fid, cone), nu), 0.1)
        ef = (force_costs or friction) if enable_force is None else enable_force
        dam = mb.DifferentialActionModelContactFwdDynamics(state, act, cm, costs, damping, ef)
    else:
        dam = mb.DifferentialActionModelFreeFwdDynamics(state, act, costs)
    if armature is not None:
        dam.armature = armature
    running = IntegratedActionModelEuler(dam, dt)
    terminal = IntegratedActionModelEuler(dam, 0.0)
    x0s = random_floating_state(model, rng, B, spread=spread)
    return x0s, [running] * T, terminal
