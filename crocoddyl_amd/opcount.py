"""Algorithmic FP64 operation counts of the multibody knots (measurement accounting
for bench.py's knot-kernel rooflines; not on the solver path).

The count follows the reference's op sequence per knot with the algorithms it calls,
priced at fixed spatial-algebra costs (flops = mul + add; a fused multiply-add is 2):

  6D motion / force transform X m           c_X   = 42
  spatial cross product (m x m, m x* f)     c_cr  = 24
  rigid-body inertia times motion I m       c_I   = 36
  6D dot product                            c_dot = 11

calc of Euler ∘ ContactFwdDynamics (contact-fwddyn.hxx:59-104, euler.hxx:41-80):
  computeAllTerms: RNEA nle (per dof: forward X v, X a, v x S qd, I a, v x* I v; backward
    S.f, X^T f) ~ 350 n; CRBA (composite X^T Ic X ~ 200 per body, per column F = Ic S and
    per ancestor X^T F + S.F) 236 n + 53 sum_j |anc(j)|; contact frame Jacobians
    42 per ancestor column per contact frame; drift accelerations ~100 per contact.
  forwardDynamics: the sparse LDL^T of M (pinocchio::cholesky::decompose) sum_k
    (d_k^2 + 2 d_k) with d_k = |anc(k)|; nc + 1 solves (4 sum_k d_k + n each);
    JMinvJt 2 nc^2 n; its LLT nc^3 / 3; lambda 2 nc^2 + 2 nc n; a = z + Y lambda 2 n nc.
  Euler step 4 n (+ exp6 on the free-flyer ~200); costs: per residual row ~20, frame
    costs + 150 (log6 / frame placement), CoM 10 n, state 2 n (+100 free-flyer).
calcDiff (contact-fwddyn.hxx:107-160, euler.hxx:83-131, cost-sum.hxx:122-160), at the
  calc's linearisation point (the reference recomputes it: computeRNEADerivatives):
  computeRNEADerivatives: 4 RNEA + 200 per (dof, ancestor) pair (the q and v columns:
    3 cross products, 4 dots, 2 transforms per pair);
  getKKTContactDynamicMatrixInverse: M^-1 from the factorisation (n solves), M^-1 Jc^T
    and JMinvJt as above, the Schur inverse nc^3, Kinv top-left 2 n nc^2 + 2 n^2 nc;
  contact derivatives (frame velocity / acceleration derivatives) 20 nc L;
  df_dx = -Kinv [dtau_dx; da0_dx] (the (n + nc) rows: a and lambda) 2 (n + nc)^2 L;
  Euler assembly 2 n L (+ Jintegrate 72 L on a free-flyer), Fu 2 n nu;
  costs: residual Jacobians (frame: Jlog6 x frame Jacobian 72 n + 42 d) and the
    Gauss-Newton products R^T diag(w h) R over each cost's columns c: nr c (c + 1)
    (symmetric half), gradients 2 nr c; state / control costs 4 per entry.
Impulse knots (impulse-fwddyn.hxx) take the calc's and calcDiff's contact terms with
the impulse rows; free-dynamics knots nc = 0.

These are estimates of the reference's arithmetic, stated so that the roofline's
flop fraction can be reproduced; bench.py reports them beside the HBM roofline and
takes the binding roof (the larger time floor).
"""
import numpy as np

C_X, C_CR, C_I, C_DOT = 42, 24, 36, 11


def dof_parents(robot):
    """Dof-level parent (-1 for a root dof) of a RobotModel in Pinocchio's order; a
    free-flyer root's six dofs form a chain."""
    from .multibody import JOINT_FREEFLYER
    par, last = [], {0: -1}
    for j in range(1, robot.njoints):
        p = last[robot.parents[j]]
        for _ in range(6 if robot.kinds[j] == JOINT_FREEFLYER else 1):
            par.append(p)
            p = len(par) - 1
        last[j] = p
    return par


def _anc_counts(par):
    d = []
    for k in range(len(par)):
        c, p = 0, par[k]
        while p >= 0:
            c, p = c + 1, par[p]
        d.append(c)
    return np.array(d, float)


def _frame_depth(robot, fid, par_d=None):
    """Dofs on the path of a frame's joint to the root."""
    from .multibody import JOINT_FREEFLYER
    j = robot.frames[fid][1]
    cnt = 0
    while j != 0:
        cnt += 6 if robot.kinds[j] == JOINT_FREEFLYER else 1
        j = robot.parents[j]
    return cnt


def _cost_terms(dam, n, nu, L, robot, par):
    """(calc flops, calcDiff flops) of a CostModelSum."""
    from . import multibody as mb
    calc = diff = 0.0
    for name in sorted(dam.costs.costs):
        it = dam.costs.costs[name]
        if not it.active:
            continue
        c = it.cost
        nr = c.activation.nr
        calc += 20 * nr
        if isinstance(c, (mb.CostModelFramePlacement, mb.CostModelFrameTranslation, mb.CostModelFrameVelocity)):
            ref = getattr(c, "Mref", None) or getattr(c, "xref", None) or getattr(c, "vref", None)
            d = _frame_depth(robot, ref.id, par)
            calc += 150
            cols = L if isinstance(c, mb.CostModelFrameVelocity) else n
            diff += 72 * n + C_X * d + nr * cols * (cols + 1) + 2 * nr * cols
        elif isinstance(c, mb.CostModelCoMPosition):
            calc += 10 * n
            diff += 10 * n * 3 + nr * n * (n + 1) + 2 * nr * n
        elif isinstance(c, mb.CostModelState):
            calc += 2 * L + (100 if robot.has_freeflyer else 0)
            diff += 4 * L + (72 * 6 if robot.has_freeflyer else 0)
        elif isinstance(c, mb.CostModelControl):
            calc += 2 * nu
            diff += 4 * nu
        else:  # contact force / friction cone: rows of lambda and d lambda / d(x, u)
            cols = L + nu
            diff += nr * cols * (cols + 1) + 2 * nr * cols
    return calc, diff


def knot_flops(model):
    """(calc, calcDiff) algorithmic flops of one knot (a device-kind multibody model:
    IntegratedActionModelEuler of a Free/ContactFwdDynamics DAM, or
    ActionModelImpulseFwdDynamics). None for the dense kinds."""
    from . import multibody as mb
    dam = getattr(model, "differential", None)
    if dam is None and isinstance(model, mb.ActionModelImpulseFwdDynamics):
        dam, imp = model, True
    elif isinstance(dam, mb.DifferentialActionModelFreeFwdDynamics):
        imp = False
    else:
        return None
    robot = dam.state.pinocchio
    par = dof_parents(robot)
    n = len(par)
    L = 2 * n
    nu = 0 if imp else dam.nu
    d = _anc_counts(par)
    sd, sd2 = float(d.sum()), float((d * d).sum())
    if imp:
        nc = dam.impulses.ni
        frames = [dam.impulses.impulses[k].impulse for k in dam.impulses.active]
    else:
        nc = dam.contacts.nc if isinstance(dam, mb.DifferentialActionModelContactFwdDynamics) else 0
        frames = ([dam.contacts.contacts[k].contact for k in dam.contacts.active]
                  if isinstance(dam, mb.DifferentialActionModelContactFwdDynamics) else [])
    fdepth = sum(_frame_depth(robot, f.frame if imp else f._ref.id) for f in frames)
    rnea = 350 * n
    crba = 236 * n + 53 * sd
    jac = C_X * fdepth + 100 * len(frames)
    chol = sd2 + 2 * sd
    solve = 4 * sd + n
    schur = (nc + 1) * solve + 2 * nc * nc * n + nc ** 3 / 3 + 2 * nc * nc + 4 * nc * n if nc else solve
    ceul = 4 * n + (200 if robot.has_freeflyer else 0)
    cc, cd = _cost_terms(dam, n, nu, L, robot, par)
    calc = rnea + crba + jac + chol + schur + ceul + cc
    rnea_d = 4 * rnea + 200 * sd
    minv = n * solve
    kkt = minv + (nc * solve + 2 * nc * nc * n + nc ** 3 + 2 * n * nc * nc + 2 * n * n * nc if nc else 0)
    cder = 20 * nc * L
    dfdx = 2 * (n + nc) ** 2 * L if nc else 2 * n * n * L
    eul = 2 * n * L + (72 * L if robot.has_freeflyer else 0) + 2 * n * nu
    diff = calc + rnea_d + kkt + cder + dfdx + eul + cd
    return float(calc), float(diff)


def horizon_flops(running, terminal):
    """Mean (calc, calcDiff) flops per knot over a horizon (None if any knot is not a
    multibody kind)."""
    vals = [knot_flops(m) for m in list(running) + [terminal]]
    if any(v is None for v in vals):
        return None
    a = np.array(vals)
    return float(a[:, 0].mean()), float(a[:, 1].mean())
