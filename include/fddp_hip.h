/*
 * fddp_hip.h — C ABI of libfddp_hip, the MI355X-native batched FDDP solver.
 *
 * This is the drop-in boundary for the reference's hot path
 *   ShootingProblem::calc/calcDiff + SolverFDDP
 * (reference: /root/reference, a Crocoddyl 1.4.0 fork). One handle owns B
 * independent optimal-control problems that share one knot sequence
 * (T running knots + 1 terminal knot) and solves them together on one GPU.
 *
 * Conventions
 *  - Every floating-point value is IEEE fp64.
 *  - Host arrays are contiguous, batch-major: vectors [b][t][i]; matrix blocks
 *    column-major exactly as Eigen stores them (element (i,j) at j*rows+i).
 *  - Every entry point returns an int status (FDDP_OK == 0, negative on an
 *    argument/runtime error; fddp_last_error() gives the message). No C++
 *    exception crosses the ABI. Numerical failures (the reference's
 *    backward_error / forward_error, src/core/solvers/ddp.cpp:246-251,
 *    fddp.cpp:175-180) are handled per batch element inside fddp_solve,
 *    exactly as SolverFDDP::solve catches them (fddp.cpp:35-60).
 *  - No torch types, no HIP types in signatures. A device stream can be
 *    obtained as an opaque pointer for callers that want to order work.
 *
 * Which reference interface each entry point replaces is cited per function.
 */
#ifndef FDDP_HIP_H_
#define FDDP_HIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- ABI version ----------------------------------------------------------
 * Bumped on every incompatible change of a declaration below; a caller compiled
 * against this header checks fddp_abi_version() == FDDP_ABI_VERSION at start-up.
 *   1  rounds 1-4
 *   2  fddp_iteration_callback returns int (nonzero stops fddp_solve)
 *   3  fddp_calc_diff / fddp_backward_pass / fddp_forward_pass */
#define FDDP_ABI_VERSION 3
int fddp_abi_version(void);

/* ---- status codes -------------------------------------------------------- */
#define FDDP_OK 0
#define FDDP_ERR_INVALID_ARG (-1)   /* reference: throw_pretty("Invalid argument") */
#define FDDP_ERR_RUNTIME (-2)       /* HIP runtime failure */
#define FDDP_ERR_UNSUPPORTED (-3)   /* knot kind / size the device path does not cover */
#define FDDP_ERR_NO_DEVICE (-4)     /* no usable gfx950 device */
#define FDDP_ERR_CALLBACK_ABORT (-5) /* an iteration callback returned nonzero: fddp_solve stopped after that
                                        iteration (out = that iteration's results); reference: an exception
                                        thrown by a CallbackAbstract leaves solve() there (fddp.cpp:92-98) */

/* ---- per-element solve status (fddp_result.status) ----------------------- */
#define FDDP_STATUS_RUNNING 0       /* maxiter reached without convergence (solve returned false) */
#define FDDP_STATUS_CONVERGED 1     /* was_feasible && stop < th_stop (fddp.cpp:100-102) */
#define FDDP_STATUS_REGMAX 2        /* xreg reached regmax (fddp.cpp:41-43, 88-90) */

/* ---- knot model kinds ---------------------------------------------------- */
/* ActionModelLQR (include/crocoddyl/core/actions/lqr.hxx:13-70). nx == ndx.
 * Parameter block (doubles): [hdr0 = drift_free (1/0), hdr1..3 = 0]
 *   Fx(nx*nx) Fu(nx*nu) f0(nx) Lxx(nx*nx) Lxu(nx*nu) Luu(nu*nu) lx(nx) lu(nu) */
#define FDDP_KNOT_LQR 1
/* ActionModelUnicycle (core/actions/unicycle.hxx:13-73). nx=ndx=3, nu=2.
 * Parameter block: [dt, w_x, w_u, 0]  (dt=0.1, cost weights (10, 1) by default) */
#define FDDP_KNOT_UNICYCLE 2
/* IntegratedActionModelEuler (core/integrator/euler.hxx:41-131) around
 * DifferentialActionModelLQR (core/actions/diff-lqr.hxx:13-82), Euclidean
 * state x=(q,v), nq = nv = nx/2.
 * Parameter block: [dt, drift_free, 0, 0]
 *   Fq(nq*nq) Fv(nq*nq) Fu(nq*nu) f0(nq) Lxx(nx*nx) Lxu(nx*nu) Luu(nu*nu) lx(nx) lu(nu) */
#define FDDP_KNOT_EULER_DIFFLQR 3
/* IntegratedActionModelEuler (euler.hxx:41-131) around
 * DifferentialActionModelFreeFwdDynamics (multibody/actions/free-fwddyn.hxx:44-118)
 * with ActuationModelFull (tau = u) and a CostModelSum (cost-sum.hxx:89-160) over
 * a kinematic tree (StateMultibody, multibody/states/multibody.hxx:54-240): revolute
 * joints, optionally below a free-flyer root (JointModelFreeFlyer: q = (p, quat
 * x y z w), v = body twist (linear, angular); nq = nv + 1). nx = nq + nv,
 * ndx = 2 nv; nu = nv (no free-flyer). Variable-size block:
 *   header [dt, nv, ncost, size (doubles, header included)]
 *   gravity(3)  armature(nv)
 *   one 27-double record per joint (a free-flyer root is ONE record for its 6
 *   dofs), parents before children (Pinocchio order):
 *     [type (0 revolute, 1 free-flyer), parent record (-1 = universe), axis(3,
 *     unit, joint frame; unused for the free-flyer), placement in the parent
 *     joint frame R(9, column-major) p(3), body mass, CoM(3, joint frame),
 *     rotational inertia about the CoM (Ixx Iyy Izz Ixy Ixz Iyz)]
 *   ncost cost records in name order (CostModelSum's std::map), each
 *     [type, weight, activation kind, size (doubles, record header included)]
 *     then the payload, then the activation parameters:
 *       kind 0 ActivationModelQuad: ones(nr); 1 WeightedQuad: w(nr);
 *       2 QuadraticBarrier: lb(nr) ub(nr); 3 WeightedQuadraticBarrier: lb ub w
 *       (core/activations/<kind>.hpp; the bounds already shrunk by beta)
 *     payloads by type:
 *     1 CostModelState (state.hxx:130-169): xref(nx); r = diff(xref, x), nr = ndx
 *     2 CostModelControl (control.hxx:56-87): uref(nu)
 *     3 CostModelFramePlacement (frame-placement.hxx:45-80): frame joint,
 *       frame placement in that joint R(9) p(3), Mref^-1 R(9) p(3); nr = 6
 *     4 CostModelFrameTranslation (frame-translation.hxx:50-81): frame joint,
 *       frame placement R(9) p(3), reference translation(3); nr = 3
 *     7 CostModelContactForce (contact-force.hxx:33-74, contact knots only):
 *       [row0, nr, fref(6)]: r = lambda[row0 .. row0+nr) - fref, row0 the
 *       contact's first row (-2: the contact exists but is inactive, lambda = 0)
 *     8 CostModelCoMPosition (com-position.hxx:49-75): cref(3)
 *     9 CostModelContactFrictionCone (contact-friction-cone.hxx:51-91, contact
 *       knots only): [row0, contact rows, nr, A(nr x 3, row-major)]: r = A lambda_lin
 *    10 CostModelFrameVelocity (frame-velocity.hxx:53-84, Euler knots): frame
 *       joint, frame placement R(9) p(3), vref(6) (LOCAL); nr = 6
 * At most 64 dofs, 64 cost records and 64 stacked residual rows with dense
 * Jacobians per knot (the calcDiff LDS plan must fit; fddp_create says why not). */
#define FDDP_KNOT_EULER_FREEFWD 4
/* IntegratedActionModelEuler around DifferentialActionModelContactFwdDynamics
 * (multibody/actions/contact-fwddyn.hxx:59-160) with ActuationModelFloatingBase
 * (actuations/floating-base.hpp:29-40: tau = [0_nun; u], nu = nv - nun; nun = 6
 * on a free-flyer root) and a ContactModelMultiple (contacts/multiple-contacts.hxx)
 * of ContactModel3D / ContactModel6D (contacts/contact-{3d,6d}.hxx, LOCAL frame,
 * Baumgarte gains). Block: the FDDP_KNOT_EULER_FREEFWD layout (header size covers
 * everything; dt = 0 is the biped's pseudo-impulse knot), then
 *   [nun, JMinvJt_damping, ncontact, flag (0; 2 = enable_force: the force
 *    Jacobians the contact-force / friction-cone costs read)]
 *   ncontact active contact records in name order, each
 *     [type (5: 3D, 6: 6D), gains[0], gains[1], size], frame joint, frame
 *     placement in that joint R(9) p(3), then 3D: reference translation(3);
 *     6D: Mref^-1 R(9) p(3)
 * At most 24 stacked contact rows (nc); the Schur complement Jc M^-1 Jc^T +
 * damping I must be positive definite (full-rank Jc or damping > 0). */
#define FDDP_KNOT_EULER_CONTACTFWD 5
/* ActionModelImpulseFwdDynamics (multibody/actions/impulse-fwddyn.hxx:53-127): an
 * action model (no integrator), nu = 0, xnext = (q, v+) with the impulse
 * dynamics [M Jc^T; Jc 0][v+; -Lambda] = [M v; -r_coeff Jc v], cost = costs(x);
 * ImpulseModelMultiple of ImpulseModel3D / 6D (impulses/impulse-{3d,6d}.hxx).
 * Block: the FDDP_KNOT_EULER_FREEFWD layout with dt = 0 (no frame-velocity or
 * force costs), then
 *   [r_coeff, JMinvJt_damping, nimpulse, 1]
 *   nimpulse active impulse records in name order, each
 *     [type (5: 3D, 6: 6D), 0, 0, size = 17], frame joint, frame placement R(9) p(3)
 * calcDiff follows the reference's formula (restitution terms left out of Fx, as
 * impulse-fwddyn.hxx:111-115). At most 24 stacked impulse rows. */
#define FDDP_KNOT_IMPULSEFWD 6

#define FDDP_PARAM_HEADER 4 /* doubles of scalar header in front of every block */

typedef struct {
  int32_t nx;      /* state dimension (ShootingProblem::get_nx, shooting.hxx:25) */
  int32_t ndx;     /* tangent dimension (nx, or nx - 1 on a free-flyer multibody state) */
  int32_t nu_max;  /* max controls over the running knots (shooting.hxx:27-34) */
  int32_t T;       /* number of running knots */
  int32_t B;       /* number of independent problems in the batch */
} fddp_dims;

typedef struct {
  int32_t kind;          /* FDDP_KNOT_* */
  int32_t nu;            /* controls of this knot's model (0 allowed for running knots) */
  int64_t param_offset;  /* offset (doubles) of this knot's block in the parameter pool */
  int64_t param_stride;  /* doubles between batch elements' blocks; 0 = block shared by all */
} fddp_knot_desc;

/* Solver thresholds; defaults = reference constructors
 * (solver-base.cpp:24-25, ddp.cpp:17-31, fddp.cpp:15). */
typedef struct {
  double th_acceptstep;    /* 0.1  */
  double th_stop;          /* 1e-9 */
  double th_grad;          /* 1e-12 */
  double th_stepdec;       /* 0.5  */
  double th_stepinc;       /* 0.01 */
  double th_acceptnegstep; /* 2    */
  double regfactor;        /* 10   */
  double regmin;           /* 1e-9 */
  double regmax;           /* 1e9  */
  int32_t n_alphas;        /* 10   */
  int32_t pad_;
  double alphas[16];       /* 2^-k, k = 0..9 */
} fddp_params;

/* Per-element outcome of fddp_solve: the reference solver's public state
 * after SolverFDDP::solve returns (solver-base.hpp getters). */
typedef struct {
  int32_t status;      /* FDDP_STATUS_* ; solve()'s bool == (status == CONVERGED) */
  int32_t iter;        /* SolverAbstract::get_iter() after return */
  int32_t is_feasible; /* get_is_feasible() */
  int32_t n_iter_run;  /* loop bodies executed (for iterations/s accounting) */
  double cost;         /* get_cost() */
  double stop;         /* get_stop() */
  double xreg;         /* get_xreg() */
  double ureg;         /* get_ureg() */
  double steplength;   /* get_steplength() */
  double dV;           /* get_dV() */
  double dVexp;        /* get_dVexp() */
  double d0, d1;       /* get_d() */
} fddp_result;

typedef struct fddp_handle_s fddp_handle;

/* Fill the reference defaults. Replaces the SolverDDP/SolverFDDP constructors
 * (ddp.cpp:15-37, fddp.cpp:14-15). */
void fddp_default_params(fddp_params* p);

/* Create a batched problem + solver on `device`. Replaces
 * ShootingProblem(x0, runningModels, terminalModel) (shooting.hxx:17-59) and
 * SolverFDDP(problem) (fddp.cpp:14, allocateData ddp.cpp:328-384).
 * knots: T+1 descriptors (running 0..T-1, terminal T). params: the parameter
 * pool (n_params doubles) referenced by the descriptors. All device memory is
 * allocated here, once. */
int fddp_create(const fddp_dims* dims, const fddp_knot_desc* knots, const double* params, int64_t n_params,
                int device, fddp_handle** out);
void fddp_destroy(fddp_handle* h);

/* Message of the last error on this thread ("" if none). */
const char* fddp_last_error(void);

/* Re-upload the parameter pool (same size). Replaces the model setters
 * (e.g. ActionModelLQR::set_Fx, lqr.hxx:128-136) for a live handle. */
int fddp_set_model_params(fddp_handle* h, const double* params, int64_t n_params);

/* Replace the knot sequence and the parameter pool of a live handle (same T,
 * nx, B; every nu <= nu_max), keeping trajectories, gains and solver state.
 * Replaces ShootingProblem::circularAppend / updateNode / updateModel
 * (shooting.hxx:235-346): the caller rotates or swaps models on its side and
 * uploads the new sequence; shared models are still one block. */
int fddp_set_knots(fddp_handle* h, const fddp_knot_desc* knots, const double* params, int64_t n_params);

/* x0 for every element: B*nx. Replaces ShootingProblem::set_x0 (shooting.hxx:391-397). */
int fddp_set_x0(fddp_handle* h, const double* x0);
int fddp_get_x0(fddp_handle* h, double* x0);

/* SolverFDDP thresholds. Replaces the setters (ddp.cpp:420-486,
 * solver-base.cpp:159-173, fddp.cpp:229-235) with the same validation. */
int fddp_set_params(fddp_handle* h, const fddp_params* p);
int fddp_get_params(fddp_handle* h, fddp_params* p);

/* Warm start. xs: B*(T+1)*nx or NULL (= state.zero()), us: B*T*nu_max or NULL
 * (= zeros). Replaces SolverAbstract::setCandidate (solver-base.cpp:42-67). */
int fddp_set_candidate(fddp_handle* h, const double* xs, const double* us, int is_feasible);
/* The same from device-resident arrays (same dense layout, device pointers on the
 * handle's device; NULL = state.zero() / zeros). Enqueued on the handle's stream,
 * no host synchronisation: a warm start kept in HBM and re-applied before every
 * solve, as the reference's benchmarks call solve(xs, us, ...) with the same
 * arrays each time (benchmark/bipedal_walk_optctrl.py:39-43,
 * quadrupedal-gaits-optctrl.cpp:60-64). */
int fddp_set_candidate_device(fddp_handle* h, const double* xs, const double* us, int is_feasible);

/* SolverFDDP::solve (fddp.cpp:19-105) from the current candidate, for every
 * element at once, each element with its own state machine. reg_init may be
 * NaN (→ regmin). out: B results (may be NULL). Runs on the handle's stream and
 * returns after the results are on the host. */
int fddp_solve(fddp_handle* h, int maxiter, int is_feasible, double reg_init, fddp_result* out);

/* Per-iteration callback of fddp_solve: the reference calls every
 * CallbackAbstract once per loop body, after the regularisation update and
 * stoppingCriteria and before the convergence test (fddp.cpp:92-98; an element
 * that aborts at regmax returns before it, fddp.cpp:41-43,88-90). `iter` is the
 * loop counter iter_ of that body; `results` the B elements' state at that point
 * (results[b].iter == iter for the reported ones); reported[b] != 0 for the
 * elements whose callbacks the reference would call in this body (the others
 * have converged or aborted earlier, or aborted in it). Runs on the calling
 * thread, between iterations (the device is idle): the callback may call the
 * getters and the step API of the same handle, not fddp_solve. Setting a
 * callback makes fddp_solve read the states back once per iteration.
 * Returns 0 to go on; nonzero stops fddp_solve after this iteration (the
 * reference's exception leaving solve() inside the loop body): fddp_solve then
 * fills `out` with this iteration's results (iter, xs, us, regularisation stay
 * where that body left them) and returns FDDP_ERR_CALLBACK_ABORT. */
typedef int (*fddp_iteration_callback)(void* user, int iter, const fddp_result* results, const int32_t* reported,
                                       int B);
/* NULL clears it. Replaces SolverAbstract::setCallbacks (solver-base.cpp:69-73). */
int fddp_set_callback(fddp_handle* h, fddp_iteration_callback cb, void* user);

/* Diagnostics of the last line search of fddp_solve (for the bench's rollout
 * accounting): the trial-group size it used (1: the serial search; g > 1: g alpha
 * trials per element evaluated together, SolverFDDP's acceptance order kept) and
 * the number of rollout dispatches it made. */
int fddp_get_line_search_info(fddp_handle* h, int* group_size, int* launches);

/* Results of the last solve / current solver state per element. */
int fddp_get_results(fddp_handle* h, fddp_result* out);
/* xs: B*(T+1)*nx, us: B*T*nu_max. on_device != 0: `out` is a device pointer
 * on the handle's device (copy is enqueued on the handle's stream). */
int fddp_get_xs(fddp_handle* h, double* out, int on_device);
int fddp_get_us(fddp_handle* h, double* out, int on_device);

/* ---- step API: the SolverDDP/SolverFDDP methods one at a time --------------
 * Used for parity tests against the reference's own step-level tests
 * (unittest/bindings/test_solvers.py:38-96). cost/dV/d/stop outputs are B (or
 * B*2) doubles, may be NULL. */
/* ShootingProblem::calc (shooting.hxx:133-161) at the current candidate. */
int fddp_problem_calc(fddp_handle* h, double* cost);
/* ShootingProblem::calcDiff (shooting.hxx:164-195) at the current candidate. */
int fddp_problem_calc_diff(fddp_handle* h, double* cost);
/* SolverDDP::computeDirection(recalc) (ddp.cpp:120-125): calcDiff (with the
 * iter==0 calc and the gaps, ddp.cpp:157-178) + backwardPass (ddp.cpp:180-253).
 * status: B ints, 0 ok / 1 backward_error (may be NULL). */
int fddp_compute_direction(fddp_handle* h, int recalc, int32_t* status);
/* The three phases of computeDirection / tryStep one at a time, as the reference's
 * SolverDDP exposes them (bindings/python/crocoddyl/core/solvers/ddp.cpp:70-82) and its
 * timing harness calls them (benchmark/arm-kinova-codegen.cpp:260-285).
 * SolverDDP::calcDiff (ddp.cpp:157-178): problem.calc when iter_ == 0, problem.calcDiff,
 * then the gaps fs (or zero gaps when the candidate just became feasible). cost: B
 * doubles (cost_, the return value), may be NULL. */
int fddp_calc_diff(fddp_handle* h, double* cost);
/* SolverDDP::backwardPass (ddp.cpp:180-253) with computeGains (ddp.cpp:298-310) and the
 * sums of SolverFDDP::updateExpectedImprovement (fddp.cpp:126-147), on the derivatives of
 * the last calc_diff. K, k, Vx, Vxx, Q* are read with fddp_get_quantity (Vx, Vxx, Q* in
 * debug mode). status: B ints, 0 ok / 1 backward_error (the reference throws; here the
 * element keeps the blocks of the failed sweep), may be NULL. */
int fddp_backward_pass(fddp_handle* h, int32_t* status);
/* SolverFDDP::forwardPass(stepLength) (fddp.cpp:149-225): the rollout of the current
 * policy into xs_try / us_try (fddp_get_xs_try / us_try) and cost_try, without the
 * cost difference tryStep returns. stepLength outside [0, 1] is an argument error
 * (fddp.cpp:150-153). cost_try: B doubles, status: B ints (1 forward_error); either
 * may be NULL. */
int fddp_forward_pass(fddp_handle* h, double step_length, double* cost_try, int32_t* status);
/* SolverFDDP::updateExpectedImprovement (fddp.cpp:126-147). */
int fddp_update_expected_improvement(fddp_handle* h);
/* SolverDDP::tryStep / SolverFDDP::forwardPass (ddp.cpp:127-130, fddp.cpp:149-225).
 * dV = cost - cost_try; status: 0 ok / 1 forward_error. */
int fddp_try_step(fddp_handle* h, double alpha, double* dV, int32_t* status);
/* SolverFDDP::expectedImprovement (fddp.cpp:107-124) after a tryStep. d: B*2. */
int fddp_expected_improvement(fddp_handle* h, double* d);
/* SolverDDP::stoppingCriteria (ddp.cpp:132-142). */
int fddp_stopping_criteria(fddp_handle* h, double* stop);
/* Solver members the step API depends on, for every element: iter_ (the
 * iter_==0 calc in SolverDDP::calcDiff, ddp.cpp:158), xreg_/ureg_ (NaN on a
 * fresh solver, solver-base.cpp:19-20) and was_feasible_. */
int fddp_set_solver_state(fddp_handle* h, int iter, double xreg, double ureg, int was_feasible);
/* xs_try/us_try of the last tryStep. */
int fddp_get_xs_try(fddp_handle* h, double* out);
int fddp_get_us_try(fddp_handle* h, double* out);

/* ---- inspection of per-knot data (ActionData members, action-base.hpp:101-142,
 * and SolverDDP getters ddp.hpp:60-271). Sizes per element per knot below.  */
#define FDDP_Q_FX 0   /* (T+1) x ndx*ndx  */
#define FDDP_Q_FU 1   /* (T+1) x ndx*nu_max */
#define FDDP_Q_LXX 2  /* (T+1) x ndx*ndx  */
#define FDDP_Q_LXU 3  /* (T+1) x ndx*nu_max */
#define FDDP_Q_LUU 4  /* (T+1) x nu_max*nu_max */
#define FDDP_Q_LX 5   /* (T+1) x ndx */
#define FDDP_Q_LU 6   /* (T+1) x nu_max */
#define FDDP_Q_XNEXT 7 /* T x nx (data[t].xnext of the current candidate) */
#define FDDP_Q_FS 8   /* (T+1) x ndx (gaps) */
#define FDDP_Q_K 9    /* T x nu_max*ndx (K_, nu x ndx col-major) */
#define FDDP_Q_KV 10  /* T x nu_max (k_) */
/* The following need fddp_set_debug(h, 1) before the backward pass. */
#define FDDP_Q_VXX 11 /* (T+1) x ndx*ndx */
#define FDDP_Q_VX 12  /* (T+1) x ndx */
#define FDDP_Q_QXX 13 /* T x ndx*ndx */
#define FDDP_Q_QXU 14 /* T x ndx*nu_max */
#define FDDP_Q_QUU 15 /* T x nu_max*nu_max */
#define FDDP_Q_QX 16  /* T x ndx */
#define FDDP_Q_QU 17  /* T x nu_max */
#define FDDP_Q_QUU_INV 18 /* T x nu_max*nu_max: SolverBoxFDDP::get_Quu_inv (box-fddp.cpp:162);
                             like the reference, a knot keeps its last value
                             (zero initially) while the box QP does not run on it */
#define FDDP_Q_COST 19 /* (T+1) x 1: data[t].cost of the current candidate (after
                          fddp_problem_calc / calc_diff or a solve) */
int fddp_get_quantity(fddp_handle* h, int which, double* out);
/* Store Vxx/Vx/Q* per knot during backward passes (costs HBM traffic). */
int fddp_set_debug(fddp_handle* h, int on);

/* ---- control limits and the box-constrained solver ------------------------ */
/* Solver variants of a handle. FDDP: SolverFDDP (fddp.cpp:14-225); control
 * limits are ignored, as SolverFDDP ignores them. BOXFDDP: SolverBoxFDDP
 * (box-fddp.cpp:15-160): on knots whose model has control limits, and once the
 * element is feasible, computeGains solves a box QP (BoxQP, box-qp.cpp:51-182)
 * warm-started at the previous k; the forward pass clamps us_try to the
 * limits. The reference's SolverBoxFDDP ctor also sets th_stop = 5e-5; this
 * ABI leaves th_stop to fddp_set_params (the facades apply the default). */
#define FDDP_SOLVER_FDDP 0
#define FDDP_SOLVER_BOXFDDP 1
/* Replaces constructing SolverBoxFDDP(problem) instead of SolverFDDP(problem)
 * (box-fddp.cpp:15-29). FDDP_ERR_UNSUPPORTED if BOXFDDP is asked with
 * nu_max > 64 (one wave holds one box QP). */
int fddp_set_solver_kind(fddp_handle* h, int kind);
int fddp_get_solver_kind(fddp_handle* h, int* kind);
/* Control limits of every running knot and element: u_lb, u_ub are
 * B*T*nu_max doubles ([b][t][i], entries i >= nu(t) ignored); -inf / +inf =
 * no limit. Replaces ActionModelAbstract::set_u_lb / set_u_ub
 * (action-base.hxx:122-144): a knot "has control limits" iff any of its
 * u_lb is finite and any of its u_ub is finite (update_has_control_limits,
 * action-base.hxx:142-144). NULL, NULL removes all limits. */
int fddp_set_control_limits(fddp_handle* h, const double* u_lb, const double* u_ub);

/* Projected-Newton box QP  x = argmin 0.5 x'Hx + q'x  s.t. lb <= x <= ub
 * (BoxQP, box-qp.hpp:29-206, box-qp.cpp:14-182). */
typedef struct {
  int32_t maxiter;       /* 100 */
  int32_t n_alphas;      /* 10 */
  double th_acceptstep;  /* 0.1 */
  double th_grad;        /* 1e-9 (SolverBoxFDDP's own QP uses 1e-5) */
  double reg;            /* 1e-9 (SolverBoxFDDP's own QP uses 0) */
  double alphas[16];     /* 2^-k, k = 0..9 */
} fddp_boxqp_params;
/* BoxQP(nx) constructor defaults (box-qp.hpp:92-93, box-qp.cpp:14-46). */
void fddp_boxqp_default_params(fddp_boxqp_params* p);
/* B independent box QPs of dimension nx (1 <= nx <= 64) solved on `device`,
 * one wave each. Host arrays: H B*nx*nx (column-major), q, lb, ub, xinit B*nx.
 * Outputs (host; any may be NULL): x B*nx (BoxQPSolution::x); free_mask B
 * (bit i set = i in BoxQPSolution::free_idx, the rest is clamped_idx);
 * inv_mask B (the free set Hff_inv was factorised on) and Hff_inv B*nx*nx,
 * the inverse embedded at inv_mask's indices (zero elsewhere): the
 * reference's compact nf x nf Hff_inv is its inv_mask rows/cols in order;
 * status B: 0 ok, 1 the LLT of a free Hessian failed (the reference throws
 * "backward_error"). Replaces BoxQP::solve (box-qp.cpp:51-182). */
int fddp_boxqp_solve(int device, int B, int nx, const double* H, const double* q, const double* lb,
                     const double* ub, const double* xinit, const fddp_boxqp_params* p, double* x,
                     uint64_t* free_mask, uint64_t* inv_mask, double* Hff_inv, int32_t* status);

/* ---- MPC plumbing -------------------------------------------------------- */
/* Receding-horizon shift on device: x0 <- xs[1]; xs[t] <- xs[t+1] (last kept);
 * us[t] <- us[t+1] (last kept). The device analogue of a user's shift between
 * warm-started solve(maxiter=1) calls (benchmark/quadrupedal-gaits-optctrl.cpp:63). */
int fddp_mpc_shift(fddp_handle* h);

/* ---- runtime ------------------------------------------------------------ */
int fddp_synchronize(fddp_handle* h);
/* Opaque hipStream_t of the handle. */
int fddp_get_stream(fddp_handle* h, void** stream);
/* Device time (ms) of the named kernel class accumulated since the last reset,
 * measured with HIP events on the handle's stream. which: 0 calc, 1 calcDiff,
 * 2 backward, 3 forward/line-search. counts: launches. */
int fddp_get_timing(fddp_handle* h, double* ms_out /*4*/, int64_t* counts_out /*4*/);
int fddp_set_timing(fddp_handle* h, int on);
/* Number of bytes of device memory owned by the handle. */
int64_t fddp_device_bytes(fddp_handle* h);

#ifdef __cplusplus
}
#endif

#endif /* FDDP_HIP_H_ */
