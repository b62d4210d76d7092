// Multibody knots on the device: IntegratedActionModelEuler ∘
// DifferentialAction{Free,Contact}FwdDynamics and ActionModelImpulseFwdDynamics
// (CostModelSum of State / Control / FramePlacement / FrameTranslation / CoMPosition /
// ContactForce costs) over a kinematic tree of revolute joints below either the
// universe or a free-flyer root (StateMultibody on SE(3) x R^n).
//
// Reference: include/crocoddyl/core/integrator/euler.hxx:41-131,
//   multibody/actions/{free,contact,impulse}-fwddyn.hxx, multibody/costs/cost-sum.hxx:89-160,
//   multibody/costs/*.hxx, multibody/states/multibody.hxx:54-240; the rigid-body
//   arithmetic the reference takes from Pinocchio (aba, computeRNEADerivatives,
//   updateFramePlacement, getFrameJacobian, integrate / difference / dIntegrate /
//   dIntegrateTransport / dDifference, exp6, log6, Jexp6, Jlog6) is computed here as:
//   * forward dynamics: a = (M + diag(armature))^-1 (tau - nle), with RNEA and the
//     composite-rigid-body algorithm in world coordinates, where every recursion is
//     an ancestor / subtree sum evaluated one dof per lane (a free-flyer is six dofs
//     that share one body), and the solve by Gauss-Jordan with one column per lane.
//     (The reference's default path is ABA, the same function.)
//   * derivatives: the world-frame analytic RNEA derivatives, one lane per tangent
//     direction (q_j or v_j): every world quantity of the subtree moved by q_j is
//     transported by the joint motion S_j, and what is left reduces to the
//     subtree composites (composite inertia, and P_k = sum_b dY_b-like terms), so
//     d tau_k / d q_j is a 6-vector dot product per pair (see dtau_direction);
//     da/dx = -Kinv (dtau/dx; da0/dx) as computeABADerivatives /
//     the contact KKT inverse (contact-fwddyn.hxx:127-140).
//   * frame-cost Jacobians: the frame's motion under S_j pushed through log6 in dual
//     numbers, which is Jlog6(rMf) * fJf (frame-placement.hxx:63-66);
//   * free-flyer state: M exp6(dq) with Eigen's quaternion extraction, log6(M0^-1 M1),
//     Jexp6 / Jlog6 columns in dual numbers, Ad(exp6(dq)^-1) (pinocchio's
//     SpecialEuclideanOperationTpl<3>).
// Parameter-block layout: include/fddp_hip.h (FDDP_KNOT_EULER_FREEFWD).
#pragma once

#include <type_traits>

#include "fddp_device.hpp"

// Everything except the workgroup drivers (knot_calc, knot_calc_diff,
// gauss_jordan) is __host__ __device__, so the same arithmetic is unit-tested
// on the CPU against the oracle (tests/test_multibody_host.py).
#define MB_HD __host__ __device__
#ifndef MB_DUMP
// (tools/mb_probe: copies an LDS matrix, rows x cols at leading dimension ld, out of
// the calcDiff for the parity diagnosis; every thread calls it between phases)
#define MB_DUMP(slot, ptr, rows, cols, ld)
#endif

// On the device every multibody record (parameter block) and the work area live in
// LDS; the record / work-area accessors re-assert it where the pointer is formed, so
// the accesses compile to ds_* even where the address-space inference loses the
// entry's assumption (flat accesses to LDS pay a full round trip each). The host
// emulation (tests/cpp/mb_host.cpp) reads ordinary memory.
// A store to the caller's output blocks, which are in HBM: through a global pointer,
// so the compiler emits global_store instead of a flat store that every later LDS
// access of the wave must wait behind (flat may alias LDS).
MB_HD __forceinline__ void mb_gstore(double* p, double v) {
#if defined(__HIP_DEVICE_COMPILE__)
  *(__attribute__((address_space(1))) double*)p = v;
#else
  *p = v;
#endif
}
// two consecutive doubles (16-B aligned) in one store
MB_HD __forceinline__ void mb_gstore2(double* p, double v0, double v1) {
#if defined(__HIP_DEVICE_COMPILE__)
  *(__attribute__((address_space(1))) double2*)p = make_double2(v0, v1);
#else
  p[0] = v0;
  p[1] = v1;
#endif
}
// A fresh register copy of v (device: an empty asm the optimiser cannot see through), so
// a value live across the whole kernel is reloaded from its spill slot once, here.
template <class T>
MB_HD __forceinline__ T mb_launder(T v) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (sizeof(T) == 8) {
    long long x;
    __builtin_memcpy(&x, &v, 8);
    asm volatile("" : "+v"(x));
    __builtin_memcpy(&v, &x, 8);
  } else {
    int x;
    __builtin_memcpy(&x, &v, 4);
    asm volatile("" : "+v"(x));
    __builtin_memcpy(&v, &x, 4);
  }
#endif
  return v;
}
template <class T>
MB_HD __forceinline__ T* mb_lds(T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return ::fddp::lds_ptr(p);
#else
  return p;
#endif
}

namespace fddp {
namespace mb {

typedef unsigned long long Mask;  // one bit per dof
constexpr int kMaxJ = 64;         // dofs (nv)
constexpr int kJRec = 27;         // doubles per joint record
constexpr int kCHdr = 4;          // doubles of a cost record's header
constexpr int kMaxJacCosts = 8;   // costs with a dense residual Jacobian (frame, CoM, free-flyer state)
constexpr int kMaxNc = 24;        // stacked contact rows (FDDP_KNOT_EULER_CONTACTFWD)
constexpr int kMbDiffNT = 256;    // threads of the knot-parallel calcDiff workgroup
enum { J_REVOLUTE = 0, J_FREEFLYER = 1 };
// Cost record types; contact records (after the costs) use 5 / 6 and the same
// frame payload as the frame costs, so frame_residual serves both.
enum {
  C_STATE = 1,
  C_CONTROL = 2,
  C_FRAME_PLACEMENT = 3,
  C_FRAME_TRANSLATION = 4,
  C_CONTACT_3D = 5,
  C_CONTACT_6D = 6,
  C_CONTACT_FORCE = 7,  // cost on a contact's force: payload [row0, nr, fref(6)] (contact-force.hxx)
  C_COM_POSITION = 8,   // r = com(q) - cref: payload [cref(3)] (com-position.hxx:49-75)
  C_FRICTION_CONE = 9,  // r = A lambda_lin: payload [row0, nc, nr, A (nr x 3 row-major)]
                        // (contact-friction-cone.hxx:51-91)
  C_FRAME_VELOCITY = 10  // r = LOCAL frame velocity - vref: frame payload + vref(6) (frame-velocity.hxx:53-84)
};
// Activation of a cost record: header slot 2 (core/activations/*.hpp)
enum { A_QUAD = 0, A_WEIGHTED_QUAD = 1, A_QUAD_BARRIER = 2, A_WEIGHTED_QUAD_BARRIER = 3 };
constexpr int kInactiveForceRow = -2;  // contact-force cost on an inactive contact: lambda = 0, no Jacobians

struct Blk {
  double dt;
  int nj;   // nv: dofs
  int nq;   // nv + 1 with a free-flyer root
  int nb;   // joint records (pinocchio joints)
  bool ff;  // record 0 is a free-flyer (dofs 0..5: base twist, body on dof 5)
  int ncost;
  const double* g;    // gravity (3)
  const double* arm;  // armature (nv)
  const double* J;    // joint records
  const double* C;    // cost records
  // contact section (DifferentialActionModelContactFwdDynamics); ncon == 0 without
  int nun;            // leading unactuated dofs: tau = [0_nun; u], nu = nj - nun
  int ncon, nc;       // active contact records, stacked rows
  double damping;     // JMinvJt_damping
  const double* K;    // contact records
  // impulse section instead (ActionModelImpulseFwdDynamics, nu = 0)
  bool impulse;
  double r_coeff;     // restitution coefficient
  bool enable_force;  // contact section flag 2: force Jacobians for CostModelContactForce
};

MB_HD inline Blk parse(const double* P) {
  Blk b;
  b.dt = P[0];
  b.nj = (int)P[1];
  b.ncost = (int)P[2];
  b.g = P + FDDP_PARAM_HEADER;
  b.arm = b.g + 3;
  b.J = b.arm + b.nj;
  b.ff = (int)b.J[0] == J_FREEFLYER;
  b.nb = b.ff ? b.nj - 5 : b.nj;
  b.nq = b.ff ? b.nj + 1 : b.nj;
  b.C = b.J + (int64_t)kJRec * b.nb;
  const double* e = b.C;
  for (int k = 0; k < b.ncost; ++k) e += (int)e[3];
  b.nun = 0;
  b.ncon = b.nc = 0;
  b.damping = 0.;
  b.K = e;
  b.impulse = false;
  b.enable_force = false;
  b.r_coeff = 0.;
  if (e - P < (int64_t)P[3]) {  // [nun | r_coeff, damping, ncontact, 0 | 1 | 2] + records
    b.impulse = (int)e[3] == 1;
    b.enable_force = (int)e[3] == 2;
    b.nun = b.impulse ? b.nj : (int)e[0];
    b.r_coeff = b.impulse ? e[0] : 0.;
    b.damping = e[1];
    b.ncon = (int)e[2];
    b.K = e + 4;
    const double* r = b.K;
    for (int k = 0; k < b.ncon; ++k) {
      b.nc += (int)r[0] == C_CONTACT_3D ? 3 : 6;
      r += (int)r[3];
    }
  }
  return b;
}

// ---- 3-vectors / rotations (column-major 3x3: R[c*3 + r]) ------------------
MB_HD __forceinline__ void cross3(const double* a, const double* b, double* o) {
  const double x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
  o[0] = x;
  o[1] = y;
  o[2] = z;
}
MB_HD __forceinline__ double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
MB_HD __forceinline__ void matvec3(const double* R, const double* v, double* o) {  // o = R v
  const double x = R[0] * v[0] + R[3] * v[1] + R[6] * v[2];
  const double y = R[1] * v[0] + R[4] * v[1] + R[7] * v[2];
  const double z = R[2] * v[0] + R[5] * v[1] + R[8] * v[2];
  o[0] = x;
  o[1] = y;
  o[2] = z;
}
MB_HD __forceinline__ void matTvec3(const double* R, const double* v, double* o) {  // o = R^T v
  const double x = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
  const double y = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
  const double z = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
  o[0] = x;
  o[1] = y;
  o[2] = z;
}
MB_HD __forceinline__ void matmul3(const double* A, const double* B, double* O) {  // O = A B
  for (int c = 0; c < 3; ++c) matvec3(A, B + 3 * c, O + 3 * c);
}
MB_HD __forceinline__ void matTmul3(const double* A, const double* B, double* O) {  // O = A^T B
  for (int c = 0; c < 3; ++c) matTvec3(A, B + 3 * c, O + 3 * c);
}

// Spatial algebra in (linear, angular) order, as Pinocchio's Motion / Force.
// actInv on a motion by M = (R, p): lin' = R^T (v - p x w), ang' = R^T w.
MB_HD __forceinline__ void motion_act_inv(const double* R, const double* p, const double* m, double* o) {
  double t[3];
  cross3(p, m + 3, t);
  t[0] = m[0] - t[0];
  t[1] = m[1] - t[1];
  t[2] = m[2] - t[2];
  matTvec3(R, t, o);
  matTvec3(R, m + 3, o + 3);
}
// act on a force (child -> parent): f' = R f, n' = R n + p x f'.
MB_HD __forceinline__ void force_act(const double* R, const double* p, const double* f, double* o) {
  double ff[3], nn[3], t[3];
  matvec3(R, f, ff);
  matvec3(R, f + 3, nn);
  cross3(p, ff, t);
  o[0] = ff[0];
  o[1] = ff[1];
  o[2] = ff[2];
  o[3] = nn[0] + t[0];
  o[4] = nn[1] + t[1];
  o[5] = nn[2] + t[2];
}
// m1 x_motion m2 = (w1 x v2 + v1 x w2, w1 x w2)
MB_HD __forceinline__ void cross_m(const double* m1, const double* m2, double* o) {
  double a[3], b[3], c[3];
  cross3(m1 + 3, m2, a);
  cross3(m1, m2 + 3, b);
  cross3(m1 + 3, m2 + 3, c);
  o[0] = a[0] + b[0];
  o[1] = a[1] + b[1];
  o[2] = a[2] + b[2];
  o[3] = c[0];
  o[4] = c[1];
  o[5] = c[2];
}
// m x_force f = (w x f, w x n + v x f)
MB_HD __forceinline__ void cross_f(const double* m, const double* f, double* o) {
  double a[3], b[3], c[3];
  cross3(m + 3, f, a);
  cross3(m + 3, f + 3, b);
  cross3(m, f, c);
  o[0] = a[0];
  o[1] = a[1];
  o[2] = a[2];
  o[3] = b[0] + c[0];
  o[4] = b[1] + c[1];
  o[5] = b[2] + c[2];
}
// Inertia (mass m, CoM c, rotational inertia Ic about the CoM: xx yy zz xy xz yz)
// times a motion: f = m (v - c x w), n = Ic w + c x f.
MB_HD __forceinline__ void inertia_mul(double m, const double* c, const double* I6, const double* mo, double* o) {
  double t[3];
  cross3(c, mo + 3, t);
  const double f0 = m * (mo[0] - t[0]), f1 = m * (mo[1] - t[1]), f2 = m * (mo[2] - t[2]);
  const double w0 = mo[3], w1 = mo[4], w2 = mo[5];
  const double n0 = I6[0] * w0 + I6[3] * w1 + I6[4] * w2;
  const double n1 = I6[3] * w0 + I6[1] * w1 + I6[5] * w2;
  const double n2 = I6[4] * w0 + I6[5] * w1 + I6[2] * w2;
  const double f[3] = {f0, f1, f2};
  cross3(c, f, t);
  o[0] = f0;
  o[1] = f1;
  o[2] = f2;
  o[3] = n0 + t[0];
  o[4] = n1 + t[1];
  o[5] = n2 + t[2];
}
MB_HD __forceinline__ double dot6(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}

// Joint record accessors: [type, parent record (-1 universe), axis(3), placement
// R(9) p(3), mass, CoM(3), I(6)]
struct JRec {
  const double* r;
  MB_HD JRec(const Blk& b, int i) : r(mb_lds(b.J + (int64_t)kJRec * i)) {}
  MB_HD int type() const { return (int)r[0]; }
  MB_HD int parent() const { return (int)r[1]; }
  MB_HD const double* axis() const { return r + 2; }
  MB_HD const double* Rpl() const { return r + 5; }
  MB_HD const double* ppl() const { return r + 14; }
  MB_HD double mass() const { return r[17]; }
  MB_HD const double* com() const { return r + 18; }
  MB_HD const double* I6() const { return r + 21; }
};

// ---- dofs and bodies --------------------------------------------------------
// Dof d is one lane. A free-flyer record expands into dofs 0..5 (base twist:
// linear 0..2 along, angular 3..5 about the base axes) that share one body, whose
// inertia sits on dof 5; placements compose along 0 -> 1 -> .. -> 5 with the base
// pose on dof 0 and identities after it. Every other record is one revolute dof.
MB_HD __forceinline__ int rec_of(const Blk& b, int d) { return b.ff ? (d < 6 ? 0 : d - 5) : d; }
// the dof that carries record r's body (and its frames)
MB_HD __forceinline__ int dof_of_rec(const Blk& b, int r) { return b.ff ? (r == 0 ? 5 : r + 5) : r; }
// configuration index of a revolute dof
MB_HD __forceinline__ int qof(const Blk& b, int d) { return b.ff ? d + 1 : d; }
// the dof carrying the parent body (-1: universe)
MB_HD __forceinline__ int body_parent(const Blk& b, int d) {
  if (b.ff && d < 6) return -1;
  const int pr = JRec(b, rec_of(b, d)).parent();
  return pr < 0 ? -1 : dof_of_rec(b, pr);
}
// placement composition parent (free-flyer dofs chain 0 -> 5)
MB_HD __forceinline__ int chain_parent(const Blk& b, int d) { return (b.ff && d < 6) ? d - 1 : body_parent(b, d); }
MB_HD __forceinline__ Mask own_mask(const Blk& b, int d) { return (b.ff && d < 6) ? Mask(0x3F) : (Mask(1) << d); }
// dofs whose body is an ancestor-or-self of d's body
MB_HD inline Mask anc_mask(const Blk& b, int d) {
  Mask m = own_mask(b, d);
  for (int k = body_parent(b, d); k >= 0; k = body_parent(b, k)) m |= own_mask(b, k);
  return m;
}
MB_HD __forceinline__ bool carries_body(const Blk& b, int d) { return !(b.ff && d < 5); }
// joint-frame axis of dof d; prismatic: translation along it (free-flyer 0..2)
MB_HD __forceinline__ bool dof_prismatic(const Blk& b, int d) { return b.ff && d < 3; }
MB_HD __forceinline__ void dof_axis(const Blk& b, int d, double* ax) {
  if (b.ff && d < 6) {
    ax[0] = d % 3 == 0 ? 1. : 0.;
    ax[1] = d % 3 == 1 ? 1. : 0.;
    ax[2] = d % 3 == 2 ? 1. : 0.;
  } else {
    const double* a = JRec(b, rec_of(b, d)).axis();
    ax[0] = a[0];
    ax[1] = a[1];
    ax[2] = a[2];
  }
}

// R = Rpl * exp(q [axis]x)  (Rodrigues: c I + s [a]x + (1 - c) a a^T)
MB_HD inline void joint_rotation(const double* Rpl, const double* ax, double q, double* R) {
  double s, c;
  sincos(q, &s, &c);
  const double oc = 1. - c;
  double Rj[9];
  Rj[0] = c + oc * ax[0] * ax[0];
  Rj[1] = oc * ax[1] * ax[0] + s * ax[2];
  Rj[2] = oc * ax[2] * ax[0] - s * ax[1];
  Rj[3] = oc * ax[0] * ax[1] - s * ax[2];
  Rj[4] = c + oc * ax[1] * ax[1];
  Rj[5] = oc * ax[2] * ax[1] + s * ax[0];
  Rj[6] = oc * ax[0] * ax[2] + s * ax[1];
  Rj[7] = oc * ax[1] * ax[2] - s * ax[0];
  Rj[8] = c + oc * ax[2] * ax[2];
  matmul3(Rpl, Rj, R);
}

// Eigen QuaternionBase::toRotationMatrix, quaternion (x, y, z, w); column-major R
MB_HD inline void quat_to_R(const double* qv, double* R) {
  const double x = qv[0], y = qv[1], z = qv[2], w = qv[3];
  const double tx = 2. * x, ty = 2. * y, tz = 2. * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w;
  const double txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  R[0] = 1. - (tyy + tzz);
  R[1] = txy + twz;
  R[2] = txz - twy;
  R[3] = txy - twz;
  R[4] = 1. - (txx + tzz);
  R[5] = tyz + twx;
  R[6] = txz + twy;
  R[7] = tyz - twx;
  R[8] = 1. - (txx + tyy);
}

// Eigen's quaternion from a rotation matrix (quaternionbase_assign_impl), with the
// index selection written as explicit selects (no runtime-indexed arrays).
MB_HD inline void R_to_quat(const double* R, double* q) {
  auto at = [&](int r, int c) { return R[c * 3 + r]; };
  const double t = at(0, 0) + at(1, 1) + at(2, 2);
  if (t > 0.) {
    double s = sqrt(t + 1.);
    q[3] = 0.5 * s;
    s = 0.5 / s;
    q[0] = (at(2, 1) - at(1, 2)) * s;
    q[1] = (at(0, 2) - at(2, 0)) * s;
    q[2] = (at(1, 0) - at(0, 1)) * s;
    return;
  }
  int i = 0;
  if (at(1, 1) > at(0, 0)) i = 1;
  if (at(2, 2) > (i == 0 ? at(0, 0) : at(1, 1))) i = 2;
  if (i == 0) {
    double s = sqrt(at(0, 0) - at(1, 1) - at(2, 2) + 1.);
    q[0] = 0.5 * s;
    s = 0.5 / s;
    q[3] = (at(2, 1) - at(1, 2)) * s;
    q[1] = (at(1, 0) + at(0, 1)) * s;
    q[2] = (at(2, 0) + at(0, 2)) * s;
  } else if (i == 1) {
    double s = sqrt(at(1, 1) - at(2, 2) - at(0, 0) + 1.);
    q[1] = 0.5 * s;
    s = 0.5 / s;
    q[3] = (at(0, 2) - at(2, 0)) * s;
    q[2] = (at(2, 1) + at(1, 2)) * s;
    q[0] = (at(0, 1) + at(1, 0)) * s;
  } else {
    double s = sqrt(at(2, 2) - at(0, 0) - at(1, 1) + 1.);
    q[2] = 0.5 * s;
    s = 0.5 / s;
    q[3] = (at(1, 0) - at(0, 1)) * s;
    q[0] = (at(0, 2) + at(2, 0)) * s;
    q[1] = (at(1, 2) + at(2, 1)) * s;
  }
}

// Phase executor: run(f) calls f(lane) for every thread of the workgroup and
// then synchronises (device), or for lanes 0..nt-1 in order (host emulation,
// tests/test_multibody_host.py). Within one phase no lane reads what another
// lane writes, so both orders give the same result. run_w0(f): a phase only
// wave 0 works in, closed by a wave-level fence instead of a workgroup barrier
// (the other waves skip ahead to the next sync()); sync(): the barrier that
// hands wave-0 results back to the whole workgroup.
// Everything the device executor runs is inlined into the kernel: LDS pointers
// keep their address space only through inlining (an outlined phase or helper
// takes them as generic pointers and reaches LDS with flat instructions, at
// global-memory latency).
struct DevExec {
  int nt;
  template <class F>
  __device__ __forceinline__ void run(F f) const {
    [[clang::always_inline]] f((int)threadIdx.x);
    __syncthreads();
  }
  template <class F>
  __device__ __forceinline__ void run_w0(F f) const {
    if (threadIdx.x < 64) {
      [[clang::always_inline]] f((int)threadIdx.x);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  __device__ void sync() const { __syncthreads(); }
  // an LDS pointer re-typed through the LDS address space (fddp_device.hpp lds_ptr)
  template <class T>
  __device__ __forceinline__ T* lds(T* p) const {
    return lds_ptr(p);
  }
};
struct HostExec {
  int nt;
  template <class F>
  void run(F f) const {
    for (int l = 0; l < nt; ++l) f(l);
  }
  template <class F>
  void run_w0(F f) const {
    for (int l = 0; l < 64 && l < nt; ++l) f(l);
  }
  void sync() const {}
  template <class T>
  T* lds(T* p) const {
    return p;
  }
};

// Gauss-Jordan on the column-major nr x nc matrix A (ld nr) without pivoting
// (the left nr x nr block is SPD): one column per lane (lane < nc), one pivot
// per phase; the left block's pivot column is only read in its step. Returns
// false if a pivot is not positive. Columns beyond 64 are taken by the same
// lanes in a second pass of each pivot step.
// Runs on wave 0 between wave-level fences; the caller's preceding phase must
// have ended in a workgroup barrier.
// Leading dimension of the nj-row matrices in LDS that are walked column per lane
// (mass matrix / KKT blocks): odd, so a wave's 64 column reads hit distinct banks.
MB_HD __forceinline__ int lda_of(int nj) { return nj | 1; }

// Device version: every thread of the workgroup takes columns tid, tid + nt, ...
// (one pass for nc <= nt), one workgroup barrier per pivot; plain arguments and no
// lambdas, so nothing of it lives in scratch. The column update runs in chunks of 8
// rows, loads first, so the LDS round trips overlap.
__device__ __forceinline__ bool gauss_jordan_dev(double* A, int nr, int ld, int nc, int* flag) {
  const int tid = (int)threadIdx.x, nt = (int)blockDim.x;
  A = lds_ptr(A);
  flag = lds_ptr(flag);
  __syncthreads();
  bool bad = false;
#pragma unroll 1
  for (int k = 0; k < nr; ++k) {
    const double piv = A[(int64_t)k * ld + k];
    bad = bad || !(piv > 0.);
    const double* pc = A + (int64_t)k * ld;
#pragma unroll 1
    for (int cc = tid; cc < nc; cc += nt) {
      if (cc <= k || bad) continue;
      double* col = A + (int64_t)cc * ld;
      const double akc = col[k] / piv;
      int r0 = 0;
#pragma unroll 1
      for (; r0 + 8 <= nr; r0 += 8) {
        double pv[8], cv[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          pv[r] = pc[r0 + r];
          cv[r] = col[r0 + r];
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) col[r0 + r] = (r0 + r == k) ? akc : cv[r] - pv[r] * akc;
      }
#pragma unroll 1
      for (; r0 < nr; ++r0) col[r0] = (r0 == k) ? akc : col[r0] - pc[r0] * akc;
    }
    __syncthreads();
  }
  if (tid == 0) *flag = bad ? 1 : 0;
  __syncthreads();
  return !bad;
}

// v from lane l (uniform l) of the wave, as a scalar
__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)bits, l);
  const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Gauss-Jordan with the rows in registers: lane r of every wave holds row r
// (nr <= 64) of the column slabs of CPW columns the wave owns (slab s of wave w:
// columns (w + s nw) CPW ..); per pivot k the wave owning column k publishes it
// through LDS (pb: 2 x 64 doubles, double-buffered, so one barrier per pivot), the
// pivot row comes from lane k by readlane. The pivot loop runs in chunks of CPW
// unrolled steps, so the owner's register of column k is static. No LDS traffic
// beyond the one published column per pivot. Returns false if a pivot is not
// positive (the LLT failure the reference reports).
// id0: A's columns from id0 on start as an identity block ([M | I]); their slabs
// are skipped until the pivot reaches them (the update is the identity there too).
template <int CPW, int SPW>
__device__ __forceinline__ bool gauss_jordan_rows(double* A, int nr, int ld, int nc, double* pb, int* flag,
                                                  int id0 = 1 << 30) {
  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = (int)(blockDim.x >> 6);
  const int nslab = (nc + CPW - 1) / CPW;
  A = lds_ptr(A);
  pb = lds_ptr(pb);
  flag = lds_ptr(flag);
  double v[SPW][CPW];
  __syncthreads();
#pragma unroll
  for (int s = 0; s < SPW; ++s) {
    const int slab = wave + s * nw;
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int c = slab * CPW + j;
      v[s][j] = (lane < nr && slab < nslab && c < nc) ? A[(int64_t)c * ld + lane] : 0.;
    }
  }
  bool bad = false;
#pragma unroll 1
  for (int kk = 0; kk < nr; kk += CPW) {
    const int kslab = kk / CPW, owner = kslab % nw, os = kslab / nw;
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int k = kk + j;
      if (k >= nr) continue;  // (uniform)
      double* pcol = pb + (k & 1) * 64;
      if (wave == owner) {
        double val = 0.;
#pragma unroll
        for (int s = 0; s < SPW; ++s)
          if (s == os) val = v[s][j];
        pcol[lane] = val;
      }
      __syncthreads();
      const double piv = pcol[k];
      const double ark = pcol[lane];  // A[r][k] of this lane's row
      bad = bad || !(piv > 0.);
      const double ipiv = 1. / piv;
#pragma unroll
      for (int s = 0; s < SPW; ++s) {
        // a slab left of the pivot holds unit columns (row k zero): the update is the
        // identity there, so it is skipped (wave-uniform)
        const int slab = wave + s * nw;
        if (slab >= nslab || slab * CPW + CPW <= k || slab * CPW - id0 > k) continue;
#pragma unroll
        for (int jj = 0; jj < CPW; ++jj) {
          const double akc = readlane_d(v[s][jj], k) * ipiv;  // pivot row, scaled
          v[s][jj] = lane == k ? akc : v[s][jj] - ark * akc;
        }
      }
    }
  }
#pragma unroll
  for (int s = 0; s < SPW; ++s) {
    const int slab = wave + s * nw;
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int c = slab * CPW + j;
      if (lane < nr && slab < nslab && c < nc) A[(int64_t)c * ld + lane] = v[s][j];
    }
  }
  if (tid == 0) *flag = bad ? 1 : 0;
  __syncthreads();
  return !bad;
}

// the device executor takes the register version when the slabs fit (overload
// resolution prefers these to the template below, which serves the host emulation)
// The slab count per wave follows nc (the block is uniform): every unrolled register
// column costs a readlane pair and an FMA per pivot, so the [M | Jc^T | r] block of
// the calc (nc = nj + nc + 1) and the small Schur block do not pay for the 3 slabs
// per wave that the calcDiff's [M | I] needs.
// SPW: the call site's bound on the slabs per wave (one instantiation per call site
// keeps the register budget of the kernels it is inlined into); blocks wider than
// SPW slabs per wave take the LDS version.
template <int SPW>
__device__ __forceinline__ bool gauss_jordan_regs(double* A, int nr, int ld, int nc, int* flag, double* pb,
                                                  int id0 = 1 << 30) {
  if (nr <= 64 && nc <= SPW * 8 * (int)(blockDim.x >> 6)) return gauss_jordan_rows<8, SPW>(A, nr, ld, nc, pb, flag, id0);
  return gauss_jordan_dev(A, nr, ld, nc, flag);
}
template <int SPW>
__device__ __forceinline__ bool gauss_jordan(const DevExec&, double* A, int nr, int ld, int nc, int* flag,
                                             double* pb, int id0 = 1 << 30) {
  return gauss_jordan_regs<SPW>(A, nr, ld, nc, flag, pb, id0);
}

// no side work for the idle waves of gj_mfma
struct GjNoSide {
  __device__ void operator()(int, int, int) const {}
};
#if defined(__HIP_DEVICE_COMPILE__) && !defined(MB_GJ_ROWS)
// Blocked Gauss-Jordan on the fp64 matrix cores. A: nr x nc column-major in LDS (ld),
// its left nr x nr block SPD. Pivot blocks of 16 rows; per block k:
//  A  every wave inverts the diagonal block D itself, in registers (the symmetric sweep:
//     a_pp <- -1/a_pp, a_ip <- a_ip/a_pp, a_pj <- a_pj/a_pp, a_ij <- a_ij - a_ip a_pj/a_pp;
//     after all 16 pivots N = -D^-1), so no barrier separates it from B;
//  B  the wave owning column tile j (j mod nw) forms R_j = N A_kj = -D^-1 A_kj and updates
//     its whole column: A_ij += A_ik R_j (i != k), A_kj <- -R_j (v_mfma_f64_16x16x4_f64);
//  C  (inverse) the diagonal column block, A_ik <- A_ik N, A_kk <- -N, deferred to its
//     owner's next pass (nobody else reads it before then): one workgroup barrier per
//     pivot block instead of one per pivot.
// N's registers serve as both MFMA operands: lane (i = lane & 15, g = lane >> 4) holds
// N[i][g + 4q], q = 0..3, which is the A fragment of k-chunk q (k = g + 4q) and, N being
// symmetric, the B fragment too; R_j's accumulators are the B fragments of the update
// with the same k order. Columns: the right-hand sides start at the 16-aligned virtual
// column nrp (their tiles never share a tile with the matrix). The pivots are the LDL^T
// pivots in order, so a non-positive one is the LLT failure the unblocked sweep reports.
// inverse: the left block becomes M^-1 in place; the right-hand sides M^-1 B either way.
#ifndef MB_GJ_MARK
#define MB_GJ_MARK(id)  // (tools/mb_probe: phase stamps)
#endif
// side(slot, lane, nlanes): independent work of the caller for the waves that own no
// column tile (wave >= nct), one slot per barrier interval (nbr + 1 of them), so the
// latency-bound pivot chain of the owners hides it.
template <class Side = GjNoSide>
__device__ __forceinline__ bool gj_mfma(double* A_, int nr, int ld, int nc, bool inverse, int* flag,
                                        Side side = Side{}) {
  typedef __attribute__((address_space(3))) double lds_d;
  typedef double f64x4 __attribute__((ext_vector_type(4)));
  lds_d* A = (lds_d*)lds_ptr(A_);
  // the shape in scalar registers (the callers read it from the LDS parameter block, i.e.
  // into vector registers): the sweep's `r0 + p < nr` then skips the padding pivots of the
  // last block by a scalar branch instead of running all 16 under a lane mask
  nr = __builtin_amdgcn_readfirstlane(nr);
  ld = __builtin_amdgcn_readfirstlane(ld);
  nc = __builtin_amdgcn_readfirstlane(nc);
  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = (int)(blockDim.x >> 6);
  const int li = lane & 15, lk = lane >> 4;
  const int nrp = (nr + 15) & ~15, nbr = nrp >> 4, nct = (nrp + nc - nr + 15) >> 4;
  auto phys = [&](int v) { return v < nr ? v : (v < nrp ? -1 : v - nrp + nr); };
  // branch-free guarded load: an in-range address always, the value selected
  auto at = [&](int r, int c) -> double {
    const bool v = r < nr && c >= 0 && c < nc;
    const double x = A[(v ? r : 0) + ld * (v ? c : 0)];
    return v ? x : 0.;
  };
  // Without side work or the inverse's trailing column updates (mb_solve), the per-step
  // workgroup barrier is replaced by a progress counter: step k + 1 needs tile k + 1 as
  // updated by step k (its sweep reads the diagonal block, every wave's update its
  // column), and nothing else another wave writes — a pivot tile is never written again
  // once passed — so only its owner is waited for, and the other waves' updates of the
  // later tiles overlap the next sweep.
  constexpr bool kNoSide = std::is_same<Side, GjNoSide>::value;
  const bool flagged = kNoSide && !inverse;
  int* prog = flag + 1;   // diagonal block of tile k ready (its sweep may start)
  int* prog2 = flag + 2;  // all of tile k ready (the updates may read it)
  if (flagged && tid == 0) *prog = *prog2 = 0;
  __syncthreads();
  MB_GJ_MARK(0);
  bool bad = false;
  double Np[4] = {0., 0., 0., 0.};
  // C: column block kc <- A_ik N (i != kc), the diagonal block <- -N
  auto col_update = [&](int kc, const double* N) {
    const int c = 16 * kc + li;
#pragma unroll 1
    for (int i = 0; i < nbr; ++i) {
      if (i == kc) continue;
      f64x4 acc = {0., 0., 0., 0.};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int kk = 16 * kc + lk + 4 * q;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(at(16 * i + li, kk < nr ? kk : -1), N[q], acc, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 16 * i + lk + 4 * q;
        if (r < nr && c < nr) A[r + ld * c] = acc[q];
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 16 * kc + li, cc = 16 * kc + lk + 4 * q;
      if (r < nr && cc < nr) A[r + ld * cc] = -N[q];
    }
  };
#pragma unroll 1
  for (int k = 0; k < nbr; ++k) {
    const int r0 = 16 * k;
    double d[4] = {0., 0., 0., 0.};
    if (flagged && k > 0 && wave < nct) {  // tile k updated through step k - 1
      lds_wait_ge(prog, k);
      asm volatile("" ::: "memory");
    }
    // A: only the waves that own a column tile need N (one sweep per SIMD, not two);
    // the padding pivots beyond nr are skipped (their identity rows stay +1, which only
    // ever multiplies the zero-loaded padding)
    if (wave < nct) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = lk + 4 * q;
        const double x = at(r0 + li, r0 + c < nr ? r0 + c : -1);
        d[q] = (r0 + li < nr && r0 + c < nr) ? x : (li == c ? 1. : 0.);
      }
#pragma unroll
      for (int p = 0; p < 16; ++p) {
        if (r0 + p < nr) {  // (uniform; the loop stays fully unrolled, d[] static)
          const int pq = p >> 2, pg = p & 3;
          const double app = readlane_d(d[pq], p + 16 * pg);
          const double aip = row_to_all_d(d[pq], pg);  // = __shfl(d[pq], li + 16 pg)
          double apc[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) apc[q] = row_bcast_d(d[q], p);  // = __shfl(d[q], p + 16 lk)
          bad = bad || !(app > 0.);
          // 1 / app from v_rcp_f64 (relative error up to ~2^-23) corrected to working
          // precision in three dependent fmas: with e = 1 - app x0, x0 (1 + e + e^2) has
          // relative error e^3 (one Newton step leaves e^2 ~ 1e-14, which the contact
          // KKT's conditioning, ~1e7, turned into 1e-7 trajectory errors). The pivot chain
          // is latency-bound (35 cycles per dependent f64 op), so not the IEEE division's
          // special-case scaling: app > 0 is all that is used.
          double ip = __builtin_amdgcn_rcp(app);
#ifdef MB_GJ_RCP_FAST
          ip = __builtin_fma(ip, __builtin_fma(-app, ip, 1.), ip);
#else
          {
            const double e = __builtin_fma(-app, ip, 1.);
            ip = __builtin_fma(ip, __builtin_fma(e, e, e), ip);
          }
#endif
          const double t = aip * ip;
          // row p: a_pc ip; the others: a_ic - t a_pc (one fma with per-lane factors);
          // column p (register pq of the lanes with lk == pg): t, the pivot itself -ip
          const bool rp = li == p;
          const double sf = rp ? ip : -t;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const double v = __builtin_fma(sf, apc[q], rp ? 0. : d[q]);
            d[q] = (q == pq && lk == pg) ? (rp ? -ip : t) : v;
          }
        }
      }
    }
    MB_GJ_MARK(1 + 3 * k);
    if (flagged && k > 0 && wave < nct) {  // all of tile k updated through step k - 1
      lds_wait_ge(prog2, k);
      asm volatile("" ::: "memory");
    }
#pragma unroll 1
    for (int j = wave; j < nct; j += nw) {
      if (inverse && j == k - 1) col_update(j, Np);
      if (j == k || (!inverse && j < k)) continue;
      const int pc = phys(16 * j + li);
      f64x4 R = {0., 0., 0., 0.};
#pragma unroll
      for (int q = 0; q < 4; ++q) R = __builtin_amdgcn_mfma_f64_16x16x4f64(d[q], at(r0 + lk + 4 * q, pc), R, 0, 0, 0);
      // row blocks from k + 1 on (rotated): the next pivot tile's diagonal block first
#pragma unroll 1
      for (int ii = 0; ii < nbr; ++ii) {
        const int i = ii + k + 1 < nbr ? ii + k + 1 : ii + k + 1 - nbr;
        if (i == k) continue;
        f64x4 acc;
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = at(16 * i + lk + 4 * q, pc);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int kk = r0 + lk + 4 * q;
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(at(16 * i + li, kk < nr ? kk : -1), R[q], acc, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = 16 * i + lk + 4 * q;
          if (r < nr && pc >= 0 && pc < nc) A[r + ld * pc] = acc[q];
        }
        if (flagged && j == k + 1 && i == k + 1) {  // the next sweep's block is ready
          if (lane == 0) lds_publish(prog, k + 1);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = r0 + lk + 4 * q;
        if (r < nr && pc >= 0 && pc < nc) A[r + ld * pc] = -R[q];
      }
      if (flagged && j == k + 1) {  // the whole next pivot tile is ready
        if (lane == 0) lds_publish(prog2, k + 1);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) Np[q] = d[q];
    if (wave >= nct) side(k, tid - 64 * nct, (nw - nct) * 64);
    MB_GJ_MARK(2 + 3 * k);
    if (!flagged) __syncthreads();
    MB_GJ_MARK(3 + 3 * k);
  }
  if (inverse)
    for (int j = wave; j < nct; j += nw)
      if (j == nbr - 1) col_update(j, Np);
  if (wave >= nct) side(nbr, tid - 64 * nct, (nw - nct) * 64);
  if (tid == 0) *lds_ptr(flag) = bad ? 1 : 0;
  __syncthreads();
  MB_GJ_MARK(20);
  return !bad;
}
#endif

// whether mb_invert works in place (then [M | I] needs no identity half)
__device__ __forceinline__ constexpr bool mb_inv_inplace(const DevExec&) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(MB_GJ_ROWS)
  return true;
#else
  return false;
#endif
}
// [M | B] (nr x nc, M SPD) -> M^-1 B in the columns beyond M (the left block is consumed)
__device__ __forceinline__ bool mb_solve(const DevExec&, double* A, int nr, int ld, int nc, int* flag, double* pb) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(MB_GJ_ROWS)
  (void)pb;
  return gj_mfma(A, nr, ld, nc, false, flag);
#else
  return gauss_jordan_regs<2>(A, nr, ld, nc, flag, pb);
#endif
}
// [M | I] (nr x 2 nr, M SPD) -> M^-1, at *Minv (device: in place of M). side: work the
// idle waves run meanwhile (gj_mfma); *nslots: the slots it ran (0: none)
template <class Side = GjNoSide>
__device__ __forceinline__ bool mb_invert(const DevExec&, double* A, int nr, int ld, int* flag, double* pb,
                                          double** Minv, Side side = Side{}, int* nslots = nullptr) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(MB_GJ_ROWS)
  (void)pb;
  *Minv = A;
  const int nbr = (nr + 15) >> 4, nw = (int)(blockDim.x >> 6);
  if (nslots) *nslots = nw > nbr ? nbr + 1 : 0;
  return gj_mfma(A, nr, ld, nr, true, flag, side);
#else
  (void)side;
  if (nslots) *nslots = 0;
  *Minv = A + (int64_t)ld * nr;
  return gauss_jordan_regs<3>(A, nr, ld, 2 * nr, flag, pb, nr);
#endif
}

template <int SPW, class X>
MB_HD __attribute__((noinline)) bool gauss_jordan(const X& ex, double* A, int nr, int ld, int nc, int* flag,
                                                 double* = nullptr, int = 0) {
  ex.run_w0([&](int lane) {
    if (lane == 0) *flag = 0;
  });
#pragma unroll 1
  for (int k = 0; k < nr; ++k) {
    ex.run_w0([&](int lane) {
      const double piv = A[(int64_t)k * ld + k];
      if (!(piv > 0.)) {
        if (lane == 0) *flag = 1;
        return;
      }
#pragma unroll 1
      for (int cc = lane; cc < nc; cc += 64) {
        if (cc <= k) continue;
        // pivot column and own column in chunks of 8 rows through registers
        // (independent loads, then the updates): no LDS round trip per row
        double* col = A + (int64_t)cc * ld;
        const double* pc = A + (int64_t)k * ld;
        const double akc = col[k] / piv;
#pragma unroll 1
        for (int r0 = 0; r0 < nr; r0 += 8) {
          double pv[8], cv[8];
#pragma unroll
          for (int r = 0; r < 8; ++r)
            if (r0 + r < nr) {
              pv[r] = pc[r0 + r];
              cv[r] = col[r0 + r];
            }
#pragma unroll
          for (int r = 0; r < 8; ++r)
            if (r0 + r < nr) col[r0 + r] = (r0 + r == k) ? akc : cv[r] - pv[r] * akc;
        }
      }
    });
  }
  ex.sync();
  return *flag == 0;
}
// the host emulation (and any other executor): the unblocked sweep on [M | B], [M | I]
template <class X>
MB_HD __forceinline__ constexpr bool mb_inv_inplace(const X&) {
  return false;
}
template <class X>
MB_HD __forceinline__ bool mb_solve(const X& ex, double* A, int nr, int ld, int nc, int* flag, double* pb) {
  return gauss_jordan<2>(ex, A, nr, ld, nc, flag, pb);
}
template <class X, class Side = int>
MB_HD __forceinline__ bool mb_invert(const X& ex, double* A, int nr, int ld, int* flag, double* pb, double** Minv,
                                     Side = Side{}, int* nslots = nullptr) {
  if (nslots) *nslots = 0;
  *Minv = A + (int64_t)ld * nr;
  return gauss_jordan<3>(ex, A, nr, ld, 2 * nr, flag, pb, nr);
}

// ---- dual numbers for the exp6 / log6 Jacobians ----------------------------
struct Dual {
  double v, d;
  Dual() = default;
  MB_HD constexpr Dual(double v_, double d_ = 0.) : v(v_), d(d_) {}
};
MB_HD __forceinline__ Dual operator+(Dual a, Dual b) { return {a.v + b.v, a.d + b.d}; }
MB_HD __forceinline__ Dual operator-(Dual a, Dual b) { return {a.v - b.v, a.d - b.d}; }
MB_HD __forceinline__ Dual operator*(Dual a, Dual b) { return {a.v * b.v, a.d * b.v + a.v * b.d}; }
MB_HD __forceinline__ Dual operator*(double s, Dual a) { return {s * a.v, s * a.d}; }
MB_HD __forceinline__ Dual operator/(Dual a, Dual b) { return {a.v / b.v, (a.d * b.v - a.v * b.d) / (b.v * b.v)}; }
MB_HD __forceinline__ Dual msqrt(Dual a) {
  const double s = sqrt(a.v);
  return {s, a.d / (2. * s)};
}
MB_HD __forceinline__ Dual masin(Dual a) { return {asin(a.v), a.d / sqrt(1. - a.v * a.v)}; }
MB_HD __forceinline__ Dual macos(Dual a) { return {acos(a.v), -a.d / sqrt(1. - a.v * a.v)}; }
MB_HD __forceinline__ Dual msin(Dual a) { return {sin(a.v), a.d * cos(a.v)}; }
MB_HD __forceinline__ Dual mcos(Dual a) { return {cos(a.v), -a.d * sin(a.v)}; }
MB_HD __forceinline__ double mval(Dual a) { return a.v; }
MB_HD __forceinline__ double msqrt(double a) { return sqrt(a); }
MB_HD __forceinline__ double masin(double a) { return asin(a); }
MB_HD __forceinline__ double macos(double a) { return acos(a); }
MB_HD __forceinline__ double msin(double a) { return sin(a); }
MB_HD __forceinline__ double mcos(double a) { return cos(a); }
MB_HD __forceinline__ double mval(double a) { return a; }

// log6(R, p) -> (lin, ang) (pinocchio::log6), R column-major. T = double, or
// Dual so that the tangent along (dR, dp) is Jlog6 * xi. Same branches as
// oracle/multibody_np.py:log3/log6.
template <class T>
MB_HD inline void log6_t(const T* R, const T* p, T* out) {
  auto at = [&](int r, int c) { return R[c * 3 + r]; };
  const T one(1.);
  const T tr = at(0, 0) + at(1, 1) + at(2, 2);
  const T c = 0.5 * (tr - one);
  const T w[3] = {at(2, 1) - at(1, 2), at(0, 2) - at(2, 0), at(1, 0) - at(0, 1)};
  const T s2 = 0.25 * (w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  T om[3];
  T sth = T(0.), thg = T(0.);  // sin(theta), theta of the generic branch (beta reuses them)
  bool generic = false;
  if (mval(s2) < 1e-8 && mval(c) > 0.) {
    const T k = 0.5 * (one + (1. / 6.) * s2 + (3. / 40.) * (s2 * s2) + (5. / 112.) * (s2 * s2 * s2));
    for (int e = 0; e < 3; ++e) om[e] = k * w[e];
  } else if (mval(s2) < 1e-8) {  // theta near pi: axis from the symmetric part (value only)
    // (explicit selects: no runtime-indexed arrays, which would live in scratch)
    const double cv = mval(c) < -1. ? -1. : mval(c);
    const double th = acos(cv);
    auto axc = [&](double d) {
      const double t = (d - cv) / (1. - cv);
      return t > 0. ? sqrt(t) : 0.;
    };
    const double a0 = axc(mval(at(0, 0))), a1 = axc(mval(at(1, 1))), a2 = axc(mval(at(2, 2)));
    const int i0 = (a1 > a0) ? ((a2 > a1) ? 2 : 1) : ((a2 > a0) ? 2 : 0);
    const double s01 = mval(at(0, 1)) + mval(at(1, 0)), s02 = mval(at(0, 2)) + mval(at(2, 0)),
                 s12 = mval(at(1, 2)) + mval(at(2, 1));
    auto sgn = [](double v) { return v >= 0. ? 1. : -1.; };
    const double g0 = i0 == 0 ? 1. : (i0 == 1 ? sgn(s01) : sgn(s02));
    const double g1 = i0 == 1 ? 1. : (i0 == 0 ? sgn(s01) : sgn(s12));
    const double g2 = i0 == 2 ? 1. : (i0 == 0 ? sgn(s02) : sgn(s12));
    const double wi = i0 == 0 ? mval(w[0]) : (i0 == 1 ? mval(w[1]) : mval(w[2]));
    const double flip = wi < 0. ? -th : th;
    om[0] = T(flip * g0 * a0);
    om[1] = T(flip * g1 * a1);
    om[2] = T(flip * g2 * a2);
  } else {
    const T s = msqrt(s2);
    T th;
    if (mval(c) > 0.5)
      th = masin(s);
    else if (mval(c) < -0.5)
      th = T(M_PI) - masin(s);
    else
      th = macos(c);
    const T k = th / (2. * s);
    for (int e = 0; e < 3; ++e) om[e] = k * w[e];
    sth = s;
    thg = th;
    generic = true;
  }
  const T t2 = om[0] * om[0] + om[1] * om[1] + om[2] * om[2];
  T beta;
  if (mval(t2) < 1e-2) {
    beta = T(1. / 12.) + (1. / 720.) * t2 + (1. / 30240.) * (t2 * t2) + (1. / 1209600.) * (t2 * t2 * t2);
  } else if (generic) {  // 1/t^2 - sin t / (2 t (1 - cos t)) with sin, cos of theta read off R
    beta = one / (thg * thg) - sth / (2. * thg * (one - c));
  } else {
    const T t = msqrt(t2);
    beta = one / t2 - msin(t) / (2. * t * (one - mcos(t)));
  }
  // v = (I - 0.5 [w]x + beta [w]x^2) p ; [w]x^2 p = w (w.p) - |w|^2 p
  const T wp = om[0] * p[0] + om[1] * p[1] + om[2] * p[2];
  const T wxp[3] = {om[1] * p[2] - om[2] * p[1], om[2] * p[0] - om[0] * p[2], om[0] * p[1] - om[1] * p[0]};
  for (int e = 0; e < 3; ++e) {
    const T w2p = om[e] * wp - t2 * p[e];
    out[e] = p[e] - 0.5 * wxp[e] + beta * w2p;
    out[3 + e] = om[e];
  }
}

// exp6(nu) -> (R, p) (pinocchio::exp6): R = cos t I + (1 - cos t)/t^2 w w^T +
// sin t / t [w]x, p = sin t / t v + (1 - sin t / t)/t^2 (w.v) w + (1 - cos t)/t^2 w x v,
// Taylor branch for t^2 < 1e-8 (as oracle/multibody_np.py:exp6). T = double or Dual.
template <class T>
MB_HD inline void exp6_t(const T* nu, T* R, T* p) {
  const T* v = nu;
  const T* w = nu + 3;
  const T t2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  T ct, st_t, a_wxv, a_w;
  if (mval(t2) < 1e-8) {
    ct = T(1.) - 0.5 * t2 + (1. / 24.) * (t2 * t2);
    st_t = T(1.) - (1. / 6.) * t2 + (1. / 120.) * (t2 * t2);
    a_wxv = T(0.5) - (1. / 24.) * t2 + (1. / 720.) * (t2 * t2);
    a_w = T(1. / 6.) - (1. / 120.) * t2 + (1. / 5040.) * (t2 * t2);
  } else {
    const T t = msqrt(t2);
    ct = mcos(t);
    st_t = msin(t) / t;
    a_wxv = (T(1.) - ct) / t2;
    a_w = (T(1.) - st_t) / t2;
  }
  // column-major R[c*3 + r] = ct d_rc + a_wxv w_r w_c + st_t [w]x(r, c)
  R[0] = ct + a_wxv * (w[0] * w[0]);
  R[1] = a_wxv * (w[1] * w[0]) + st_t * w[2];
  R[2] = a_wxv * (w[2] * w[0]) - st_t * w[1];
  R[3] = a_wxv * (w[0] * w[1]) - st_t * w[2];
  R[4] = ct + a_wxv * (w[1] * w[1]);
  R[5] = a_wxv * (w[2] * w[1]) + st_t * w[0];
  R[6] = a_wxv * (w[0] * w[2]) + st_t * w[1];
  R[7] = a_wxv * (w[1] * w[2]) - st_t * w[0];
  R[8] = ct + a_wxv * (w[2] * w[2]);
  const T wv = w[0] * v[0] + w[1] * v[1] + w[2] * v[2];
  const T wxv[3] = {w[1] * v[2] - w[2] * v[1], w[2] * v[0] - w[0] * v[2], w[0] * v[1] - w[1] * v[0]};
  for (int e = 0; e < 3; ++e) p[e] = st_t * v[e] + a_w * wv * w[e] + a_wxv * wxv[e];
}

// pinocchio SpecialEuclideanOperationTpl<3>::integrate: M1 = M0 exp6(dq); the
// quaternion re-extracted from M1's rotation, flipped into q0's hemisphere and
// first-order normalised. q7 = (p, quat xyzw); out may not alias q7.
MB_HD inline void ff_integrate(const double* q7, const double* dq, double* out) {
  double R0[9], Re[9], pe[3], R1[9], t[3];
  quat_to_R(q7 + 3, R0);
  exp6_t<double>(dq, Re, pe);
  matmul3(R0, Re, R1);
  matvec3(R0, pe, t);
  out[0] = q7[0] + t[0];
  out[1] = q7[1] + t[1];
  out[2] = q7[2] + t[2];
  double qn[4];
  R_to_quat(R1, qn);
  const double dd = qn[0] * q7[3] + qn[1] * q7[4] + qn[2] * q7[5] + qn[3] * q7[6];
  const double sg = dd < 0. ? -1. : 1.;
  const double n2 = qn[0] * qn[0] + qn[1] * qn[1] + qn[2] * qn[2] + qn[3] * qn[3];
  const double al = sg * (3. - n2) * 0.5;
  for (int e = 0; e < 4; ++e) out[3 + e] = qn[e] * al;
}
// pinocchio SpecialEuclideanOperationTpl<3>::difference: log6(M0^-1 M1).
MB_HD inline void ff_difference(const double* q0, const double* q1, double* out) {
  double R0[9], R1[9], Rr[9], dp[3], pr[3];
  quat_to_R(q0 + 3, R0);
  quat_to_R(q1 + 3, R1);
  matTmul3(R0, R1, Rr);
  dp[0] = q1[0] - q0[0];
  dp[1] = q1[1] - q0[1];
  dp[2] = q1[2] - q0[2];
  matTvec3(R0, dp, pr);
  log6_t<double>(Rr, pr, out);
}
// column k of Jexp6(nu) (pinocchio Jexp6, the right Jacobian: exp6(nu + e eps)
// = exp6(nu) exp6(J e eps)): the twist of exp6(nu)^-1 d exp6(nu + eps e_k).
MB_HD inline void jexp6_col(const double* nu, int k, double* col) {
  Dual n[6], R[9], p[3];
  for (int e = 0; e < 6; ++e) n[e] = Dual{nu[e], e == k ? 1. : 0.};
  exp6_t<Dual>(n, R, p);
  double Rv[9], dR[9], dp[3], Om[9];
  for (int e = 0; e < 9; ++e) {
    Rv[e] = R[e].v;
    dR[e] = R[e].d;
  }
  for (int e = 0; e < 3; ++e) dp[e] = p[e].d;
  matTvec3(Rv, dp, col);
  matTmul3(Rv, dR, Om);  // [xi_ang]x
  col[3] = Om[5];        // (2,1)
  col[4] = Om[6];        // (0,2)
  col[5] = Om[1];        // (1,0)
}
// column k of Jlog6(M) (pinocchio Jlog6: log6(M exp6(e eps)) = log6(M) + J e eps)
MB_HD inline void jlog6_col(const double* R, const double* p, int k, double* col) {
  double xi[6] = {0., 0., 0., 0., 0., 0.};
  xi[k] = 1.;
  double dR[9], dp[3];
  for (int c = 0; c < 3; ++c) {  // dR = R [xi_ang]x
    double t[3];
    const double e[3] = {c == 0 ? 1. : 0., c == 1 ? 1. : 0., c == 2 ? 1. : 0.};
    cross3(xi + 3, e, t);
    matvec3(R, t, dR + 3 * c);
  }
  matvec3(R, xi, dp);
  Dual RD[9], PD[3], o[6];
  for (int e = 0; e < 9; ++e) RD[e] = Dual{R[e], dR[e]};
  for (int e = 0; e < 3; ++e) PD[e] = Dual{p[e], dp[e]};
  log6_t<Dual>(RD, PD, o);
  for (int e = 0; e < 6; ++e) col[e] = o[e].d;
}

// ---------------------------------------------------------------------------
// World-frame values. Spatial quantities are expressed at the world origin in
// world axes, so every recursion of RNEA/CRBA becomes a sum over the ancestors or
// the subtree of a dof
//   v_i = sum_{k in anc(i)} S_k qd_k,  a_i = -g + sum_{k in anc(i)} (S_k qdd_k + v_k x S_k qd_k),
//   tau_i = S_i . sum_{k in sub(i)} f_k,  Ic_i = sum_{k in sub(i)} I_k,
//   M_ij = S_i . (Ic_j S_j)  (i in anc(j)),
// which each lane evaluates for its own dof: no serial chain through LDS.
// anc(i) holds every dof of the ancestor-or-self bodies (all six free-flyer
// dofs for the base), so v_k is the full body velocity. The placements
// oMi = oMparent * liMi are composed by each lane walking its ancestors (w_walk).
// ---------------------------------------------------------------------------
// The world values of a dof in two records of kWRec doubles (40 used, 2 of padding): the
// L record holds what outlives the recursions (placement oMi, motion subspace, velocity,
// acceleration, composite inertia), the D record what the recursions alone use (the local
// placement, body mass / CoM / inertia, the RNEA's forces and terms). The workgroup's lanes
// read and write their own dof's records (lane stride kWRec): at a multiple of 32 doubles
// every lane of a 64-bit access would map to the same bank pair; at 42 (84 dwords) the lanes
// spread over 16 bank pairs (2-way) with the records 16-byte aligned. (One 80-double record
// per dof, its round-5 layout, was a 16-way conflict: C5 rollout 28.55 -> 26.81 ms,
// calcDiff 25.60 -> 25.26 ms when padded.) The D records may lie apart from the L records
// (`aux`): the rollout's calc puts its factorisation over them once the recursions are done
// (knot_calc_dense_x); by default they follow the L records, the ancestor masks and root_a.
constexpr int kWRec = 42;
constexpr int kMaxCosts = 64;
struct WVals {
  double* base;
  int nj;
  double* parts;  // per-wave partial sums of the recursions: 4 x 6 per dof (kPartDoubles)
  double* aux;    // the D records
  MB_HD WVals(double* b, int n, double* p, double* a = nullptr)
      : base(b), nj(n), parts(p), aux(a ? a : b + lsize(n)) {}
  MB_HD double* L(int i) const { return mb_lds(base + kWRec * i); }
  MB_HD double* Dr(int i) const { return mb_lds(aux + kWRec * i); }
  MB_HD double* oR(int i) const { return L(i); }  // oMi
  MB_HD double* op(int i) const { return L(i) + 9; }
  MB_HD double* S(int i) const { return L(i) + 12; }   // dof motion subspace (world)
  MB_HD double* v(int i) const { return L(i) + 18; }
  MB_HD double* a(int i) const { return L(i) + 24; }
  MB_HD double* cm(int i) const { return L(i) + 30; }  // composite inertia, origin form: m, h = m c, I_O (6)
  MB_HD double* ch(int i) const { return L(i) + 31; }
  MB_HD double* cI(int i) const { return L(i) + 34; }
  MB_HD double* R(int i) const { return Dr(i); }  // liMi rotation
  MB_HD double* p(int i) const { return Dr(i) + 9; }
  MB_HD double* m(int i) const { return Dr(i) + 12; }   // body mass (0 on the massless free-flyer dofs)
  MB_HD double* c(int i) const { return Dr(i) + 13; }   // body CoM (world)
  MB_HD double* Ic(int i) const { return Dr(i) + 16; }  // body inertia about its CoM, world axes (6)
  MB_HD double* F(int i) const { return Dr(i) + 22; }   // body force, then accumulated joint force
  MB_HD double* cq(int i) const { return Dr(i) + 28; }  // S_i qdd_i + v_i x S_i qd_i
  MB_HD double* fb(int i) const { return Dr(i) + 34; }  // body force I a + v x* I v
  // per-wave partial sums of the ancestor / subtree recursions (wave w's share of the dofs)
  MB_HD double* part(int w, int i) const { return mb_lds(parts + 6 * ((int64_t)w * nj + i)); }
  MB_HD Mask* anc(int i) const { return (Mask*)(base + kWRec * nj) + i; }  // ancestors-or-self dofs
  MB_HD double* root_a() const { return mb_lds(base + kWRec * nj + nj); }
  // the L records, the masks and root_a; the D records
  MB_HD static int64_t lsize(int nj) { return pad2((int64_t)kWRec * nj + nj + 6); }
  MB_HD static int64_t dsize(int nj) { return (int64_t)kWRec * nj; }
  MB_HD static int64_t doubles(int nj) { return lsize(nj) + dsize(nj); }
};

// The per-wave partial sums (RNEA recursions: 6 per dof, composites: 10 per dof) come
// from at most kPartWaves waves (their LDS areas are sized for that); larger workgroups
// leave the other waves idle in those phases.
constexpr int kPartWaves = 4;
MB_HD __forceinline__ int part_waves(int nt) { return (nt >> 6) < kPartWaves ? (nt >> 6) : kPartWaves; }
// (6 per dof for the RNEA sums, 10 for the composites)
MB_HD __forceinline__ int64_t part_doubles(int nj) { return (int64_t)kPartWaves * 10 * nj; }

// lane i < nj: local placement (buffer A starts as liMi), ancestor bits.
MB_HD inline void w_joint_local(const Blk& b, const WVals& W, const double* q, int i) {
  double R[9], p[3];
  if (b.ff && i < 6) {
    if (i == 0) {  // base pose: root placement * (R(quat), p)
      const JRec J(b, 0);
      double Rq[9], t[3];
      quat_to_R(q + 3, Rq);
      matmul3(J.Rpl(), Rq, R);
      matvec3(J.Rpl(), q, t);
      for (int e = 0; e < 3; ++e) p[e] = J.ppl()[e] + t[e];
    } else {
      for (int e = 0; e < 9; ++e) R[e] = (e % 4 == 0) ? 1. : 0.;
      for (int e = 0; e < 3; ++e) p[e] = 0.;
    }
  } else {
    const JRec J(b, rec_of(b, i));
    double ax[3], Rpl[9];
    for (int e = 0; e < 3; ++e) ax[e] = J.axis()[e];
    for (int e = 0; e < 9; ++e) Rpl[e] = J.Rpl()[e];
    joint_rotation(Rpl, ax, q[qof(b, i)], R);
    for (int e = 0; e < 3; ++e) p[e] = J.ppl()[e];
  }
  for (int e = 0; e < 9; ++e) {
    W.R(i)[e] = R[e];
    W.oR(i)[e] = R[e];
  }
  for (int e = 0; e < 3; ++e) {
    W.p(i)[e] = p[e];
    W.op(i)[e] = p[e];
  }
  if (i == 0) {
    for (int e = 0; e < 6; ++e) W.root_a()[e] = e < 3 ? -b.g[e] : 0.;
  }
  *W.anc(i) = anc_mask(b, i);
}

// lane i < nj: oMi = L_root ... L_i, the local placements of i's ancestors composed
// by walking its ancestor mask from i towards the root (parents precede children):
// one phase, no barrier per level, and the loads do not wait on the products (the
// pointer-jumping rounds this replaced took ceil(log2 nj) barrier phases). The free-flyer's
// dofs 1..5 carry identity placements and are skipped (exact).
MB_HD inline void w_walk(const Blk& b, const WVals& W, int i) {
  double R[9], p[3];
  for (int e = 0; e < 9; ++e) R[e] = W.R(i)[e];
  for (int e = 0; e < 3; ++e) p[e] = W.p(i)[e];
  Mask m = *W.anc(i) & ~(1ull << i);
  if (b.ff) m &= ~0x3Eull;
  while (m) {
    const int k = 63 - __builtin_clzll(m);
    m &= ~(1ull << k);
    double Rk[9], pk[3], Rn[9], t[3];
    for (int e = 0; e < 9; ++e) Rk[e] = W.R(k)[e];
    for (int e = 0; e < 3; ++e) pk[e] = W.p(k)[e];
    matmul3(Rk, R, Rn);
    matvec3(Rk, p, t);
    for (int e = 0; e < 9; ++e) R[e] = Rn[e];
    for (int e = 0; e < 3; ++e) p[e] = pk[e] + t[e];
  }
  for (int e = 0; e < 9; ++e) W.oR(i)[e] = R[e];
  for (int e = 0; e < 3; ++e) W.op(i)[e] = p[e];
}

// lane i < nj: world motion subspace and body inertia from oMi (oR/op).
MB_HD inline void w_joint_world(const Blk& b, const WVals& W, int i) {
  double oR[9], op[3], w[3], ax[3];
  for (int e = 0; e < 9; ++e) oR[e] = W.oR(i)[e];
  for (int e = 0; e < 3; ++e) op[e] = W.op(i)[e];
  dof_axis(b, i, ax);
  matvec3(oR, ax, w);
  if (dof_prismatic(b, i)) {
    for (int e = 0; e < 3; ++e) {
      W.S(i)[e] = w[e];
      W.S(i)[3 + e] = 0.;
    }
  } else {
    double vl[3];
    cross3(op, w, vl);  // velocity of the world origin: w x (0 - op) = op x w
    for (int e = 0; e < 3; ++e) {
      W.S(i)[e] = vl[e];
      W.S(i)[3 + e] = w[e];
    }
  }
  double* o = W.Ic(i);
  if (!carries_body(b, i)) {
    *W.m(i) = 0.;
    for (int e = 0; e < 3; ++e) W.c(i)[e] = op[e];
    for (int e = 0; e < 6; ++e) o[e] = 0.;
    return;
  }
  const JRec J(b, rec_of(b, i));
  double c[3], t[3];
  matvec3(oR, J.com(), t);
  for (int e = 0; e < 3; ++e) c[e] = op[e] + t[e];
  // Ic_w = oR Ic oR^T
  const double* s = J.I6();
  const double Is[9] = {s[0], s[3], s[4], s[3], s[1], s[5], s[4], s[5], s[2]};
  double tmp[9], Iw[9];
  matmul3(oR, Is, tmp);
  for (int r = 0; r < 3; ++r)
    for (int cc = 0; cc < 3; ++cc) Iw[cc * 3 + r] = tmp[r] * oR[cc] + tmp[3 + r] * oR[3 + cc] + tmp[6 + r] * oR[6 + cc];
  for (int e = 0; e < 3; ++e) W.c(i)[e] = c[e];
  *W.m(i) = J.mass();
  o[0] = Iw[0];
  o[1] = Iw[4];
  o[2] = Iw[8];
  o[3] = Iw[3];
  o[4] = Iw[6];
  o[5] = Iw[7];
}

// wave w's contiguous share [w c, (w + 1) c), c = ceil(nj / nw), of nj dofs
MB_HD __forceinline__ void k_range(int nj, int w, int nw, int& k0, int& k1) {
  const int c = (nj + nw - 1) / nw;
  k0 = w * c;
  k1 = k0 + c < nj ? k0 + c : nj;
}
// Per-record work on one lane each, from the top of the workgroup down: record k on
// lane nt - 1 - 64 (k mod W) - k / W (W waves), i.e. one record per wave before any wave
// takes a second (a wave runs its divergent lanes' paths one after another).
MB_HD __forceinline__ int spread_lane(int k, int nt) {
  const int nwv = nt >> 6;
  return nt - 1 - 64 * (k % nwv) - k / nwv;
}
MB_HD __forceinline__ int spread_item(int lane, int nt) {
  const int u = nt - 1 - lane, nwv = nt >> 6;
  return (u & 63) * nwv + (u >> 6);
}
// composite inertia of dof i's subtree times a motion x: (m v - h x w, I_O w + h x v)
MB_HD __forceinline__ void comp_mul(const WVals& W, int i, const double* x, double* o) {
  const double m = *W.cm(i);
  const double* h = W.ch(i);
  const double* I = W.cI(i);
  double t[3];
  cross3(h, x + 3, t);
  for (int e = 0; e < 3; ++e) o[e] = m * x[e] - t[e];
  cross3(h, x, t);
  o[3] = I[0] * x[3] + I[3] * x[4] + I[4] * x[5] + t[0];
  o[4] = I[3] * x[3] + I[1] * x[4] + I[5] * x[5] + t[1];
  o[5] = I[4] * x[3] + I[5] * x[4] + I[2] * x[5] + t[2];
}

// lane i < nj: v_i = sum over ancestors-or-self of S_k qd_k
MB_HD inline void w_velocity(const WVals& W, const double* qd, int i) {
  double v[6] = {0., 0., 0., 0., 0., 0.};
  const Mask am = *W.anc(i);
  // every dof's terms loaded, the others' selected away (not branched around), so the
  // unrolled iterations' LDS loads overlap; the sums keep their order
#pragma unroll 2
  for (int k = 0; k < W.nj; ++k) {
    const bool in = (am >> k) & 1ull;
    const double w = qd[k];
    for (int e = 0; e < 6; ++e) {
      const double t = W.S(k)[e] * w;
      v[e] += in ? t : 0.;
    }
  }
  for (int e = 0; e < 6; ++e) W.v(i)[e] = v[e];
}

// lane i < nj: cq_i = S_i qdd_i + v_i x (S_i qd_i)
MB_HD inline void w_accel_term(const WVals& W, const double* qd, const double* qdd, int i) {
  double S[6], v[6], Sw[6], t6[6];
  const double w = qd[i], qa = qdd ? qdd[i] : 0.;
  for (int e = 0; e < 6; ++e) {
    S[e] = W.S(i)[e];
    v[e] = W.v(i)[e];
    Sw[e] = S[e] * w;
  }
  cross_m(v, Sw, t6);
  for (int e = 0; e < 6; ++e) W.cq(i)[e] = S[e] * qa + t6[e];
}

// lane i < nj: a_i = -g + sum over ancestors-or-self of cq_k, then the body
// force f_i = I_i a_i + v_i x* (I_i v_i) - fext_i
MB_HD inline void w_accel_force(const WVals& W, int i, const double* fx = nullptr) {
  double a[6];
  for (int e = 0; e < 6; ++e) a[e] = W.root_a()[e];
  const Mask am = *W.anc(i);
#pragma unroll 2
  for (int k = 0; k < W.nj; ++k) {  // (selected, not branched: as w_velocity)
    const bool in = (am >> k) & 1ull;
    for (int e = 0; e < 6; ++e) {
      const double t = W.cq(k)[e];
      a[e] += in ? t : 0.;
    }
  }
  double v[6], f[6], Iv[6], t6[6], c[3], I6[6];
  for (int e = 0; e < 6; ++e) {
    W.a(i)[e] = a[e];
    v[e] = W.v(i)[e];
    I6[e] = W.Ic(i)[e];
  }
  for (int e = 0; e < 3; ++e) c[e] = W.c(i)[e];
  const double m = *W.m(i);
  inertia_mul(m, c, I6, a, f);
  inertia_mul(m, c, I6, v, Iv);
  cross_f(v, Iv, t6);
  for (int e = 0; e < 6; ++e) W.fb(i)[e] = f[e] + t6[e] - (fx ? fx[6 * i + e] : 0.);
}

// lane i < nj: F_i = sum over the subtree of the body forces, tau_i = S_i . F_i
MB_HD inline void w_joint_force(const Blk& b, const WVals& W, double* tau, int i) {
  double F[6] = {0., 0., 0., 0., 0., 0.};
#pragma unroll 2
  for (int k = 0; k < b.nj; ++k) {  // (selected, not branched: as w_velocity)
    const bool in = (*W.anc(k) >> i) & 1ull;
    for (int e = 0; e < 6; ++e) {
      const double t = W.fb(k)[e];
      F[e] += in ? t : 0.;
    }
  }
  for (int e = 0; e < 6; ++e) W.F(i)[e] = F[e];
  tau[i] = dot6(W.S(i), F);
}

// lane j < nj of wave w (of nw): CRBA column j in world frame, F = Ic_j S_j, M_ij = S_i . F
// for the ancestors-or-self i < j of j (+ armature on the diagonal), the rows i < j split
// in nw contiguous ranges, one per wave (the waves run side by side: the per-lane chain
// of LDS loads is a quarter as long). A: ld lda, zeroed.
// The column is formed about the point P = joint j's origin, not the world origin: the
// subtree's composite inertia is summed from the bodies' offsets c_b - P, and the motion
// subspaces are shifted to P (S_i at P: [w_i x (P - p_i); w_i], a prismatic dof [w_i; 0]).
// About the world origin the entries of a light distal link (a gripper, 1e-4 kg m^2, 1 m
// from the origin) are the difference of terms ~ m |c|^2 ~ 0.3, which cost ~3 digits of
// M and, through cond(M) ~ 1e6, of M^-1 and Fu (the round-4 parity trace); at P the
// lever arms are the link's own size.
// Phase 1 (lane j of wave w < nw): wave w's share of j's subtree bodies into its
// partial (W.parts, 10 per dof: m, h, I about P_j), as w_composite.
MB_HD inline void w_crba_composite_part(const Blk& b, const WVals& W, int j, int w, int nw) {
  double P[3], m = 0., h[3] = {0., 0., 0.}, I[6] = {0., 0., 0., 0., 0., 0.};
  for (int e = 0; e < 3; ++e) P[e] = W.op(j)[e];
  int k0 = b.ff ? 5 : 0, k1 = b.nj;
  if (nw > 1) k_range(b.nj, w, nw, k0, k1);
  if (b.ff && k0 < 5) k0 = 5;
  // (every body of the share read, the others weighted 0: the loads overlap)
#pragma unroll 2
  for (int k = k0; k < k1; ++k) {
    const double sel = ((*W.anc(k) >> j) & 1ull) ? 1. : 0.;
    const double mk = *W.m(k);
    double c[3], Ic[6];
    for (int e = 0; e < 3; ++e) c[e] = W.c(k)[e] - P[e];
    for (int e = 0; e < 6; ++e) Ic[e] = W.Ic(k)[e];
    const double cc = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
    m += sel * mk;
    for (int e = 0; e < 3; ++e) h[e] += sel * (mk * c[e]);
    I[0] += sel * (Ic[0] + mk * (cc - c[0] * c[0]));
    I[1] += sel * (Ic[1] + mk * (cc - c[1] * c[1]));
    I[2] += sel * (Ic[2] + mk * (cc - c[2] * c[2]));
    I[3] += sel * (Ic[3] - mk * c[0] * c[1]);
    I[4] += sel * (Ic[4] - mk * c[0] * c[2]);
    I[5] += sel * (Ic[5] - mk * c[1] * c[2]);
  }
  double* o = mb_lds(W.parts + 10 * ((int64_t)w * b.nj + j));
  o[0] = m;
  for (int e = 0; e < 3; ++e) o[1 + e] = h[e];
  for (int e = 0; e < 6; ++e) o[4 + e] = I[e];
}
// Phase 2 (lane j of wave w of nw): the partials of the npw waves combined in wave order,
// F = Ic_j S_j about P_j, M_ij = S_i(P_j) . F for the ancestors-or-self i < j of j (+
// armature on the diagonal), the rows i < j split in nw contiguous ranges, one per wave.
// A: ld lda, zeroed.
// store_world: wave 0 also stores the subtree composite about the world origin (W.cm /
// ch / cI, the calcDiff's recursions): h_O = h + m P, I_O = I + 2 (h.P) 1 - (h P^T +
// P h^T) + m (|P|^2 1 - P P^T) (the same terms as summing the bodies about the origin).
// (the partials of the npw waves combined in wave order)
MB_HD __forceinline__ void w_crba_combine(const WVals& W, int nj, int j, int npw, double* v) {
  const double* p0 = mb_lds(W.parts + 10 * (int64_t)j);
  for (int e = 0; e < 10; ++e) v[e] = p0[e];
  for (int ww = 1; ww < npw; ++ww) {
    const double* p = mb_lds(W.parts + 10 * ((int64_t)ww * nj + j));
    for (int e = 0; e < 10; ++e) v[e] += p[e];
  }
}
// combined: the composite about P_j already in W.cm / ch / cI (w_crba_store_local; the
// partials may be overwritten meanwhile)
MB_HD inline void w_crba_column(const Blk& b, const WVals& W, int j, double* A, int lda, int w, int nw, int npw,
                                bool store_world = false, bool combined = false) {
  double P[3], v[10];
  for (int e = 0; e < 3; ++e) P[e] = W.op(j)[e];
  if (combined) {
    v[0] = *W.cm(j);
    for (int e = 0; e < 3; ++e) v[1 + e] = W.ch(j)[e];
    for (int e = 0; e < 6; ++e) v[4 + e] = W.cI(j)[e];
  } else {
    w_crba_combine(W, b.nj, j, npw, v);
  }
  const double m = v[0];
  const double* h = v + 1;
  const double* I = v + 4;
  if (store_world && w == 0) {
    const double hp = h[0] * P[0] + h[1] * P[1] + h[2] * P[2], pp = P[0] * P[0] + P[1] * P[1] + P[2] * P[2];
    *W.cm(j) = m;
    for (int e = 0; e < 3; ++e) W.ch(j)[e] = h[e] + m * P[e];
    // (I ordering: xx, yy, zz, xy, xz, yz)
    W.cI(j)[0] = I[0] + 2. * (hp - h[0] * P[0]) + m * (pp - P[0] * P[0]);
    W.cI(j)[1] = I[1] + 2. * (hp - h[1] * P[1]) + m * (pp - P[1] * P[1]);
    W.cI(j)[2] = I[2] + 2. * (hp - h[2] * P[2]) + m * (pp - P[2] * P[2]);
    W.cI(j)[3] = I[3] - (h[0] * P[1] + P[0] * h[1]) - m * P[0] * P[1];
    W.cI(j)[4] = I[4] - (h[0] * P[2] + P[0] * h[2]) - m * P[0] * P[2];
    W.cI(j)[5] = I[5] - (h[1] * P[2] + P[1] * h[2]) - m * P[1] * P[2];
  }
  // S_i shifted to P: [S_i.lin + S_i.ang x P; S_i.ang] (a revolute dof's axis w through
  // p_i moves P at w x (P - p_i) = S_i.lin + w x P; a prismatic dof has S_i.ang = 0).
  // The products are dimension-one in the lever arms, so forming them from the world-origin
  // S_i costs only the rounding of the placements (unlike the quadratic m |c|^2 terms).
  // Scalars throughout: a shifted-S array written under a branch lands in scratch memory.
  const double* Sjw = W.S(j);
  const double sj3 = Sjw[3], sj4 = Sjw[4], sj5 = Sjw[5];
  const double sj0 = Sjw[0] + (sj4 * P[2] - sj5 * P[1]);
  const double sj1 = Sjw[1] + (sj5 * P[0] - sj3 * P[2]);
  const double sj2 = Sjw[2] + (sj3 * P[1] - sj4 * P[0]);
  // F = Ic_j S_j about P: (m v - h x w, I w + h x v)
  const double F0 = m * sj0 - (h[1] * sj5 - h[2] * sj4);
  const double F1 = m * sj1 - (h[2] * sj3 - h[0] * sj5);
  const double F2 = m * sj2 - (h[0] * sj4 - h[1] * sj3);
  const double F3 = I[0] * sj3 + I[3] * sj4 + I[4] * sj5 + (h[1] * sj2 - h[2] * sj1);
  const double F4 = I[3] * sj3 + I[1] * sj4 + I[5] * sj5 + (h[2] * sj0 - h[0] * sj2);
  const double F5 = I[4] * sj3 + I[5] * sj4 + I[2] * sj5 + (h[0] * sj1 - h[1] * sj0);
  if (w == 0) A[(int64_t)j * lda + j] = (sj0 * F0 + sj1 * F1 + sj2 * F2) + (sj3 * F3 + sj4 * F4 + sj5 * F5) + b.arm[j];
  const Mask am = *W.anc(j);
  const int ch = (j + nw - 1) / nw, i0 = w * ch, i1 = i0 + ch < j ? i0 + ch : j;
  // every i < j visited, the non-ancestors storing their zero (only lane j writes the
  // pair {i, j}), so the loop has no branch and the unrolled loads overlap
#pragma unroll 2
  for (int i = i0; i < i1; ++i) {
    const double* Si = W.S(i);
    const double a3 = Si[3], a4 = Si[4], a5 = Si[5];
    const double l0 = Si[0] + (a4 * P[2] - a5 * P[1]);
    const double l1 = Si[1] + (a5 * P[0] - a3 * P[2]);
    const double l2 = Si[2] + (a3 * P[1] - a4 * P[0]);
    const double d = (l0 * F0 + l1 * F1 + l2 * F2) + (a3 * F3 + a4 * F4 + a5 * F5);
    const double Mij = ((am >> i) & 1ull) ? d : 0.;
    A[(int64_t)j * lda + i] = Mij;
    A[(int64_t)i * lda + j] = Mij;
  }
}

// lane j: the subtree composite about P_j (the combined partials) into W.cm / ch / cI, so
// that the columns can overwrite the partials (the rollout's calc, knot_calc_dense_x)
MB_HD inline void w_crba_store_local(const WVals& W, int nj, int j, int npw) {
  double v[10];
  w_crba_combine(W, nj, j, npw, v);
  *W.cm(j) = v[0];
  for (int e = 0; e < 3; ++e) W.ch(j)[e] = v[1 + e];
  for (int e = 0; e < 6; ++e) W.cI(j)[e] = v[4 + e];
}

// ---- the RNEA recursions split over the waves ---------------------------------
// Each ancestor (or subtree) sum of lane i runs over the dofs k in wave w's contiguous
// range [w c, (w + 1) c), c = ceil(nj / nw), into part(w, i); the next phase combines
// the nw partials in wave order. (The sums' association changes, not their terms.)
MB_HD __forceinline__ void combine6(const WVals& W, int i, int nw, double* o) {
  for (int e = 0; e < 6; ++e) o[e] = W.part(0, i)[e];
  for (int w = 1; w < nw; ++w)
    for (int e = 0; e < 6; ++e) o[e] += W.part(w, i)[e];
}
// lane i, wave w: sum over ancestors-or-self k in w's range of S_k qd_k
MB_HD inline void w_velocity_part(const WVals& W, const double* qd, int i, int w, int nw) {
  double v[6] = {0., 0., 0., 0., 0., 0.};
  const Mask am = *W.anc(i);
  int k0, k1;
  k_range(W.nj, w, nw, k0, k1);
#pragma unroll 2
  for (int k = k0; k < k1; ++k) {
    const bool in = (am >> k) & 1ull;
    const double qk = qd[k];
    for (int e = 0; e < 6; ++e) {
      const double t = W.S(k)[e] * qk;
      v[e] += in ? t : 0.;
    }
  }
  for (int e = 0; e < 6; ++e) W.part(w, i)[e] = v[e];
}
// lane i, wave w: sum over ancestors-or-self k in w's range of cq_k
MB_HD inline void w_accel_part(const WVals& W, int i, int w, int nw) {
  double a[6] = {0., 0., 0., 0., 0., 0.};
  const Mask am = *W.anc(i);
  int k0, k1;
  k_range(W.nj, w, nw, k0, k1);
#pragma unroll 2
  for (int k = k0; k < k1; ++k) {
    const bool in = (am >> k) & 1ull;
    for (int e = 0; e < 6; ++e) {
      const double t = W.cq(k)[e];
      a[e] += in ? t : 0.;
    }
  }
  for (int e = 0; e < 6; ++e) W.part(w, i)[e] = a[e];
}
// lane i, wave w: sum over the subtree bodies k in w's range of the body forces
MB_HD inline void w_force_part(const WVals& W, int i, int w, int nw) {
  double F[6] = {0., 0., 0., 0., 0., 0.};
  int k0, k1;
  k_range(W.nj, w, nw, k0, k1);
#pragma unroll 2
  for (int k = k0; k < k1; ++k) {
    const bool in = (*W.anc(k) >> i) & 1ull;
    for (int e = 0; e < 6; ++e) {
      const double t = W.fb(k)[e];
      F[e] += in ? t : 0.;
    }
  }
  for (int e = 0; e < 6; ++e) W.part(w, i)[e] = F[e];
}
// lane i: v_i from the partials, then cq_i = S_i qdd_i + v_i x (S_i qd_i)
MB_HD inline void w_velocity_accel_term(const WVals& W, const double* qd, const double* qdd, int i, int nw) {
  double v[6];
  combine6(W, i, nw, v);
  for (int e = 0; e < 6; ++e) W.v(i)[e] = v[e];
  double S[6], Sw[6], t6[6];
  const double wq = qd[i], qa = qdd ? qdd[i] : 0.;
  for (int e = 0; e < 6; ++e) {
    S[e] = W.S(i)[e];
    Sw[e] = S[e] * wq;
  }
  cross_m(v, Sw, t6);
  for (int e = 0; e < 6; ++e) W.cq(i)[e] = S[e] * qa + t6[e];
}
// lane i: a_i = -g + the partials, then the body force f_i = I_i a_i + v_i x* (I_i v_i) - fext_i
MB_HD inline void w_accel_body_force(const WVals& W, int i, int nw, const double* fx) {
  double a[6], p[6];
  combine6(W, i, nw, p);
  for (int e = 0; e < 6; ++e) a[e] = W.root_a()[e] + p[e];
  double v[6], f[6], Iv[6], t6[6], c[3], I6[6];
  for (int e = 0; e < 6; ++e) {
    W.a(i)[e] = a[e];
    v[e] = W.v(i)[e];
    I6[e] = W.Ic(i)[e];
  }
  for (int e = 0; e < 3; ++e) c[e] = W.c(i)[e];
  const double m = *W.m(i);
  inertia_mul(m, c, I6, a, f);
  inertia_mul(m, c, I6, v, Iv);
  cross_f(v, Iv, t6);
  for (int e = 0; e < 6; ++e) W.fb(i)[e] = f[e] + t6[e] - (fx ? fx[6 * i + e] : 0.);
}
// lane i: F_i from the partials, tau_i = S_i . F_i
MB_HD inline void w_joint_force_comb(const WVals& W, double* tau, int i, int nw) {
  double F[6];
  combine6(W, i, nw, F);
  for (int e = 0; e < 6; ++e) W.F(i)[e] = F[e];
  tau[i] = dot6(W.S(i), F);
}

// Cost records
struct CRec {
  const double* r;
  MB_HD int type() const { return (int)mb_lds(r)[0]; }
  MB_HD double weight() const { return mb_lds(r)[1]; }
  MB_HD int size() const { return (int)mb_lds(r)[3]; }
  MB_HD const double* d() const { return mb_lds(r + kCHdr); }
};

// dof carrying the frame of a frame / contact payload d = [joint record, R 9, p 3, ...]
MB_HD __forceinline__ int frame_dof(const Blk& b, const double* d) { return dof_of_rec(b, (int)d[0]); }

// oMf of a frame payload
MB_HD inline void frame_placement(const Blk& b, const WVals& V, const double* d, double* R, double* p) {
  const int j = frame_dof(b, d);
  matmul3(V.oR(j), d + 1, R);
  matvec3(V.oR(j), d + 10, p);
  p[0] += V.op(j)[0];
  p[1] += V.op(j)[1];
  p[2] += V.op(j)[2];
}

// Residual of a frame cost and, with S != null (the world motion of a dof that
// moves the frame), its Jacobian column. Returns the residual size (6 placement,
// 3 translation).
MB_HD inline int frame_residual(const Blk& b, const WVals& V, const CRec& C, const double* S, double* r, double* Jc) {
  const double* d = C.d();
  double Rf[9], pf[3];
  frame_placement(b, V, d, Rf, pf);
  double dR[9] = {0., 0., 0., 0., 0., 0., 0., 0., 0.}, dp[3] = {0., 0., 0.};
  if (S) {  // motion of oMf under S: dp = S_lin + S_ang x pf, dR = [S_ang]x Rf
    double t[3];
    cross3(S + 3, pf, t);
    for (int e = 0; e < 3; ++e) dp[e] = S[e] + t[e];
    for (int c = 0; c < 3; ++c) cross3(S + 3, Rf + 3 * c, dR + 3 * c);
  }
  if (C.type() == C_FRAME_TRANSLATION || C.type() == C_CONTACT_3D) {
    const double* pref = d + 13;
    for (int e = 0; e < 3; ++e) {
      r[e] = pf[e] - pref[e];
      if (Jc) Jc[e] = dp[e];
    }
    for (int e = 3; e < 6; ++e) {
      r[e] = 0.;
      if (Jc) Jc[e] = 0.;
    }
    return 3;
  }
  // rMf = Mref^-1 oMf
  const double* Rri = d + 13;
  const double* pri = d + 22;
  double Rr[9], pr[3], dRr[9], dpr[3];
  matmul3(Rri, Rf, Rr);
  matvec3(Rri, pf, pr);
  pr[0] += pri[0];
  pr[1] += pri[1];
  pr[2] += pri[2];
  matmul3(Rri, dR, dRr);
  matvec3(Rri, dp, dpr);
  Dual RD[9], PD[3], o[6];
  for (int e = 0; e < 9; ++e) RD[e] = Dual{Rr[e], dRr[e]};
  for (int e = 0; e < 3; ++e) PD[e] = Dual{pr[e], dpr[e]};
  log6_t<Dual>(RD, PD, o);
  for (int e = 0; e < 6; ++e) {
    r[e] = o[e].v;
    if (Jc) Jc[e] = S ? o[e].d : 0.;
  }
  return 6;
}

// Residual size of a cost record.
MB_HD inline int cost_nr(const Blk& b, const CRec& C, int nu) {
  const int t = C.type();
  if (t == C_CONTACT_FORCE) return (int)C.d()[1];
  if (t == C_FRICTION_CONE) return (int)C.d()[2];
  if (t == C_STATE) return 2 * b.nj;
  if (t == C_CONTROL) return nu;
  return (t == C_FRAME_PLACEMENT || t == C_FRAME_VELOCITY) ? 6 : 3;
}
// The activation of a cost record (its parameters end the record):
//   Quad / WeightedQuad (quadratic.hpp, weighted-quadratic.hpp:42-71): w (ones if
//     unweighted); a = 0.5 w r^2, Ar = w r, Arr = w
//   QuadraticBarrier (quadratic-barrier.hpp:88-117): lb, ub; with rl = min(r - lb, 0),
//     ru = max(r - ub, 0): a = 0.5 (rl^2 + ru^2), Ar = rl + ru, Arr = [r <= lb or r >= ub]
//   WeightedQuadraticBarrier (weighted-quadratic-barrier.hpp:35-70): lb, ub, w;
//     a = 0.5 w^2 (rl^2 + ru^2), Ar = w^2 (rl + ru), Arr = w [r <= lb or r >= ub]
// Per residual row i: value2 (twice its share of a: callers sum the rows, then
// halve), sgrad (X * Ar_i, as (X w) r for the quadratic kinds), hess (Arr_ii).
struct Act {
  int kind, nr;
  const double* p;
  MB_HD __forceinline__ double value2(int i, double r) const {
    const double* p = mb_lds(this->p);
    if (kind <= A_WEIGHTED_QUAD) return p[i] * r * r;
    const double rl = fmin(r - p[i], 0.), ru = fmax(r - p[nr + i], 0.);
    const double v = rl * rl + ru * ru;
    return kind == A_WEIGHTED_QUAD_BARRIER ? p[2 * nr + i] * p[2 * nr + i] * v : v;
  }
  MB_HD __forceinline__ double sgrad(int i, double r, double X) const {
    const double* p = mb_lds(this->p);
    if (kind <= A_WEIGHTED_QUAD) return X * p[i] * r;
    const double g = fmin(r - p[i], 0.) + fmax(r - p[nr + i], 0.);
    return X * (kind == A_WEIGHTED_QUAD_BARRIER ? p[2 * nr + i] * p[2 * nr + i] * g : g);
  }
  MB_HD __forceinline__ double hess(int i, double r) const {
    const double* p = mb_lds(this->p);
    if (kind <= A_WEIGHTED_QUAD) return p[i];
    const double h = (r - p[i] <= 0.) ? 1. : ((r - p[nr + i] >= 0.) ? 1. : 0.);
    return kind == A_WEIGHTED_QUAD_BARRIER ? p[2 * nr + i] * h : h;
  }
};
MB_HD inline Act cost_act(const Blk& b, const CRec& C, int nu) {
  const int nr = cost_nr(b, C, nu), kind = (int)C.r[2];
  const int np = kind <= A_WEIGHTED_QUAD ? nr : (kind == A_QUAD_BARRIER ? 2 * nr : 3 * nr);
  return Act{kind, nr, C.r + C.size() - np};
}
// costs whose residual Jacobian is dense over the configuration tangent (stored
// per cost: rows x jw, jw = nj, or 2 nj when a frame-velocity cost needs the
// velocity columns too): frame costs, CoM, frame velocity, and the free-flyer
// block of a state cost
MB_HD __forceinline__ bool jac_cost(const Blk& b, int type) {
  return type == C_FRAME_PLACEMENT || type == C_FRAME_TRANSLATION || type == C_COM_POSITION ||
         type == C_FRAME_VELOCITY || (type == C_STATE && b.ff);
}
MB_HD __forceinline__ int jac_rows(int type) {
  return (type == C_FRAME_TRANSLATION || type == C_COM_POSITION) ? 3 : 6;
}
MB_HD inline int count_jac_costs(const Blk& b, bool* vel_cols = nullptr) {
  int n = 0;
  bool fv = false;
  const double* cr = b.C;
  for (int k = 0; k < b.ncost; ++k) {
    const CRec C{cr};
    if (jac_cost(b, C.type())) ++n;
    if (C.type() == C_FRAME_VELOCITY) fv = true;
    cr += C.size();
  }
  if (vel_cols) *vel_cols = fv;
  return n;
}
// costs on the contact multipliers: CostModelContactForce, CostModelContactFrictionCone
MB_HD __forceinline__ bool force_cost(int type) { return type == C_CONTACT_FORCE || type == C_FRICTION_CONE; }
// Residual rows with a dense Jacobian (jac costs; force costs on an active contact
// when the force Jacobians are computed): the rows of the stacked R of calcDiff.
MB_HD inline int count_cost_rows(const Blk& b, int nu) {
  int n = 0;
  const bool fd = b.enable_force && b.nc > 0 && !b.impulse;
  const double* cr = b.C;
  for (int k = 0; k < b.ncost; ++k) {
    const CRec C{cr};
    if (jac_cost(b, C.type())) n += jac_rows(C.type());
    if (fd && force_cost(C.type()) && (int)C.d()[0] >= 0) n += cost_nr(b, C, nu);
    cr += C.size();
  }
  return n;
}
// row i of a force cost's residual from the multipliers lam of the contact rows
// [row0, row0 + nc) (lam unread for an inactive contact: lambda = 0):
//   contact force: lambda_i - fref_i (contact-force.hxx:33-50: jMf.actInv(f) is the multiplier);
//   friction cone: A_i . lambda_lin (contact-friction-cone.hxx:58)
MB_HD __forceinline__ double force_res(const CRec& C, const double* lam, int i) {
  const double* d = C.d();
  const int row0 = (int)d[0];
  if (C.type() == C_CONTACT_FORCE) return (row0 >= 0 ? lam[row0 + i] : 0.) - d[2 + i];
  if (row0 < 0) return 0.;
  const double* A = d + 3 + 3 * i;
  return A[0] * lam[row0] + A[1] * lam[row0 + 1] + A[2] * lam[row0 + 2];
}
// row i of a force cost's Jacobian column from the multiplier Jacobian column
// dl[row * ld] (the same linear map as force_res, without the offset)
MB_HD __forceinline__ double force_jac(const CRec& C, const double* dl, int64_t ld, int i) {
  const double* d = C.d();
  const int row0 = (int)d[0];
  if (C.type() == C_CONTACT_FORCE) return dl[(int64_t)(row0 + i) * ld];
  const double* A = d + 3 + 3 * i;
  return A[0] * dl[(int64_t)row0 * ld] + A[1] * dl[(int64_t)(row0 + 1) * ld] + A[2] * dl[(int64_t)(row0 + 2) * ld];
}
// activation value of a force cost (inactive contact: lambda = 0)
MB_HD inline double force_cost_activation(const Blk& b, const CRec& C, const double* lam, int nu) {
  const Act act = cost_act(b, C, nu);
  double a = 0.;
  for (int e = 0; e < act.nr; ++e) a += act.value2(e, force_res(C, lam, e));
  return 0.5 * a;
}

// Residual of a frame cost, value only (calc). Returns the residual size.
MB_HD __forceinline__ int frame_residual_value(const Blk& b, const WVals& V, const CRec& C, double* r) {
  const double* d = C.d();
  double Rf[9], pf[3];
  frame_placement(b, V, d, Rf, pf);
  if (C.type() == C_FRAME_TRANSLATION || C.type() == C_CONTACT_3D) {
    for (int e = 0; e < 3; ++e) r[e] = pf[e] - d[13 + e];
    return 3;
  }
  double Rr[9], pr[3];
  matmul3(d + 13, Rf, Rr);
  matvec3(d + 13, pf, pr);
  for (int e = 0; e < 3; ++e) pr[e] += d[22 + e];
  log6_t<double>(Rr, pr, r);
  return 6;
}

// Centre of mass (pinocchio::centerOfMass) from the world body CoMs
MB_HD inline void com_value(const Blk& b, const WVals& W, double* c) {
  double m = 0., h[3] = {0., 0., 0.};
  for (int k = 0; k < b.nj; ++k) {
    if (!carries_body(b, k)) continue;
    const double mk = *W.m(k);
    m += mk;
    for (int e = 0; e < 3; ++e) h[e] += mk * W.c(k)[e];
  }
  for (int e = 0; e < 3; ++e) c[e] = h[e] / m;
}

// free-flyer block of a state residual: log6(Mref^-1 M) (multibody.hxx:69)
MB_HD inline void ff_rel(const double* xref, const double* x, double* Rr, double* pr) {
  double R0[9], R1[9], dp[3];
  quat_to_R(xref + 3, R0);
  quat_to_R(x + 3, R1);
  matTmul3(R0, R1, Rr);
  for (int e = 0; e < 3; ++e) dp[e] = x[e] - xref[e];
  matTvec3(R0, dp, pr);
}

// entry i of the state residual diff(xref, x) beyond the free-flyer block
MB_HD __forceinline__ double state_res(const Blk& b, const double* xref, const double* x, int i) {
  if (i < b.nj) return x[qof(b, i)] - xref[qof(b, i)];
  return x[b.nq + i - b.nj] - xref[b.nq + i - b.nj];
}

// LOCAL velocity of a frame payload d minus vref (pinocchio::getFrameVelocity,
// frame-velocity.hxx:57-59), from the world body velocities in V.
MB_HD inline void frame_velocity_res(const Blk& b, const WVals& V, const double* d, double* r) {
  const int j = frame_dof(b, d);
  double Rf[9], pf[3], m6[6];
  frame_placement(b, V, d, Rf, pf);
  for (int e = 0; e < 6; ++e) m6[e] = V.v(j)[e];
  motion_act_inv(Rf, pf, m6, r);
  for (int e = 0; e < 6; ++e) r[e] -= d[13 + e];
}

// Activation value of one cost record (kinematics in V; velocities in V only with
// vel: frame-velocity costs are skipped without). Force costs return 0: they need
// the multipliers and are added after the contact solve.
MB_HD __forceinline__ double cost_activation(const Blk& b, const WVals& V, const CRec& C, const double* x,
                                             const double* u, int nu, bool vel = true) {
  const Act act = cost_act(b, C, nu);
  double a = 0.;
  if (C.type() == C_STATE) {
    const int ndx = 2 * b.nj;
    int i0 = 0;
    if (b.ff) {
      double Rr[9], pr[3], r[6];
      ff_rel(C.d(), x, Rr, pr);
      log6_t<double>(Rr, pr, r);
      for (int e = 0; e < 6; ++e) a += act.value2(e, r[e]);
      i0 = 6;
    }
    for (int i = i0; i < ndx; ++i) a += act.value2(i, state_res(b, C.d(), x, i));
  } else if (C.type() == C_CONTROL) {
    for (int i = 0; i < nu; ++i) a += act.value2(i, u[i] - C.d()[i]);
  } else if (force_cost(C.type())) {
    return 0.;
  } else if (C.type() == C_COM_POSITION) {
    double c[3];
    com_value(b, V, c);
    for (int i = 0; i < 3; ++i) a += act.value2(i, c[i] - C.d()[i]);
  } else if (C.type() == C_FRAME_VELOCITY) {
    if (!vel) return 0.;
    double r[6];
    frame_velocity_res(b, V, C.d(), r);
    for (int i = 0; i < 6; ++i) a += act.value2(i, r[i]);
  } else {
    double r[6] = {0., 0., 0., 0., 0., 0.};
    const int nr = frame_residual_value(b, V, C, r);
#pragma unroll
    for (int i = 0; i < 6; ++i)  // fixed trip count: r stays in registers
      if (i < nr) a += act.value2(i, r[i]);
  }
  return 0.5 * a;
}

// The long vector residuals (state, control) are summed lane-parallel in the calc:
// wide_cost says which records (the first kMaxWide such records) take that path.
constexpr int kMaxWide = 2;
MB_HD __forceinline__ bool wide_cost(const CRec& C, int nwide) {
  return (C.type() == C_STATE || C.type() == C_CONTROL) && nwide < kMaxWide;
}
// Lane l's share of twice the activation of a wide record: the rows i = l (mod L)
// (lane 0 also the free-flyer block of a state residual, log6 of the base).
MB_HD __forceinline__ double cost_activation_part(const Blk& b, const CRec& C, const double* x, const double* u,
                                                  int nu, int l, int L) {
  const Act act = cost_act(b, C, nu);
  double a = 0.;
  if (C.type() == C_STATE) {
    const int ndx = 2 * b.nj, i0 = b.ff ? 6 : 0;
    if (b.ff && l == 0) {
      double Rr[9], pr[3], r[6];
      ff_rel(C.d(), x, Rr, pr);
      log6_t<double>(Rr, pr, r);
      for (int e = 0; e < 6; ++e) a += act.value2(e, r[e]);
    }
    for (int i = i0 + l; i < ndx; i += L) a += act.value2(i, state_res(b, C.d(), x, i));
  } else {
    for (int i = l; i < nu; i += L) a += act.value2(i, u[i] - C.d()[i]);
  }
  return a;
}

// Cost value of the DAM (one thread; kinematics and velocities in V): sum of
// weight * activation in record (name) order (cost-sum.hxx:89-117).
MB_HD inline double cost_value(const Blk& b, const WVals& V, const double* x, const double* u, int nu) {
  double total = 0.;
  const double* cr = b.C;
  for (int k = 0; k < b.ncost; ++k) {
    const CRec C{cr};
    total += C.weight() * cost_activation(b, V, C, x, u, nu);
    cr += C.size();
  }
  return total;
}

// ---- contacts (ContactModel3D / 6D in the LOCAL frame) ----------------------
// Row offset of contact record k and its record pointer.
MB_HD inline const double* contact_rec(const Blk& b, int k, int* row0) {
  const double* r = b.K;
  int row = 0;
  for (int i = 0; i < k; ++i) {
    row += (int)r[0] == C_CONTACT_3D ? 3 : 6;
    r += (int)r[3];
  }
  *row0 = row;
  return r;
}

// a0 of a contact (contact-3d.hxx:35-43, contact-6d.hxx:31-44) in two parts,
// so that neither holds log6 and the frame motions live at once: the
// Baumgarte position term kp * (p - p_ref) | kp * log6(Mref^-1 oMf) (needs only
// the placements), then the frame drift acceleration (classical for 3D, gravity
// removed) + kd * v from the world velocity / acceleration of the body.
MB_HD __attribute__((always_inline)) inline void contact_a0_position(const Blk& b, const WVals& W, const CRec& C, double* a0) {
  const double kp = C.r[1];
  double r[6] = {0., 0., 0., 0., 0., 0.};
  if (kp != 0.) frame_residual_value(b, W, C, r);
  const int n = C.type() == C_CONTACT_3D ? 3 : 6;
  for (int e = 0; e < n; ++e) a0[e] = kp * r[e];
}
MB_HD __attribute__((always_inline)) inline void contact_a0_drift(const Blk& b, const WVals& W, const CRec& C, double* a0) {
  const double* d = C.d();
  const int j = frame_dof(b, d);
  double Rf[9], pf[3], m6[6], vf[6], af[6];
  frame_placement(b, W, d, Rf, pf);
  for (int e = 0; e < 6; ++e) m6[e] = W.v(j)[e];
  motion_act_inv(Rf, pf, m6, vf);
  for (int e = 0; e < 6; ++e) m6[e] = W.a(j)[e] - W.root_a()[e];  // data.a has no gravity
  motion_act_inv(Rf, pf, m6, af);
  const double kd = C.r[2];
  if (C.type() == C_CONTACT_3D) {
    double wxv[3];
    cross3(vf + 3, vf, wxv);
    for (int e = 0; e < 3; ++e) a0[e] += af[e] + wxv[e] + kd * vf[e];
  } else {
    for (int e = 0; e < 6; ++e) a0[e] += af[e] + kd * vf[e];
  }
}

// World force (at the origin) of contact record C for the multipliers lam
// (updateForce: jMf.act(Force(lambda[, 0])), contact-3d.hxx:59-67).
MB_HD inline void contact_world_force(const Blk& b, const WVals& W, const CRec& C, const double* lam, double* o) {
  double Rf[9], pf[3], f[6];
  frame_placement(b, W, C.d(), Rf, pf);
  const bool c3 = C.type() == C_CONTACT_3D;
  for (int e = 0; e < 6; ++e) f[e] = (c3 && e >= 3) ? 0. : lam[e];
  force_act(Rf, pf, f, o);
}

// lane j < nj: sum of the contact forces acting on dof j's body (world) into fx[6j..]
MB_HD inline void contact_joint_forces(const Blk& b, const WVals& W, const double* lam, double* fx, int j) {
  double F[6] = {0., 0., 0., 0., 0., 0.};
  const double* r = b.K;
  int row = 0;
  for (int k = 0; k < b.ncon; ++k) {
    const CRec C{r};
    if (frame_dof(b, C.d()) == j) {
      double o[6];
      contact_world_force(b, W, C, lam + row, o);
      for (int e = 0; e < 6; ++e) F[e] += o[e];
    }
    row += C.type() == C_CONTACT_3D ? 3 : 6;
    r += C.size();
  }
  for (int e = 0; e < 6; ++e) fx[6 * j + e] = F[e];
}

// lane c < nj: column c of the stacked contact Jacobian Jc (nc x nj,
// Jc[row * nj + c]) — the LOCAL frame Jacobian (pinocchio getFrameJacobian LOCAL,
// contact-3d.hxx:29 / contact-6d.hxx:29): the world motion S_c moved to the frame
// (SE3::actInv of oMf), zero unless c moves the frame's body; with At != null also
// into the columns [nj + row] of A (ld lda).
MB_HD __attribute__((always_inline)) inline void contact_jac_lane(const Blk& b, const WVals& W, int c, double* Jc, double* At,
                                                      int lda = 0) {
  double Sc[6];
  for (int e = 0; e < 6; ++e) Sc[e] = W.S(c)[e];
  const double* r = b.K;
  int row = 0;
  for (int k = 0; k < b.ncon; ++k) {
    const CRec C{r};
    const int j = frame_dof(b, C.d());
    double o[6] = {0., 0., 0., 0., 0., 0.};
    if ((*W.anc(j) >> c) & 1ull) {
      double Rf[9], pf[3];
      frame_placement(b, W, C.d(), Rf, pf);
      motion_act_inv(Rf, pf, Sc, o);
    }
    const int n = C.type() == C_CONTACT_3D ? 3 : 6;
    for (int e = 0; e < n; ++e) {
      Jc[(int64_t)(row + e) * b.nj + c] = o[e];
      if (At) At[(int64_t)(b.nj + row + e) * lda + c] = o[e];
    }
    row += n;
    r += C.size();
  }
}

// Placements, world quantities, composite inertias and M (into A, zeroed by
// the caller) for configuration q; `costs(wave, l)` runs on waves >= 1 in
// the phase after the kinematics (nullptr-like no-op allowed).
// `early(wave, l)` runs on waves >= 1 beside the local placements (work on x / u only).
#if defined(__HIP_DEVICE_COMPILE__)
// ---- fp64 matrix-core products (v_mfma_f64_16x16x4_f64) ---------------------------
// Fragment maps (MI355X guide, f64 16x16x4): A[i = lane & 15][k = lane >> 4],
// B[k = lane >> 4][j = lane & 15], C/D col = lane & 15, row = (lane >> 4) + 4 reg.
// Every wave of the workgroup takes 16 x 16 output tiles round-robin; loads outside
// the operands read as exact zeros, so padded rows / columns stay zero.
typedef double mb_f64x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ mb_f64x4 mb_mfma(double a, double b, mb_f64x4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
typedef __attribute__((address_space(3))) double mb_lds_d;
#endif

// ---- tree-sparse LTDL of the joint-space inertia (RBDA 6.3) ------------------------
// M (nj x nj, column-major at ld lda, both triangles as the CRBA writes them) has the
// branch-induced sparsity of the kinematic tree: M_ij != 0 only when i is an ancestor-
// or-self of j or j of i, in the dof tree whose parent of d is chain_parent(b, d) (the
// free-flyer's six dofs form a chain). Featherstone's LTDL factorisation M = L^T D L
// keeps L (unit lower triangular) on that pattern, and the reference's solvers reach
// M^-1 through Pinocchio's sparse Cholesky of M (contact-fwddyn.hxx:94,132: forwardDynamics
// / getKKTContactDynamicMatrixInverse; free-fwddyn.hxx:64: aba). A dof's row is final once
// all its descendants are eliminated, and dofs of one depth are never ancestor and
// descendant of each other, so a whole depth level is eliminated in one step, deepest
// first: the chain of dependent steps is the tree depth (16 on Talos) instead of the nj (38)
// pivots of a dense factorisation, and each step is one FMA per pattern entry.
// G = L^-1 (same pattern) follows level by level from the root, and
//   M^-1 = G D^-1 G^T,   M^-1 B = G (D^-1 (G^T B)),
// whose sums run over common ancestors only.
// Storage: L, then G, in place of M's lower triangle on the pattern, D on the diagonal;
// M's upper triangle is left as it was. The factorisation and G run on wave 0 alone
// (run_w0 steps, one wave-level fence per level); the products on the whole workgroup.
struct TreeWork {
  Mask* cm;      // nj: chain ancestors-or-self of each dof (index order = depth order)
  Mask* dsc;     // nj: strict descendants
  Mask* lev;     // 64: the dofs of each depth
  double* dinv;  // nj: 1 / D
  int* bad;      // set on a non-positive D (the LLT failure)
};
MB_HD __forceinline__ Mask chain_mask(const Blk& b, const WVals& W, int d) {
  return (b.ff && d < 6) ? ((Mask(2) << d) - 1) : *W.anc(d);
}
MB_HD __forceinline__ int mask_depth(Mask m) { return __builtin_popcountll(m) - 1; }
MB_HD __forceinline__ int mask_low(Mask m) { return __builtin_ctzll(m); }
// 1 / d to working precision: v_rcp_f64 corrected by x0 (1 + e + e^2), e = 1 - d x0
// (relative error e^3, as the blocked Gauss-Jordan's pivots)
MB_HD __forceinline__ double mb_recip(double d) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double x0 = __builtin_amdgcn_rcp(d);
  const double e = __builtin_fma(-d, x0, 1.);
  return __builtin_fma(x0, __builtin_fma(e, e, e), x0);
#else
  return 1. / d;
#endif
}
// the tree's depth (uniform: every thread computes it from the ancestor masks)
MB_HD inline int tree_depth(const Blk& b, const WVals& W) {
  int md = 0;
  for (int k = 0; k < b.nj; ++k) {
    const int d = mask_depth(chain_mask(b, W, k));
    md = d > md ? d : md;
  }
  return md;
}
// M -> (L, D) in place, then L -> G = L^-1 in place; tw.dinv = 1 / D. md: tree_depth.
// The level steps as executor phases (the host emulation; the device for trees deeper
// than its register fast path, tree_ltdl_wave).
template <class X>
MB_HD inline void tree_ltdl_steps(const X& ex, const Blk& b, const WVals& W, double* A_, int lda, const TreeWork& tw,
                                  int md) {
  const int nj = b.nj;
  double* A = ex.lds(A_);
  ex.run_w0([&](int lane) {
    if (lane < nj) {
      const Mask c = chain_mask(b, W, lane);
      Mask d = 0;
      for (int k = lane + 1; k < nj; ++k) d |= ((chain_mask(b, W, k) >> lane) & 1ull) << k;
      tw.cm[lane] = c;
      tw.dsc[lane] = d;
    }
    Mask lv = 0;  // lane l: the dofs at depth l
    for (int k = 0; k < nj; ++k) lv |= Mask(mask_depth(chain_mask(b, W, k)) == lane ? 1 : 0) << k;
    tw.lev[lane] = lv;
    if (lane == 0) *tw.bad = 0;
  });
  // Level L, deepest first: (a) every row i above level L takes the contributions of its
  // descendants k at depth L (rows final since the deeper levels), H_ij -= H_ki H_kj / D_k
  // for j in the ancestors-or-self of i; (b) the rows of level L + 1 (final now) are
  // scaled to L_kj = H_kj / D_k. (a) reads the rows of level L and writes rows above it,
  // (b) rewrites the rows of level L + 1: no lane reads what another writes.
#pragma unroll 1
  for (int L = md; L >= -1; --L)
    ex.run_w0([&](int i) {
      if (i >= nj) return;
      const Mask ci = tw.cm[i];
      const int di = mask_depth(ci);
      if (di < L) {
        Mask km = tw.dsc[i] & tw.lev[L];
        while (km) {
          const int k = mask_low(km);
          km &= km - 1;
          const double f = A[k + lda * i] * mb_recip(A[k + lda * k]);
          Mask jm = ci;
          while (jm) {
            const int j = mask_low(jm);
            jm &= jm - 1;
            A[i + lda * j] -= f * A[k + lda * j];
          }
        }
      } else if (di == L + 1) {
        const double d = A[i + lda * i];
        const double inv = mb_recip(d);
        if (!(d > 0.)) *tw.bad = 1;
        tw.dinv[i] = inv;
        Mask jm = ci & ~(Mask(1) << i);
        while (jm) {
          const int j = mask_low(jm);
          jm &= jm - 1;
          A[i + lda * j] *= inv;
        }
      }
    });
  // G = L^-1: G_k = e_k - sum_{m in anc(k)} L_km G_m, level L from the root: row k (deeper
  // than L) takes the term of its ancestor m at depth L, whose row is final; position (k, m)
  // holds L_km until this step and G_km from it on.
#pragma unroll 1
  for (int L = 0; L < md; ++L)
    ex.run_w0([&](int k) {
      if (k >= nj) return;
      const Mask ck = tw.cm[k];
      if (mask_depth(ck) <= L) return;
      const int m = mask_low(ck & tw.lev[L]);
      const double l = A[k + lda * m];
      Mask im = ck & ((Mask(1) << m) - 1);
      while (im) {
        const int i = mask_low(im);
        im &= im - 1;
        A[k + lda * i] -= l * A[m + lda * i];
      }
      A[k + lda * m] = -l;
    });
  ex.sync();
}
constexpr int kTreeKD = 16;  // depth bound of the device fast path (below)
#if defined(__HIP_DEVICE_COMPILE__)
// Device fast path of tree_ltdl for trees of depth < kTreeKD, on wave 0 in one phase:
// lane i holds row i of the factor in registers, path-indexed (entry s = the column of
// i's ancestor at depth s; s = depth(i) the diagonal), so every update is a static-index
// register FMA; the rows other lanes need (a level's rows, then G's rows) go through LDS
// (PR: nj x kTreeKD), the levels and descendant sets are wave ballots, and one wave-level
// fence separates the levels. Same results as the generic steps up to the summation order
// of a row's contributions.
#ifndef MB_GJ_MARK
#define MB_GJ_MARK(id)  // (tools/mb_probe: phase stamps)
#endif
typedef __attribute__((address_space(3))) Mask mb_lds_mask;
typedef __attribute__((address_space(3))) int mb_lds_int;
__device__ __forceinline__ void tree_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// (the LDS operands arrive typed as LDS; the own row lives in registers during the
// elimination, then L in the row's LDS copy, so only G's row is in registers after it)
// (MB_TREE_NOINLINE builds it out of line: inlined into the rollout kernel at its
// 256-VGPR cap, the register allocation trips the backend's "even aligned vector
// registers" check; the rollout takes the dense solve instead, k_fwd.hip MB_CALC_DENSE.)
#ifdef MB_TREE_NOINLINE
#define MB_TREE_INL __attribute__((noinline))
#else
#define MB_TREE_INL __forceinline__
#endif
__device__ __forceinline__ Mask readlane_mask(Mask v, int l) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
  return (Mask(hi) << 32) | lo;
}
__device__ MB_TREE_INL void tree_ltdl_wave(const mb_lds_mask* anc, int ff, int nj, mb_lds_d* A, int lda,
                                           int md, mb_lds_d* PR, mb_lds_d* dinv_out, mb_lds_int* bad_out) {
  // Written for the instruction stream of one wave: every register array index is static
  // (the levels are unrolled, so level L touches only the path entries s < L), the
  // level's dofs are a uniform (scalar) loop with their rows read as LDS broadcasts, and
  // every LDS access is unconditional within its lanes.
  constexpr int KD = kTreeKD;
  const int pld = md + 1;  // PR row stride (a row has depth + 1 <= md + 1 entries)
  MB_GJ_MARK(0);
  const int lane = (int)threadIdx.x & 63;
  const bool act = lane < nj;
  const int rl = act ? lane : 0;  // (inactive lanes read row 0 and store nothing)
  const Mask cmi = act ? ((ff && lane < 6) ? ((Mask(2) << lane) - 1) : anc[lane]) : Mask(1);
  const int di = act ? mask_depth(cmi) : -1;
  // the ancestors by depth (col[s], s <= di; col[di] = the dof itself; beyond: the dof)
  int col[KD];
  {
    Mask cur = cmi;
#pragma unroll
    for (int s = 0; s < KD; ++s) {
      const int c = (int)__builtin_ctzll(cur | (Mask(1) << 63));
      col[s] = c < nj ? c : rl;
      cur &= cur - 1;
    }
  }
  // row i of M, path-indexed (entries beyond the diagonal are never read)
  double R[KD];
#pragma unroll
  for (int s = 0; s < KD; ++s) R[s] = A[rl + lda * col[s]];
  mb_lds_d* pr = PR + pld * rl;
  MB_GJ_MARK(1);
  double dinv = 0.;
  bool bad = false;
  // the rows of depth L are final: stored for the level that reads them, with 1 / D
  // (L static: the diagonal is R[L], and the row has L + 1 entries)
  auto finalize = [&](auto Lc) __attribute__((always_inline)) {
    constexpr int L = decltype(Lc)::value;
    if (act && di == L) {
#pragma unroll
      for (int s = 0; s <= L; ++s) pr[s] = R[s];
      const double d = R[L];
      dinv = mb_recip(d);
      bad = bad || !(d > 0.);
      dinv_out[lane] = dinv;
    }
  };
  // (the deepest level: every row of depth md is final from the start)
#pragma unroll
  for (int s = 0; s < KD; ++s)
    if (act && di == md && s <= md) pr[s] = R[s];
  if (act && di == md) {
    double d = 0.;
#pragma unroll
    for (int s = 0; s < KD; ++s) d = s == di ? R[s] : d;
    dinv = mb_recip(d);
    bad = bad || !(d > 0.);
    dinv_out[lane] = dinv;
  }
  tree_wave_sync();
  MB_GJ_MARK(2);
  // elimination, deepest level first: row i takes the contributions of its descendants k
  // at depth L, H_is -= (H_ki / D_k) H_ks over the path entries s <= depth(i) < L
  auto level = [&](auto Lc) __attribute__((always_inline)) {
    constexpr int L = decltype(Lc)::value;
    if (L > md) return;
    Mask lev = __ballot(act && di == L);  // the dofs at depth L (uniform)
    const bool mine = act && di < L;
    while (lev) {
      const int k = mask_low(lev);
      lev &= lev - 1;
      const Mask ck = readlane_mask(cmi, k);
      if (mine && ((ck >> lane) & 1ull)) {
        const mb_lds_d* pk = PR + pld * k;
        const double f = pk[di] * dinv_out[k];
#pragma unroll
        for (int s = 0; s < L; ++s) R[s] = __builtin_fma(-f, pk[s], R[s]);
      }
    }
    finalize(std::integral_constant<int, L - 1>{});
    tree_wave_sync();
    MB_GJ_MARK(3 + md - L);
  };
  static_assert(KD == 16, "the levels below are unrolled for kTreeKD = 16");
  level(std::integral_constant<int, 15>{});
  level(std::integral_constant<int, 14>{});
  level(std::integral_constant<int, 13>{});
  level(std::integral_constant<int, 12>{});
  level(std::integral_constant<int, 11>{});
  level(std::integral_constant<int, 10>{});
  level(std::integral_constant<int, 9>{});
  level(std::integral_constant<int, 8>{});
  level(std::integral_constant<int, 7>{});
  level(std::integral_constant<int, 6>{});
  level(std::integral_constant<int, 5>{});
  level(std::integral_constant<int, 4>{});
  level(std::integral_constant<int, 3>{});
  level(std::integral_constant<int, 2>{});
  level(std::integral_constant<int, 1>{});
  MB_GJ_MARK(19);
  // L = row i / D_i below the diagonal (registers; the final row values are in R)
  double Lr[KD];
#pragma unroll
  for (int s = 0; s < KD; ++s) Lr[s] = R[s] * dinv;
  // G = L^-1 from the root: row k takes the term of its ancestor at depth t (whose G row,
  // final after step t - 1, is read from PR); the rows of depth t + 1 are final after step t
  double Gr[KD];
#pragma unroll
  for (int s = 0; s < KD; ++s) Gr[s] = 0.;
  tree_wave_sync();
#pragma unroll
  for (int t = 0; t < KD - 1; ++t) {
    if (t < md) {
      if (act && di > t) {
        const mb_lds_d* pm = PR + pld * col[t];
        double g[KD];
#pragma unroll
        for (int s = 0; s < t; ++s) g[s] = pm[s];
        const double l = Lr[t];
#pragma unroll
        for (int s = 0; s < t; ++s) Gr[s] = __builtin_fma(-l, g[s], Gr[s]);
        Gr[t] = -l;
        if (di == t + 1)
#pragma unroll
          for (int s = 0; s <= t; ++s) pr[s] = Gr[s];
      }
      tree_wave_sync();
    }
  }
  MB_GJ_MARK(20);
  // G below the diagonal into A's pattern entries (D stays on the diagonal)
  if (act)
#pragma unroll
    for (int s = 0; s < KD - 1; ++s)
      if (s < di) A[lane + lda * col[s]] = Gr[s];
  if (lane == 0) *bad_out = 0;
  tree_wave_sync();
  if (bad) *bad_out = 1;
  MB_GJ_MARK(21);
}
#endif
#if defined(__HIP_DEVICE_COMPILE__)
// G's entry (r, m) from the dense storage tree_ltdl leaves (G below the diagonal on the
// pattern, exact zeros elsewhere below it, D on the diagonal: G_rr = 1), zero above the
// diagonal and outside nj
__device__ __forceinline__ double tree_gd(const mb_lds_d* A, int lda, int nj, int r, int m) {
  const bool in = r < nj && m < nj;
  const double v = A[in ? r + lda * m : 0];
  return (!in || m > r) ? 0. : (m == r ? 1. : v);
}
// Minv = G D^-1 G^T on the matrix cores: the upper 16 x 16 tiles, each entry with r <= c
// stored at (r, c) and (c, r) (exactly symmetric); a tile's k-range stops at the smaller
// block (G is lower triangular)
__device__ __forceinline__ void tree_minv_mfma(const double* A_, int lda, int nj, const double* dinv_, double* Mi_) {
  const mb_lds_d* A = (const mb_lds_d*)lds_ptr(A_);
  const mb_lds_d* dinv = (const mb_lds_d*)lds_ptr(dinv_);
  mb_lds_d* Mi = (mb_lds_d*)lds_ptr(Mi_);
  const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6, nw = (int)blockDim.x >> 6;
  const int li = lane & 15, lk = lane >> 4, nt = (nj + 15) >> 4, ntiles = nt * (nt + 1) / 2;
#pragma unroll 1
  for (int tile = wave; tile < ntiles; tile += nw) {
    int ti = 0, rem = tile;
    while (rem >= nt - ti) {
      rem -= nt - ti;
      ++ti;
    }
    const int tj = ti + rem;
    const int r = 16 * ti + li, c = 16 * tj + li;
    const int kmax = 16 * ti + 16 < nj ? 16 * ti + 16 : nj;
    mb_f64x4 acc0 = {0., 0., 0., 0.}, acc1 = {0., 0., 0., 0.};  // two chains (even / odd k-steps)
#pragma unroll 2
    for (int kb = 0; kb < kmax; kb += 8) {
      const int m0 = kb + lk, m1 = kb + 4 + lk;
      const double w0 = m0 < nj ? dinv[m0] : 0., w1 = m1 < nj ? dinv[m1] : 0.;
      acc0 = mb_mfma(tree_gd(A, lda, nj, r, m0), tree_gd(A, lda, nj, c, m0) * w0, acc0);
      if (kb + 4 < kmax) acc1 = mb_mfma(tree_gd(A, lda, nj, r, m1), tree_gd(A, lda, nj, c, m1) * w1, acc1);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = 16 * ti + lk + 4 * q, col = 16 * tj + li;
      const double v = acc0[q] + acc1[q];
      if (row < nj && col < nj && row <= col) {
        Mi[row + lda * col] = v;
        Mi[col + lda * row] = v;
      }
    }
  }
}
// The right-hand sides B (nj x nb at A + lda nj) -> M^-1 B in place on the matrix cores:
// T = D^-1 G^T B (T: nj x nb, ld nj), a workgroup barrier, X = G T. Every thread calls.
__device__ __forceinline__ void tree_solve_mfma(const double* A_, int lda, int nj, int nb, const double* dinv_,
                                                double* T_) {
  const mb_lds_d* A = (const mb_lds_d*)lds_ptr(A_);
  const mb_lds_d* dinv = (const mb_lds_d*)lds_ptr(dinv_);
  mb_lds_d* T = (mb_lds_d*)lds_ptr(T_);
  mb_lds_d* B = (mb_lds_d*)lds_ptr(A_ + (int64_t)lda * nj);
  const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6, nw = (int)blockDim.x >> 6;
  const int li = lane & 15, lk = lane >> 4, tr = (nj + 15) >> 4, tc = (nb + 15) >> 4;
  // T tile (tm, tcc): rows m, k over r >= 16 tm
#pragma unroll 1
  for (int tile = wave; tile < tr * tc; tile += nw) {
    const int tm = tile / tc, tcc = tile - tm * tc;
    const int m = 16 * tm + li, c = 16 * tcc + li;
    mb_f64x4 acc0 = {0., 0., 0., 0.}, acc1 = {0., 0., 0., 0.};
#pragma unroll 2
    for (int kb = 16 * tm; kb < nj; kb += 8) {
      const int r0 = kb + lk, r1 = kb + 4 + lk;
      const double b0 = (r0 < nj && c < nb) ? B[r0 + lda * c] : 0.;
      const double b1 = (r1 < nj && c < nb) ? B[r1 + lda * c] : 0.;
      acc0 = mb_mfma(tree_gd(A, lda, nj, r0, m), b0, acc0);
      if (kb + 4 < nj) acc1 = mb_mfma(tree_gd(A, lda, nj, r1, m), b1, acc1);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = 16 * tm + lk + 4 * q, col = 16 * tcc + li;
      if (row < nj && col < nb) T[row + nj * col] = (acc0[q] + acc1[q]) * dinv[row];
    }
  }
  __syncthreads();
  // X tile (tr_, tcc): rows r, k over m <= 16 tr_ + 15
#pragma unroll 1
  for (int tile = wave; tile < tr * tc; tile += nw) {
    const int ti = tile / tc, tcc = tile - ti * tc;
    const int r = 16 * ti + li, c = 16 * tcc + li;
    const int kmax = 16 * ti + 16 < nj ? 16 * ti + 16 : nj;
    mb_f64x4 acc0 = {0., 0., 0., 0.}, acc1 = {0., 0., 0., 0.};
#pragma unroll 2
    for (int kb = 0; kb < kmax; kb += 8) {
      const int m0 = kb + lk, m1 = kb + 4 + lk;
      const double t0 = (m0 < nj && c < nb) ? T[m0 + nj * c] : 0.;
      const double t1 = (m1 < nj && c < nb) ? T[m1 + nj * c] : 0.;
      acc0 = mb_mfma(tree_gd(A, lda, nj, r, m0), t0, acc0);
      if (kb + 4 < kmax) acc1 = mb_mfma(tree_gd(A, lda, nj, r, m1), t1, acc1);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = 16 * ti + lk + 4 * q, col = 16 * tcc + li;
      if (row < nj && col < nb) B[row + lda * col] = acc0[q] + acc1[q];
    }
  }
  __syncthreads();
}
#endif
// M -> (L, D) -> G = L^-1 in place, tw.dinv = 1 / D (tree_ltdl_steps / tree_ltdl_wave).
// PR: (md + 1) * nj doubles of scratch (the device fast path's rows; the generic steps
// use tw.cm / tw.dsc instead, so the two may share their space).
// Independent work of the caller for the waves the factorisation leaves idle: side(slot,
// lane, nlanes) on waves >= 1 (lane counted from wave 1), slots 0 .. nslots - 1 one after
// another, the side waves meeting at an LDS counter (ctr, zeroed by the caller in an
// earlier phase) between slots. Without the device fast path the slots run afterwards as
// ordinary phases.
struct TreeNoSide {
  MB_HD void operator()(int, int, int) const {}
};
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ void tree_side_barrier(int* ctr_, int target) {
  mb_lds_int* ctr = (mb_lds_int*)lds_ptr(ctr_);
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
}
#endif
template <class X, class Side = TreeNoSide>
MB_HD __forceinline__ void tree_ltdl(const X& ex, const Blk& b, const WVals& W, double* A, int lda, const TreeWork& tw,
                                     int md, double* PR, Side side = Side{}, int nslots = 0, int* ctr = nullptr) {
#if defined(__HIP_DEVICE_COMPILE__)
#ifndef MB_TREE_NO_WAVE
  if (md < kTreeKD) {
    double* const Al = ex.lds(A);
    double* const PRl = ex.lds(PR);
    ex.run([&](int tid) {
      if (tid < 64) {
        tree_ltdl_wave((const mb_lds_mask*)ex.lds(W.anc(0)), b.ff ? 1 : 0, b.nj, (mb_lds_d*)Al, lda, md,
                       (mb_lds_d*)PRl, (mb_lds_d*)ex.lds(tw.dinv), (mb_lds_int*)ex.lds(tw.bad));
      } else if (nslots > 0) {
        const int sl = tid - 64, snt = ex.nt - 64;
#pragma unroll 1
        for (int slot = 0; slot < nslots; ++slot) {
          if (slot > 0) tree_side_barrier(ctr, (snt >> 6) * slot);
          side(slot, sl, snt);
        }
      }
    });
    return;
  }
#endif
#endif
  (void)PR;
  tree_ltdl_steps(ex, b, W, A, lda, tw, md);
  for (int slot = 0; slot < nslots; ++slot)
    ex.run([&](int lane) {
      if (lane >= 64) side(slot, lane - 64, ex.nt - 64);
    });
}
// G's entry (r, m), m an ancestor-or-self of r (the diagonal holds D: G_rr = 1)
MB_HD __forceinline__ double tree_g(const double* A, int lda, int r, int m) { return m == r ? 1. : A[r + lda * m]; }
// Minv (ld lda) = G D^-1 G^T from tree_ltdl, exactly symmetric (the sum for (r, c) and
// (c, r) has the same terms in the same order). Returns false on a non-positive pivot.
// (device: on the matrix cores, tree_minv_mfma)
template <class X>
MB_HD inline bool tree_minv(const X& ex, const Blk& b, const double* A_, int lda, const TreeWork& tw, double* Mi_) {
#if defined(__HIP_DEVICE_COMPILE__)
  ex.run([&](int) { tree_minv_mfma(A_, lda, b.nj, tw.dinv, Mi_); });
  return *tw.bad == 0;
#endif
  const int nj = b.nj;
  const double* A = ex.lds(A_);
  double* Mi = ex.lds(Mi_);
  ex.run([&](int lane) {
    for (int e = lane; e < nj * nj; e += ex.nt) {
      const int c = e / nj, r = e - nj * c;
      Mask mm = tw.cm[r] & tw.cm[c];
      double s = 0.;
      while (mm) {
        const int m = mask_low(mm);
        mm &= mm - 1;
        s += (tree_g(A, lda, r, m) * tree_g(A, lda, c, m)) * tw.dinv[m];
      }
      Mi[r + lda * c] = s;
    }
  });
  return *tw.bad == 0;
}
// B (nj x nb at A + lda nj, ld lda: the right-hand sides beside M) -> M^-1 B in place,
// through T = D^-1 G^T B (nj x nb, ld nj). Returns false on a non-positive pivot.
template <class X>
MB_HD inline bool tree_solve(const X& ex, const Blk& b, double* A_, int lda, int nb, const TreeWork& tw, double* T_) {
#if defined(__HIP_DEVICE_COMPILE__)
  ex.run([&](int) { tree_solve_mfma(A_, lda, b.nj, nb, tw.dinv, T_); });
  return *tw.bad == 0;
#endif
  const int nj = b.nj;
  double* A = ex.lds(A_);
  double* T = ex.lds(T_);
  double* B = A + (int64_t)lda * nj;
  ex.run([&](int lane) {
    for (int e = lane; e < nj * nb; e += ex.nt) {
      const int c = e / nj, m = e - nj * c;
      const double* bc = B + (int64_t)lda * c;
      Mask rm = tw.dsc[m];
      double s0 = bc[m], s1 = 0.;  // (two partial sums: the root's row has nj terms)
      while (rm) {
        const int r = mask_low(rm);
        rm &= rm - 1;
        s0 += A[r + lda * m] * bc[r];
        if (!rm) break;
        const int r2 = mask_low(rm);
        rm &= rm - 1;
        s1 += A[r2 + lda * m] * bc[r2];
      }
      T[m + nj * c] = (s0 + s1) * tw.dinv[m];
    }
  });
  ex.run([&](int lane) {
    for (int e = lane; e < nj * nb; e += ex.nt) {
      const int c = e / nj, r = e - nj * c;
      const double* tc = T + (int64_t)nj * c;
      Mask mm = tw.cm[r] & ~(Mask(1) << r);
      double s = tc[r];
      while (mm) {
        const int m = mask_low(mm);
        mm &= mm - 1;
        s += A[r + lda * m] * tc[m];
      }
      B[r + (int64_t)lda * c] = s;
    }
  });
  return *tw.bad == 0;
}

template <class X, class EarlyF, class CostF>
MB_HD inline void world_kinematics(const X& ex, const Blk& b, const WVals& W, const double* q, double* A, int lda,
                                   EarlyF early, CostF costs, bool world_composite = false) {
  const int nj = b.nj;
  ex.run([&](int lane) {
    if (lane < nj) w_joint_local(b, W, q, lane);
    if (lane >= 64) early(lane >> 6, lane & 63);
  });
  ex.run([&](int lane) {
    if (lane < nj) {
      w_walk(b, W, lane);
      w_joint_world(b, W, lane);
    }
  });
  // CRBA about each column's joint: the subtree composites in wave partials (beside them,
  // the cost records on waves >= 1), then the columns (rows split over all the waves); with
  // `world_composite` (the calcDiff) the columns' lanes also store the subtree composites
  // about the world origin
  const int npw = part_waves(ex.nt);
  ex.run([&](int lane) {
    const int w = lane >> 6, j = lane & 63;
    if (j < nj && w < npw) w_crba_composite_part(b, W, j, w, npw);
    if (w >= 1) costs(w, j);
  });
  ex.run([&](int lane) {
    const int w = lane >> 6, j = lane & 63;
    if (j < nj) w_crba_column(b, W, j, A, lda, w, ex.nt >> 6, npw, world_composite);
  });
}

// Joint torques of RNEA(q, qd, qdd) (qdd == nullptr: 0) with the kinematics in W;
// fx (6 per dof, world frame at the origin, may be null): external forces,
// as pinocchio::rnea(model, data, q, v, a, fext).
template <class X>
MB_HD inline void world_rnea(const X& ex, const Blk& b, const WVals& W, const double* qd, const double* qdd,
                             double* tau, const double* fx = nullptr) {
  const int nj = b.nj, nw = part_waves(ex.nt);
  // every ancestor / subtree sum split over the waves (w_*_part), combined by lane i
  ex.run([&](int lane) {
    const int w = lane >> 6, i = lane & 63;
    if (i < nj && w < nw) w_velocity_part(W, qd, i, w, nw);
  });
  ex.run([&](int lane) {
    if (lane < nj) w_velocity_accel_term(W, qd, qdd, lane, nw);
  });
  ex.run([&](int lane) {
    const int w = lane >> 6, i = lane & 63;
    if (i < nj && w < nw) w_accel_part(W, i, w, nw);
  });
  ex.run([&](int lane) {
    if (lane < nj) w_accel_body_force(W, lane, nw, fx);
  });
  ex.run([&](int lane) {
    const int w = lane >> 6, i = lane & 63;
    if (i < nj && w < nw) w_force_part(W, i, w, nw);
  });
  ex.run([&](int lane) {
    if (lane < nj) w_joint_force_comb(W, tau, lane, nw);
  });
}

// Euler step of the state (euler.hxx:64-68 + StateMultibody::integrate): lane i < nj
// writes v_next[i] and the configuration entries of dof i (lane 0 the free-flyer's
// seven: M exp6(v dt + a dt^2)). a: the acceleration (every lane reads a[0..5]).
MB_HD inline void euler_step(const Blk& b, const double* x, const double* a, double dt, double* xnext, int i) {
  const int nq = b.nq;
  const double v = x[nq + i], ai = a[i];
  xnext[nq + i] = v + ai * dt;
  if (b.ff && i < 6) {
    if (i == 0) {
      double dq[6];
      for (int e = 0; e < 6; ++e) dq[e] = x[nq + e] * dt + a[e] * (dt * dt);
      ff_integrate(x, dq, xnext);
    }
  } else {
    const int qi = qof(b, i);
    xnext[qi] = x[qi] + (v * dt + ai * dt * dt);
  }
}

// LDS (doubles) of the calc scratch for nj dofs and nc contact rows.
MB_HD inline int64_t calc_work_doubles(int nj, int nc = 0) {
  return pad2(WVals::doubles(nj)) + (int64_t)lda_of(nj) * (nj + nc + 1) + 2 * nj + kMaxCosts + 8 + (int64_t)nc * nj + nc +
         (int64_t)nc * (nc + 1) + 128 + part_doubles(nj);
}

// The calc's cost records other than the wide ones (knot_calc_x): record item i on lane
// i / 3 of side wave i % 3 (sl: the lane counted from the first side wave, snt: the side
// lanes), each record's weighted value into cv[k]. It rebuilds the block's views from the
// LDS pointers, so it can be built out of line (MB_TREE_NOINLINE, as tree_ltdl_wave).
#if defined(__HIP_DEVICE_COMPILE__) && defined(MB_TREE_NOINLINE)
__device__ __attribute__((noinline))
#else
MB_HD __forceinline__
#endif
void calc_cost_records(const double* P_, double* w_, double* parts_, const double* x_, const double* ub_, double* cv_,
                       int sl, int snt) {
  const double* P = mb_lds(P_);
  const Blk b = parse(P);
  const WVals W{mb_lds(w_), b.nj, mb_lds(parts_)};
  const double* x = mb_lds(x_);
  const double* ub = mb_lds(ub_);
  double* cv = mb_lds(cv_);
  const int nu = b.nj - b.nun, nc = b.nc;
  const bool imp = b.impulse;
  const int nsw = snt >> 6, item = nsw * (sl & 63) + (sl >> 6);
  const double* cr = b.C;
  int nn = 0, nw = 0;
  for (int k = 0; k < b.ncost; ++k) {
    const CRec C{cr};
    if (wide_cost(C, nw)) {
      ++nw;
    } else {
      if (item == nn) {
        double v = C.type() == C_FRAME_VELOCITY && imp ? 0. : cost_activation(b, W, C, x, ub, nu);
        if (force_cost(C.type()) && nc == 0) v = force_cost_activation(b, C, nullptr, nu);
        cv[k] = C.weight() * v;
      }
      ++nn;
    }
    cr += C.size();
  }
}

// model->calc(data, x, u) for the Euler∘FreeFwdDynamics knot (euler.hxx:41-80,
// free-fwddyn.hxx:44-79): a = (M + diag(armature))^-1 (u - nle) in world frame;
// with contacts, Euler∘ContactFwdDynamics (contact-fwddyn.hxx:59-104):
// pinocchio::forwardDynamics by the Schur complement,
//   [Y | z] = M^-1 [Jc^T | tau - nle],  S = Jc Y + damping I,
//   lambda = -S^-1 (Jc z + a0),  a = z + Y lambda.
// Needs >= 256 threads (4 waves): independent work of one phase runs on
// different waves (divergent lanes of one wave would serialise) — wave 0 the
// recursions and composite inertias, waves 1-3 the cost records (state / control residuals row-parallel).
// Every thread must call (phases end in barriers). x, u readable by all lanes;
// writes xnext[0..nx) and returns the knot cost. `w`: calc_work_doubles(nj, nc).
template <class X>
MB_HD __forceinline__ double knot_calc_x(const X& ex, const double* P, int nx, const double* x, const double* u, bool use_u,
                                double* xnext, double* w) {
  w = ex.lds(w);  // the work area and the parameter block live in LDS
  P = ex.lds(P);
  const Blk b = parse(P);
  const bool imp = b.impulse;  // impulse: [M | Jc^T] only, z = v
  const int nj = b.nj, nq = b.nq, nc = b.nc, nu = nj - b.nun, ncol = imp ? nj + nc : nj + nc + 1;
  const int lda = lda_of(nj);
  double* A = w + pad2(WVals::doubles(nj));  // nj x (nj + nc + 1), ld lda: [M | Jc^T | tau - nle]
  double* tau = A + (int64_t)lda * ncol;
  double* ub = tau + nj;  // u (zero if !use_u)
  double* cv = ub + nj;   // per-cost activations
  double* red = cv + kMaxCosts;
  int* flag = (int*)(red + 2);
  double* Jc = red + 8;                  // nc x nj
  double* a0 = Jc + (int64_t)nc * nj;    // nc
  double* S = a0 + nc;                   // nc x (nc + 1), ld nc: [S | Jc z + a0]
  double* pb = S + (int64_t)nc * (nc + 1);  // Gauss-Jordan pivot-column buffer (128)
  const WVals W{w, nj, pb + 128};            // the recursions' per-wave partials after it
  ex.run([&](int lane) {
    if (lane < nu) ub[lane] = use_u ? u[lane] : 0.;
    for (int e = lane; e < lda * ncol; e += ex.nt) A[e] = 0.;
  });
  // the wide records (state / control residuals: x, u only) row-parallel on waves 3 and 1
  // beside the local placements, their lane partials into pb (free until the
  // factorisation); the other records on the waves the factorisation leaves idle (below)
  world_kinematics(ex, b, W, x, A, lda, [&](int wave, int l) {
    const double* cr = b.C;
    int nw = 0;
    for (int k = 0; k < b.ncost; ++k) {
      const CRec C{cr};
      if (wide_cost(C, nw)) {
        if (wave == (nw == 0 ? 3 : 1)) pb[64 * nw + l] = cost_activation_part(b, C, x, ub, nu, l, 64);
        ++nw;
      }
      cr += C.size();
    }
  }, [&](int wave, int l) {
    // (dense solve: the other records but the frame velocities first,) the contacts'
    // position terms (log6 for the 6D ones): item i on lane i / 3 of wave 1 + i % 3, so
    // that no wave runs two of them (a wave pays for the sum of its divergent lanes' paths)
    if (wave > 3) return;
    const int item = 3 * l + (wave - 1);
    const int kc = item;
    if (!imp && kc >= 0 && kc < b.ncon) {
      int row0;
      const CRec C{contact_rec(b, kc, &row0)};
      contact_a0_position(b, W, C, a0 + row0);
    }
  });
  if (!imp) world_rnea(ex, b, W, x + nq, nullptr, tau);
  ex.run([&](int lane) {
    if (lane < nj) {
      const double ti = lane < b.nun ? 0. : ub[lane - b.nun];  // ActuationModelFloatingBase: tau = [0; u]
      if (!imp) A[(int64_t)lda * (nj + nc) + lane] = ti - tau[lane];
      if (nc) contact_jac_lane(b, W, lane, Jc, A, lda);
    }
    if (!imp && lane >= 64 && lane < 64 + b.ncon) {
      int row0;
      const CRec C{contact_rec(b, lane - 64, &row0)};
      contact_a0_drift(b, W, C, a0 + row0);
    }
    if (lane == 128) {  // the wide records' values from their lane partials (pb is the
                        // factorisation's scratch next)
      const double* cr = b.C;
      int nw = 0;
      for (int k = 0; k < b.ncost; ++k) {
        const CRec C{cr};
        if (wide_cost(C, nw)) {
          double a = 0.;
          for (int l = 0; l < 64; ++l) a += pb[64 * nw + l];
          cv[k] = C.weight() * (0.5 * a);
          ++nw;
        }
        cr += C.size();
      }
    }
  });
  // Every other record's weighted value into cv[k], on the waves the factorisation leaves
  // idle: record item i on lane i / 3 of side wave i % 3 (the frame placements / CoM are
  // long serial evaluations, which would otherwise sit on the knot's critical path); the
  // force costs without active contact rows (lambda = 0) here, with contacts after the
  // Schur solve; frame velocities with the body velocities (impulse knots: rejected by the
  // host). The knot cost is their sum in record order (cost-sum.hxx:89-117), at the end.
  auto cost_side = [&](int, int sl, int snt) { calc_cost_records(P, w, W.parts, x, ub, cv, sl, snt); };
  // [Y | z] = M^-1 [Jc^T | tau - nle] by the tree-sparse LTDL of M; its scratch: the depth
  // levels in pb, the dof masks, 1 / D and the intermediate D^-1 G^T B in the recursions'
  // per-wave partials (dead from here on)
  double* const tp = ex.lds(W.parts);
  const TreeWork tw{(Mask*)tp, (Mask*)tp + nj, (Mask*)ex.lds(pb), tp + 2 * nj, ex.lds(flag)};
  // (the device fast path's rows, then D^-1 G^T B, both after the masks and 1 / D)
  tree_ltdl(ex, b, W, A, lda, tw, tree_depth(b, W), tp + 3 * nj, cost_side, 1);
  bool ok = tree_solve(ex, b, A, lda, ncol - nj, tw, tp + 3 * nj);
  // z, then a (impulse: v+, in tau's slot; z = M^-1 M v = v)
  double* a = imp ? tau : A + (int64_t)lda * (nj + nc);
  if (nc > 0) {
    ex.run([&](int lane) {
      for (int e = lane; e < nc * (nc + 1); e += ex.nt) {
        const int col = e / nc, row = e % nc;
        // column col of Y, or z (impulse: v, and the restitution term r Jc v)
        const double* yc = (imp && col == nc) ? x + nq : A + (int64_t)lda * (nj + col);
        double s = 0.;
        for (int i = 0; i < nj; ++i) s += Jc[(int64_t)row * nj + i] * yc[i];
        S[e] = col < nc ? s + (row == col ? b.damping : 0.) : (imp ? (1. + b.r_coeff) * s : s + a0[row]);
      }
    });
    ok = gauss_jordan<1>(ex, S, nc, nc, nc + 1, flag, pb) && ok;
    ex.run([&](int lane) {
      // contact-force costs (lambda = -S^-1 r, in S's last column, negated): record k's
      // value on lane 64 + k into cv[k], summed in record order with the next phase
      const int kf = lane - 64;
      if (kf >= 0 && kf < b.ncost && !imp) {
        const double* cr = b.C;
        for (int k = 0; k < kf; ++k) cr += CRec{cr}.size();
        const CRec C{cr};
        if (force_cost(C.type())) {
          double lamv[kMaxNc];
          for (int k = 0; k < nc; ++k) lamv[k] = -S[(int64_t)nc * nc + k];
          cv[kf] = C.weight() * force_cost_activation(b, C, lamv, nu);
        }
      }
      if (lane >= nj) return;
      double s = imp ? x[nq + lane] : a[lane];
      for (int k = 0; k < nc; ++k) s -= A[(int64_t)lda * (nj + k) + lane] * S[(int64_t)nc * nc + k];
      a[lane] = s;
    });
  }
  const double dt = b.dt;
  if (!ok)  // a singular mass matrix / Schur complement surfaces as forward_error
    ex.run([&](int i) {
      if (i < nj) a[i] = NAN;
    });
  ex.run([&](int i) {
    if (i == 64) {  // the knot cost: the records' values in record order
      double total = 0.;
      for (int k = 0; k < b.ncost; ++k) total += cv[k];
      red[0] = total;
    }
    if (i >= nj) return;
    if (imp) {  // impulse-fwddyn.hxx:80-81: xnext = (q, v+)
      xnext[nq + i] = nc > 0 ? a[i] : x[nq + i];
      if (!ok) xnext[nq + i] = NAN;
      xnext[i] = x[i];
      if (i == nj - 1 && b.ff) xnext[nq - 1] = x[nq - 1];
      return;
    }
    if (dt != 0.) {
      euler_step(b, x, a, dt, xnext, i);
    } else {
      xnext[i] = x[i];
      xnext[nq + i] = x[nq + i];
      if (i == nj - 1 && b.ff) xnext[nq - 1] = x[nq - 1];
    }
  });
  const double cc = red[0];
  (void)nx;
  return dt != 0. ? dt * cc : cc;
}

// LDS (doubles) of the rollout's calc (knot_calc_dense_x): the L records, the small arrays,
// then one region that first holds the D records and the recursions' partials and, from the
// CRBA columns on, [M | Jc^T | tau - nle], Jc and the Schur block.
MB_HD inline int64_t calc_dense_doubles(int nj, int nc = 0) {
  const int64_t small = 2 * nj + kMaxCosts + 8 + nc + 128;
  const int64_t rec = WVals::dsize(nj) + part_doubles(nj);
  const int64_t fac = (int64_t)lda_of(nj) * (nj + nc + 1) + (int64_t)nc * nj + (int64_t)nc * (nc + 1);
  return WVals::lsize(nj) + pad2(small) + pad2(rec > fac ? rec : fac);
}

// model->calc as knot_calc_x, with the dense factorisation (the blocked Gauss-Jordan of
// gj_mfma on [M | Jc^T | tau - nle]) and a smaller LDS footprint: the rollout's workgroups
// share a CU three at a time on the C5 walk (calc_dense_doubles: 40 KB against
// calc_work_doubles' 60 KB). The phases run in the order
//   local placements | walk, world frames | RNEA (tau = nle) | CRBA composites + cost records |
//   composites stored | CRBA columns into A | Jc, a0, tau column | solve | Schur | a, xnext
// so that the D records and the partials are dead when the columns write A over them.
// Every value is formed by the same arithmetic as in knot_calc_x's dense solve of round 5.
template <class X>
MB_HD __forceinline__ double knot_calc_dense_x(const X& ex, const double* P, int nx, const double* x, const double* u,
                                               bool use_u, double* xnext, double* w) {
  w = ex.lds(w);
  P = ex.lds(P);
  const Blk b = parse(P);
  const bool imp = b.impulse;  // impulse: [M | Jc^T] only, z = v
  const int nj = b.nj, nq = b.nq, nc = b.nc, nu = nj - b.nun, ncol = imp ? nj + nc : nj + nc + 1;
  const int lda = lda_of(nj);
  double* tau = w + WVals::lsize(nj);
  double* ub = tau + nj;  // u (zero if !use_u)
  double* cv = ub + nj;   // per-cost activations
  double* red = cv + kMaxCosts;
  int* flag = (int*)(red + 2);
  double* a0 = red + 8;     // nc
  double* pb = a0 + nc;     // the wide records' lane partials; the Schur block's pivot buffer
  double* R2 = w + WVals::lsize(nj) + pad2(2 * nj + kMaxCosts + 8 + nc + 128);
  const WVals W{w, nj, R2 + WVals::dsize(nj), R2};
  double* A = R2;                          // from the columns on: nj x ncol, ld lda
  double* Jc = A + (int64_t)lda * ncol;    // nc x nj
  double* S = Jc + (int64_t)nc * nj;       // nc x (nc + 1), ld nc: [S | Jc z + a0]
  const int npw = part_waves(ex.nt);
  ex.run([&](int lane) {
    if (lane < nu) ub[lane] = use_u ? u[lane] : 0.;
  });
  // local placements; the wide records (state / control residuals: x, u only) row-parallel
  // on waves 3 and 1, their lane partials into pb
  ex.run([&](int lane) {
    if (lane < nj) w_joint_local(b, W, x, lane);
    if (lane >= 64) {
      const int wave = lane >> 6, l = lane & 63;
      const double* cr = b.C;
      int nw = 0;
      for (int k = 0; k < b.ncost; ++k) {
        const CRec C{cr};
        if (wide_cost(C, nw)) {
          if (wave == (nw == 0 ? 3 : 1)) pb[64 * nw + l] = cost_activation_part(b, C, x, ub, nu, l, 64);
          ++nw;
        }
        cr += C.size();
      }
    }
  });
  ex.run([&](int lane) {
    if (lane < nj) {
      w_walk(b, W, lane);
      w_joint_world(b, W, lane);
    }
  });
  if (!imp) world_rnea(ex, b, W, x + nq, nullptr, tau);
  // CRBA composites in wave partials; beside them, on waves 1-3, the other cost records
  // (force costs without active contact rows: lambda = 0; frame velocities: impulse knots
  // skip them, as the host rejects them there) and the contacts' position terms (log6 for the
  // 6D ones): item i on lane i / 3 of wave 1 + i % 3, so that no wave runs two of them
  ex.run([&](int lane) {
    const int wave = lane >> 6, l = lane & 63;
    if (l < nj && wave < npw) w_crba_composite_part(b, W, l, wave, npw);
    if (wave < 1 || wave > 3) return;
    const int item = 3 * l + (wave - 1);
    int nn = 0;
    const double* cr = b.C;
    int nw = 0;
    for (int k = 0; k < b.ncost; ++k) {
      const CRec C{cr};
      if (wide_cost(C, nw)) {
        ++nw;
      } else {
        if (item == nn) {
          double v = cost_activation(b, W, C, x, ub, nu, !imp);
          if (force_cost(C.type()) && nc == 0) v = force_cost_activation(b, C, nullptr, nu);
          cv[k] = C.weight() * v;
        }
        ++nn;
      }
      cr += C.size();
    }
    const int kc = item - nn;
    if (!imp && kc >= 0 && kc < b.ncon) {
      int row0;
      const CRec C{contact_rec(b, kc, &row0)};
      contact_a0_position(b, W, C, a0 + row0);
    }
  });
  ex.run([&](int lane) {
    if (lane < nj) w_crba_store_local(W, nj, lane, npw);
  });
  // (from here on the D records and the partials are dead: A, Jc, S over them)
  ex.run([&](int lane) {
    const int wv = lane >> 6, j = lane & 63;
    if (j < nj) w_crba_column(b, W, j, A, lda, wv, ex.nt >> 6, npw, false, true);
  });
  ex.run([&](int lane) {
    if (lane < nj) {
      const double ti = lane < b.nun ? 0. : ub[lane - b.nun];  // ActuationModelFloatingBase: tau = [0; u]
      if (!imp) A[(int64_t)lda * (nj + nc) + lane] = ti - tau[lane];
      if (nc) contact_jac_lane(b, W, lane, Jc, A, lda);
    }
    if (!imp && lane >= 64 && lane < 64 + b.ncon) {
      int row0;
      const CRec C{contact_rec(b, lane - 64, &row0)};
      contact_a0_drift(b, W, C, a0 + row0);
    }
    if (lane == 128) {  // the wide records' values from their lane partials
      const double* cr = b.C;
      int nw = 0;
      for (int k = 0; k < b.ncost; ++k) {
        const CRec C{cr};
        if (wide_cost(C, nw)) {
          double a = 0.;
          for (int l = 0; l < 64; ++l) a += pb[64 * nw + l];
          cv[k] = C.weight() * (0.5 * a);
          ++nw;
        }
        cr += C.size();
      }
    }
  });
  bool ok = mb_solve(ex, A, nj, lda, ncol, flag, pb);
  // z, then a (impulse: v+, in tau's slot; z = M^-1 M v = v)
  double* a = imp ? tau : A + (int64_t)lda * (nj + nc);
  if (nc > 0) {
    ex.run([&](int lane) {
      for (int e = lane; e < nc * (nc + 1); e += ex.nt) {
        const int col = e / nc, row = e % nc;
        const double* yc = (imp && col == nc) ? x + nq : A + (int64_t)lda * (nj + col);
        double s = 0.;
        for (int i = 0; i < nj; ++i) s += Jc[(int64_t)row * nj + i] * yc[i];
        S[e] = col < nc ? s + (row == col ? b.damping : 0.) : (imp ? (1. + b.r_coeff) * s : s + a0[row]);
      }
    });
    ok = gauss_jordan<1>(ex, S, nc, nc, nc + 1, flag, pb) && ok;
    ex.run([&](int lane) {
      const int kf = lane - 64;
      if (kf >= 0 && kf < b.ncost && !imp) {
        const double* cr = b.C;
        for (int k = 0; k < kf; ++k) cr += CRec{cr}.size();
        const CRec C{cr};
        if (force_cost(C.type())) {
          double lamv[kMaxNc];
          for (int k = 0; k < nc; ++k) lamv[k] = -S[(int64_t)nc * nc + k];
          cv[kf] = C.weight() * force_cost_activation(b, C, lamv, nu);
        }
      }
      if (lane >= nj) return;
      double s = imp ? x[nq + lane] : a[lane];
      for (int k = 0; k < nc; ++k) s -= A[(int64_t)lda * (nj + k) + lane] * S[(int64_t)nc * nc + k];
      a[lane] = s;
    });
  }
  const double dt = b.dt;
  if (!ok)
    ex.run([&](int i) {
      if (i < nj) a[i] = NAN;
    });
  ex.run([&](int i) {
    if (i == 64) {
      double total = 0.;
      for (int k = 0; k < b.ncost; ++k) total += cv[k];
      red[0] = total;
    }
    if (i >= nj) return;
    if (imp) {
      xnext[nq + i] = nc > 0 ? a[i] : x[nq + i];
      if (!ok) xnext[nq + i] = NAN;
      xnext[i] = x[i];
      if (i == nj - 1 && b.ff) xnext[nq - 1] = x[nq - 1];
      return;
    }
    if (dt != 0.) {
      euler_step(b, x, a, dt, xnext, i);
    } else {
      xnext[i] = x[i];
      xnext[nq + i] = x[nq + i];
      if (i == nj - 1 && b.ff) xnext[nq - 1] = x[nq - 1];
    }
  });
  const double cc = red[0];
  (void)nx;
  return dt != 0. ? dt * cc : cc;
}

template <int NT>
__device__ __forceinline__ double knot_calc(const double* P, int nx, const double* x, const double* u, bool use_u, double* xnext,
                                   double* w) {
  static_assert(NT >= 256, "the multibody calc splits its phases over 4 waves");
#ifdef MB_CALC_DENSE
  return knot_calc_dense_x(DevExec{NT}, P, nx, x, u, use_u, xnext, w);
#else
  return knot_calc_x(DevExec{NT}, P, nx, x, u, use_u, xnext, w);
#endif
}

// ---------------------------------------------------------------------------
// calcDiff: one kMbDiffNT-thread workgroup per (element, knot).
//
// World-frame RNEA derivatives. Perturbing q_j moves the whole subtree of dof j's
// body rigidly by S_j, so every world quantity X of that subtree changes by the
// transport S_j x X (x* for forces) plus an intrinsic part; with
//   V_P, A_P: velocity / acceleration (gravity included) of the parent body of j,
//   u_j = S_j x V_P,  c_j = -S_j x A_P + u_j x V_P,  w_j = (V_b(j) + V_P) x S_j,
// the body accelerations and velocities change by
//   dA_b/dq_j = S_j x A_b + c_j - u_j x V_b,  dV_b/dq_j = S_j x V_b - u_j,
//   dA_b/dv_j = w_j + S_j x V_b,              dV_b/dv_j = S_j,
// for every body b below j, and the transport cancels in tau_k = S_k . F_k, so
//   k below j (incl. j's body):   dtau_k/dq_j = Q_k . c_j - P_k . u_j,   dtau_k/dv_j = Q_k . w_j + P_k . S_j
//   k strict ancestor of j:       dtau_k/dx_j = S_k . G_j
// with Q_k = Ycrb_k S_k (composite inertia), P_k = sum_{b in sub(k)} [V_b x* (Y_b S_k)
// - Y_b (V_b x S_k)] - S_k x* sum_{b in sub(k)} Y_b V_b, and G_j = S_j x* F_j +
// Ycrb_j c_j - B_j u_j (q) / Ycrb_j w_j + B_j S_j (v), B_j x = sum_{b in sub(j)}
// [-Y_b (V_b x x) + x x* (Y_b V_b) + V_b x* (Y_b x)]. Contact forces are fixed in
// their frames (computeRNEADerivatives with fext) and enter through F.
// ---------------------------------------------------------------------------
struct DiffLayout {
  int64_t wv, A, dtau, da, qp, vec, J, red, total;
  // cost-derivative area (after the dynamics, over the dead world values when it
  // fits): group table, per-row Arr / Ar factors, the stacked residual Jacobians
  int64_t R;
  // contact area (nc > 0): Jc nc x nj, a0 nc, lambda nc, Y = Minv Jc^T and
  // H = Y S^-1 (nj x nc each), [S | I | r] nc x (2nc + 1), da0/dx nc x L, fx 6 nj
  int64_t Jc, a0, lam, Y, H, Sx, da0, fx, zv, dfx, dfu;
  // the per-wave partials of the recursions (kinematics / the RNEA at the solved a), the
  // per-body velocity-product maps and their subtree sums; half: doubles per half of A
  int64_t pk, pr, nb, ns, half;
  // the cost table's diagonal terms and residual rows (after the table, or apart from it),
  // and the LDS copy of dtau the da product reads (the spilled plan: over the world values)
  int64_t Rr, dts;
  int spill;       // kSpill* flags the plan was made with
  int64_t ht;      // host emulation: its factorisation scratch (70 nj)
  int64_t htotal;  // host emulation: total plus its own areas (da, the factorisation scratch)
};
// The spilled calcDiff plan (the Talos-size trees): the LDS plan keeps what the phases read
// at random, and the arrays each written once and streamed once go to the knot's own
// output blocks in global memory, dead there until the blocks are written (after their
// last read): dtau/dx into Lxx (read by the da product, the Gauss-Newton blocks write Lxx
// after it), the body maps and their subtree sums into Fx (read up to the tangent
// directions; the da product writes Fx), the jac-cost Jacobians into Lxu (kSpillJ: read by
// the residual rows, before the Gauss-Newton blocks), d lambda / dx, du into Fu (kSpillF:
// read by the residual rows; Fu is written last). The product's epilogue writes Fx
// itself, so da needs no area; Minv and the contact arrays share the factorisation's A
// area. Two workgroups share a CU under it (<= 80 KB with the parameter block).
constexpr int kSpillBlocks = 1, kSpillJ = 2, kSpillF = 4;
// vec area: x (nq + nj <= 2 nj + 1), u (nj), nle / z / a / tau (3 nj), jac-cost
// residuals (6 per cost), Jexp6 / Ad(exp6^-1) (72)
// Cost-derivative area (doubles) for nrows stacked residual rows over L + nu columns.
constexpr int kMaxCostRows = 64;
// (4 columns of slack: the GEMM reads rows four columns at a time)
MB_HD __forceinline__ int cost_rows_ld(int nj, int nu) { return (int)pad2(2 * nj + nu) + 4; }
constexpr int kMaxCostCols = 3 * kMaxJ;  // diagonal terms per column of [x tangent | u]
MB_HD __forceinline__ int64_t cost_table_doubles() { return 4 * kMaxCosts + 5 * kMaxCostRows; }
MB_HD __forceinline__ int64_t cost_area_doubles(int nj, int nu, int nrows) {
  return cost_table_doubles() + kMaxCostCols + (int64_t)nrows * cost_rows_ld(nj, nu);
}
__host__ __device__ inline DiffLayout diff_layout(int nj, int njac, int nc = 0, bool vel_cols = false, int nu = 0,
                                                  int nrows = 0, int spill = 0) {
  const int L = 2 * nj;
  DiffLayout l;
  l.spill = spill;
  const int64_t jsz = (int64_t)6 * (vel_cols ? L : nj) * (njac > 0 ? njac : 1);  // jac-cost Jacobians [cost][6][jw]
  const int64_t ca = cost_area_doubles(nj, nu, nrows);
  const int64_t wvs = pad2(WVals::doubles(nj));
  if (!(spill & kSpillBlocks)) {
    // dtau [k][L] (first the per-body N_b, h_b: 42 per dof); the da area (first the subtree
    // sums Nsub, Hsub; da itself on the host: the device's product writes Fx directly)
    // (da rows at the odd stride L + 1: the Fx assembly reads a column of it per wave)
    const int64_t dsz = pad2((int64_t)nj * (L + 1) > 42 * (int64_t)nj ? (int64_t)nj * (L + 1) : 42 * (int64_t)nj);
    // the world values, then dtau: both dead after the da phase, so the cost-derivative
    // area can run over both
    l.wv = 0;
    l.dtau = l.wv + wvs;
    l.half = pad2((int64_t)lda_of(nj) * nj);
    l.A = l.dtau + dsz;  // [M | Minv], ld lda_of(nj)
    l.da = l.A + 2 * l.half;
    l.pk = l.pr = l.nb = l.dtau;
    l.ns = l.da;
    l.qp = l.da + dsz;
    l.vec = l.qp + (int64_t)12 * nj;      // Q_k, P_k
    l.J = l.vec + pad2(6 * nj + 1 + 6 * kMaxJacCosts + 72);
    l.red = l.J + jsz;
    l.total = l.red + 8 + 128;  // reductions, Gauss-Jordan pivot-column buffer
    l.Jc = l.total;
    l.a0 = l.Jc + (int64_t)nc * nj;
    l.lam = l.a0 + nc;
    l.Y = l.lam + nc;
    l.H = l.Y + (int64_t)nj * nc;
    l.Sx = l.H + (int64_t)nj * nc;
    l.da0 = l.Sx + (int64_t)nc * (2 * nc + 1);
    l.fx = l.da0 + (int64_t)nc * L;
    l.zv = l.fx + 6 * nj;  // impulse: v+ - v
    l.dfx = l.zv + nj;     // d lambda / dx (nc x L), d lambda / du (nc x nj): CostModelContactForce
    l.dfu = l.dfx + (int64_t)nc * L;
    l.total = nc > 0 ? l.dfu + (int64_t)nc * nj : l.total;
    // the table (written on spare lanes during the da phase, beside the dtau reads) within
    // the world values; the diagonal terms and R rows (written after it) also over dtau
    if (cost_table_doubles() <= wvs && ca <= wvs + dsz) {
      l.R = l.wv;
    } else {
      l.R = pad2(l.total);
      l.total = l.R + ca;
    }
    l.Rr = l.R + cost_table_doubles();
    l.dts = l.dtau;
    l.ht = pad2(l.total);  // host: the factorisation scratch
    l.htotal = l.ht + pad2((int64_t)70 * nj);
    return l;
  }
  // spilled plan; live ranges (phases of knot_calc_diff_x):
  //   world values        kinematics .. tangent directions; then the cost area
  //   A, first half       M and its factors .. M^-1; then Y (z / Y .. Kinv), the partials
  //                       of the RNEA at the solved a, then da0 / dlambda/dx, du (tangent
  //                       directions .. residual rows) when they fit, else their own area
  //   A, second half      the recursions' partials (kinematics), the factorisation's
  //                       scratch, then M^-1 / Kinv top-left .. Fu
  //   contact area        Jc, a0, lambda, H, [S | I | r], joint forces, v+ - v
  l.half = pad2(lda_of(nj) * (int64_t)nj > part_doubles(nj) ? lda_of(nj) * (int64_t)nj : part_doubles(nj));
  l.wv = 0;
  l.A = wvs;
  l.pk = l.A + l.half;
  l.pr = l.A;
  l.dtau = l.nb = l.ns = -1;  // in the output blocks
  l.qp = l.A + 2 * l.half;
  l.vec = l.qp + (int64_t)12 * nj;
  l.red = l.vec + pad2(6 * nj + 1 + 6 * kMaxJacCosts + 72);
  l.total = l.red + 8 + 128;
  l.J = -1;
  if (!(spill & kSpillJ)) {
    l.J = l.total;
    l.total = pad2(l.J + jsz);
  }
  l.Jc = l.total;
  l.a0 = l.Jc + (int64_t)nc * nj;
  l.lam = l.a0 + nc;
  l.H = l.lam + nc;
  l.Sx = l.H + (int64_t)nj * nc;
  l.fx = l.Sx + (int64_t)nc * (2 * nc + 1);
  l.zv = l.fx + 6 * nj;
  if (nc > 0) l.total = pad2(l.zv + nj);
  const int64_t ysz = (int64_t)nj * nc, d0 = pad2((int64_t)nc * L), dfs = pad2((int64_t)nc * L) + (int64_t)nc * nj;
  l.Y = ysz <= l.half ? l.A : l.total;
  if (nc > 0 && l.Y == l.total) l.total = pad2(l.total + ysz);
  l.da0 = d0 <= l.half ? l.A : l.total;
  if (nc > 0 && l.da0 == l.total) l.total = pad2(l.total + d0);
  // d lambda / dx, du: the knot's Fu block (kSpillF: written after the residual rows read
  // them), else after da0 when both fit the half, else their own area
  if (spill & kSpillF) {
    l.dfx = l.dfu = -1;
  } else {
    l.dfx = (l.da0 == l.A && d0 + dfs <= l.half) ? l.A + d0 : l.total;
    if (nc > 0 && l.dfx == l.total) l.total = pad2(l.total + dfs);
    l.dfu = l.dfx + pad2((int64_t)nc * L);
  }
  // The cost area: where the world values are dead (from the da phase on). With room in
  // the first half of A after da0 (and d lambda / dx, du not there) the table (written
  // during the da phase) goes there, and the da phase reads dtau from an LDS copy over the
  // world values (dts: its loads then never wait behind the Fx stores, as global loads
  // do); the diagonal terms and the rows (from the next phase on) over the world values.
  // Else the whole area over the world values and the first half, when it fits.
  const bool f_in_half = nc > 0 && l.dfx >= l.A && l.dfx < l.A + l.half;
  const int64_t tab0 = (nc > 0 ? d0 : 0), rsz = ca - cost_table_doubles();
  l.dts = -1;
  if (!f_in_half && tab0 + cost_table_doubles() <= l.half && (int64_t)nj * L <= wvs && rsz <= wvs) {
    l.R = l.A + tab0;
    l.Rr = l.wv;
    l.dts = l.wv;
  } else if (cost_table_doubles() + kMaxCostCols <= wvs && ca <= wvs + (f_in_half ? 0 : l.half)) {
    l.R = l.wv;
    l.Rr = l.R + cost_table_doubles();
  } else {
    l.R = pad2(l.total);
    l.total = l.R + ca;
    l.Rr = l.R + cost_table_doubles();
  }
  // host emulation: the da area and the factorisation's scratch of its own
  l.da = pad2(l.total);
  l.ht = l.da + pad2((int64_t)nj * (L + 1));
  l.htotal = l.ht + pad2((int64_t)70 * nj);
  return l;
}
// The spill flags of a handle's plan: spill when the all-LDS plan (with the parameter block
// of psz doubles) exceeds half the CU's LDS, the tree is large enough for the body maps
// and their sums (84 nj doubles) to fit in the Fx block (4 nj^2); the Jacobians go to
// Lxu (2 nj m), d lambda / dx, du to Fu (2 nj m) when they fit.
MB_HD inline int diff_spill(int nj, int njac, int nc, bool vcols, int nu, int nrows, int64_t psz, int m) {
  const DiffLayout a = diff_layout(nj, njac, nc, vcols, nu, nrows, 0);
  if ((pad2(a.total) + pad2(psz)) * 8 <= 80 * 1024 || 84 * (int64_t)nj > 4 * (int64_t)nj * nj) return 0;
  const int64_t jsz = (int64_t)6 * (vcols ? 2 * nj : nj) * (njac > 0 ? njac : 1);
  const int64_t fsz = pad2((int64_t)nc * 2 * nj) + (int64_t)nc * nj;
  return kSpillBlocks | (jsz <= (int64_t)2 * nj * m ? kSpillJ : 0) | (nc > 0 && fsz <= (int64_t)2 * nj * m ? kSpillF : 0);
}

// Live ranges of the calcDiff's LDS arrays (knot_calc_diff_x's phases, in order), for the
// static check of its plans (diff_layout_check): arrays whose areas overlap must not be
// live in a common phase.
enum DiffPhase {
  DP_INIT, DP_KIN, DP_CONTACT, DP_FACTOR, DP_MINV, DP_ZY, DP_SX, DP_SGJ, DP_LAMH, DP_KINV, DP_RNEA2, DP_CALC,
  DP_QPJAC, DP_TANG, DP_DA, DP_RROWS, DP_GN, DP_END
};
struct DiffRegion {
  const char* name;
  int64_t off, size;
  int first, last;
};
// The regions of plan l (host emulation areas excluded); returns their count (<= 40).
MB_HD inline int diff_layout_regions(const DiffLayout& l, int nj, int njac, int nc, bool vcols, int nu, int nrows,
                                     DiffRegion* r) {
  const int L = 2 * nj;
  const bool sp = l.spill & kSpillBlocks;
  const int64_t wvs = WVals::doubles(nj), jsz = (int64_t)6 * (vcols ? L : nj) * (njac > 0 ? njac : 1);
  int k = 0;
  auto add = [&](const char* n, int64_t off, int64_t size, int first, int last) {
    if (off >= 0 && size > 0) r[k++] = DiffRegion{n, off, size, first, last};
  };
  add("world values", l.wv, wvs, DP_INIT, DP_TANG);
  add("M / its factors", l.A, (int64_t)lda_of(nj) * nj, DP_KIN, DP_MINV);
  // (the fast path's rows, or the generic steps' masks; then the recursions' partials are
  // dead, and M^-1 is written)
  // ((depth + 1) nj <= min(kTreeKD, nj) nj doubles, or 2 nj)
  const int64_t fs = (int64_t)nj * (kTreeKD < nj ? kTreeKD : nj);
  add("factorisation scratch", l.A + l.half, fs > 2 * nj ? fs : 2 * nj, DP_FACTOR, DP_FACTOR);
  add("Minv / Kinv", l.A + l.half, (int64_t)lda_of(nj) * nj, DP_MINV, DP_END);
  add("partials (kinematics)", l.pk, part_doubles(nj), DP_KIN, DP_KIN);
  add("partials (RNEA at a)", l.pr, part_doubles(nj), DP_RNEA2, DP_RNEA2);
  add("qp", l.qp, (int64_t)12 * nj, DP_FACTOR, DP_TANG);
  add("vec", l.vec, 6 * nj + 1 + 6 * kMaxJacCosts + 72, DP_INIT, DP_END);
  add("red / pivots", l.red, 8 + 128, DP_INIT, DP_END);
  if (!(l.spill & kSpillJ)) add("jac-cost Jacobians", l.J, jsz, DP_FACTOR, DP_RROWS);
  if (!sp) {
    // (built beside the factorisation, or after the RNEA at a when no wave is idle then)
    add("body maps (side)", l.nb, (int64_t)42 * nj, DP_FACTOR, DP_FACTOR);
    add("body maps", l.nb, (int64_t)42 * nj, DP_QPJAC, DP_QPJAC);
    add("subtree sums", l.ns, (int64_t)42 * nj, DP_FACTOR, DP_TANG);
    add("dtau", l.dtau, (int64_t)nj * L, DP_TANG, DP_DA);
  }
  if (nc > 0) {
    add("Jc", l.Jc, (int64_t)nc * nj, DP_CONTACT, DP_DA);
    add("a0", l.a0, nc, DP_CONTACT, DP_SX);
    add("lambda", l.lam, nc, DP_LAMH, DP_END);
    add("Y", l.Y, (int64_t)nj * nc, DP_ZY, DP_KINV);
    add("H", l.H, (int64_t)nj * nc, DP_LAMH, DP_DA);
    add("[S | I | r]", l.Sx, (int64_t)nc * (2 * nc + 1), DP_SX, DP_DA);
    add("da0", l.da0, (int64_t)nc * L, DP_TANG, DP_DA);
    add("contact joint forces", l.fx, 6 * nj, DP_KINV, DP_RNEA2);
    add("v+ - v", l.zv, nj, DP_KINV, DP_RNEA2);
    if (!(l.spill & kSpillF)) {
      add("d lambda / dx", l.dfx, (int64_t)nc * L, DP_DA, DP_RROWS);
      add("d lambda / du", l.dfu, (int64_t)nc * nj, DP_DA, DP_RROWS);
    }
  }
  add("cost table", l.R, cost_table_doubles(), DP_DA, DP_END);
  add("cost diagonal / rows", l.Rr, cost_area_doubles(nj, nu, nrows) - cost_table_doubles(), DP_RROWS, DP_END);
  if (sp && l.dts >= 0) add("dtau (LDS copy)", l.dts, (int64_t)nj * L, DP_DA, DP_DA);
  return k;
}
// 0 when no two regions of the plan overlap in both LDS and live range (and all lie in
// [0, total)); else the index + 1 of the first region in conflict (a, b: the pair).
MB_HD inline int diff_layout_check(const DiffLayout& l, int nj, int njac, int nc, bool vcols, int nu, int nrows,
                                   int* a = nullptr, int* b = nullptr) {
  DiffRegion r[40];
  const int n = diff_layout_regions(l, nj, njac, nc, vcols, nu, nrows, r);
  for (int i = 0; i < n; ++i) {
    if (r[i].off + r[i].size > l.total) {
      if (a) *a = i, *b = i;
      return i + 1;
    }
    for (int j = i + 1; j < n; ++j) {
      const bool mem = r[i].off < r[j].off + r[j].size && r[j].off < r[i].off + r[i].size;
      const bool live = r[i].first <= r[j].last && r[j].first <= r[i].last;
      if (mem && live) {
        if (a) *a = i, *b = j;
        return i + 1;
      }
    }
  }
  return 0;
}

// The velocity-product terms of the derivatives are linear maps of the subtree
// bodies: with N_b x = V_b x* (Y_b x) - Y_b (V_b x x) and h_b = Y_b V_b,
//   P_k = Nsub_k S_k - S_k x* Hsub_k,   B_j x = Nsub_j x + x x* Hsub_j,
// Nsub / Hsub the subtree sums. lane d < nj: N_d (column-major 6x6) and h_d of d's
// body (zero on the massless free-flyer dofs) into nb[42 d ..].
MB_HD inline void body_nh_lane(const Blk& b, const WVals& W, int d, double* nb) {
  double* o = nb + 42 * d;
  if (!carries_body(b, d)) {
    for (int e = 0; e < 42; ++e) o[e] = 0.;
    return;
  }
  const double m = *W.m(d);
  double c[3], I6[6], V[6];
  for (int e = 0; e < 3; ++e) c[e] = W.c(d)[e];
  for (int e = 0; e < 6; ++e) {
    I6[e] = W.Ic(d)[e];
    V[e] = W.v(d)[e];
  }
  for (int col = 0; col < 6; ++col) {
    double x[6] = {0., 0., 0., 0., 0., 0.}, Yx[6], t1[6], VxX[6], t2[6];
    x[col] = 1.;
    inertia_mul(m, c, I6, x, Yx);
    cross_f(V, Yx, t1);
    cross_m(V, x, VxX);
    inertia_mul(m, c, I6, VxX, t2);
    for (int e = 0; e < 6; ++e) o[6 * col + e] = t1[e] - t2[e];
  }
  inertia_mul(m, c, I6, V, o + 36);
}
// lane j < nj of wave w (of nw): components [11 w, 11 w + 11) of Nsub_j, Hsub_j (sums over
// the bodies below dof j) into ns[42 j ..]; every body read, the others weighted 0 (no
// branch: the unrolled loads overlap), the 42 components split over the waves
template <int kC = 11>  // components per pass (11 for 4 waves, 6 for 8: one pass per wave)
MB_HD inline void subtree_nh_lane(const Blk& b, const WVals& W, int j, const double* nb, double* ns, int w = 0,
                                  int nw = 1) {
  // wave w's components [w per, (w + 1) per), per = ceil(42 / nw), in chunks of kC
  const int per = (42 + nw - 1) / nw, e0 = w * per, e1 = e0 + per < 42 ? e0 + per : 42;
  double acc[kC];
  for (int e = 0; e < kC; ++e) acc[e] = 0.;
  for (int c0 = e0; c0 < e1; c0 += kC) {
#pragma unroll 2
    for (int bb = 0; bb < b.nj; ++bb) {
      const bool in = ((*W.anc(bb) >> j) & 1ull) && carries_body(b, bb);
      const double* o = nb + 42 * bb + c0;
#pragma unroll
      for (int e = 0; e < kC; ++e) {
        const double v = c0 + e < e1 ? o[e] : 0.;
        acc[e] += in ? v : 0.;
      }
    }
#pragma unroll
    for (int e = 0; e < kC; ++e) {
      if (c0 + e < e1) ns[42 * j + c0 + e] = acc[e];
      acc[e] = 0.;
    }
  }
}
// B_j x = Nsub_j x + x x* Hsub_j
MB_HD __forceinline__ void bsub_mul_ns(const double* ns, int j, const double* x, double* o) {
  const double* N = ns + 42 * j;
  double t[6];
  cross_f(x, N + 36, t);
  for (int e = 0; e < 6; ++e) {
    double v = t[e];
    for (int col = 0; col < 6; ++col) v += N[6 * col + e] * x[col];
    o[e] = v;
  }
}
// lane k < nj: Q_k = Ycrb_k S_k, P_k = Nsub_k S_k - S_k x* Hsub_k. qp[12 k ..].
MB_HD inline void qp_lane_ns(const WVals& W, int k, const double* ns, double* qp) {
  double S[6], Q[6], t6[6];
  for (int e = 0; e < 6; ++e) S[e] = W.S(k)[e];
  comp_mul(W, k, S, Q);
  const double* N = ns + 42 * k;
  cross_f(S, N + 36, t6);
  for (int e = 0; e < 6; ++e) {
    double v = -t6[e];
    for (int col = 0; col < 6; ++col) v += N[6 * col + e] * S[col];
    qp[12 * k + e] = Q[e];
    qp[12 * k + 6 + e] = v;
  }
}

// lane k < nj: Q_k = Ycrb_k S_k, P_k (header comment). qp[12 k ..].
MB_HD inline void qp_lane(const Blk& b, const WVals& W, int k, double* qp) {
  double S[6], Q[6], P[6] = {0., 0., 0., 0., 0., 0.}, Hc[6] = {0., 0., 0., 0., 0., 0.};
  for (int e = 0; e < 6; ++e) S[e] = W.S(k)[e];
  comp_mul(W, k, S, Q);
  for (int bb = 0; bb < b.nj; ++bb) {
    if (!((*W.anc(bb) >> k) & 1ull) || !carries_body(b, bb)) continue;
    const double m = *W.m(bb);
    double c[3], I6[6], V[6], YS[6], VxS[6], YVxS[6], t6[6], h[6];
    for (int e = 0; e < 3; ++e) c[e] = W.c(bb)[e];
    for (int e = 0; e < 6; ++e) {
      I6[e] = W.Ic(bb)[e];
      V[e] = W.v(bb)[e];
    }
    inertia_mul(m, c, I6, S, YS);
    cross_m(V, S, VxS);
    inertia_mul(m, c, I6, VxS, YVxS);
    cross_f(V, YS, t6);
    inertia_mul(m, c, I6, V, h);
    for (int e = 0; e < 6; ++e) {
      P[e] += t6[e] - YVxS[e];
      Hc[e] += h[e];
    }
  }
  double t6[6];
  cross_f(S, Hc, t6);
  for (int e = 0; e < 6; ++e) {
    qp[12 * k + e] = Q[e];
    qp[12 * k + 6 + e] = P[e] - t6[e];
  }
}

// B_j x = sum_{b in sub(j)} [-Y_b (V_b x x) + x x* (Y_b V_b) + V_b x* (Y_b x)]
MB_HD inline void bsub_mul(const Blk& b, const WVals& W, int j, const double* x, double* o) {
  for (int e = 0; e < 6; ++e) o[e] = 0.;
  for (int bb = 0; bb < b.nj; ++bb) {
    if (!((*W.anc(bb) >> j) & 1ull) || !carries_body(b, bb)) continue;
    const double m = *W.m(bb);
    double c[3], I6[6], V[6], t[6], Yt[6], h[6], s1[6], Yx[6], s2[6];
    for (int e = 0; e < 3; ++e) c[e] = W.c(bb)[e];
    for (int e = 0; e < 6; ++e) {
      I6[e] = W.Ic(bb)[e];
      V[e] = W.v(bb)[e];
    }
    cross_m(V, x, t);
    inertia_mul(m, c, I6, t, Yt);
    inertia_mul(m, c, I6, V, h);
    cross_f(x, h, s1);
    inertia_mul(m, c, I6, x, Yx);
    cross_f(V, Yx, s2);
    for (int e = 0; e < 6; ++e) o[e] += s1[e] + s2[e] - Yt[e];
  }
}

// Direction dd (q_j for dd < nj, v_j otherwise): column dd of dtau/dx
// (dtau[k * L + dd]), and the motion derivatives of the contact / impulse frames.
// Parent-body quantities: V_P, A_P (gravity included; the root: 0, root_a).
MB_HD inline void parent_motion(const Blk& b, const WVals& W, int j, double* VP, double* AP) {
  const int p = body_parent(b, j);
  for (int e = 0; e < 6; ++e) {
    VP[e] = p >= 0 ? W.v(p)[e] : 0.;
    AP[e] = p >= 0 ? W.a(p)[e] : W.root_a()[e];
  }
}

// part / np: this lane's share of the rows k (the direction's setup is repeated per part)
MB_HD inline void dtau_direction(const Blk& b, const WVals& W, const double* qp, int dd, int L, double* dtau,
                                  const double* ns = nullptr, int part = 0, int np = 1) {
  const int nj = b.nj, j = dd < nj ? dd : dd - nj;
  const bool isq = dd < nj;
  double S[6], VP[6], AP[6], u[6], cj[6], G[6], t6[6], t7[6];
  for (int e = 0; e < 6; ++e) S[e] = W.S(j)[e];
  parent_motion(b, W, j, VP, AP);
  if (isq) {
    cross_m(S, VP, u);
    cross_m(S, AP, t6);
    cross_m(u, VP, t7);
    for (int e = 0; e < 6; ++e) cj[e] = t7[e] - t6[e];
    // G_j = S_j x* F_j + Ycrb_j c_j - B_j u_j
    double F[6], Bu[6];
    for (int e = 0; e < 6; ++e) F[e] = W.F(j)[e];
    cross_f(S, F, G);
    comp_mul(W, j, cj, t6);
    if (ns)
      bsub_mul_ns(ns, j, u, Bu);
    else
      bsub_mul(b, W, j, u, Bu);
    for (int e = 0; e < 6; ++e) G[e] += t6[e] - Bu[e];
  } else {
    // w_j = (V_b(j) + V_P) x S_j ; G_j = Ycrb_j w_j + B_j S_j
    double Vs[6], BS[6];
    for (int e = 0; e < 6; ++e) Vs[e] = W.v(j)[e] + VP[e];
    cross_m(Vs, S, cj);  // (w_j in cj)
    comp_mul(W, j, cj, G);
    if (ns)
      bsub_mul_ns(ns, j, S, BS);
    else
      bsub_mul(b, W, j, S, BS);
    for (int e = 0; e < 6; ++e) G[e] += BS[e];
    for (int e = 0; e < 6; ++e) u[e] = S[e];  // P_k . S_j
  }
  const Mask aj = *W.anc(j);
  int k0 = 0, k1 = nj;
  if (np > 1) k_range(nj, part, np, k0, k1);
  for (int k = k0; k < k1; ++k) {
    double val = 0.;
    if ((*W.anc(k) >> j) & 1ull) {  // k's body below j's (or the same body)
      const double* Q = qp + 12 * k;
      const double* P = Q + 6;
      val = isq ? dot6(Q, cj) - dot6(P, u) : dot6(Q, cj) + dot6(P, u);
    } else if ((aj >> k) & 1ull) {  // k's body a strict ancestor of j's
      val = dot6(W.S(k), G);
    }
    dtau[(int64_t)k * L + dd] = val;
  }
}

// Direction dd: da0/dx column (contact-3d.hxx:46-71, contact-6d.hxx:48-66) at the
// solved acceleration (getJointAccelerationDerivatives after computeRNEADerivatives):
// the frame motion derivative moved to the frame, the classical term of a 3D
// contact, the Baumgarte terms. da0[row * L + dd].
MB_HD inline void contact_direction(const Blk& b, const WVals& W, int dd, int L, double* da0) {
  const int nj = b.nj, j = dd < nj ? dd : dd - nj;
  const bool isq = dd < nj;
  double S[6], VP[6], AP[6], u[6], c0[6], t6[6], t7[6];
  for (int e = 0; e < 6; ++e) S[e] = W.S(j)[e];
  parent_motion(b, W, j, VP, AP);
  for (int e = 0; e < 6; ++e) AP[e] -= W.root_a()[e];  // gravity-free (data.a)
  if (isq) {
    cross_m(S, VP, u);
    cross_m(S, AP, t6);
    cross_m(u, VP, t7);
    for (int e = 0; e < 6; ++e) c0[e] = t7[e] - t6[e];
  } else {
    double Vs[6];
    for (int e = 0; e < 6; ++e) Vs[e] = W.v(j)[e] + VP[e];
    cross_m(Vs, S, c0);  // w_j
  }
  const double* r = b.K;
  int row = 0;
  for (int k = 0; k < b.ncon; ++k) {
    const CRec C{r};
    const double* d = C.d();
    const int fb = frame_dof(b, d);
    const int n = C.type() == C_CONTACT_3D ? 3 : 6;
    if (!((*W.anc(fb) >> j) & 1ull)) {
      for (int e = 0; e < n; ++e) da0[(int64_t)(row + e) * L + dd] = 0.;
      row += n;
      r += C.size();
      continue;
    }
    double Rf[9], pf[3], V[6], dV[6], dA[6], vf[6], dvf[6], daf[6];
    frame_placement(b, W, d, Rf, pf);
    for (int e = 0; e < 6; ++e) V[e] = W.v(fb)[e];
    if (isq) {  // dV = -u_j, dA = c0_j - u_j x V_b (intrinsic parts)
      cross_m(u, V, t6);
      for (int e = 0; e < 6; ++e) {
        dV[e] = -u[e];
        dA[e] = c0[e] - t6[e];
      }
    } else {  // dV = S_j, dA = w_j + S_j x V_b
      cross_m(S, V, t6);
      for (int e = 0; e < 6; ++e) {
        dV[e] = S[e];
        dA[e] = c0[e] + t6[e];
      }
    }
    motion_act_inv(Rf, pf, V, vf);
    motion_act_inv(Rf, pf, dV, dvf);
    motion_act_inv(Rf, pf, dA, daf);
    const double kp = C.r[1], kd = C.r[2];
    if (C.type() == C_CONTACT_3D) {
      double t1[3], t2[3], pv[3] = {0., 0., 0.};
      cross3(dvf + 3, vf, t1);
      cross3(vf + 3, dvf, t2);
      if (isq && kp != 0.) {  // world velocity of the frame origin: oRf Jc
        cross3(S + 3, pf, pv);
        for (int e = 0; e < 3; ++e) pv[e] += S[e];
      }
      for (int e = 0; e < 3; ++e)
        da0[(int64_t)(row + e) * L + dd] = daf[e] + t1[e] + t2[e] + kd * dvf[e] + kp * pv[e];
    } else {
      double rr[6], Jk[6] = {0., 0., 0., 0., 0., 0.};
      if (isq && kp != 0.) frame_residual(b, W, C, S, rr, Jk);
      for (int e = 0; e < 6; ++e) da0[(int64_t)(row + e) * L + dd] = daf[e] + kd * dvf[e] + kp * Jk[e];
    }
    row += n;
    r += C.size();
  }
}

// d(Jc v+)/dq_j for the impulse records (impulse-3d.hxx:33-39 / impulse-6d.hxx:30-36:
// getJointVelocityDerivatives at v+, moved into the frame): -Ad(oMf)^-1 (S_j x V+_P)
// with W.v holding the velocities at v+. dv0[row * L + j].
MB_HD inline void impulse_direction(const Blk& b, const WVals& W, int j, int L, double* dv0) {
  double S[6], VP[6], AP[6], u[6];
  for (int e = 0; e < 6; ++e) S[e] = W.S(j)[e];
  parent_motion(b, W, j, VP, AP);
  cross_m(S, VP, u);
  for (int e = 0; e < 6; ++e) u[e] = -u[e];
  const double* r = b.K;
  int row = 0;
  for (int k = 0; k < b.ncon; ++k) {
    const CRec C{r};
    const int fb = frame_dof(b, C.d());
    const int n = C.type() == C_CONTACT_3D ? 3 : 6;
    double o[6] = {0., 0., 0., 0., 0., 0.};
    if ((*W.anc(fb) >> j) & 1ull) {
      double Rf[9], pf[3];
      frame_placement(b, W, C.d(), Rf, pf);
      motion_act_inv(Rf, pf, u, o);
    }
    for (int e = 0; e < n; ++e) dv0[(int64_t)(row + e) * L + j] = o[e];
    row += n;
    r += C.size();
  }
}

// lane j < nj: column j of every jac-cost Jacobian (Jf[(f*6 + e)*jw + j]; a
// frame-velocity cost also its velocity column nj + j) and, on lane 0, their
// residuals (rf[6 f + e]); lanes j < 6 of a free-flyer knot also the Euler step's
// Jexp6(dq) column j (Je, col-major 6x6) and, on lane 0, Ad(exp6(dq)^-1) (Ai).
// only: -1 every jac cost, -2 none (the free-flyer Euler terms alone), f >= 0 jac cost f
// alone (one (dof, cost) item per lane)
MB_HD inline void jac_lane(const Blk& b, const WVals& W, const double* x, int j, double* Jf, int jw, double* rf,
                           const double* dqff, double* Je, double* Ai, int only = -1) {
  const int nj = b.nj;
  double S[6];
  for (int e = 0; e < 6; ++e) S[e] = W.S(j)[e];
  const double* cr = b.C;
  int f = 0;
  for (int k = 0; k < b.ncost && only != -2; ++k) {
    const CRec C{cr};
    const int t = C.type();
    if (jac_cost(b, t) && only >= 0 && f != only) {
      ++f;
    } else if (jac_cost(b, t)) {
      double r[6] = {0., 0., 0., 0., 0., 0.}, Jc[6] = {0., 0., 0., 0., 0., 0.};
      if (t == C_FRAME_PLACEMENT || t == C_FRAME_TRANSLATION) {
        const bool sup = (*W.anc(frame_dof(b, C.d())) >> j) & 1ull;
        frame_residual(b, W, C, sup ? S : nullptr, r, Jc);
      } else if (t == C_FRAME_VELOCITY) {  // getFrameVelocityDerivatives (LOCAL)
        // dv_f/dq_j = -Ad(oMf)^-1 (S_j x V_P) (the transport of the subtree cancels),
        // dv_f/dv_j = Ad(oMf)^-1 S_j, for the dofs that move the frame's body
        const double* d = C.d();
        double Jv[6] = {0., 0., 0., 0., 0., 0.};
        if ((*W.anc(frame_dof(b, d)) >> j) & 1ull) {
          double Rf[9], pf[3], VP[6], AP[6], u6[6];
          frame_placement(b, W, d, Rf, pf);
          parent_motion(b, W, j, VP, AP);
          cross_m(S, VP, u6);
          for (int e = 0; e < 6; ++e) u6[e] = -u6[e];
          motion_act_inv(Rf, pf, u6, Jc);
          motion_act_inv(Rf, pf, S, Jv);
        }
        for (int e = 0; e < 6; ++e) Jf[((int64_t)f * 6 + e) * jw + nj + j] = Jv[e];
        if (j == 0) frame_velocity_res(b, W, d, r);
      } else if (t == C_COM_POSITION) {  // Jcom col j = (m_sub S_lin + S_ang x h_sub) / m_total
        double mt = 0.;
        for (int bb = 0; bb < nj; ++bb)
          if (carries_body(b, bb)) mt += *W.m(bb);
        double tt[3];
        cross3(S + 3, W.ch(j), tt);
        const double m = *W.cm(j);
        for (int e = 0; e < 3; ++e) Jc[e] = (m * S[e] + tt[e]) / mt;
        if (j == 0) {
          double c[3];
          com_value(b, W, c);
          for (int e = 0; e < 3; ++e) r[e] = c[e] - C.d()[e];
        }
      } else {  // free-flyer block of a state cost: Jlog6(Mref^-1 M) (Jdiff second, multibody.hxx:118-126)
        double Rr[9], pr[3];
        ff_rel(C.d(), x, Rr, pr);
        if (j < 6) jlog6_col(Rr, pr, j, Jc);
        if (j == 0) log6_t<double>(Rr, pr, r);
      }
      const int nr = jac_rows(t);
#pragma unroll
      for (int e = 0; e < 6; ++e)
        if (e < nr) {
          Jf[((int64_t)f * 6 + e) * jw + j] = Jc[e];
          if (j == 0) rf[6 * f + e] = r[e];
        }
      ++f;
    }
    cr += C.size();
  }
  if (dqff && j < 6) {
    jexp6_col(dqff, j, Je + 6 * j);
    if (j == 0) {  // Ad(M^-1) of M = exp6(dq): [[R^T, -R^T [p]x], [0, R^T]]
      double R[9], p[3];
      exp6_t<double>(dqff, R, p);
      for (int c = 0; c < 6; ++c)
        for (int r = 0; r < 6; ++r) Ai[c * 6 + r] = 0.;
      for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) {
          const double Rt = R[r * 3 + c];  // (R^T)(r, c)
          Ai[c * 6 + r] = Rt;
          Ai[(c + 3) * 6 + r + 3] = Rt;
        }
      for (int c = 0; c < 3; ++c) {  // -R^T [p]x, column c: -R^T (p x e_c)
        const double e[3] = {c == 0 ? 1. : 0., c == 1 ? 1. : 0., c == 2 ? 1. : 0.};
        double t[3], o[3];
        cross3(p, e, t);
        matTvec3(R, t, o);
        for (int r = 0; r < 3; ++r) Ai[(c + 3) * 6 + r] = -o[r];
      }
    }
  }
}

// model->calcDiff for one knot by one workgroup (euler.hxx:83-131,
// free-fwddyn.hxx:82-118, contact-fwddyn.hxx:107-160, impulse-fwddyn.hxx:85-127,
// cost-sum.hxx:122-160). Writes full blocks (entries beyond nu zero). A mass
// matrix that is not positive definite leaves NaN in Fx/Fu, which the backward
// pass reports as backward_error. `w`: diff_layout(nj, njac, nc).total doubles of LDS.
// xnext_out / cost_out (may be null): the knot's calc (xnext, cost) as well;
// Fx == nullptr: calc only (no derivative block is written).
#if defined(__HIP_DEVICE_COMPILE__)
// ---- fp64 matrix-core products of the calcDiff (v_mfma_f64_16x16x4_f64) -------
// (fragment maps and mb_mfma: with the tree-sparse LTDL above)
typedef __attribute__((address_space(1))) double mb_glb_d;
// The Fx block (euler.hxx:100-112 with JintegrateTransport / Jintegrate;
// impulse-fwddyn.hxx:111-115) straight from the da product's accumulators:
// da = -(Kinv_tl dtau + H da0) (contact-fwddyn.hxx:127-140 as computeABADerivatives / the
// KKT inverse), computed transposed, tile rows = the tangent directions c, tile columns =
// the dofs i: a lane's accumulators are da(i, c) for one i and four c, and the 16 lanes of
// a row group store 16 consecutive rows of a column of the column-major Fx. With the
// contact-force costs (nfd = nc) the same product's rows nj + k' ([H^T | -S^-1]) give
// d lambda / dx (contact-fwddyn.hxx:131-137), row-major nc x L into dfx (LDS, or the Fu
// block in the spilled plan: a generic pointer).
// mode: bit 0 impulse, 1 integrated (dt != 0), 2 free-flyer Euler (Jexp6 rows), 3 ok.
// dtau: read from LDS at dts; in the spilled plan dtg is its global copy (the knot's Lxx
// block) and each wave first copies the direction blocks of its tiles into dts (so the
// tiles' loads are LDS loads, which never wait behind the Fx stores); dtg == nullptr:
// dtau is in LDS already. dts == nullptr: the product reads dtg (global) directly.
template <bool GA>  // GA: the A operand read from global memory (dtg) instead of the LDS copy
__device__ __attribute__((noinline)) void da_fx_mfma(const mb_lds_d* Minv, int lda, const mb_lds_d* H,
                                                     const double* dtg, mb_lds_d* dts, const mb_lds_d* da0, int nj,
                                                     int nc, int L, int mode, double dt, const mb_lds_d* Sinv, int nfd,
                                                     double* dfx, const mb_lds_d* Je, const mb_lds_d* Ai,
                                                     const mb_lds_d* Jc, double* Fx, const mb_lds_d* Z) {
  const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6, nw = (int)blockDim.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int NR = nj + nfd, tr = (NR + 15) >> 4, tc = (L + 15) >> 4, K = nj + nc, N = 2 * nj;
  const bool imp = mode & 1, integ = mode & 2, ffe = mode & 4, ok = mode & 8;
  const double mul_v = ok ? -1. : (double)NAN, dt2 = dt * dt;
  const int vcols = imp ? nj : L;  // impulse knots: the v columns of da are zero
  mb_glb_d* const F = (mb_glb_d*)Fx;
  const mb_glb_d* const G = (const mb_glb_d*)dtg;
  // tiles direction-block major, a contiguous range per wave: its tiles share their A
  // operands (at most two direction blocks)
  MB_GJ_MARK(22);
  const int per = (tr * tc + nw - 1) / nw, t0 = wave * per;
  const int t1 = (wave + 1) * per < tr * tc ? (wave + 1) * per : tr * tc;
  if (!GA && G && t0 < t1) {  // this wave's direction blocks of dtau into LDS (loads first)
    const int j0 = t0 / tr, j1 = (t1 - 1) / tr;
    for (int tj = j0; tj <= j1; ++tj) {
      const int c = 16 * tj + li;
      // (nj <= 40: the copy's area, 2 nj^2 doubles, fits the world values' only then)
      double v[10];
#pragma unroll
      for (int s = 0; s < 10; ++s) {
        const int k = 4 * s + lk;
        v[s] = (k < nj && c < L) ? (double)G[k * L + c] : 0.;
      }
#pragma unroll
      for (int s = 0; s < 10; ++s) {
        const int k = 4 * s + lk;
        if (k < nj && c < L) dts[k * L + c] = v[s];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  MB_GJ_MARK(25);
#pragma unroll 1
  for (int tile = t0; tile < t1; ++tile) {
    const int tj = tile / tr, ti = tile - tj * tr;
    const int i = 16 * ti + li, ca = 16 * tj + li;
    const bool rv = i < nj, rf = !rv && i < NR, cv = ca < L;
    mb_f64x4 acc = {0., 0., 0., 0.};
    // operands from clamped addresses, every load unconditional, then selected (a load
    // under a lane-dependent condition becomes a branch that waits for it: one LDS round
    // trip per k-step); the k-steps in chunks of 8, the chunk's loads first
    const int cac = ca < L ? ca : L - 1;
    const int ic = i < nj ? i : nj - 1, ir = i - nj < 0 ? 0 : (i - nj < nfd ? i - nj : (nfd > 0 ? nfd - 1 : 0));
    if constexpr (!GA) {
      // two k-ranges, each with one operand source per lane and a per-lane stride (no
      // per-step address selects, which became branches): k < nj (A = dtau, B = Kinv_tl
      // rows / H^T columns), then k' = k - nj < nc (A = da0, B = H rows / -S^-1); the
      // padding k-steps masked; loads of 4 k-steps first, then their MFMAs
      const mb_lds_d* pa = dts + (lk * L + cac);
      const mb_lds_d* pb = rv ? Minv + (lk * lda + ic) : (rf ? H + (ir * nj + lk) : Z);
      const int sb = rv ? 4 * lda : (rf ? 4 : 0);
#pragma unroll 1
      for (int k0 = 0; k0 < nj; k0 += 16) {
        double av[4], bw[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          av[s] = pa[(k0 + 4 * s) * L];
          bw[s] = pb[(k0 / 4 + s) * sb];
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int k = k0 + 4 * s + lk;
          if (k0 + 4 * s < nj) acc = mb_mfma(cv && k < nj ? av[s] : 0., rv || rf ? bw[s] : 0., acc);
        }
      }
      const mb_lds_d* qa = da0 + (lk * L + cac);
      const mb_lds_d* qb = rv ? H + (lk * nj + ic) : (rf ? Sinv + (lk * nc + ir) : Z);
      const int sq = rv ? 4 * nj : (rf ? 4 * nc : 0);
      const double sg = rf ? -1. : 1.;
#pragma unroll 1
      for (int k0 = 0; k0 < nc; k0 += 16) {
        double av[4], bw[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          av[s] = qa[(k0 + 4 * s) * L];
          bw[s] = qb[(k0 / 4 + s) * sq];
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int k = k0 + 4 * s + lk;
          if (k0 + 4 * s < nc) acc = mb_mfma(cv && k < nc ? av[s] : 0., rv || rf ? sg * bw[s] : 0., acc);
        }
      }
    } else {
    // (chunks of 4 k-steps: the chunk's 24 loads issued, pinned by one empty asm that
    // consumes them all, then selected: sunk into the selects' conditions the loads became
    // branches that each wait for their load)
#pragma unroll 1
    for (int k0 = 0; k0 < K; k0 += 16) {
      double x1[4], x2[4], m1[4], h1[4], h2[4], s2[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int k = k0 + 4 * s + lk;
        const int kc = k < nj ? k : nj - 1, kn = k - nj < 0 ? 0 : (k - nj < nc ? k - nj : (nc > 0 ? nc - 1 : 0));
        // A(c, k) = [dtau; da0](k, c)
        x1[s] = GA ? (double)G[kc * L + cac] : (double)dts[kc * L + cac];
        x2[s] = da0[kn * L + cac];
        // B(k, i) = [Kinv_tl | H](i, k), the force rows nj + k': [H^T | -S^-1](k', k) (S symmetric)
        m1[s] = Minv[kc * lda + ic];
        h1[s] = H[kn * nj + ic];
        h2[s] = H[ir * nj + kc];
        s2[s] = Sinv[kn * nc + ir];
      }
      asm volatile(""
                   : "+v"(x1[0]), "+v"(x1[1]), "+v"(x1[2]), "+v"(x1[3]), "+v"(x2[0]), "+v"(x2[1]), "+v"(x2[2]),
                     "+v"(x2[3]), "+v"(m1[0]), "+v"(m1[1]), "+v"(m1[2]), "+v"(m1[3]), "+v"(h1[0]), "+v"(h1[1]),
                     "+v"(h1[2]), "+v"(h1[3]), "+v"(h2[0]), "+v"(h2[1]), "+v"(h2[2]), "+v"(h2[3]), "+v"(s2[0]),
                     "+v"(s2[1]), "+v"(s2[2]), "+v"(s2[3]));
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int k = k0 + 4 * s + lk;
        const bool km = k < nj, kh = !km && k < K;
        const double av = !cv ? 0. : (km ? x1[s] : (kh ? x2[s] : 0.));
        const double bw = rv ? (km ? m1[s] : (kh ? h1[s] : 0.)) : (rf ? (km ? h2[s] : (kh ? -s2[s] : 0.)) : 0.);
        if (k0 + 4 * s < K) acc = mb_mfma(av, bw, acc);
      }
    }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = 16 * tj + lk + 4 * q;
      // da(i, c) (a failed factorisation: NaN; impulse: 0 in the v columns)
      const double dav = acc[q] * (c >= vcols ? 0. * mul_v : mul_v);
      // the free-flyer Euler rows i < 6 mix da(0..5, c): lanes li = 0..5 of this row group
      double d6[6];
      if (ffe && ti == 0)
#pragma unroll
        for (int r = 0; r < 6; ++r) d6[r] = __shfl(dav, (lane & 48) | r);
      if (i >= nj && i < NR && c < L) dfx[(i - nj) * L + c] = acc[q];
      if (i >= nj || c >= L) continue;
      double fq, fv;  // Fx(i, c), Fx(nj + i, c)
      if (imp) {  // [[I, 0], [-G dtau_dq - H dv0_dq, G M = I - H Jc]]
        fq = c == i ? 1. : 0.;
        if (c < nj) {
          fv = dav;
        } else {
          double s = 0.;
          for (int k = 0; k < nc; ++k) s += H[k * nj + i] * Jc[k * nj + (c - nj)];
          fv = ok ? (c - nj == i ? 1. : 0.) - s : (double)NAN;
        }
      } else if (!integ) {
        fq = c == i ? 1. : 0.;
        fv = c == nj + i ? 1. : 0.;
      } else {
        if (ffe && i < 6) {  // Jexp6(dq) (da dt^2 + [0 dt I]) + Ad(exp6(dq)^-1)
          double s2 = c < 6 ? Ai[c * 6 + i] : 0.;
#pragma unroll
          for (int r = 0; r < 6; ++r) s2 += Je[r * 6 + i] * (d6[r] * dt2 + (c == nj + r ? dt : 0.));
          fq = s2;
        } else {
          fq = dav * dt2 + (c == nj + i ? dt : 0.) + (c == i ? 1. : 0.);
        }
        fv = dav * dt + (c == nj + i ? 1. : 0.);
      }
      F[(int64_t)c * N + i] = fq;
      F[(int64_t)c * N + nj + i] = fv;
    }
  }
  MB_GJ_MARK(23);
}
// The Gauss-Newton blocks sc * (R^T diag(w h) R + the diagonal state / control terms)
// (cost-sum.hxx:122-160) over the combined column space [x tangent (L) | u (m)]: the
// upper-triangle 16 x 16 tiles (bi <= bj) of the (L + m)^2 product; Lxx and Luu are
// written from the upper triangle and mirrored, Lxu from the x-row / u-column tiles.
// wrow[r]: the row's weight times its activation Hessian (w h).
// (noinline: its registers apart from the kernel body's, which is at the VGPR cap here)
__device__ __attribute__((noinline)) void gn_blocks_mfma(const double* Rm, int ldR, const double* wrow, int nrows,
                                                         int L, int nu, int m, double sc, double* Lxx, double* Lxu,
                                                         double* Luu, const double* diag) {
  const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6, nw = (int)blockDim.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int NC = L + m, cv = L + nu, NT = (NC + 15) >> 4, ntiles = NT * (NT + 1) / 2, n = L;
  Rm = lds_ptr(Rm);
  wrow = lds_ptr(wrow);
  diag = lds_ptr(diag);
#pragma unroll 1
  for (int tile = wave; tile < ntiles; tile += nw) {
    int bi = 0, rem = tile;
    while (rem >= NT - bi) {
      rem -= NT - bi;
      ++bi;
    }
    const int bj = bi + rem;
    const int ca = 16 * bi + li, cb = 16 * bj + li;
    // (clamped addresses, unconditional loads, then selects: a lane-dependent condition
    // around a load becomes a branch that waits for it)
    const int cac = ca < ldR ? ca : ldR - 1, cbc = cb < ldR ? cb : ldR - 1;
    mb_f64x4 acc = {0., 0., 0., 0.};
    // (the tile's transpose: the accumulator rows run over bj, its columns over bi, so
    // lane li holds row 16 bi + li and the 16 lanes of a column store 128 contiguous
    // bytes of the column-major blocks); chunks of 4 k-steps, the chunk's 12 loads issued
    // first and pinned by one empty asm (not sunk into the selects' branches)
#pragma unroll 1
    for (int k0 = 0; k0 < nrows; k0 += 16) {
      double x[4], y[4], wr[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int r = k0 + 4 * s + lk, rc = r < nrows ? r : nrows - 1;
        const mb_lds_d* Rr = (const mb_lds_d*)Rm + (int64_t)rc * ldR;
        x[s] = Rr[cbc];
        y[s] = Rr[cac];
        wr[s] = ((const mb_lds_d*)wrow)[rc];
      }
      asm volatile(""
                   : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]),
                     "+v"(wr[0]), "+v"(wr[1]), "+v"(wr[2]), "+v"(wr[3]));
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int r = k0 + 4 * s + lk;
        const double a = (r < nrows && cb < cv) ? x[s] : 0.;
        const double bv = (r < nrows && ca < cv) ? y[s] * wr[s] : 0.;
        if (k0 + 4 * s < nrows) acc = mb_mfma(a, bv, acc);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = 16 * bi + li, j = 16 * bj + lk + 4 * q;
      if (i > j || j >= NC) continue;
      const double v = sc * (i == j ? acc[q] + diag[i] : acc[q]);
      if (j < L) {  // Lxx (symmetric)
        mb_gstore(Lxx + (int64_t)j * n + i, v);
        if (i < j) mb_gstore(Lxx + (int64_t)i * n + j, v);
      } else if (i < L) {  // Lxu
        mb_gstore(Lxu + (int64_t)(j - L) * n + i, v);
      } else {  // Luu (symmetric)
        mb_gstore(Luu + (int64_t)(j - L) * m + (i - L), v);
        if (i < j) mb_gstore(Luu + (int64_t)(i - L) * m + (j - L), v);
      }
    }
  }
}

// The subtree sums of the velocity-product maps (subtree_nh_lane) on the matrix cores:
// Nsub (nj x 42) = T nb with the subtree indicator T[j][b] = 1 when dof j is an ancestor-
// or-self of b and b carries a body; waves w of nw (the caller's numbering) take the
// 16 x 16 output tiles round-robin. (The sums' association changes, not their terms.)
// (AS: the address space of the maps and sums, LDS or the spilled plan's Fx block)
template <class AS>
__device__ __forceinline__ void subtree_nh_mfma(const Blk& b, const WVals& W, const double* nb_, double* ns_, int w,
                                                int nw) {
  const AS* nb = (const AS*)(std::is_same<AS, mb_lds_d>::value ? lds_ptr(nb_) : nb_);
  AS* ns = (AS*)(std::is_same<AS, mb_lds_d>::value ? lds_ptr(ns_) : ns_);
  const int lane = (int)threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
  const int nj = b.nj, tr = (nj + 15) >> 4, tc = 3;  // 42 components in 3 tiles
#pragma unroll 1
  for (int tile = w; tile < tr * tc; tile += nw) {
    const int ti = tile / tc, tj = tile - ti * tc;
    const int j = 16 * ti + li, c = 16 * tj + li;
    mb_f64x4 acc = {0., 0., 0., 0.};
    // the k-steps in chunks of 8: every operand of a chunk loaded first, then its MFMA
    // chain (one LDS round trip per chunk, not per k-step)
#pragma unroll 1
    for (int k0 = 0; k0 < nj; k0 += 32) {
      double av[8], bv[8];
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int bb = k0 + 4 * s + lk;
        const int bs = bb < nj ? bb : 0;
        const double nv = nb[42 * bs + (c < 42 ? c : 0)];
        const bool in = bb < nj && j < nj && carries_body(b, bs) && ((*W.anc(bs) >> j) & 1ull);
        av[s] = in ? 1. : 0.;
        bv[s] = bb < nj && c < 42 ? nv : 0.;
      }
#pragma unroll
      for (int s = 0; s < 8; ++s)
        if (k0 + 4 * s < nj) acc = mb_mfma(av[s], bv[s], acc);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = 16 * ti + lk + 4 * q;
      if (row < nj && c < 42) ns[42 * row + c] = acc[q];
    }
  }
}
#endif

// SP: the spilled plan fixed at compile time (0 / 1: the device kernels, one variant per
// plan) or taken from `spill` (-1: the host emulation)
template <class X, int SP = -1>
MB_HD __forceinline__ void knot_calc_diff_x(const X& ex, const double* P, int nx, int m, const double* xg, const double* ug,
                                   bool use_u, double* w, double* Fx, double* Fu, double* Lxx, double* Lxu,
                                   double* Luu, double* Lx, double* Lu, double* xnext_out = nullptr,
                                   double* cost_out = nullptr, const double* xu_pre = nullptr, int spill = 0) {
  w = ex.lds(w);  // the work area and the parameter block live in LDS
  P = ex.lds(P);
  const Blk b = parse(P);
  const bool imp = b.impulse;  // ActionModelImpulseFwdDynamics (impulse-fwddyn.hxx:53-127)
  const int nj = b.nj, nq = b.nq, n = 2 * nj, L = 2 * nj, nc = b.nc, nu = nj - b.nun;
  const int lda = lda_of(nj);
  bool vcols;
  const int njac = count_jac_costs(b, &vcols);
  const int jw = vcols ? L : nj;  // columns of the stored jac-cost Jacobians
  const int nrows = count_cost_rows(b, nu);
  // (calc only, Fx == nullptr: the same plan; it ends before any spilled array is used)
  if (SP == 0) spill = 0;
  if (SP == 1) spill |= kSpillBlocks;
  const DiffLayout l = diff_layout(nj, njac, nc, vcols, nu, nrows, spill);
  const bool spilled = SP >= 0 ? SP == 1 : (spill & kSpillBlocks) != 0;
  // the recursions' per-wave partials (free areas of their phases: DiffLayout)
  const WVals W{w + l.wv, nj, w + l.pk};
  double* A = w + l.A;
  // dtau/dx, the body maps and their subtree sums: LDS, or (spilled) the knot's Lxx / Fx
  // blocks, written there after their last read (DiffLayout)
  double* dtau = spilled ? Lxx : w + l.dtau;
  double* nbm = spilled ? Fx : w + l.nb;
  double* nsub = spilled ? Fx + pad2((int64_t)42 * nj) : w + l.ns;
  double* da = w + l.da;  // (host emulation only)
  const int Ld = L + 1;   // row stride of da (odd: conflict-free column reads)
  double* qp = w + l.qp;
  double* x = w + l.vec;
  double* u = x + nq + nj;
  double* nle = u + nj;   // nle, then RNEA's tau (unused)
  double* av = nle + nj;  // z, then a (impulse: v+)
  double* rf = av + nj;   // jac-cost residuals, 6 per cost
  double* Je = rf + 6 * kMaxJacCosts;  // Jexp6(dq) 6x6
  double* Ai = Je + 36;                // Ad(exp6(dq)^-1) 6x6
  double* Jf = (spill & kSpillJ) ? Lxu : w + l.J;
  double* red = w + l.red;
  int* flag = (int*)(red + 4);
  double* Jc = w + l.Jc;
  double* a0 = w + l.a0;
  double* lam = w + l.lam;
  double* Y = w + l.Y;
  double* H = w + l.H;
  double* Sx = w + l.Sx;
  double* da0 = w + l.da0;
  double* fx = w + l.fx;
  double* zv = w + l.zv;
  ex.run([&](int lane) {
    // xu_pre (device, nq + nj <= nt): this thread's x[lane] / u[lane] loaded by the caller
    // beside the parameter-block copy (one global round trip instead of two)
    if (lane == 0) *(int*)(red + 5) = 0;  // the factorisation's side-work counter
    if (lane == 1) red[7] = 0.;           // an LDS zero (the da product's padding operand)
    if (xu_pre) {
      if (lane < nq + nj) x[lane] = xu_pre[0];
      if (lane < nj) u[lane] = (use_u && lane < nu) ? xu_pre[1] : 0.;
    } else {
      for (int e = lane; e < nq + nj; e += ex.nt) x[e] = xg[e];
      if (lane < nj) u[lane] = (use_u && lane < nu) ? ug[lane] : 0.;  // (impulse: a zero velocity)
    }
  });
  // world-frame kinematics, M into the left half of [M | I], nle
  world_kinematics(ex, b, W, x, A, lda, [](int, int) {}, [](int, int) {}, true);
  if (!imp) world_rnea(ex, b, W, x + nq, nullptr, nle);
  if (nc > 0)  // contact rows at the drift (ddq = 0; ContactModelMultiple::calc)
    ex.run([&](int lane) {
      if (lane < nj) contact_jac_lane(b, W, lane, Jc, nullptr);
      // the a0 terms on the next wave (not after the Jacobian columns on wave 0: a wave
      // runs its divergent lanes' paths one after another)
      for (int k = lane - 64; k >= 0 && k < (imp ? 0 : b.ncon); k += ex.nt) {
        int row0;
        const CRec C{contact_rec(b, k, &row0)};
        contact_a0_position(b, W, C, a0 + row0);
        contact_a0_drift(b, W, C, a0 + row0);
      }
    });
  MB_DUMP(0, A, nj, nj, lda);        // M (+ armature)
  if (!imp) MB_DUMP(1, nle, nj, 1, nj);
  if (nc > 0) {
    MB_DUMP(2, Jc, nj, nc, nj);         // Jc^T (nj x nc)
    MB_DUMP(3, a0, nc, 1, nc);
  }
  double* pb = red + 8;
  // M^-1 by the tree-sparse LTDL of M (tree_ltdl), into the second half of the A area
  // (column-major nj x nj, ld lda); with contacts: d a / d tau after the Schur step.
  double* Minv = A + l.half;
  // The velocity-product maps of the derivatives (per-body N_b, h_b into the dtau area;
  // their subtree sums into the da area; P_k, Q_k) and the cost-Jacobian columns need the
  // velocities and composite inertias only: on the device the waves the factorisation
  // leaves idle build them meanwhile, one map per slot (vp: how many are built), the
  // Jacobian columns beside the body maps when the idle waves are at least two (jac_side).
  // (unused by impulse knots)
  auto vp_side = [&](int slot, int sl, int snt) {
    if (slot == 0) {
      if (!imp)
        for (int d = sl; d < nj; d += 64) body_nh_lane(b, W, d, nbm);
      if (snt >= 128)
        for (int id = sl - 64; id >= 0 && id < nj * njac; id += snt - 64)
          jac_lane(b, W, x, id % nj, Jf, jw, rf, nullptr, nullptr, nullptr, id / nj);
    } else if (slot == 1 && !imp) {
#if defined(__HIP_DEVICE_COMPILE__)
      if (spilled)
        subtree_nh_mfma<mb_glb_d>(b, W, nbm, nsub, sl >> 6, snt >> 6);
      else
        subtree_nh_mfma<mb_lds_d>(b, W, nbm, nsub, sl >> 6, snt >> 6);
#endif
    } else if (slot == 2 && !imp) {
      for (int j = sl; j < nj; j += snt) qp_lane_ns(W, j, nsub, qp);
    }
  };
#if defined(__HIP_DEVICE_COMPILE__)
  // scratch of the factorisation: the depth levels and 1 / D in pb; in the M^-1 area (free
  // until tree_minv, nj lda >= nj^2 doubles) the fast path's rows ((md + 1) nj) or the
  // generic steps' dof masks (2 nj), which never run together
  const int md = tree_depth(b, W);
  // (calc only: no derivative work beside the factorisation)
  const int vp = (md < kTreeKD && ex.nt >= 128 && Fx) ? 3 : 0;
  const bool jac_side = vp > 0 && ex.nt - 64 >= 128;
  double* const tp = ex.lds(Minv);
  const TreeWork tw{(Mask*)tp, (Mask*)tp + nj, (Mask*)ex.lds(pb), ex.lds(pb) + 64, ex.lds(flag)};
  tree_ltdl(ex, b, W, A, lda, tw, md, tp, vp_side, vp, (int*)(red + 5));
#else
  // (host emulation: the factorisation's scratch in an area of its own, no side work)
  const int vp = 0;
  const bool jac_side = false;
  double* const tp = w + l.ht;
  const TreeWork tw{(Mask*)tp, (Mask*)tp + nj, (Mask*)ex.lds(pb), tp + 2 * nj, ex.lds(flag)};
  tree_ltdl(ex, b, W, A, lda, tw, tree_depth(b, W), tp + 3 * nj);
#endif
  bool ok = tree_minv(ex, b, A, lda, tw, Minv);
  Minv = ex.lds(Minv);
  MB_DUMP(4, Minv, nj, nj, lda);
  // z = (M + A)^-1 (tau - nle) (the acceleration without contacts); Y = Minv Jc^T
  ex.run([&](int lane) {
    if (lane < nj && imp) {
      av[lane] = x[nq + lane];  // z = M^-1 (M v) = v
      zv[lane] = 0.;
      if (lane == 0)
        for (int e = 0; e < 6; ++e) W.root_a()[e] = 0.;  // the impulse RNEA has no gravity
    } else if (lane < nj) {
      double s = 0.;
      for (int k = 0; k < nj; ++k) s += Minv[(int64_t)k * lda + lane] * ((k < b.nun ? 0. : u[k - b.nun]) - nle[k]);
      av[lane] = ok ? s : NAN;
    }
    for (int e = lane; e < nj * nc; e += ex.nt) {
      const int k = e / nj, i = e % nj;
      double s = 0.;
      for (int r = 0; r < nj; ++r) s += Minv[(int64_t)r * lda + i] * Jc[(int64_t)k * nj + r];
      Y[e] = s;
    }
  });
  if (nc > 0) {
    // [S | I | Jc z + a0], S = Jc Y + damping I; Gauss-Jordan -> [. | S^-1 | S^-1 r]
    ex.run([&](int lane) {
      for (int e = lane; e < nc * (2 * nc + 1); e += ex.nt) {
        const int col = e / nc, row = e % nc;
        double v;
        if (col < nc) {
          double s = 0.;
          for (int i = 0; i < nj; ++i) s += Jc[(int64_t)row * nj + i] * Y[(int64_t)col * nj + i];
          v = s + (row == col ? b.damping : 0.);
        } else if (col < 2 * nc) {
          v = (col - nc == row) ? 1. : 0.;
        } else {
          double s = 0.;
          for (int i = 0; i < nj; ++i) s += Jc[(int64_t)row * nj + i] * av[i];
          v = imp ? (1. + b.r_coeff) * s : s + a0[row];  // impulse: Jc v+ = -r Jc v
        }
        Sx[e] = v;
      }
    });
    ok = gauss_jordan<1>(ex, Sx, nc, nc, 2 * nc + 1, flag, pb) && ok;
    // lambda = -S^-1 r, a = z + Y lambda, H = Y S^-1 (= Kinv top-right)
    ex.run([&](int lane) {
      const double* Sinv = Sx + (int64_t)nc * nc;
      const double* sr = Sx + (int64_t)2 * nc * nc;
      if (lane < nc) lam[lane] = -sr[lane];
      if (lane < nj) {
        double s = av[lane];
        for (int k = 0; k < nc; ++k) s -= Y[(int64_t)k * nj + lane] * sr[k];
        av[lane] = ok ? s : NAN;
      }
      for (int e = lane; e < nj * nc; e += ex.nt) {
        const int k = e / nj, i = e % nj;
        double s = 0.;
        for (int m2 = 0; m2 < nc; ++m2) s += Y[(int64_t)m2 * nj + i] * Sinv[(int64_t)k * nc + m2];
        H[e] = s;
      }
    });
    // Kinv top-left Minv - H Y^T (in place); contact forces per dof (world)
    ex.run([&](int lane) {
      for (int e = lane; e < nj * nj; e += ex.nt) {
        const int c = e / nj, i = e % nj;
        double s = Minv[(int64_t)c * lda + i];
        for (int k = 0; k < nc; ++k) s -= H[(int64_t)k * nj + i] * Y[(int64_t)k * nj + c];
        Minv[(int64_t)c * lda + i] = s;
      }
      if (lane < nj) {
        contact_joint_forces(b, W, lam, fx, lane);
        if (imp) zv[lane] = av[lane] - x[nq + lane];  // v+ - v
      }
    });
  }
  MB_DUMP(5, Minv, nj, nj, lda);  // Kinv top-left (with contacts)
  MB_DUMP(6, av, nj, 1, nj);      // a
  if (nc > 0) {
    MB_DUMP(7, Y, nj, nc, nj);
    MB_DUMP(8, Sx + (int64_t)nc * nc, nc, nc, nc);  // S^-1
    MB_DUMP(9, H, nj, nc, nj);
  }
  // velocities, accelerations and forces at the solved a (the linearisation point
  // of computeABADerivatives / computeRNEADerivatives with fext)
  // (impulse: RNEA(q, 0, v+ - v) without gravity, impulse-fwddyn.hxx:102-104)
  // (the partials in the first half of A in the spilled plan: M is dead, Y too)
  world_rnea(ex, b, WVals{W.base, nj, w + l.pr}, imp ? u : x + nq, imp ? zv : av, nle, nc > 0 ? fx : nullptr);
  if (xnext_out || cost_out) {  // the knot's calc, fused (iteration 0 of a solve, or calc only)
    ex.run([&](int lane) {
      const double dt = b.dt;
      if (xnext_out && lane < nj) {
        if (imp) {
          xnext_out[lane] = x[lane];
          if (lane == nj - 1 && b.ff) xnext_out[nq - 1] = x[nq - 1];
          xnext_out[nq + lane] = av[lane];
        } else if (dt != 0.) {
          euler_step(b, x, av, dt, xnext_out, lane);
        } else {
          xnext_out[lane] = x[lane];
          if (lane == nj - 1 && b.ff) xnext_out[nq - 1] = x[nq - 1];
          xnext_out[nq + lane] = x[nq + lane];
        }
      }
      if (cost_out && !Fx && lane == 0) {  // calc only (with derivatives: from the residuals below)
        double cc = cost_value(b, W, x, u, nu);
        const double* cr = b.C;
        for (int k = 0; k < b.ncost; ++k) {
          const CRec C{cr};
          if (force_cost(C.type())) cc += C.weight() * force_cost_activation(b, C, lam, nu);
          cr += C.size();
        }
        *cost_out = dt != 0. ? dt * cc : cc;
      }
    });
  }
  if (!Fx) return;  // calc only
  const double dt = b.dt, dt2 = dt * dt;
  const bool integ = dt != 0.;
  const bool ffe = b.ff && integ && !imp;  // Euler on the free-flyer: Jexp6 / Ad(exp6^-1)
  // per-dof Q_k, P_k (lanes < nj) and the jac-cost Jacobians / residuals; the
  // free-flyer Euler step's Jexp6 and Ad(exp6(dq)^-1) (dq = v dt + a dt^2)
  // per-body velocity-product maps, then their subtree sums (DiffLayout nb / ns)
  // (the maps the factorisation's idle waves did not build)
  if (!imp && vp < 1)
    ex.run([&](int lane) {
      if (lane < nj) body_nh_lane(b, W, lane, nbm);
    });
  if (!imp && vp < 2)
    ex.run([&](int lane) {
      const int w = lane >> 6, j = lane & 63;
#if defined(__HIP_DEVICE_COMPILE__)
      (void)j;
      if (spilled)
        subtree_nh_mfma<mb_glb_d>(b, W, nbm, nsub, w, ex.nt >> 6);
      else
        subtree_nh_mfma<mb_lds_d>(b, W, nbm, nsub, w, ex.nt >> 6);
#else
      if (j < nj) {
        if (ex.nt >= 512)
          subtree_nh_lane<6>(b, W, j, nbm, nsub, w, ex.nt >> 6);
        else
          subtree_nh_lane<11>(b, W, j, nbm, nsub, w, ex.nt >> 6);
      }
#endif
    });
  // the velocity-product maps (if still to do) on the lower half of the workgroup, the
  // cost / Euler Jacobians on the rest (independent: they run side by side)
  ex.run([&](int lane) {
    const int h = !imp && vp < 3 ? ex.nt / 2 : 0;
    if (lane < h) {
      for (int j = lane; j < nj; j += h) qp_lane_ns(W, j, nsub, qp);
      return;
    }
    double dq[6];
    if (ffe)
      for (int e = 0; e < 6; ++e) dq[e] = x[nq + e] * dt + av[e] * dt2;
    if (jac_side) {  // the Jacobian columns are done: the free-flyer Euler terms only
      if (ffe && lane - h < 6) jac_lane(b, W, x, lane - h, Jf, jw, rf, dq, Je, Ai, -2);
      return;
    }
    for (int j = lane - h; j < nj; j += ex.nt - h) jac_lane(b, W, x, j, Jf, jw, rf, ffe ? dq : nullptr, Je, Ai);
  });
  if (imp) {  // V = 0 in the impulse RNEA: P_k = 0, Q_k = Ycrb_k S_k
    ex.run([&](int lane) {
      if (lane >= nj) return;
      comp_mul(W, lane, W.S(lane), qp + 12 * lane);
      for (int e = 0; e < 6; ++e) qp[12 * lane + 6 + e] = 0.;
    });
  }
  // tangent directions: dtau/dx (impulse: q only) and da0/dx side by side: one lane per
  // da0 direction (at most half the workgroup), the rest for dtau
  ex.run([&](int lane) {
    const int hc = (nc > 0 && !imp) ? (L < ex.nt / 2 ? L : ex.nt / 2) : 0;
    const int h = ex.nt - hc;
    if (lane < h) {
      // (direction, row part) per lane: a direction's rows split over up to 3 lanes when
      // the half-workgroup has the lanes for it
      const int nd = imp ? nj : L;
      const int np = h >= 3 * nd ? 3 : (h >= 2 * nd ? 2 : 1);
      for (int id = lane; id < nd * np; id += h)
        dtau_direction(b, W, qp, id % nd, L, dtau, imp ? nullptr : nsub, id / nd, np);
    } else {
      for (int dd = lane - h; dd < L; dd += hc) contact_direction(b, W, dd, L, da0);
    }
  });
  if (imp && nc > 0) {  // velocities at v+, then d(Jc v+)/dq
    ex.run([&](int lane) {
      if (lane < nj) w_velocity(W, av, lane);
    });
    ex.run([&](int lane) {
      for (int j = lane; j < nj; j += ex.nt) impulse_direction(b, W, j, L, da0);
    });
  }
  // d lambda / dx, d lambda / du for CostModelContactForce (contact-fwddyn.hxx:131-137, with
  // enable_force): Kinv bottom-left = H^T, bottom-right = -S^-1; dtau/du = [0; I]
  const bool fd = b.enable_force && nc > 0 && !imp;
  // (kSpillF: in the knot's Fu block, written last)
  double* dfx = (spill & kSpillF) ? Fu : w + l.dfx;
  double* dfu = (spill & kSpillF) ? Fu + pad2((int64_t)nc * L) : w + l.dfu;
  const double sc = integ ? dt : 1.;
  // cost-derivative area (layout: group table 4 kMaxCosts | Arr, Ar mul, Ar val,
  // source per row | R rows)
  double* cg = w + l.R;
  double* ch = cg + 4 * kMaxCosts;
  double* cam = ch + kMaxCostRows;
  double* cav = cam + kMaxCostRows;
  double* csrc = cav + kMaxCostRows;
  double* cgi = csrc + kMaxCostRows;  // group of each row
  double* cdg = w + l.Rr;             // device: the state / control diagonal terms per column
  double* Rm = cdg + kMaxCostCols;
  const int ldR = cost_rows_ld(nj, nu);
  // da = -Kinv_tl dtau - H da0 (impulse: -G dtau_dq - H dv0_dq on the q columns) on all
  // lanes but the last ncost, which build the cost-derivative table meanwhile (its area may be
  // the world-value area, dead since the tangent-direction phase)
  ex.run([&](int lane) {
    const int nl = ex.nt - (b.ncost > 0 ? b.ncost : 1);
#if defined(__HIP_DEVICE_COMPILE__)
    // on the matrix cores, every wave (the whole workgroup is converged here), the product's
    // epilogue writing the Fx block
    {
      const int mode = (imp ? 1 : 0) | (integ ? 2 : 0) | (ffe ? 4 : 0) | (ok ? 8 : 0);
      const mb_lds_d* SiL = (const mb_lds_d*)lds_ptr(Sx + (int64_t)nc * nc);
      // dtau: LDS (all-LDS plan), or the Lxx block copied into the LDS staging area / read
      // in place (spilled plan without room for the copy)
      // (an explicit flag: the copy's area may sit at LDS address 0)
      const double* dtg = spilled ? dtau : nullptr;
      const bool staged = !spilled || l.dts >= 0;
      mb_lds_d* dts = !spilled ? (mb_lds_d*)lds_ptr(dtau) : (mb_lds_d*)lds_ptr(w + (l.dts >= 0 ? l.dts : 0));
      const mb_lds_d* Z = (const mb_lds_d*)lds_ptr(red + 7);  // (0, set in the first phase)
      if (staged)
        da_fx_mfma<false>((const mb_lds_d*)lds_ptr(Minv), lda, (const mb_lds_d*)lds_ptr(H), dtg, dts,
                          (const mb_lds_d*)lds_ptr(da0), nj, nc, L, mode, dt, SiL, fd ? nc : 0, dfx,
                          (const mb_lds_d*)lds_ptr(Je), (const mb_lds_d*)lds_ptr(Ai), (const mb_lds_d*)lds_ptr(Jc),
                          Fx, Z);
      else
        da_fx_mfma<true>((const mb_lds_d*)lds_ptr(Minv), lda, (const mb_lds_d*)lds_ptr(H), dtg, dts,
                         (const mb_lds_d*)lds_ptr(da0), nj, nc, L, mode, dt, SiL, fd ? nc : 0, dfx,
                         (const mb_lds_d*)lds_ptr(Je), (const mb_lds_d*)lds_ptr(Ai), (const mb_lds_d*)lds_ptr(Jc),
                         Fx, Z);
    }
    constexpr bool dfx_done = true;
    (void)nl;
#else
    constexpr bool dfx_done = false;
    // two entries per lane at a time: two independent dot-product chains, so the LDS
    // loads of one overlap the other's FMAs (each entry's summation order unchanged)
    const int ne = nj * L;
    for (int e0 = lane; e0 < ne && lane < nl; e0 += 2 * nl) {
      const int e1 = e0 + nl < ne ? e0 + nl : e0;
      const int r0 = e0 / L, c0 = e0 % L, r1 = e1 / L, c1 = e1 % L;
      double s0 = 0., s1 = 0.;
      for (int k = 0; k < nj; ++k) {
        s0 += Minv[(int64_t)k * lda + r0] * dtau[(int64_t)k * L + c0];
        s1 += Minv[(int64_t)k * lda + r1] * dtau[(int64_t)k * L + c1];
      }
      for (int k = 0; k < nc; ++k) {
        s0 += H[(int64_t)k * nj + r0] * da0[(int64_t)k * L + c0];
        s1 += H[(int64_t)k * nj + r1] * da0[(int64_t)k * L + c1];
      }
      if (imp && c0 >= nj) s0 = 0.;
      if (imp && c1 >= nj) s1 = 0.;
      da[(int64_t)r0 * Ld + c0] = ok ? -s0 : NAN;
      if (e1 != e0) da[(int64_t)r1 * Ld + c1] = ok ? -s1 : NAN;
    }
#endif
    if (fd) {
      const double* Sinv = Sx + (int64_t)nc * nc;
      for (int e = lane; e < (dfx_done ? 0 : nc * L); e += ex.nt) {
        const int k = e / L, c = e % L;
        double s = 0.;
        for (int i = 0; i < nj; ++i) s += H[(int64_t)k * nj + i] * dtau[(int64_t)i * L + c];
        for (int m2 = 0; m2 < nc; ++m2) s -= Sinv[(int64_t)m2 * nc + k] * da0[(int64_t)m2 * L + c];
        dfx[e] = s;
      }
      for (int e = lane; e < nc * nj; e += ex.nt) {
        const int k = e / nj, c = e % nj;
        dfu[e] = c < nu ? -H[(int64_t)k * nj + b.nun + c] : 0.;
      }
    }
    // the cost-derivative table: groups in cost (name) order, each the rows of one cost
    // with a dense residual Jacobian, or the diagonal of a state / control cost; per row
    // Arr (hess), and Ar as amul * aval (the quadratic kinds' (w, r), so the gradient
    // keeps the order (X w) r of the reference's R^T (w r)). Cost k on lane
    // spread_lane(k) after the da tiles (host: lane nt-1-k, which has no da entries), from
    // its group / row / jac-cost offsets, prefix-counted.
#if defined(__HIP_DEVICE_COMPILE__)
    const int kk = spread_item(lane, ex.nt);  // (every lane ran the da tiles)
    if (kk < (b.ncost > 0 ? b.ncost : 1)) {
#else
    if (lane >= nl) {
      const int kk = ex.nt - 1 - lane;
#endif
      int g = 0, row = 0, f = 0;
      const double* cr = b.C;
      for (int k = 0; k < kk; ++k) {  // offsets of record kk
        const CRec C{cr};
        const int t = C.type();
        if (jac_cost(b, t)) {
          row += jac_rows(t);
          ++g;
          ++f;
        }
        if (t == C_STATE || t == C_CONTROL) ++g;
        if (fd && force_cost(t) && (int)C.d()[0] >= 0) {
          row += cost_act(b, C, nu).nr;
          ++g;
        }
        cr += C.size();
      }
      if (kk < b.ncost) {
        const CRec C{cr};
        const int t = C.type();
        const Act act = cost_act(b, C, nu);
        const double co = (double)(cr - P);
        if (jac_cost(b, t)) {
          const int r0 = row;
          for (int e = 0; e < jac_rows(t); ++e, ++row) {
            const double rv = rf[6 * f + e];
            ch[row] = act.hess(e, rv);
            cam[row] = act.kind <= A_WEIGHTED_QUAD ? act.p[e] : 1.;
            cav[row] = act.kind <= A_WEIGHTED_QUAD ? rv : act.sgrad(e, rv, 1.);
            csrc[row] = (double)(f * 8 + e);
            cgi[row] = g;
          }
          cg[4 * g] = r0;
          cg[4 * g + 1] = row;
          cg[4 * g + 2] = co;
          cg[4 * g + 3] = t == C_FRAME_VELOCITY ? 1. : 0.;  // 0: q columns only, 1: x columns
          ++g;
          ++f;
        }
        if (t == C_STATE || t == C_CONTROL) {  // diagonal part (state: beyond the free-flyer block)
          cg[4 * g] = -1.;
          cg[4 * g + 1] = t == C_STATE ? 0. : 1.;
          cg[4 * g + 2] = co;
          cg[4 * g + 3] = 0.;
          ++g;
        }
        if (fd && force_cost(t) && (int)C.d()[0] >= 0) {
          const int r0 = row;
          for (int e = 0; e < act.nr; ++e, ++row) {
            const double rv = force_res(C, lam, e);
            ch[row] = act.hess(e, rv);
            cam[row] = act.kind <= A_WEIGHTED_QUAD ? act.p[e] : 1.;
            cav[row] = act.kind <= A_WEIGHTED_QUAD ? rv : act.sgrad(e, rv, 1.);
            csrc[row] = -1. - e;
            cgi[row] = g;
          }
          cg[4 * g] = r0;
          cg[4 * g + 1] = row;
          cg[4 * g + 2] = co;
          cg[4 * g + 3] = 2.;  // x and u columns
          ++g;
        }
      }
      if (kk == (b.ncost > 0 ? b.ncost - 1 : 0)) cg[4 * kMaxCosts - 1] = g;  // the group count
    }
#if defined(__HIP_DEVICE_COMPILE__)
    MB_GJ_MARK(24);
#endif
  });
  // Output blocks in row pairs over all lanes: consecutive lanes write consecutive
  // 16-B pairs of the column-major blocks (n even, blocks 16-B aligned); the lane's
  // (column, row pair) advances by nt pairs without a division. Columns c0.. of [Fx | Fu],
  // after the residual rows (DiffLayout kSpillF): the host's last phase writes both; on the
  // device the da product wrote Fx, and Fu is written at the end of the last phase.
  auto assemble = [&](int lane, int c0) __attribute__((always_inline)) {
    // the operands re-asserted as LDS here: without it the inference lost them and they
    // were flat loads, each waiting (vmcnt) for the output stores issued before it
    const double* const daL = ex.lds(da);
    const double* const MinvL = ex.lds(Minv);
    const double* const HL = ex.lds(H);
    const double* const JcL = ex.lds(Jc);
    const double* const JeL = ex.lds(Je);
    const double* const AiL = ex.lds(Ai);
    // this phase's invariants laundered into fresh registers: kept in spill slots across
    // the kernel they were reloaded in every iteration, and a scratch reload after an
    // output store waits (vmcnt, in order) for that store to reach memory
    const int NJ = mb_launder(nj), NC = mb_launder(nc), LD = mb_launder(Ld), NU = mb_launder(nu);
    const int LDA = mb_launder(lda), NUN = mb_launder(b.nun), N = mb_launder(n), M = mb_launder(m);
    const double DT = mb_launder(dt), DT2 = mb_launder(dt2);
    const int flags = mb_launder((imp ? 1 : 0) | (integ ? 2 : 0) | (ffe ? 4 : 0) | (ok ? 8 : 0));
    const bool IMP = flags & 1, INTEG = flags & 2, FFE = flags & 4, OK = flags & 8;
    double* const FX = Fx;
    double* const FU = Fu;
    // Fx(i, c): Euler assembly (euler.hxx:100-112) with JintegrateTransport / Jintegrate
    // (both inlined, capturing copies: a closure left in scratch made every captured value a
    // scratch load of its address and a flat load of the value)
    auto fx_at = [=](int i, int c) __attribute__((always_inline)) -> double {
      if (IMP) {  // [[I, 0], [-G dtau_dq - H dv0_dq, G M = I - H Jc]] (impulse-fwddyn.hxx:111-115)
        if (i < NJ) return c == i ? 1. : 0.;
        if (c < NJ) return daL[(int64_t)(i - NJ) * LD + c];
        double s = 0.;
        for (int k = 0; k < NC; ++k) s += HL[(int64_t)k * NJ + (i - NJ)] * JcL[(int64_t)k * NJ + (c - NJ)];
        return OK ? (c - NJ == i - NJ ? 1. : 0.) - s : NAN;
      }
      if (!INTEG) return c == i ? 1. : 0.;
      if (i < NJ && FFE && i < 6) {  // Jexp6(dq) (da dt^2 + [0 dt I]) + Ad(exp6(dq)^-1)
        double s = c < 6 ? AiL[c * 6 + i] : 0.;
        for (int r = 0; r < 6; ++r) s += JeL[r * 6 + i] * (daL[(int64_t)r * LD + c] * DT2 + (c == NJ + r ? DT : 0.));
        return s;
      }
      if (i < NJ) return daL[(int64_t)i * LD + c] * DT2 + (c == NJ + i ? DT : 0.) + (c == i ? 1. : 0.);
      return daL[(int64_t)(i - NJ) * LD + c] * DT + (c == i ? 1. : 0.);
    };
    // Fu(i, c) = Kinv_tl(i mod nj, nun + c) dt^2 | dt (dtau/du = [0; I]), Jexp6 on
    // the free-flyer rows
    auto fu_at = [=](int i, int c) __attribute__((always_inline)) -> double {
      if (!(INTEG && c < NU && !IMP)) return 0.;
      if (i < NJ && FFE && i < 6) {
        double s = 0.;
        for (int r = 0; r < 6; ++r) s += JeL[r * 6 + i] * MinvL[(int64_t)(NUN + c) * LDA + r];
        return OK ? s * DT2 : NAN;
      }
      const double mi = OK ? MinvL[(int64_t)(NUN + c) * LDA + (i < NJ ? i : i - NJ)] : NAN;
      return i < NJ ? mi * DT2 : mi * DT;
    };
    // the free-flyer Euler rows (Jexp6 products, 6 terms each) on lanes of their own,
    // so the row pairs below all take the short path (a wave pays for its slowest lane)
    const int r6 = FFE ? 6 : 0;
    for (int e = lane + r6 * c0; e < r6 * (N + M); e += ex.nt) {
      const int c = e / 6, i = e - 6 * c;
      if (c < N)
        mb_gstore(FX + (int64_t)c * N + i, fx_at(i, c));
      else
        mb_gstore(FU + (int64_t)(c - N) * N + i, fu_at(i, c - N));
    }
    const int p0 = r6 >> 1, hp = (N >> 1) - p0, dq = ex.nt / hp, dr = ex.nt % hp;
    for (int c = c0 + lane / hp, ip = lane % hp; c < N + M;) {
      const int i = 2 * (p0 + ip);
      if (c < N)
        mb_gstore2(FX + (int64_t)c * N + i, fx_at(i, c), fx_at(i + 1, c));
      else
        mb_gstore2(FU + (int64_t)(c - N) * N + i, fu_at(i, c - N), fu_at(i + 1, c - N));
      c += dq;
      ip += dr;
      if (ip >= hp) ip -= hp, ++c;
    }
  };
  // the stacked residual Jacobians R (nrows x (L + nu), ld ldR): jac-cost rows from
  // their q (or x) columns, force-cost rows from d lambda / dx, du
  const int ngr = (int)cg[4 * kMaxCosts - 1];
  ex.run([&](int lane) {
    // entry e of the rows (the Jacobians and d lambda / dx, du may be in global memory:
    // four entries' loads issued before their stores)
    auto rentry = [&](int e) __attribute__((always_inline)) -> double {
      const int row = e / ldR, c = e % ldR;
      const int src = (int)csrc[row];
      double v = 0.;
      if (src >= 0) {  // jac cost f, row e2
        const int f = src >> 3, e2 = src & 7;
        const bool xc = c < nj || (c < L && jw == L);
        v = xc ? Jf[((int64_t)f * 6 + e2) * jw + c] : 0.;
        // a q-only cost stored with jw = L carries zeros in its velocity columns
        if (c >= nj && c < L && jw == L && cg[4 * (int)cgi[row] + 3] == 0.) v = 0.;
      } else {  // force cost row -1 - src of its group
        const CRec C{P + (int64_t)cg[4 * (int)cgi[row] + 2]};
        const int e2 = -1 - src;
        if (c < L)
          v = force_jac(C, dfx + c, L, e2);
        else if (c - L < nu)
          v = force_jac(C, dfu + (c - L), nj, e2);
      }
      return c < L + nu ? v : 0.;
    };
    const int ne = nrows * ldR;
    for (int e0 = lane; e0 < ne; e0 += 2 * ex.nt) {
      double v4[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) v4[u] = e0 + u * ex.nt < ne ? rentry(e0 + u * ex.nt) : 0.;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int e = e0 + u * ex.nt;
        if (e >= ne) break;
        Rm[e] = v4[u];
#if defined(__HIP_DEVICE_COMPILE__) && !defined(MB_NO_MFMA_GN)
        // the matrix-core GEMM takes each row's weight times its activation Hessian (w h)
        if (e % ldR == 0) {
          const int row = e / ldR;
          const CRec C{P + (int64_t)cg[4 * (int)cgi[row] + 2]};
          ch[row] *= C.weight();
        }
#endif
      }
    }
#if defined(__HIP_DEVICE_COMPILE__) && !defined(MB_NO_MFMA_GN)
    // the diagonal terms of the state / control costs (beyond the free-flyer block), per
    // column of [x tangent | u], in cost order
    for (int i = lane; i < L + m; i += ex.nt) {
      double d = 0.;
      for (int g = 0; g < ngr; ++g) {
        if ((int)cg[4 * g] >= 0) continue;
        const CRec C{P + (int64_t)cg[4 * g + 2]};
        if (cg[4 * g + 1] == 0. && i < L && !(b.ff && i < 6))
          d += C.weight() * cost_act(b, C, nu).hess(i, state_res(b, C.d(), x, i));
        else if (cg[4 * g + 1] == 1. && i >= L && i - L < nu)
          d += C.weight() * cost_act(b, C, nu).hess(i - L, u[i - L] - C.d()[i - L]);
      }
      cdg[i] = d;
    }
#endif
  });
  const double *const Rm_ = Rm, *const ch_ = ch, *const cg_ = cg, *const cam_ = cam, *const cav_ = cav, *const P_ = P,
                      *const x_ = x, *const u_ = u, *const cdg_ = cdg;
  // Gauss-Newton blocks (cost-sum.hxx:122-160) as a small GEMM over the rows, in
  // cost order: Lxx / Lxu / Luu entries four rows i at a time, then Lx / Lu.
  ex.run([&](int lane) {
    // the operands re-asserted as LDS where they are used (the inference does not carry
    // the entry's assumption this far: the loads were flat, each one a full round trip)
    const double* const Rm = ex.lds(Rm_);
    const double* const ch = ex.lds(ch_);
    const double* const cg = ex.lds(cg_);
    const double* const cam = ex.lds(cam_);
    const double* const cav = ex.lds(cav_);
    const double* const P = ex.lds(P_);
    const double* const x = ex.lds(x_);
    const double* const u = ex.lds(u_);
#if defined(__HIP_DEVICE_COMPILE__) && !defined(MB_NO_MFMA_GN)
    gn_blocks_mfma(Rm, ldR, ch, nrows, L, nu, m, sc, Lxx, Lxu, Luu, cdg_);
    MB_GJ_MARK(26);
#else
    const int n4 = (n + 3) / 4, m4 = (m + 3) / 4;
    // Lxx is symmetric: only its row blocks i0 <= j are tasks (column j has j / 4 + 1 of
    // them; columns 4a .. 4a+3 follow 2a(a+1) tasks), each entry above the diagonal also
    // stored mirrored
    int tx = 0;
    for (int jj = 0; jj < n; ++jj) tx += jj / 4 + 1;
    const int txu = n4 * m, tuu = m4 * m;
    for (int task = lane; task < tx + txu + tuu; task += ex.nt) {
      int blk, i0, j;
      if (task < tx) {
        int a = (int)((sqrt(1. + 2. * task) - 1.) * 0.5);
        while (2 * (a + 1) * (a + 2) <= task) ++a;
        while (a > 0 && 2 * a * (a + 1) > task) --a;
        const int rem = task - 2 * a * (a + 1);
        blk = 0, j = 4 * a + rem / (a + 1), i0 = 4 * (rem % (a + 1));
      } else if (task < tx + txu) {
        blk = 1, i0 = 4 * ((task - tx) % n4), j = (task - tx) / n4;
      } else {
        blk = 2, i0 = 4 * ((task - tx - txu) % m4), j = (task - tx - txu) / m4;
      }
      // R columns of the rows (i) and of the column (j): x tangent or u (L + c)
      const int ci = blk == 2 ? L + i0 : i0;
      const int cj = blk == 0 ? j : L + j;
      const bool jin = blk == 0 || j < nu;
      double lv[4] = {0., 0., 0., 0.};
      for (int g = 0; g < ngr; ++g) {
        const int r0 = (int)cg[4 * g];
        const CRec C{P + (int64_t)cg[4 * g + 2]};
        if (r0 >= 0) {
          const int r1 = (int)cg[4 * g + 1];
          double s2[4] = {0., 0., 0., 0.};
          // rows in guarded batches of 4, loads first: a group (3-6 rows here) costs one
          // or two LDS round trips instead of one per row (the sums keep row order)
#pragma unroll 1
          for (int rb = r0; rb < r1; rb += 4) {
            double2 a01[4], a23[4];
            double hr[4], rj[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int r = rb + q < r1 ? rb + q : r0;
              const double* Rr = Rm + (int64_t)r * ldR;
              // rows are 16-B aligned (ldR even) and ci is a multiple of 4 (blk 2: L even)
              a01[q] = *reinterpret_cast<const double2*>(Rr + ci);
              a23[q] = *reinterpret_cast<const double2*>(Rr + ci + 2);
              hr[q] = ch[r];
              rj[q] = jin ? Rr[cj] : 0.;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              if (rb + q >= r1) break;
              s2[0] += a01[q].x * hr[q] * rj[q];
              s2[1] += a01[q].y * hr[q] * rj[q];
              s2[2] += a23[q].x * hr[q] * rj[q];
              s2[3] += a23[q].y * hr[q] * rj[q];
            }
          }
          const double wt = C.weight();
#pragma unroll
          for (int q = 0; q < 4; ++q) lv[q] += wt * s2[q];
        } else if ((cg[4 * g + 1] == 0.) == (blk == 0) && blk != 1) {  // state (Lxx) / control (Luu) diagonal
          const Act act = cost_act(b, C, nu);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int i = i0 + q;
            if (i != j) continue;
            if (blk == 0 && !(b.ff && j < 6)) lv[q] += C.weight() * act.hess(j, state_res(b, C.d(), x, j));
            if (blk == 2 && j < nu) lv[q] += C.weight() * act.hess(j, u[j] - C.d()[j]);
          }
        }
      }
      const int rows = blk == 2 ? m : n;
      double* out = blk == 0 ? Lxx : (blk == 1 ? Lxu : Luu);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = i0 + q;
        if (i >= rows || (blk == 0 && i > j)) continue;
        const bool zero = (blk == 1 && j >= nu) || (blk == 2 && (i >= nu || j >= nu));
        const double v = zero ? 0. : (blk == 1 || integ ? sc * lv[q] : lv[q]);
        mb_gstore(out + (int64_t)j * rows + i, v);
        if (blk == 0 && i < j) mb_gstore(out + (int64_t)i * rows + j, v);
      }
    }
#endif
    // Lx (x columns) and Lu (u columns): R^T Ar in cost order
    for (int c = lane; c < n + m; c += ex.nt) {
      const bool isu = c >= n;
      const int j = isu ? c - n : c;
      double acc = 0.;
      if (!isu || j < nu) {
        const int cc = isu ? L + j : j;
        for (int g = 0; g < ngr; ++g) {
          const int r0 = (int)cg[4 * g];
          const CRec C{P + (int64_t)cg[4 * g + 2]};
          const double wt = C.weight();
          if (r0 >= 0) {
            const int r1 = (int)cg[4 * g + 1];
#pragma unroll 1
            for (int rb = r0; rb < r1; rb += 4) {  // guarded batches of 4 (as above)
              double rv[4], am[4], av[4];
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const int r = rb + q < r1 ? rb + q : r0;
                rv[q] = Rm[(int64_t)r * ldR + cc];
                am[q] = cam[r];
                av[q] = cav[r];
              }
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                if (rb + q >= r1) break;
                acc += wt * rv[q] * am[q] * av[q];
              }
            }
          } else if (!isu && cg[4 * g + 1] == 0. && !(b.ff && j < 6)) {
            acc += cost_act(b, C, nu).sgrad(j, state_res(b, C.d(), x, j), wt);
          } else if (isu && cg[4 * g + 1] == 1.) {
            acc += cost_act(b, C, nu).sgrad(j, u[j] - C.d()[j], wt);
          }
        }
      }
      mb_gstore((isu ? Lu : Lx) + j, integ ? sc * acc : acc);
    }
#if defined(__HIP_DEVICE_COMPILE__)
    MB_GJ_MARK(27);
    assemble(lane, n);  // Fu
    MB_GJ_MARK(28);
#else
    (void)lane;
#endif
    // the fused calc's cost (cost-sum.hxx:89-117): record k's weighted activation on
    // lane spread_lane(k) (one record per wave first), into the dead pivot buffer
    // (pb[0, 64)); jac-cost residuals from the Jacobian phase.
    // The wide records (state / control, wide_cost) row-parallel instead: 32 lanes each
    // from lane 128 on (from lane 0 in a 128-thread workgroup), their partials into
    // pb[64 + 32 w + l], summed below.
    if (cost_out) {
      const double* cr = b.C;
      const int wbase = ex.nt >= 256 ? 128 : 0;
      int f = 0, nw = 0;
      for (int k = 0; k < b.ncost; ++k) {
        const CRec C{cr};
        const int t = C.type();
        const bool wide = wide_cost(C, nw);
        const int wl = lane - wbase - 32 * nw;  // this lane's share of wide record nw
        if (wide ? (wl >= 0 && wl < 32) : lane == spread_lane(k, ex.nt)) {
          const Act act = cost_act(b, C, nu);
          double a = 0.;
          if (jac_cost(b, t) && (!wide || wl == 0)) {
            const int nr = jac_rows(t);
            for (int i = 0; i < nr; ++i) a += act.value2(i, rf[6 * f + i]);
          }
          if (t == C_STATE) {
            for (int i = (b.ff ? 6 : 0) + (wide ? wl : 0); i < n; i += wide ? 32 : 1)
              a += act.value2(i, state_res(b, C.d(), x, i));
          } else if (t == C_CONTROL) {
            for (int i = wide ? wl : 0; i < nu; i += wide ? 32 : 1) a += act.value2(i, u[i] - C.d()[i]);
          } else if (force_cost(t)) {
            a = 2. * force_cost_activation(b, C, lam, nu);
          }
          if (wide)
            pb[64 + 32 * nw + wl] = a;
          else
            pb[k] = C.weight() * (0.5 * a);
        }
        f += jac_cost(b, t) ? 1 : 0;
        nw += wide ? 1 : 0;
        cr += C.size();
      }
    }
  });
  if (cost_out)  // summed in cost order
    ex.run([&](int lane) {
      if (lane != 0) return;
      double total = 0.;
      const double* cr = b.C;
      int nw = 0;
      for (int k = 0; k < b.ncost; ++k) {
        const CRec C{cr};
        if (wide_cost(C, nw)) {
          double a = 0.;
          for (int l = 0; l < 32; ++l) a += pb[64 + 32 * nw + l];
          total += C.weight() * (0.5 * a);
          ++nw;
        } else {
          total += pb[k];
        }
        cr += C.size();
      }
      *cost_out = integ ? dt * total : total;
    });
#if !defined(__HIP_DEVICE_COMPILE__)
  ex.run([&](int lane) { assemble(lane, 0); });  // Fx, Fu (after the residual rows: kSpillF)
#endif
  (void)nx;
}

template <int NT, int SP>
__device__ __forceinline__ void knot_calc_diff(const double* P, int nx, int m, const double* xg, const double* ug, bool use_u,
                                      double* w, double* Fx, double* Fu, double* Lxx, double* Lxu, double* Luu,
                                      double* Lx, double* Lu, double* xnext_out, double* cost_out,
                                      const double* xu_pre = nullptr, int spill = 0) {
  static_assert(NT >= 128 && NT % 64 == 0, "the calcDiff phases take >= 2 waves");
  knot_calc_diff_x<DevExec, SP>(DevExec{NT}, P, nx, m, xg, ug, use_u, w, Fx, Fu, Lxx, Lxu, Luu, Lx, Lu, xnext_out,
                                cost_out, xu_pre, spill);
}

}  // namespace mb
}  // namespace fddp
