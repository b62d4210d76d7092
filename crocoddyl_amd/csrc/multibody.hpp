// Multibody knots on the device: IntegratedActionModelEuler ∘
// DifferentialActionModelFreeFwdDynamics (ActuationModelFull, CostModelSum of
// State / Control / FramePlacement / FrameTranslation costs) over a fixed-base
// kinematic tree of revolute joints.
//
// Reference: include/crocoddyl/core/integrator/euler.hxx:41-131,
//   multibody/actions/free-fwddyn.hxx:44-118, multibody/costs/cost-sum.hxx:89-160,
//   multibody/costs/{state,control,frame-placement,frame-translation}.hxx; the rigid-body
//   arithmetic the reference takes from Pinocchio (aba, computeABADerivatives,
//   updateFramePlacement, getFrameJacobian, log6, Jlog6) is computed here as:
//   * forward dynamics: a = (M + diag(armature))^-1 (tau - nle), with RNEA and the
//     composite-rigid-body algorithm in world coordinates, where every recursion is
//     an ancestor / subtree sum evaluated one joint per lane, and the solve by
//     Gauss-Jordan with one column per lane. (The reference's default path is ABA,
//     the same function.)
//   * derivatives: the RNEA linearised along each state direction (one lane per
//     q_j / v_j direction, tangents kept in LDS), da/dx = -(M + A)^-1 dtau/dx — the
//     identity computeABADerivatives implements;
//   * frame-cost Jacobians: the local frame Jacobian column of joint j pushed through
//     log6 in dual numbers, which is Jlog6(rMf) * fJf (frame-placement.hxx:63-66).
// Parameter-block layout: include/fddp_hip.h (FDDP_KNOT_EULER_FREEFWD).
#pragma once

#include "fddp_device.hpp"

// Everything except the workgroup drivers (knot_calc, knot_calc_diff,
// gauss_jordan) is __host__ __device__, so the same arithmetic is unit-tested
// on the CPU against the oracle (tests/test_multibody_host.py).
#define MB_HD __host__ __device__

namespace fddp {
namespace mb {

constexpr int kMaxJ = 32;       // joints (2 nv directions <= 64 lanes)
constexpr int kJRec = 26;       // doubles per joint record
constexpr int kCHdr = 4;        // doubles of a cost record's header
constexpr int kMaxFrameCosts = 8;
constexpr int kValsPerJoint = 52;  // R 9, p 3, oR 9, op 3, v 6, a 6, F 6, composite m 1, c 3, I 6
constexpr int kMaxNc = 24;         // stacked contact rows (FDDP_KNOT_EULER_CONTACTFWD)
// Cost record types; contact records (after the costs) use 5 / 6 and the same
// frame payload as the frame costs, so frame_residual serves both.
enum {
  C_STATE = 1,
  C_CONTROL = 2,
  C_FRAME_PLACEMENT = 3,
  C_FRAME_TRANSLATION = 4,
  C_CONTACT_3D = 5,
  C_CONTACT_6D = 6,
  C_CONTACT_FORCE = 7  // cost on a contact's force: payload [row0, nr, fref(6)] (contact-force.hxx)
};

struct Blk {
  double dt;
  int nj, ncost;
  const double* g;    // gravity (3)
  const double* arm;  // armature (nj)
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
  b.C = b.J + (int64_t)kJRec * b.nj;
  const double* e = b.C;
  for (int k = 0; k < b.ncost; ++k) e += (int)e[3];
  b.nun = 0;
  b.ncon = b.nc = 0;
  b.damping = 0.;
  b.K = e;
  b.impulse = false;
  b.enable_force = false;
  b.r_coeff = 0.;
  if (e - P < (int64_t)P[3]) {  // [nun | r_coeff, damping, ncontact, 0 | 1] + records
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

// Spatial algebra in (linear, angular) order, as Pinocchio's Motion / Force.
// liMi = (R, p): pose of the child joint frame in the parent frame.
// actInv on a motion (child <- parent): lin' = R^T (v - p x w), ang' = R^T w.
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

// Joint record accessors
struct JRec {
  const double* r;
  MB_HD JRec(const Blk& b, int i) : r(b.J + (int64_t)kJRec * i) {}
  MB_HD int parent() const { return (int)r[0]; }
  MB_HD const double* axis() const { return r + 1; }
  MB_HD const double* Rpl() const { return r + 4; }
  MB_HD const double* ppl() const { return r + 13; }
  MB_HD double mass() const { return r[16]; }
  MB_HD const double* com() const { return r + 17; }
  MB_HD const double* I6() const { return r + 20; }
};

// Per-knot value storage (LDS), kValsPerJoint doubles per joint, then the
// universe's velocity (0) and acceleration (-gravity) as the root's parent.
struct Vals {
  double* base;
  int nj;
  MB_HD double* root_v() const { return base + kValsPerJoint * nj; }
  MB_HD double* root_a() const { return root_v() + 6; }
  MB_HD double* R(int i) const { return base + kValsPerJoint * i; }
  MB_HD double* p(int i) const { return R(i) + 9; }
  MB_HD double* oR(int i) const { return R(i) + 12; }
  MB_HD double* op(int i) const { return R(i) + 21; }
  MB_HD double* v(int i) const { return R(i) + 24; }
  MB_HD double* a(int i) const { return R(i) + 30; }
  MB_HD double* F(int i) const { return R(i) + 36; }
  MB_HD double* cm(int i) const { return R(i) + 42; }   // composite mass
  MB_HD double* cc(int i) const { return R(i) + 43; }   // composite CoM
  MB_HD double* cI(int i) const { return R(i) + 46; }   // composite inertia about its CoM (6)
};

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

// Phase executor: run(f) calls f(lane) for every thread of the workgroup and
// then synchronises (device), or for lanes 0..nt-1 in order (host emulation,
// tests/test_multibody_host.py). Within one phase no lane reads what another
// lane writes, so both orders give the same result. run_w0(f): a phase only
// wave 0 works in, closed by a wave-level fence instead of a workgroup barrier
// (the other waves skip ahead to the next sync()); sync(): the barrier that
// hands wave-0 results back to the whole workgroup.
struct DevExec {
  int nt;
  template <class F>
  __device__ void run(F f) const {
    f((int)threadIdx.x);
    __syncthreads();
  }
  template <class F>
  __device__ void run_w0(F f) const {
    if (threadIdx.x < 64) {
      f((int)threadIdx.x);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  __device__ void sync() const { __syncthreads(); }
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
};

// Gauss-Jordan on the column-major nr x nc matrix A (ld nr) without pivoting
// (the left nr x nr block is SPD): one column per lane (lane < nc), one pivot
// per phase; the left block's pivot column is only read in its step. Returns
// false if a pivot is not positive.
// Runs on wave 0 (nc <= 64 columns) between wave-level fences; the caller's
// preceding phase must have ended in a workgroup barrier.
template <class X>
MB_HD __attribute__((noinline)) bool gauss_jordan(const X& ex, double* A, int nr, int nc, int* flag) {
  ex.run_w0([&](int lane) {
    if (lane == 0) *flag = 0;
  });
#pragma unroll 1
  for (int k = 0; k < nr; ++k) {
    ex.run_w0([&](int lane) {
      const double piv = A[(int64_t)k * nr + k];
      if (!(piv > 0.)) {
        if (lane == 0) *flag = 1;
      } else if (lane < nc && lane > k) {
        // pivot column and own column in chunks of 8 rows through registers
        // (independent loads, then the updates): no LDS round trip per row
        double* col = A + (int64_t)lane * nr;
        const double* pc = A + (int64_t)k * nr;
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

// ---- dual numbers for the log6 Jacobian -----------------------------------
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

// Cost records
struct CRec {
  const double* r;
  MB_HD int type() const { return (int)r[0]; }
  MB_HD double weight() const { return r[1]; }
  MB_HD int size() const { return (int)r[3]; }
  MB_HD const double* d() const { return r + kCHdr; }
};

// oMf of a frame record d = [joint, R 9, p 3, ...]; VT: any values type with oR(i), op(i)
template <class VT>
MB_HD inline void frame_placement(const VT& V, const double* d, double* R, double* p) {
  const int j = (int)d[0];
  matmul3(V.oR(j), d + 1, R);
  matvec3(V.oR(j), d + 10, p);
  p[0] += V.op(j)[0];
  p[1] += V.op(j)[1];
  p[2] += V.op(j)[2];
}

// Residual of a frame cost (and, with jcol >= 0, its Jacobian column d r / d q_jcol).
// Returns the residual size (6 placement, 3 translation).
MB_HD inline int frame_residual(const Blk& b, const Vals& V, const CRec& C, int jcol, double* r, double* Jc) {
  const double* d = C.d();
  double Rf[9], pf[3];
  frame_placement(V, d, Rf, pf);
  double dR[9] = {0., 0., 0., 0., 0., 0., 0., 0., 0.}, dp[3] = {0., 0., 0.};
  bool sup = false;
  if (jcol >= 0) {  // is jcol an ancestor-or-self of the frame's joint?
    for (int i = (int)d[0]; i >= 0; i = JRec(b, i).parent())
      if (i == jcol) {
        sup = true;
        break;
      }
    if (sup) {  // world axis w, velocity of the frame origin w x (op_f - op_j)
      double w[3], dd[3], vl[3];
      matvec3(V.oR(jcol), JRec(b, jcol).axis(), w);
      dd[0] = pf[0] - V.op(jcol)[0];
      dd[1] = pf[1] - V.op(jcol)[1];
      dd[2] = pf[2] - V.op(jcol)[2];
      cross3(w, dd, vl);
      dp[0] = vl[0];
      dp[1] = vl[1];
      dp[2] = vl[2];
      // dR = R_f [xi_ang]x with xi_ang = R_f^T w, i.e. [w]x R_f
      for (int c = 0; c < 3; ++c) {
        const double* Rc = Rf + 3 * c;
        double t[3];
        cross3(w, Rc, t);
        dR[3 * c] = t[0];
        dR[3 * c + 1] = t[1];
        dR[3 * c + 2] = t[2];
      }
    }
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
    if (Jc) Jc[e] = sup ? o[e].d : 0.;
  }
  return 6;
}

// Residual size of a cost record, and its activation weights (the last nr
// doubles of the record).
MB_HD inline int cost_nr(const CRec& C, int nx, int nu) {
  const int t = C.type();
  if (t == C_CONTACT_FORCE) return (int)C.d()[1];
  return t == C_STATE ? nx : (t == C_CONTROL ? nu : (t == C_FRAME_PLACEMENT ? 6 : 3));
}
MB_HD inline const double* cost_weights(const CRec& C, int nx, int nu) { return C.r + C.size() - cost_nr(C, nx, nu); }
// 0.5 r^T W r of a contact-force cost, r = lambda[row0 .. row0 + nr) - fref
// (contact-force.hxx:33-50: jMf.actInv(f) is the multiplier itself).
MB_HD inline double force_cost_activation(const CRec& C, const double* lam, int nx, int nu) {
  const double* d = C.d();
  const int row0 = (int)d[0], nr = (int)d[1];
  const double* w = cost_weights(C, nx, nu);
  double a = 0.;
  for (int e = 0; e < nr; ++e) {
    const double r = lam[row0 + e] - d[2 + e];
    a += w[e] * r * r;
  }
  return 0.5 * a;
}

// Residual of a frame cost, value only (calc). Returns the residual size.
template <class VT>
MB_HD __forceinline__ int frame_residual_value(const VT& V, const CRec& C, double* r) {
  const double* d = C.d();
  double Rf[9], pf[3];
  frame_placement(V, d, Rf, pf);
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

// 0.5 r^T W r of one cost record (kinematics in V).
template <class VT>
MB_HD __forceinline__ double cost_activation(const VT& V, const CRec& C, const double* x, const double* u, int nx, int nu) {
  const double* w = cost_weights(C, nx, nu);
  double a = 0.;
  if (C.type() == C_STATE) {
    for (int i = 0; i < nx; ++i) {
      const double r = x[i] - C.d()[i];
      a += w[i] * r * r;
    }
  } else if (C.type() == C_CONTROL) {
    for (int i = 0; i < nu; ++i) {
      const double r = u[i] - C.d()[i];
      a += w[i] * r * r;
    }
  } else if (C.type() == C_CONTACT_FORCE) {
    return 0.;  // needs the multipliers: added after the contact solve
  } else {
    double r[6] = {0., 0., 0., 0., 0., 0.};
    const int nr = frame_residual_value(V, C, r);
#pragma unroll
    for (int i = 0; i < 6; ++i)  // fixed trip count: r stays in registers
      if (i < nr) a += w[i] * r[i] * r[i];
  }
  return 0.5 * a;
}

// Cost value of the DAM (one thread; kinematics in V): sum of weight * 0.5 r^T W r
// in record (name) order (cost-sum.hxx:89-117).
template <class VT>
MB_HD inline double cost_value(const Blk& b, const VT& V, const double* x, const double* u, int nx, int nu) {
  double total = 0.;
  const double* cr = b.C;
  for (int k = 0; k < b.ncost; ++k) {
    const CRec C{cr};
    total += C.weight() * cost_activation(V, C, x, u, nx, nu);
    cr += C.size();
  }
  return total;
}

// ---------------------------------------------------------------------------
// World-frame dynamics (the calc path). Spatial quantities are expressed at
// the world origin in world axes, so every recursion of RNEA/CRBA becomes a
// sum over the ancestors or the subtree of a joint
//   v_i = sum_{k <= i} S_k qd_k,  a_i = -g + sum_{k <= i} (S_k qdd_k + v_k x S_k qd_k),
//   tau_i = S_i . sum_{k in subtree(i)} f_k,  Ic_i = sum_{k in subtree(i)} I_k,
//   M_ij = S_i . (Ic_j S_j)  (i ancestor of j),
// which each lane evaluates for its own joint: no serial chain through LDS.
// The placements oMi = oMparent * liMi are composed by pointer jumping
// (ceil(log2 nj) rounds). Same functions as the local-frame value_pass,
// rounded differently (tests/test_multibody_host.py checks both vs the oracle).
// ---------------------------------------------------------------------------
constexpr int kWPerJoint = 96;
constexpr int kMaxCosts = 64;
struct WVals {
  double* base;
  int nj;
  MB_HD double* R(int i) const { return base + kWPerJoint * i; }  // liMi rotation
  MB_HD double* p(int i) const { return R(i) + 9; }
  MB_HD double* oR(int i) const { return R(i) + 12; }  // oMi (also pointer-jumping buffer A)
  MB_HD double* op(int i) const { return R(i) + 21; }
  MB_HD double* S(int i) const { return R(i) + 24; }   // joint motion subspace (world)
  MB_HD double* m(int i) const { return R(i) + 30; }   // body mass
  MB_HD double* c(int i) const { return R(i) + 31; }   // body CoM (world)
  MB_HD double* Ic(int i) const { return R(i) + 34; }  // body inertia about its CoM, world axes (6)
  MB_HD double* v(int i) const { return R(i) + 40; }
  MB_HD double* a(int i) const { return R(i) + 46; }
  MB_HD double* F(int i) const { return R(i) + 52; }   // body force, then accumulated joint force
  MB_HD double* cm(int i) const { return R(i) + 58; }  // composite inertia, origin form: m, h = m c, I_O (6)
  MB_HD double* ch(int i) const { return R(i) + 59; }
  MB_HD double* cI(int i) const { return R(i) + 62; }
  MB_HD double* cq(int i) const { return R(i) + 68; }  // S_i qdd_i + v_i x S_i qd_i
  MB_HD double* Rb(int i) const { return R(i) + 74; }  // pointer-jumping buffer B
  MB_HD double* pb(int i) const { return R(i) + 83; }
  MB_HD double* jA(int i) const { return R(i) + 86; }  // jump targets of buffers A / B
  MB_HD double* jB(int i) const { return R(i) + 87; }
  MB_HD double* fb(int i) const { return R(i) + 90; }  // body force I a + v x* I v
  MB_HD unsigned* anc(int i) const { return (unsigned*)(base + kWPerJoint * nj) + i; }  // ancestors-or-self bits
  MB_HD double* root_a() const { return base + kWPerJoint * nj + (nj + 1) / 2 + 1; }
  MB_HD static int64_t doubles(int nj) { return (int64_t)kWPerJoint * nj + (nj + 1) / 2 + 1 + 6; }
};

MB_HD inline int jump_rounds(int nj) {
  int r = 0;
  while ((1 << r) < nj) ++r;
  return r;
}

MB_HD __forceinline__ double dot6(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}

// lane i < nj: local placement (buffer A starts as liMi), ancestor bits.
MB_HD inline void w_joint_local(const Blk& b, const WVals& W, const double* q, int i) {
  const JRec J(b, i);
  double ax[3], Rpl[9], R[9];
  for (int e = 0; e < 3; ++e) ax[e] = J.axis()[e];
  for (int e = 0; e < 9; ++e) Rpl[e] = J.Rpl()[e];
  joint_rotation(Rpl, ax, q[i], R);
  for (int e = 0; e < 9; ++e) {
    W.R(i)[e] = R[e];
    W.oR(i)[e] = R[e];
  }
  for (int e = 0; e < 3; ++e) {
    W.p(i)[e] = J.ppl()[e];
    W.op(i)[e] = J.ppl()[e];
  }
  *W.jA(i) = (double)J.parent();
  if (i == 0) {
    for (int e = 0; e < 6; ++e) W.root_a()[e] = e < 3 ? -b.g[e] : 0.;
  }
  unsigned m = 1u << i;
  for (int k = J.parent(); k >= 0; k = JRec(b, k).parent()) m |= 1u << k;
  *W.anc(i) = m;
}

// lane i < nj, round r: T_i <- T_j(i) o T_i, j(i) <- j(j(i)) (A -> B on even
// rounds, B -> A on odd ones).
MB_HD inline void w_jump(const WVals& W, int i, int r) {
  const bool ab = (r & 1) == 0;
  double* sR = ab ? W.oR(i) : W.Rb(i);
  double* sp = ab ? W.op(i) : W.pb(i);
  double* dR = ab ? W.Rb(i) : W.oR(i);
  double* dp = ab ? W.pb(i) : W.op(i);
  const int j = (int)*(ab ? W.jA(i) : W.jB(i));
  double R[9], p[3];
  for (int e = 0; e < 9; ++e) R[e] = sR[e];
  for (int e = 0; e < 3; ++e) p[e] = sp[e];
  if (j >= 0) {
    double Rj[9], pj[3], Ro[9], t[3];
    const double* jR = ab ? W.oR(j) : W.Rb(j);
    const double* jp = ab ? W.op(j) : W.pb(j);
    for (int e = 0; e < 9; ++e) Rj[e] = jR[e];
    for (int e = 0; e < 3; ++e) pj[e] = jp[e];
    matmul3(Rj, R, Ro);
    matvec3(Rj, p, t);
    for (int e = 0; e < 9; ++e) dR[e] = Ro[e];
    for (int e = 0; e < 3; ++e) dp[e] = pj[e] + t[e];
    *(ab ? W.jB(i) : W.jA(i)) = *(ab ? W.jA(j) : W.jB(j));
  } else {
    for (int e = 0; e < 9; ++e) dR[e] = R[e];
    for (int e = 0; e < 3; ++e) dp[e] = p[e];
    *(ab ? W.jB(i) : W.jA(i)) = -1.;
  }
}

// lane i < nj: oMi into oR/op (from buffer B after an odd number of rounds),
// world motion subspace and body inertia.
MB_HD inline void w_joint_world(const Blk& b, const WVals& W, int i, bool from_b) {
  const JRec J(b, i);
  double oR[9], op[3], w[3], vl[3], c[3], t[3];
  for (int e = 0; e < 9; ++e) oR[e] = from_b ? W.Rb(i)[e] : W.oR(i)[e];
  for (int e = 0; e < 3; ++e) op[e] = from_b ? W.pb(i)[e] : W.op(i)[e];
  if (from_b) {
    for (int e = 0; e < 9; ++e) W.oR(i)[e] = oR[e];
    for (int e = 0; e < 3; ++e) W.op(i)[e] = op[e];
  }
  matvec3(oR, J.axis(), w);
  cross3(op, w, vl);  // velocity of the world origin: w x (0 - op) = op x w
  matvec3(oR, J.com(), t);
  for (int e = 0; e < 3; ++e) c[e] = op[e] + t[e];
  // Ic_w = oR Ic oR^T
  const double* s = J.I6();
  const double Is[9] = {s[0], s[3], s[4], s[3], s[1], s[5], s[4], s[5], s[2]};
  double tmp[9], Iw[9];
  matmul3(oR, Is, tmp);
  for (int r = 0; r < 3; ++r)
    for (int cc = 0; cc < 3; ++cc) Iw[cc * 3 + r] = tmp[r] * oR[cc] + tmp[3 + r] * oR[3 + cc] + tmp[6 + r] * oR[6 + cc];
  for (int e = 0; e < 3; ++e) {
    W.S(i)[e] = vl[e];
    W.S(i)[3 + e] = w[e];
    W.c(i)[e] = c[e];
  }
  *W.m(i) = J.mass();
  double* o = W.Ic(i);
  o[0] = Iw[0];
  o[1] = Iw[4];
  o[2] = Iw[8];
  o[3] = Iw[3];
  o[4] = Iw[6];
  o[5] = Iw[7];
}

// lane i < nj: composite inertia of the subtree of i in origin form
// (m, h = m c, I_O = Ic + m (|c|^2 I - c c^T)): additive over the subtree.
MB_HD inline void w_composite(const Blk& b, const WVals& W, int i) {
  double m = 0., h[3] = {0., 0., 0.}, I[6] = {0., 0., 0., 0., 0., 0.};
  for (int k = i; k < b.nj; ++k) {
    if (!((*W.anc(k) >> i) & 1u)) continue;
    const double mk = *W.m(k);
    double c[3], Ic[6];
    for (int e = 0; e < 3; ++e) c[e] = W.c(k)[e];
    for (int e = 0; e < 6; ++e) Ic[e] = W.Ic(k)[e];
    const double cc = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
    m += mk;
    for (int e = 0; e < 3; ++e) h[e] += mk * c[e];
    I[0] += Ic[0] + mk * (cc - c[0] * c[0]);
    I[1] += Ic[1] + mk * (cc - c[1] * c[1]);
    I[2] += Ic[2] + mk * (cc - c[2] * c[2]);
    I[3] += Ic[3] - mk * c[0] * c[1];
    I[4] += Ic[4] - mk * c[0] * c[2];
    I[5] += Ic[5] - mk * c[1] * c[2];
  }
  *W.cm(i) = m;
  for (int e = 0; e < 3; ++e) W.ch(i)[e] = h[e];
  for (int e = 0; e < 6; ++e) W.cI(i)[e] = I[e];
}

// lane i < nj: v_i = sum over ancestors-or-self of S_k qd_k
MB_HD inline void w_velocity(const WVals& W, const double* qd, int i) {
  double v[6] = {0., 0., 0., 0., 0., 0.};
  const unsigned am = *W.anc(i);
  for (int k = 0; k <= i; ++k) {
    if (!((am >> k) & 1u)) continue;
    const double w = qd[k];
    for (int e = 0; e < 6; ++e) v[e] += W.S(k)[e] * w;
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
// force f_i = I_i a_i + v_i x* (I_i v_i)
MB_HD inline void w_accel_force(const WVals& W, int i, const double* fx = nullptr) {
  double a[6];
  for (int e = 0; e < 6; ++e) a[e] = W.root_a()[e];
  const unsigned am = *W.anc(i);
  for (int k = 0; k <= i; ++k) {
    if (!((am >> k) & 1u)) continue;
    for (int e = 0; e < 6; ++e) a[e] += W.cq(k)[e];
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
  for (int k = i; k < b.nj; ++k) {
    if (!((*W.anc(k) >> i) & 1u)) continue;
    for (int e = 0; e < 6; ++e) F[e] += W.fb(k)[e];
  }
  for (int e = 0; e < 6; ++e) W.F(i)[e] = F[e];
  tau[i] = dot6(W.S(i), F);
}

// lane j < nj: CRBA column j in world frame: F = Ic_j S_j, M_ij = S_i . F for
// the ancestors-or-self i of j (+ armature on the diagonal). A: ld lda, zeroed.
MB_HD inline void w_crba_column(const Blk& b, const WVals& W, int j, double* A, int lda) {
  double S[6], F[6], t[3];
  for (int e = 0; e < 6; ++e) S[e] = W.S(j)[e];
  const double m = *W.cm(j);
  const double* h = W.ch(j);
  const double* I = W.cI(j);
  // (m v - h x w, I_O w + h x v)
  cross3(h, S + 3, t);
  for (int e = 0; e < 3; ++e) F[e] = m * S[e] - t[e];
  cross3(h, S, t);
  F[3] = I[0] * S[3] + I[3] * S[4] + I[4] * S[5] + t[0];
  F[4] = I[3] * S[3] + I[1] * S[4] + I[5] * S[5] + t[1];
  F[5] = I[4] * S[3] + I[5] * S[4] + I[2] * S[5] + t[2];
  A[(int64_t)j * lda + j] = dot6(S, F) + b.arm[j];
  const unsigned am = *W.anc(j);
  for (int i = 0; i < j; ++i) {
    if (!((am >> i) & 1u)) continue;
    const double Mij = dot6(W.S(i), F);
    A[(int64_t)j * lda + i] = Mij;
    A[(int64_t)i * lda + j] = Mij;
  }
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

// Column c of the contact's LOCAL frame Jacobian (pinocchio getFrameJacobian
// LOCAL, contact-3d.hxx:29 / contact-6d.hxx:29): the world motion S_c moved to
// the frame (SE3::actInv of oMf), zero unless c supports the frame's joint.
template <class VT>
MB_HD inline void contact_jac_col(const VT& V, const unsigned* anc_j, const double* d, int c, const double* Sc,
                                  double* o) {
  if (!((*anc_j >> c) & 1u)) {
    for (int e = 0; e < 6; ++e) o[e] = 0.;
    return;
  }
  double Rf[9], pf[3];
  frame_placement(V, d, Rf, pf);
  motion_act_inv(Rf, pf, Sc, o);
}

// a0 of a contact (contact-3d.hxx:35-43, contact-6d.hxx:31-44) in two parts,
// so that neither holds log6 and the frame motions live at once: the
// Baumgarte position term kp * (p - p_ref) | kp * log6(Mref^-1 oMf) (needs only
// the placements), then the frame drift acceleration (classical for 3D, gravity
// removed) + kd * v from the world velocity / acceleration of the joint.
MB_HD __attribute__((noinline)) void contact_a0_position(const WVals& W, const CRec& C, double* a0) {
  const double kp = C.r[1];
  double r[6] = {0., 0., 0., 0., 0., 0.};
  if (kp != 0.) frame_residual_value(W, C, r);
  const int n = C.type() == C_CONTACT_3D ? 3 : 6;
  for (int e = 0; e < n; ++e) a0[e] = kp * r[e];
}
MB_HD __attribute__((noinline)) void contact_a0_drift(const WVals& W, const CRec& C, double* a0) {
  const double* d = C.d();
  const int j = (int)d[0];
  double Rf[9], pf[3], m6[6], vf[6], af[6];
  frame_placement(W, d, Rf, pf);
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
MB_HD inline void contact_world_force(const WVals& W, const CRec& C, const double* lam, double* o) {
  double Rf[9], pf[3], f[6];
  frame_placement(W, C.d(), Rf, pf);
  const bool c3 = C.type() == C_CONTACT_3D;
  for (int e = 0; e < 6; ++e) f[e] = (c3 && e >= 3) ? 0. : lam[e];
  force_act(Rf, pf, f, o);
}

// lane j < nj: sum of the contact forces acting on joint j (world) into fx[6j..]
MB_HD inline void contact_joint_forces(const Blk& b, const WVals& W, const double* lam, double* fx, int j) {
  double F[6] = {0., 0., 0., 0., 0., 0.};
  const double* r = b.K;
  int row = 0;
  for (int k = 0; k < b.ncon; ++k) {
    const CRec C{r};
    if ((int)C.d()[0] == j) {
      double o[6];
      contact_world_force(W, C, lam + row, o);
      for (int e = 0; e < 6; ++e) F[e] += o[e];
    }
    row += C.type() == C_CONTACT_3D ? 3 : 6;
    r += C.size();
  }
  for (int e = 0; e < 6; ++e) fx[6 * j + e] = F[e];
}

// lane c < nj: column c of the stacked contact Jacobian Jc (nc x nj,
// Jc[row * nj + c]); with At != null also into the columns [nj + row] of A (ld nj).
MB_HD __attribute__((noinline)) void contact_jac_lane(const Blk& b, const WVals& W, int c, double* Jc, double* At) {
  double Sc[6];
  for (int e = 0; e < 6; ++e) Sc[e] = W.S(c)[e];
  const double* r = b.K;
  int row = 0;
  for (int k = 0; k < b.ncon; ++k) {
    const CRec C{r};
    const int j = (int)C.d()[0];
    double o[6];
    contact_jac_col(W, W.anc(j), C.d(), c, Sc, o);
    const int n = C.type() == C_CONTACT_3D ? 3 : 6;
    for (int e = 0; e < n; ++e) {
      Jc[(int64_t)(row + e) * b.nj + c] = o[e];
      if (At) At[(int64_t)(b.nj + row + e) * b.nj + c] = o[e];
    }
    row += n;
    r += C.size();
  }
}

// Placements, world quantities, composite inertias and M (into A, zeroed by
// the caller) for configuration q; `costs(wave, l)` runs on waves >= 2 in
// the phase after the kinematics (nullptr-like no-op allowed).
template <class X, class CostF>
MB_HD inline void world_kinematics(const X& ex, const Blk& b, const WVals& W, const double* q, double* A,
                                   CostF costs) {
  const int nj = b.nj, R = jump_rounds(nj);
  ex.run([&](int lane) {
    if (lane < nj) w_joint_local(b, W, q, lane);
  });
  for (int r = 0; r < R; ++r)
    ex.run([&](int lane) {
      if (lane < nj) w_jump(W, lane, r);
    });
  ex.run([&](int lane) {
    if (lane < nj) w_joint_world(b, W, lane, (R & 1) != 0);
  });
  ex.run([&](int lane) {
    const int wave = lane >> 6, l = lane & 63;
    if (wave == 0 && l < nj) w_composite(b, W, l);
    if (wave >= 2) costs(wave, l);
  });
  ex.run([&](int lane) {
    if (lane < nj) w_crba_column(b, W, lane, A, nj);
  });
}

// Joint torques of RNEA(q, qd, qdd) (qdd == nullptr: 0) with the kinematics in W;
// fx (6 per joint, world frame at the origin, may be null): external forces,
// as pinocchio::rnea(model, data, q, v, a, fext).
template <class X>
MB_HD inline void world_rnea(const X& ex, const Blk& b, const WVals& W, const double* qd, const double* qdd,
                             double* tau, const double* fx = nullptr) {
  const int nj = b.nj;
  ex.run([&](int lane) {
    if (lane < nj) w_velocity(W, qd, lane);
  });
  ex.run([&](int lane) {
    if (lane < nj) w_accel_term(W, qd, qdd, lane);
  });
  ex.run([&](int lane) {
    if (lane < nj) w_accel_force(W, lane, fx);
  });
  ex.run([&](int lane) {
    if (lane < nj) w_joint_force(b, W, tau, lane);
  });
}

// LDS (doubles) of the calc scratch for nj joints and nc contact rows.
MB_HD inline int64_t calc_work_doubles(int nj, int nc = 0) {
  return WVals::doubles(nj) + (int64_t)nj * (nj + nc + 1) + 2 * nj + kMaxCosts + 8 + (int64_t)nc * nj + nc +
         (int64_t)nc * (nc + 1);
}

// model->calc(data, x, u) for the Euler∘FreeFwdDynamics knot (euler.hxx:41-80,
// free-fwddyn.hxx:44-79): a = (M + diag(armature))^-1 (u - nle) in world frame;
// with contacts, Euler∘ContactFwdDynamics (contact-fwddyn.hxx:59-104):
// pinocchio::forwardDynamics by the Schur complement,
//   [Y | z] = M^-1 [Jc^T | tau - nle],  S = Jc Y + damping I,
//   lambda = -S^-1 (Jc z + a0),  a = z + Y lambda.
// Needs >= 256 threads (4 waves): independent work of one phase runs on
// different waves (divergent lanes of one wave would serialise) — wave 0 the
// recursions, wave 1 composite inertias and CRBA, waves 2-3 the cost records.
// Every thread must call (phases end in barriers). x, u readable by all lanes;
// writes xnext[0..nx) and returns the knot cost. `w`: calc_work_doubles(nj, nc).
template <class X>
MB_HD inline double knot_calc_x(const X& ex, const double* P, int nx, const double* x, const double* u, bool use_u,
                                double* xnext, double* w) {
  const Blk b = parse(P);
  const bool imp = b.impulse;  // impulse: [M | Jc^T] only, z = v
  const int nj = b.nj, nc = b.nc, nu = nj - b.nun, ncol = imp ? nj + nc : nj + nc + 1;
  const WVals W{w, nj};
  double* A = w + WVals::doubles(nj);  // nj x (nj + nc + 1), ld nj: [M | Jc^T | tau - nle]
  double* tau = A + (int64_t)nj * ncol;
  double* ub = tau + nj;  // u (zero if !use_u)
  double* cv = ub + nj;   // per-cost activations
  double* red = cv + kMaxCosts;
  int* flag = (int*)(red + 2);
  double* Jc = red + 8;                  // nc x nj
  double* a0 = Jc + (int64_t)nc * nj;    // nc
  double* S = a0 + nc;                   // nc x (nc + 1), ld nc: [S | Jc z + a0]
  ex.run([&](int lane) {
    if (lane < nu) ub[lane] = use_u ? u[lane] : 0.;
    for (int e = lane; e < nj * ncol; e += ex.nt) A[e] = 0.;
  });
  // cost records k on wave 2 + (k & 1), lane k >> 1, once the placements exist
  world_kinematics(ex, b, W, x, A, [&](int wave, int l) {
    const double* cr = b.C;
    for (int k = 0; k < b.ncost; ++k) {
      const CRec C{cr};
      if (wave == 2 + (k & 1) && l == (k >> 1)) cv[k] = C.weight() * cost_activation(W, C, x, ub, nx, nu);
      cr += C.size();
    }
    const int kc = l - 32;  // contact position terms on the upper half of wave 2
    if (!imp && wave == 2 && kc >= 0 && kc < b.ncon) {
      int row0;
      const CRec C{contact_rec(b, kc, &row0)};
      contact_a0_position(W, C, a0 + row0);
    }
  });
  if (!imp) world_rnea(ex, b, W, x + nj, nullptr, tau);
  ex.run([&](int lane) {
    if (lane < nj) {
      const double ti = lane < b.nun ? 0. : ub[lane - b.nun];  // ActuationModelFloatingBase: tau = [0; u]
      if (!imp) A[(int64_t)nj * (nj + nc) + lane] = ti - tau[lane];
      if (nc) contact_jac_lane(b, W, lane, Jc, A);
    }
    if (!imp && lane >= 64 && lane < 64 + b.ncon) {
      int row0;
      const CRec C{contact_rec(b, lane - 64, &row0)};
      contact_a0_drift(W, C, a0 + row0);
    }
    if (lane == 128) {
      double total = 0.;
      for (int k = 0; k < b.ncost; ++k) total += cv[k];
      red[0] = total;
    }
  });
  bool ok = gauss_jordan(ex, A, nj, ncol, flag);
  // z, then a (impulse: v+, in tau's slot; z = M^-1 M v = v)
  double* a = imp ? tau : A + (int64_t)nj * (nj + nc);
  if (nc > 0) {
    ex.run([&](int lane) {
      for (int e = lane; e < nc * (nc + 1); e += ex.nt) {
        const int col = e / nc, row = e % nc;
        // column col of Y, or z (impulse: v, and the restitution term r Jc v)
        const double* yc = (imp && col == nc) ? x + nj : A + (int64_t)nj * (nj + col);
        double s = 0.;
        for (int i = 0; i < nj; ++i) s += Jc[(int64_t)row * nj + i] * yc[i];
        S[e] = col < nc ? s + (row == col ? b.damping : 0.) : (imp ? (1. + b.r_coeff) * s : s + a0[row]);
      }
    });
    ok = gauss_jordan(ex, S, nc, nc + 1, flag) && ok;
    ex.run([&](int lane) {
      if (lane == 64 && !imp) {  // contact-force costs (lambda = -S^-1 r, in S's last column, negated)
        double lamv[kMaxNc];
        for (int k = 0; k < nc; ++k) lamv[k] = -S[(int64_t)nc * nc + k];
        double add = 0.;
        const double* cr = b.C;
        for (int k = 0; k < b.ncost; ++k) {
          const CRec C{cr};
          if (C.type() == C_CONTACT_FORCE) add += C.weight() * force_cost_activation(C, lamv, nx, nu);
          cr += C.size();
        }
        red[0] += add;
      }
      if (lane >= nj) return;
      double s = imp ? x[nj + lane] : a[lane];
      for (int k = 0; k < nc; ++k) s -= A[(int64_t)nj * (nj + k) + lane] * S[(int64_t)nc * nc + k];
      a[lane] = s;
    });
  }
  const double cc = red[0];
  const double dt = b.dt;
  ex.run([&](int i) {
    if (i >= nj) return;
    if (imp) {  // impulse-fwddyn.hxx:80-81: xnext = (q, v+)
      xnext[i] = x[i];
      xnext[nj + i] = ok ? (nc > 0 ? a[i] : x[nj + i]) : NAN;
      return;
    }
    const double ai = ok ? a[i] : NAN;  // a singular mass matrix surfaces as forward_error
    if (dt != 0.) {
      const double v = x[nj + i];
      xnext[i] = x[i] + (v * dt + ai * dt * dt);
      xnext[nj + i] = v + ai * dt;
    } else {
      xnext[i] = x[i];
      xnext[nj + i] = x[nj + i];
    }
  });
  return dt != 0. ? dt * cc : cc;
}

template <int NT>
__device__ inline double knot_calc(const double* P, int nx, const double* x, const double* u, bool use_u, double* xnext,
                                   double* w) {
  static_assert(NT >= 256, "the multibody calc splits its phases over 4 waves");
  return knot_calc_x(DevExec{NT}, P, nx, x, u, use_u, xnext, w);
}

// ---------------------------------------------------------------------------
// calcDiff: one 64-thread workgroup per (element, knot).
// ---------------------------------------------------------------------------
struct DiffLayout {
  int64_t wv, vals, A, tang, dtau, J, xu, red, ct, total;
  // contact area (nc > 0): Jc nc x nj, a0 nc, lambda nc, Y = Minv Jc^T and
  // H = Y S^-1 (nj x nc each), [S | I | r] nc x (2nc + 1), da0/dx nc x L, fx 6 nj
  int64_t Jc, a0, lam, Y, H, Sx, da0, fx, zv, dfx, dfu;
};
__host__ __device__ inline DiffLayout diff_layout(int nj, int nframe, int nc = 0) {
  const int L = 2 * nj;
  DiffLayout l;
  l.wv = 0;
  l.vals = l.wv + pad2(WVals::doubles(nj));
  l.A = l.vals + (int64_t)kValsPerJoint * nj + 12;
  l.tang = l.A + (int64_t)nj * 2 * nj;          // [M | I] -> [. | Minv]
  l.dtau = l.tang + (int64_t)18 * nj * L;       // per lane: dv, da, df per joint, [i][c][L]
  l.J = l.dtau + ((int64_t)nj * L > 3 * nj ? (int64_t)nj * L : 3 * nj);  // dtau [i][L] (nle, a first)
  l.xu = l.J + (int64_t)6 * nj * (nframe > 0 ? nframe : 1);  // frame-cost Jacobians [cost][6][nj] + residuals
  l.red = l.xu + 3 * nj + 6 * kMaxFrameCosts + 8;  // x (2nj), u (nj), frame residuals
  l.ct = l.red + 8;  // red: flag
  l.Jc = l.ct;
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
  l.total = nc > 0 ? l.dfu + (int64_t)nc * nj : l.ct;
  return l;
}

// Linearised RNEA along direction (q_j if dir == 0, v_j if dir == 1), values in V.
// Tangents kept at T[(i*18 + c)*L + lane]. Writes dtau[i*L + lane].
MB_HD inline void rnea_tangent(const Blk& b, const Vals& V, const double* qd, int dir, int j, double* T, int L,
                                    int lane, double* dtau) {
  const int nj = b.nj;
  auto slot = [&](int i, int c) -> double& { return T[((int64_t)i * 18 + c) * L + lane]; };
  for (int i = 0; i < nj; ++i) {
    const JRec J(b, i);
    const int lam = J.parent();
    const double* ax = J.axis();
    const double* R = V.R(i);
    const double* p = V.p(i);
    double dv[6], da[6], t6[6], u6[6];
    if (lam >= 0) {
      double pv[6], pa[6];
      for (int e = 0; e < 6; ++e) {
        pv[e] = slot(lam, e);
        pa[e] = slot(lam, 6 + e);
      }
      motion_act_inv(R, p, pv, dv);
      motion_act_inv(R, p, pa, da);
    } else {
      for (int e = 0; e < 6; ++e) dv[e] = da[e] = 0.;
    }
    const double S[6] = {0., 0., 0., ax[0], ax[1], ax[2]};
    if (i == j) {
      if (dir == 0) {  // d(X^-1 m)/dq = -S x (X^-1 m)
        motion_act_inv(R, p, lam >= 0 ? V.v(lam) : V.root_v(), u6);
        cross_m(S, u6, t6);
        for (int e = 0; e < 6; ++e) dv[e] -= t6[e];
        motion_act_inv(R, p, lam >= 0 ? V.a(lam) : V.root_a(), u6);
        cross_m(S, u6, t6);
        for (int e = 0; e < 6; ++e) da[e] -= t6[e];
      } else {
        dv[3] += ax[0];
        dv[4] += ax[1];
        dv[5] += ax[2];
      }
    }
    // d(v x S qd) = dv x S qd  (+ v x S when dir == v, i == j)
    const double w = qd[i];
    const double Sw[6] = {0., 0., 0., ax[0] * w, ax[1] * w, ax[2] * w};
    cross_m(dv, Sw, t6);
    for (int e = 0; e < 6; ++e) da[e] += t6[e];
    if (dir == 1 && i == j) {
      cross_m(V.v(i), S, t6);
      for (int e = 0; e < 6; ++e) da[e] += t6[e];
    }
    // df = I da + dv x* (I v) + v x* (I dv)
    double df[6], Iv[6], Idv[6];
    inertia_mul(J.mass(), J.com(), J.I6(), da, df);
    inertia_mul(J.mass(), J.com(), J.I6(), V.v(i), Iv);
    inertia_mul(J.mass(), J.com(), J.I6(), dv, Idv);
    cross_f(dv, Iv, t6);
    cross_f(V.v(i), Idv, u6);
    for (int e = 0; e < 6; ++e) {
      slot(i, e) = dv[e];
      slot(i, 6 + e) = da[e];
      slot(i, 12 + e) = df[e] + t6[e] + u6[e];
    }
  }
  for (int i = nj - 1; i >= 0; --i) {
    const JRec J(b, i);
    double F[6];
    for (int e = 0; e < 6; ++e) F[e] = slot(i, 12 + e);
    dtau[(int64_t)i * L + lane] = dot3(J.axis(), F + 3);
    const int lam = J.parent();
    if (lam < 0) continue;
    if (dir == 0 && i == j) {  // d(X F)/dq = X (S x* F)
      const double S[6] = {0., 0., 0., J.axis()[0], J.axis()[1], J.axis()[2]};
      double t6[6];
      cross_f(S, V.F(i), t6);
      for (int e = 0; e < 6; ++e) F[e] += t6[e];
    }
    double t6[6];
    force_act(V.R(i), V.p(i), F, t6);
    for (int e = 0; e < 6; ++e) slot(lam, 12 + e) += t6[e];
  }
}

// da0/dx along the tangent direction of this lane (q_c if dir == 0, v_c if
// dir == 1), from the joint tangents of rnea_tangent (at ddq = a fixed, as
// getJointAccelerationDerivatives after computeRNEADerivatives): the frame
// motion tangents (jMf.actInv), the classical-acceleration term of a 3D
// contact, the gravity that RNEA's tangents carry removed, and the Baumgarte
// terms (contact-3d.hxx:46-71, contact-6d.hxx:48-66). da0[row * L + lane].
MB_HD inline void contact_tangent(const Blk& b, const Vals& V, const WVals& W, int dir, int c, const double* T,
                                  int L, int lane, double* da0) {
  const double* r = b.K;
  int row = 0;
  for (int k = 0; k < b.ncon; ++k) {
    const CRec C{r};
    const double* d = C.d();
    const int j = (int)d[0];
    double dv[6], da[6];
    for (int e = 0; e < 6; ++e) {
      dv[e] = T[((int64_t)j * 18 + e) * L + lane];
      da[e] = T[((int64_t)j * 18 + 6 + e) * L + lane];
    }
    const bool sup = (*W.anc(j) >> c) & 1u;
    if (dir == 0 && sup) {  // d(-R_j^T g)/dq_c = R_j^T (w_c x g)
      double wc[3], wg[3], t[3];
      matvec3(V.oR(c), JRec(b, c).axis(), wc);
      cross3(wc, b.g, wg);
      matTvec3(V.oR(j), wg, t);
      for (int e = 0; e < 3; ++e) da[e] -= t[e];
    }
    double dvf[6], daf[6], vf[6], vj[6];
    for (int e = 0; e < 6; ++e) vj[e] = V.v(j)[e];
    motion_act_inv(d + 1, d + 10, dv, dvf);
    motion_act_inv(d + 1, d + 10, da, daf);
    motion_act_inv(d + 1, d + 10, vj, vf);
    const double kp = C.r[1], kd = C.r[2];
    double rr[6], Jk[6] = {0., 0., 0., 0., 0., 0.};
    if (kp != 0. && dir == 0 && sup) frame_residual(b, V, C, c, rr, Jk);
    if (C.type() == C_CONTACT_3D) {
      double t1[3], t2[3];
      cross3(dvf + 3, vf, t1);
      cross3(vf + 3, dvf, t2);
      for (int e = 0; e < 3; ++e)
        da0[(int64_t)(row + e) * L + lane] = daf[e] + t1[e] + t2[e] + kd * dvf[e] + kp * Jk[e];
      row += 3;
    } else {
      for (int e = 0; e < 6; ++e) da0[(int64_t)(row + e) * L + lane] = daf[e] + kd * dvf[e] + kp * Jk[e];
      row += 6;
    }
    r += C.size();
  }
}

// d(Jc v+)/dq_c for the impulse records (impulse-3d.hxx:33-39 / impulse-6d.hxx:30-36:
// getJointVelocityDerivatives at v+, moved into the frame): the joint velocity
// tangent along q_c walked from the root to each record's joint (vp: joint-frame
// velocities at v+, 6 per joint; qdp = v+). dv0[row * L + lane].
MB_HD inline void impulse_tangent(const Blk& b, const Vals& V, const WVals& W, const double* vp, const double* qdp,
                                  int c, int L, int lane, double* dv0) {
  const double* r = b.K;
  int row = 0;
  for (int k = 0; k < b.ncon; ++k) {
    const CRec C{r};
    const double* d = C.d();
    const int j = (int)d[0];
    const unsigned am = *W.anc(j);
    double dv[6] = {0., 0., 0., 0., 0., 0.};
    for (int i = 0; i <= j; ++i) {  // ancestors-or-self in root-to-j order (parents precede children)
      if (!((am >> i) & 1u)) continue;
      double t6[6];
      motion_act_inv(V.R(i), V.p(i), dv, t6);
      if (i == c) {  // d(X^-1 v_parent)/dq_i = -S x (X^-1 v_parent), X^-1 v_parent = v_i - S qd_i
        const double* ax = JRec(b, i).axis();
        const double S[6] = {0., 0., 0., ax[0], ax[1], ax[2]};
        double u6[6], w6[6];
        for (int e = 0; e < 6; ++e) u6[e] = vp[6 * i + e] - S[e] * qdp[i];
        cross_m(S, u6, w6);
        for (int e = 0; e < 6; ++e) t6[e] -= w6[e];
      }
      for (int e = 0; e < 6; ++e) dv[e] = t6[e];
    }
    double dvf[6];
    motion_act_inv(d + 1, d + 10, dv, dvf);
    const int n = C.type() == C_CONTACT_3D ? 3 : 6;
    for (int e = 0; e < n; ++e) dv0[(int64_t)(row + e) * L + lane] = dvf[e];
    row += n;
    r += C.size();
  }
}

// model->calcDiff for one knot by one 64-thread workgroup (euler.hxx:83-131,
// free-fwddyn.hxx:82-118, cost-sum.hxx:122-160). Writes full blocks (entries
// beyond nu zero); Lxu is zero (no cost couples x and u). A mass matrix that is
// not positive definite leaves NaN in Fx/Fu, which the backward pass reports
// as backward_error. `w`: diff_layout(nj, nframe).total doubles of LDS.
// xnext_out / cost_out (may be null): the knot's calc (xnext, cost) as well;
// Fx == nullptr: calc only (no derivative block is written).
template <class X>
MB_HD inline void knot_calc_diff_x(const X& ex, const double* P, int nx, int m, const double* xg, const double* ug,
                                   bool use_u, double* w, double* Fx, double* Fu, double* Lxx, double* Lxu,
                                   double* Luu, double* Lx, double* Lu, double* xnext_out = nullptr,
                                   double* cost_out = nullptr) {
  const Blk b = parse(P);
  const bool imp = b.impulse;  // ActionModelImpulseFwdDynamics (impulse-fwddyn.hxx:53-127)
  const int nj = b.nj, n = nx, L = 2 * nj, nc = b.nc, nu = nj - b.nun;
  int nframe = 0;
  {
    const double* cr = b.C;
    for (int k = 0; k < b.ncost; ++k) {
      const CRec C{cr};
      if (C.type() == C_FRAME_PLACEMENT || C.type() == C_FRAME_TRANSLATION) ++nframe;
      cr += C.size();
    }
  }
  const DiffLayout l = diff_layout(nj, nframe, nc);
  const WVals W{w + l.wv, nj};
  const Vals V{w + l.vals, nj};
  double* A = w + l.A;
  double* T = w + l.tang;
  double* dtau = w + l.dtau;
  double* Jf = w + l.J;
  double* x = w + l.xu;
  double* u = x + 2 * nj;
  double* rf = u + nj;  // frame residuals, 6 per frame cost
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
    if (lane < nx) x[lane] = xg[lane];
    if (lane < nj) u[lane] = (use_u && lane < nu) ? ug[lane] : 0.;  // (impulse: a zero velocity)
    for (int e = lane; e < 2 * nj * nj; e += ex.nt) {
      const int c = e / nj, r = e % nj;
      A[e] = (c == nj + r) ? 1. : 0.;
    }
  });
  // world-frame kinematics, M into the left half of [M | I], nle -> dtau[0..nj)
  world_kinematics(ex, b, W, x, A, [](int, int) {});
  if (!imp) world_rnea(ex, b, W, x + nj, nullptr, dtau);
  if (nc > 0)  // contact rows at the drift (ddq = 0; ContactModelMultiple::calc)
    ex.run([&](int lane) {
      if (lane < nj) contact_jac_lane(b, W, lane, Jc, nullptr);
      for (int k = lane; k < (imp ? 0 : b.ncon); k += ex.nt) {
        int row0;
        const CRec C{contact_rec(b, k, &row0)};
        contact_a0_position(W, C, a0 + row0);
        contact_a0_drift(W, C, a0 + row0);
      }
    });
  bool ok = gauss_jordan(ex, A, nj, 2 * nj, flag);
  double* Minv = A + (int64_t)nj * nj;  // column-major nj x nj; with contacts: d a / d tau after the Schur step
  // z = (M + A)^-1 (tau - nle) -> dtau[nj..2nj) (the acceleration without contacts);
  // Y = Minv Jc^T
  ex.run([&](int lane) {
    if (lane < nj && imp) {
      dtau[nj + lane] = x[nj + lane];  // z = M^-1 (M v) = v
      zv[lane] = 0.;
      if (lane == 0)
        for (int e = 0; e < 6; ++e) W.root_a()[e] = 0.;  // the impulse RNEA has no gravity
    } else if (lane < nj) {
      double s = 0.;
      for (int k = 0; k < nj; ++k) s += Minv[(int64_t)k * nj + lane] * ((k < b.nun ? 0. : u[k - b.nun]) - dtau[k]);
      dtau[nj + lane] = ok ? s : NAN;
    }
    for (int e = lane; e < nj * nc; e += ex.nt) {
      const int k = e / nj, i = e % nj;
      double s = 0.;
      for (int r = 0; r < nj; ++r) s += Minv[(int64_t)r * nj + i] * Jc[(int64_t)k * nj + r];
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
          for (int i = 0; i < nj; ++i) s += Jc[(int64_t)row * nj + i] * dtau[nj + i];
          v = imp ? (1. + b.r_coeff) * s : s + a0[row];  // impulse: Jc v+ = -r Jc v
        }
        Sx[e] = v;
      }
    });
    ok = gauss_jordan(ex, Sx, nc, 2 * nc + 1, flag) && ok;
    // lambda = -S^-1 r, a = z + Y lambda, H = Y S^-1 (= Kinv top-right)
    ex.run([&](int lane) {
      const double* Sinv = Sx + (int64_t)nc * nc;
      const double* sr = Sx + (int64_t)2 * nc * nc;
      if (lane < nc) lam[lane] = -sr[lane];
      if (lane < nj) {
        double s = dtau[nj + lane];
        for (int k = 0; k < nc; ++k) s -= Y[(int64_t)k * nj + lane] * sr[k];
        dtau[nj + lane] = ok ? s : NAN;
      }
      for (int e = lane; e < nj * nc; e += ex.nt) {
        const int k = e / nj, i = e % nj;
        double s = 0.;
        for (int m2 = 0; m2 < nc; ++m2) s += Y[(int64_t)m2 * nj + i] * Sinv[(int64_t)k * nc + m2];
        H[e] = s;
      }
    });
    // Kinv top-left Minv - H Y^T (in place); contact forces per joint (world)
    ex.run([&](int lane) {
      for (int e = lane; e < nj * nj; e += ex.nt) {
        const int c = e / nj, i = e % nj;
        double s = Minv[e];
        for (int k = 0; k < nc; ++k) s -= H[(int64_t)k * nj + i] * Y[(int64_t)k * nj + c];
        Minv[e] = s;
      }
      if (lane < nj) {
        contact_joint_forces(b, W, lam, fx, lane);
        if (imp) zv[lane] = dtau[nj + lane] - x[nj + lane];  // v+ - v
      }
    });
  }
  // accelerations and forces at the solved a (the linearisation point of
  // computeABADerivatives / computeRNEADerivatives with fext); tau lands in
  // dtau[2nj..3nj) and is not used
  // (impulse: RNEA(q, 0, v+ - v) without gravity, impulse-fwddyn.hxx:102-104)
  world_rnea(ex, b, W, imp ? u : x + nj, imp ? zv : dtau + nj, dtau + 2 * nj, nc > 0 ? fx : nullptr);
  // joint-frame values for the tangent recursion: liMi, oMi, and v, a, F moved
  // from world to joint coordinates (SE3::actInv of oMi)
  ex.run([&](int i) {
    if (i == 0)
      for (int e = 0; e < 6; ++e) {
        V.root_v()[e] = 0.;
        V.root_a()[e] = (e < 3 && !imp) ? -b.g[e] : 0.;
      }
    if (i >= nj) return;
    double oR[9], op[3], t6[6], m6[6];
    for (int e = 0; e < 9; ++e) {
      oR[e] = W.oR(i)[e];
      V.R(i)[e] = W.R(i)[e];
      V.oR(i)[e] = oR[e];
    }
    for (int e = 0; e < 3; ++e) {
      op[e] = W.op(i)[e];
      V.p(i)[e] = W.p(i)[e];
      V.op(i)[e] = op[e];
    }
    for (int e = 0; e < 6; ++e) m6[e] = W.v(i)[e];
    motion_act_inv(oR, op, m6, t6);
    for (int e = 0; e < 6; ++e) V.v(i)[e] = t6[e];
    for (int e = 0; e < 6; ++e) m6[e] = W.a(i)[e];
    motion_act_inv(oR, op, m6, t6);
    for (int e = 0; e < 6; ++e) V.a(i)[e] = t6[e];
    // force actInv: f' = R^T f, n' = R^T (n - p x f)
    double f[3], nn[3], c[3];
    for (int e = 0; e < 3; ++e) {
      f[e] = W.F(i)[e];
      nn[e] = W.F(i)[3 + e];
    }
    cross3(op, f, c);
    for (int e = 0; e < 3; ++e) nn[e] -= c[e];
    matTvec3(oR, f, t6);
    matTvec3(oR, nn, t6 + 3);
    for (int e = 0; e < 6; ++e) V.F(i)[e] = t6[e];
  });
  if (xnext_out || cost_out) {  // the knot's calc, fused (iteration 0 of a solve, or calc only)
    ex.run([&](int lane) {
      const double dt = b.dt;
      if (xnext_out && lane < nj && imp) {
        xnext_out[lane] = x[lane];
        xnext_out[nj + lane] = dtau[nj + lane];
      } else if (xnext_out && lane < nj) {
        const double ai = dtau[nj + lane];
        if (dt != 0.) {
          const double v = x[nj + lane];
          xnext_out[lane] = x[lane] + (v * dt + ai * dt * dt);
          xnext_out[nj + lane] = v + ai * dt;
        } else {
          xnext_out[lane] = x[lane];
          xnext_out[nj + lane] = x[nj + lane];
        }
      }
      if (cost_out && !Fx && lane == 0) {  // calc only (with derivatives: from the residuals below)
        double cc = cost_value(b, W, x, u, nx, nu);
        const double* cr = b.C;
        for (int k = 0; k < b.ncost; ++k) {
          const CRec C{cr};
          if (C.type() == C_CONTACT_FORCE && nc > 0) cc += C.weight() * force_cost_activation(C, lam, nx, nu);
          cr += C.size();
        }
        *cost_out = dt != 0. ? dt * cc : cc;
      }
    });
  }
  if (!Fx) return;  // calc only
  if (imp && nc > 0)  // joint-frame velocities at v+ (into fx, free after the RNEA); zv = v+
    ex.run([&](int lane) {
      if (lane >= nj) return;
      w_velocity(W, dtau + nj, lane);
      double m6[6], t6[6];
      for (int e = 0; e < 6; ++e) m6[e] = W.v(lane)[e];
      motion_act_inv(W.oR(lane), W.op(lane), m6, t6);
      for (int e = 0; e < 6; ++e) fx[6 * lane + e] = t6[e];
      zv[lane] = dtau[nj + lane];
    });
  // tangents (lanes < 2 nj; impulse: q directions only) and frame-cost residuals /
  // Jacobian columns (lanes < nj)
  ex.run([&](int lane) {
    if (lane < (imp ? nj : L)) {
      rnea_tangent(b, V, imp ? u : x + nj, lane < nj ? 0 : 1, lane % nj, T, L, lane, dtau);
      if (nc > 0 && imp) impulse_tangent(b, V, W, fx, zv, lane, L, lane, da0);
      else if (nc > 0) contact_tangent(b, V, W, lane < nj ? 0 : 1, lane % nj, T, L, lane, da0);
    }
    if (lane >= nj) return;
    const double* cr = b.C;
    int f = 0;
    for (int k = 0; k < b.ncost; ++k) {
      const CRec C{cr};
      if (C.type() == C_FRAME_PLACEMENT || C.type() == C_FRAME_TRANSLATION) {
        double r[6], Jc[6];
        const int nr = frame_residual(b, V, C, lane, r, Jc);
#pragma unroll
        for (int e = 0; e < 6; ++e)
          if (e < nr) {
            Jf[((int64_t)f * 6 + e) * nj + lane] = Jc[e];
            if (lane == 0) rf[6 * f + e] = r[e];
          }
        ++f;
      }
      cr += C.size();
    }
  });
  // d lambda / dx, d lambda / du for CostModelContactForce (contact-fwddyn.hxx:131-137, with
  // enable_force): Kinv bottom-left = H^T, bottom-right = -S^-1; dtau/du = [0; I]
  const bool fd = b.enable_force && nc > 0 && !imp;
  double* dfx = w + l.dfx;
  double* dfu = w + l.dfu;
  if (fd)
    ex.run([&](int lane) {
      const double* Sinv = Sx + (int64_t)nc * nc;
      for (int e = lane; e < nc * L; e += ex.nt) {
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
    });
  const double dt = b.dt, dt2 = dt * dt;
  const bool integ = dt != 0.;
  const double sc = integ ? dt : 1.;
  // Output blocks, entry by entry over all lanes (consecutive lanes write
  // consecutive addresses of the column-major blocks).
  ex.run([&](int lane) {
    // Fx(i, c): da/dx = -Minv dtau(:, c), Euler assembly (euler.hxx:100-112)
    for (int e = lane; e < n * n; e += ex.nt) {
      const int c = e / n, i = e % n, r = i < nj ? i : i - nj;
      double f;
      if (imp) {  // [[I, 0], [-G dtau_dq - H dv0_dq, G M = I - H Jc]] (impulse-fwddyn.hxx:111-115)
        if (i < nj) {
          f = c == i ? 1. : 0.;
        } else if (c < nj) {
          double s = 0.;
          for (int k = 0; k < nj; ++k) s += Minv[(int64_t)k * nj + r] * dtau[(int64_t)k * L + c];
          for (int k = 0; k < nc; ++k) s += H[(int64_t)k * nj + r] * da0[(int64_t)k * L + c];
          f = ok ? -s : NAN;
        } else {
          double s = 0.;
          for (int k = 0; k < nc; ++k) s += H[(int64_t)k * nj + r] * Jc[(int64_t)k * nj + (c - nj)];
          f = ok ? (c - nj == r ? 1. : 0.) - s : NAN;
        }
      } else if (integ) {
        double s = 0.;
        for (int k = 0; k < nj; ++k) s += Minv[(int64_t)k * nj + r] * dtau[(int64_t)k * L + c];
        for (int k = 0; k < nc; ++k) s += H[(int64_t)k * nj + r] * da0[(int64_t)k * L + c];
        const double da = ok ? -s : NAN;
        f = i < nj ? da * dt2 + (c == nj + i ? dt : 0.) + (c == i ? 1. : 0.) : da * dt + (c == i ? 1. : 0.);
      } else {
        f = c == i ? 1. : 0.;
      }
      Fx[e] = f;
    }
    // Fu(i, c) = Minv(i mod nj, nun + c) dt^2 | dt (dtau/du = [0; I]); Lxu = 0
    for (int e = lane; e < n * m; e += ex.nt) {
      const int c = e / n, i = e % n;
      double f = 0.;
      if (integ && c < nu) {
        const double mi = ok ? Minv[(int64_t)(b.nun + c) * nj + (i < nj ? i : i - nj)] : NAN;
        f = i < nj ? mi * dt2 : mi * dt;
      }
      Fu[e] = f;
      double lxu = 0.;  // only contact-force costs couple x and u
      if (fd && c < nu) {
        const double* cr = b.C;
        for (int k = 0; k < b.ncost; ++k) {
          const CRec C{cr};
          if (C.type() == C_CONTACT_FORCE) {
            const int row0 = (int)C.d()[0], nr = (int)C.d()[1];
            const double* wv = cost_weights(C, nx, nu);
            double s2 = 0.;
            for (int r = 0; r < nr; ++r)
              s2 += dfx[(int64_t)(row0 + r) * L + i] * wv[r] * dfu[(int64_t)(row0 + r) * nj + c];
            lxu += C.weight() * s2;
          }
          cr += C.size();
        }
      }
      Lxu[e] = sc * lxu;
    }
    // Lxx(i, j): Gauss-Newton, cost-sum.hxx:122-160
    for (int e = lane; e < n * n; e += ex.nt) {
      const int j = e / n, i = e % n;
      double l = 0.;
      const double* cr = b.C;
      int f = 0;
      for (int k = 0; k < b.ncost; ++k) {
        const CRec C{cr};
        const double wt = C.weight();
        const double* wv = cost_weights(C, nx, nu);
        if (C.type() == C_STATE) {
          if (i == j) l += wt * wv[j];
        } else if (C.type() == C_FRAME_PLACEMENT || C.type() == C_FRAME_TRANSLATION) {
          if (i < nj && j < nj) {
            const int nr = C.type() == C_FRAME_PLACEMENT ? 6 : 3;
            const double* Jk = Jf + (int64_t)f * 6 * nj;
            double s2 = 0.;
            for (int r = 0; r < nr; ++r) s2 += Jk[(int64_t)r * nj + i] * wv[r] * Jk[(int64_t)r * nj + j];
            l += wt * s2;
          }
          ++f;
        } else if (C.type() == C_CONTACT_FORCE && fd) {
          const int row0 = (int)C.d()[0], nr = (int)C.d()[1];
          double s2 = 0.;
          for (int r = 0; r < nr; ++r)
            s2 += dfx[(int64_t)(row0 + r) * L + i] * wv[r] * dfx[(int64_t)(row0 + r) * L + j];
          l += wt * s2;
        }
        cr += C.size();
      }
      Lxx[e] = integ ? sc * l : l;
    }
    // Luu (diagonal), Lu, Lx
    for (int e = lane; e < m * m; e += ex.nt) {
      const int j = e / m, i = e % m;
      double l = 0.;
      if (i < nu && j < nu) {
        const double* cr = b.C;
        for (int k = 0; k < b.ncost; ++k) {
          const CRec C{cr};
          if (C.type() == C_CONTROL && i == j) l += C.weight() * cost_weights(C, nx, nu)[j];
          if (C.type() == C_CONTACT_FORCE && fd) {
            const int row0 = (int)C.d()[0], nr = (int)C.d()[1];
            const double* wv = cost_weights(C, nx, nu);
            double s2 = 0.;
            for (int r = 0; r < nr; ++r)
              s2 += dfu[(int64_t)(row0 + r) * nj + i] * wv[r] * dfu[(int64_t)(row0 + r) * nj + j];
            l += C.weight() * s2;
          }
          cr += C.size();
        }
      }
      Luu[e] = integ ? sc * l : l;
    }
    if (lane < m) {
      const int j = lane;
      double lu = 0.;
      if (j < nu) {
        const double* cr = b.C;
        for (int k = 0; k < b.ncost; ++k) {
          const CRec C{cr};
          if (C.type() == C_CONTROL) lu += C.weight() * cost_weights(C, nx, nu)[j] * (u[j] - C.d()[j]);
          if (C.type() == C_CONTACT_FORCE && fd) {
            const int row0 = (int)C.d()[0], nr = (int)C.d()[1];
            const double* wv = cost_weights(C, nx, nu);
            for (int r = 0; r < nr; ++r)
              lu += C.weight() * dfu[(int64_t)(row0 + r) * nj + j] * wv[r] * (lam[row0 + r] - C.d()[2 + r]);
          }
          cr += C.size();
        }
      }
      Lu[j] = integ ? sc * lu : lu;
    }
    {
      const int j = lane;
      if (j < n) {
        double lx = 0.;
        const double* cr = b.C;
        int f = 0;
        for (int k = 0; k < b.ncost; ++k) {
          const CRec C{cr};
          const double wt = C.weight();
          const double* wv = cost_weights(C, nx, nu);
          if (C.type() == C_STATE) {
            lx += wt * wv[j] * (x[j] - C.d()[j]);
          } else if (C.type() == C_FRAME_PLACEMENT || C.type() == C_FRAME_TRANSLATION) {
            const int nr = C.type() == C_FRAME_PLACEMENT ? 6 : 3;
            if (j < nj) {
              const double* Jk = Jf + (int64_t)f * 6 * nj;
              for (int r = 0; r < nr; ++r) lx += wt * Jk[(int64_t)r * nj + j] * wv[r] * rf[6 * f + r];
            }
            ++f;
          } else if (C.type() == C_CONTACT_FORCE && fd) {
            const int row0 = (int)C.d()[0], nr = (int)C.d()[1];
            for (int r = 0; r < nr; ++r)
              lx += wt * dfx[(int64_t)(row0 + r) * L + j] * wv[r] * (lam[row0 + r] - C.d()[2 + r]);
          }
          cr += C.size();
        }
        Lx[j] = integ ? sc * lx : lx;
      }
    }
    // the fused calc's cost: frame residuals from the Jacobian phase (cost-sum.hxx:89-117)
    if (cost_out && lane == 0) {
      double total = 0.;
      const double* cr = b.C;
      int f = 0;
      for (int k = 0; k < b.ncost; ++k) {
        const CRec C{cr};
        const double* wv = cost_weights(C, nx, nu);
        double a = 0.;
        if (C.type() == C_STATE) {
          for (int i = 0; i < nx; ++i) a += wv[i] * (x[i] - C.d()[i]) * (x[i] - C.d()[i]);
        } else if (C.type() == C_CONTROL) {
          for (int i = 0; i < nu; ++i) a += wv[i] * (u[i] - C.d()[i]) * (u[i] - C.d()[i]);
        } else if (C.type() == C_CONTACT_FORCE) {
          if (nc > 0) a = 2. * force_cost_activation(C, lam, nx, nu);
        } else {
          const int nr = C.type() == C_FRAME_PLACEMENT ? 6 : 3;
          for (int i = 0; i < nr; ++i) a += wv[i] * rf[6 * f + i] * rf[6 * f + i];
          ++f;
        }
        total += C.weight() * (0.5 * a);
        cr += C.size();
      }
      *cost_out = integ ? dt * total : total;
    }
  });
}

__device__ inline void knot_calc_diff(const double* P, int nx, int m, const double* xg, const double* ug, bool use_u,
                                      double* w, double* Fx, double* Fu, double* Lxx, double* Lxu, double* Luu,
                                      double* Lx, double* Lu, double* xnext_out, double* cost_out) {
  knot_calc_diff_x(DevExec{64}, P, nx, m, xg, ug, use_u, w, Fx, Fu, Lxx, Lxu, Luu, Lx, Lu, xnext_out, cost_out);
}

}  // namespace mb
}  // namespace fddp
