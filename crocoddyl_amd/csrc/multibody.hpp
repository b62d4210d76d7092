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
//   * forward dynamics: a = (M + diag(armature))^-1 (tau - nle), M by the composite-
//     rigid-body algorithm (one column per lane, walking the ancestors), nle by a
//     recursive Newton-Euler value pass, the solve by Gauss-Jordan with one column
//     per lane. (The reference's default path is ABA, the same function.)
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
enum { C_STATE = 1, C_CONTROL = 2, C_FRAME_PLACEMENT = 3, C_FRAME_TRANSLATION = 4 };

struct Blk {
  double dt;
  int nj, ncost;
  const double* g;    // gravity (3)
  const double* arm;  // armature (nj)
  const double* J;    // joint records
  const double* C;    // cost records
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

// Recursive Newton-Euler value pass (one thread). Placements (liMi, oMi),
// velocities, accelerations (qdd == nullptr: zero) and the accumulated joint
// forces; tau = S^T F. With `composite`, also the composite inertia of every
// subtree (CRBA). rnea (Featherstone Table 5.1), crba (Table 6.2).
MB_HD inline void value_pass(const Blk& b, const double* q, const double* qd, const double* qdd, const Vals& V,
                                  double* tau, bool kin, bool composite) {
  const int nj = b.nj;
  for (int e = 0; e < 6; ++e) {
    V.root_v()[e] = 0.;
    V.root_a()[e] = e < 3 ? -b.g[e] : 0.;
  }
  for (int i = 0; i < nj; ++i) {
    const JRec J(b, i);
    const int lam = J.parent();
    const double* ax = J.axis();
    double* R = V.R(i);
    double* p = V.p(i);
    if (kin) {
      joint_rotation(J.Rpl(), ax, q[i], R);
      p[0] = J.ppl()[0];
      p[1] = J.ppl()[1];
      p[2] = J.ppl()[2];
      if (lam >= 0) {
        matmul3(V.oR(lam), R, V.oR(i));
        double t[3];
        matvec3(V.oR(lam), p, t);
        V.op(i)[0] = V.op(lam)[0] + t[0];
        V.op(i)[1] = V.op(lam)[1] + t[1];
        V.op(i)[2] = V.op(lam)[2] + t[2];
      } else {
        for (int e = 0; e < 9; ++e) V.oR(i)[e] = R[e];
        for (int e = 0; e < 3; ++e) V.op(i)[e] = p[e];
      }
    }
    const double* vp = lam >= 0 ? V.v(lam) : V.root_v();
    const double* ap = lam >= 0 ? V.a(lam) : V.root_a();
    double* v = V.v(i);
    double* a = V.a(i);
    const double w = qd[i];
    motion_act_inv(R, p, vp, v);
    v[3] += ax[0] * w;
    v[4] += ax[1] * w;
    v[5] += ax[2] * w;
    motion_act_inv(R, p, ap, a);
    const double qa = qdd ? qdd[i] : 0.;
    a[3] += ax[0] * qa;
    a[4] += ax[1] * qa;
    a[5] += ax[2] * qa;
    // + v x (S qd)
    const double sv[6] = {0., 0., 0., ax[0] * w, ax[1] * w, ax[2] * w};
    double t6[6];
    cross_m(v, sv, t6);
    for (int e = 0; e < 6; ++e) a[e] += t6[e];
    // f = I a + v x* (I v)
    double Iv[6], f[6];
    inertia_mul(J.mass(), J.com(), J.I6(), a, f);
    inertia_mul(J.mass(), J.com(), J.I6(), v, Iv);
    cross_f(v, Iv, t6);
    for (int e = 0; e < 6; ++e) V.F(i)[e] = f[e] + t6[e];
    if (composite) {
      *V.cm(i) = J.mass();
      for (int e = 0; e < 3; ++e) V.cc(i)[e] = J.com()[e];
      for (int e = 0; e < 6; ++e) V.cI(i)[e] = J.I6()[e];
    }
  }
  for (int i = nj - 1; i >= 0; --i) {
    const JRec J(b, i);
    const double* F = V.F(i);
    tau[i] = dot3(J.axis(), F + 3);
    const int lam = J.parent();
    if (lam < 0) continue;
    double t6[6];
    force_act(V.R(i), V.p(i), F, t6);
    for (int e = 0; e < 6; ++e) V.F(lam)[e] += t6[e];
    if (composite) {  // composite inertia of the subtree, carried to the parent and summed
      const double m1 = *V.cm(i), m0 = *V.cm(lam);
      const double* R = V.R(i);
      double c1[3], I1[9], tmp[9];
      matvec3(R, V.cc(i), c1);
      c1[0] += V.p(i)[0];
      c1[1] += V.p(i)[1];
      c1[2] += V.p(i)[2];
      const double* s = V.cI(i);
      const double Is[9] = {s[0], s[3], s[4], s[3], s[1], s[5], s[4], s[5], s[2]};
      matmul3(R, Is, tmp);
      // I1 = tmp R^T
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) I1[c * 3 + r] = tmp[r] * R[c] + tmp[3 + r] * R[3 + c] + tmp[6 + r] * R[6 + c];
      const double m = m0 + m1;
      if (m > 0.) {
        const double* c0 = V.cc(lam);
        const double cn[3] = {(m0 * c0[0] + m1 * c1[0]) / m, (m0 * c0[1] + m1 * c1[1]) / m,
                              (m0 * c0[2] + m1 * c1[2]) / m};
        const double d0[3] = {c0[0] - cn[0], c0[1] - cn[1], c0[2] - cn[2]};
        const double d1[3] = {c1[0] - cn[0], c1[1] - cn[1], c1[2] - cn[2]};
        const double q0 = dot3(d0, d0), q1 = dot3(d1, d1);
        double* o = V.cI(lam);
        // parallel-axis shift of both to the new CoM: I + m (|d|^2 I - d d^T)
        o[0] = o[0] + m0 * (q0 - d0[0] * d0[0]) + I1[0] + m1 * (q1 - d1[0] * d1[0]);
        o[1] = o[1] + m0 * (q0 - d0[1] * d0[1]) + I1[4] + m1 * (q1 - d1[1] * d1[1]);
        o[2] = o[2] + m0 * (q0 - d0[2] * d0[2]) + I1[8] + m1 * (q1 - d1[2] * d1[2]);
        o[3] = o[3] - m0 * d0[0] * d0[1] + I1[3] - m1 * d1[0] * d1[1];
        o[4] = o[4] - m0 * d0[0] * d0[2] + I1[6] - m1 * d1[0] * d1[2];
        o[5] = o[5] - m0 * d0[1] * d0[2] + I1[7] - m1 * d1[1] * d1[2];
        *V.cm(lam) = m;
        V.cc(lam)[0] = cn[0];
        V.cc(lam)[1] = cn[1];
        V.cc(lam)[2] = cn[2];
      }
    }
  }
}

// CRBA column j (thread j < nj): F = Ic_j S_j, M_jj = S_j^T F, then carried up
// the ancestors i: M_ij = M_ji = S_i^T F. A: column-major, ld = lda; the
// caller zeroes A first (entries of unrelated joints stay 0).
MB_HD inline void crba_column(const Blk& b, const Vals& V, int j, double* A, int lda) {
  const JRec Jj(b, j);
  const double S[6] = {0., 0., 0., Jj.axis()[0], Jj.axis()[1], Jj.axis()[2]};
  double F[6], t6[6];
  inertia_mul(*V.cm(j), V.cc(j), V.cI(j), S, F);
  A[(int64_t)j * lda + j] = dot3(Jj.axis(), F + 3) + b.arm[j];
  int i = j;
  while (true) {
    const int lam = JRec(b, i).parent();
    if (lam < 0) break;
    force_act(V.R(i), V.p(i), F, t6);
    for (int e = 0; e < 6; ++e) F[e] = t6[e];
    i = lam;
    const double Mij = dot3(JRec(b, i).axis(), F + 3);
    A[(int64_t)j * lda + i] = Mij;
    A[(int64_t)i * lda + j] = Mij;
  }
}

// Phase executor: run(f) calls f(lane) for every thread of the workgroup and
// then synchronises (device), or for lanes 0..nt-1 in order (host emulation,
// tests/test_multibody_host.py). Within one phase no lane reads what another
// lane writes, so both orders give the same result.
struct DevExec {
  int nt;
  template <class F>
  __device__ void run(F f) const {
    f((int)threadIdx.x);
    __syncthreads();
  }
};
struct HostExec {
  int nt;
  template <class F>
  void run(F f) const {
    for (int l = 0; l < nt; ++l) f(l);
  }
};

// Gauss-Jordan on the column-major nr x nc matrix A (ld nr) without pivoting
// (the left nr x nr block is SPD): one column per lane (lane < nc), one pivot
// per phase; the left block's pivot column is only read in its step. Returns
// false if a pivot is not positive.
template <class X>
MB_HD inline bool gauss_jordan(const X& ex, double* A, int nr, int nc, int* flag) {
  ex.run([&](int lane) {
    if (lane == 0) *flag = 0;
  });
  for (int k = 0; k < nr; ++k) {
    ex.run([&](int lane) {
      const double piv = A[(int64_t)k * nr + k];
      if (!(piv > 0.)) {
        if (lane == 0) *flag = 1;
      } else if (lane < nc && lane > k) {
        double* col = A + (int64_t)lane * nr;
        const double* pc = A + (int64_t)k * nr;
        const double akc = col[k] / piv;
        for (int r = 0; r < nr; ++r)
          if (r != k) col[r] -= pc[r] * akc;
        col[k] = akc;
      }
    });
  }
  return *flag == 0;
}

// ---- dual numbers for the log6 Jacobian -----------------------------------
struct Dual {
  double v, d;
};
MB_HD __forceinline__ Dual operator+(Dual a, Dual b) { return {a.v + b.v, a.d + b.d}; }
MB_HD __forceinline__ Dual operator-(Dual a, Dual b) { return {a.v - b.v, a.d - b.d}; }
MB_HD __forceinline__ Dual operator*(Dual a, Dual b) { return {a.v * b.v, a.d * b.v + a.v * b.d}; }
MB_HD __forceinline__ Dual operator*(double s, Dual a) { return {s * a.v, s * a.d}; }
MB_HD __forceinline__ Dual operator/(Dual a, Dual b) { return {a.v / b.v, (a.d * b.v - a.v * b.d) / (b.v * b.v)}; }
MB_HD __forceinline__ Dual dsqrt(Dual a) {
  const double s = sqrt(a.v);
  return {s, a.d / (2. * s)};
}
MB_HD __forceinline__ Dual dasin(Dual a) { return {asin(a.v), a.d / sqrt(1. - a.v * a.v)}; }
MB_HD __forceinline__ Dual dacos(Dual a) { return {acos(a.v), -a.d / sqrt(1. - a.v * a.v)}; }
MB_HD __forceinline__ Dual dsin(Dual a) { return {sin(a.v), a.d * cos(a.v)}; }
MB_HD __forceinline__ Dual dcos(Dual a) { return {cos(a.v), -a.d * sin(a.v)}; }

// log6(R, p) -> (lin, ang) (pinocchio::log6), R column-major; in dual numbers
// so that the tangent along (dR, dp) is Jlog6 * xi. Same branches as
// oracle/multibody_np.py:log3/log6.
MB_HD inline void log6_dual(const Dual* R, const Dual* p, Dual* out) {
  auto at = [&](int r, int c) { return R[c * 3 + r]; };
  const Dual tr = at(0, 0) + at(1, 1) + at(2, 2);
  const Dual c = 0.5 * (tr - Dual{1., 0.});
  Dual w[3] = {at(2, 1) - at(1, 2), at(0, 2) - at(2, 0), at(1, 0) - at(0, 1)};
  const Dual s2 = 0.25 * (w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  Dual om[3];
  if (s2.v < 1e-8 && c.v > 0.) {
    const Dual k = 0.5 * (Dual{1., 0.} + (1. / 6.) * s2 + (3. / 40.) * (s2 * s2) + (5. / 112.) * (s2 * s2 * s2));
    for (int e = 0; e < 3; ++e) om[e] = k * w[e];
  } else if (s2.v < 1e-8) {  // theta near pi: axis from the symmetric part (value only)
    // (explicit selects: no runtime-indexed arrays, which would live in scratch)
    const double cv = c.v < -1. ? -1. : c.v;
    const double th = acos(cv);
    auto axc = [&](double d) {
      const double t = (d - cv) / (1. - cv);
      return t > 0. ? sqrt(t) : 0.;
    };
    const double a0 = axc(at(0, 0).v), a1 = axc(at(1, 1).v), a2 = axc(at(2, 2).v);
    const int i0 = (a1 > a0) ? ((a2 > a1) ? 2 : 1) : ((a2 > a0) ? 2 : 0);
    const double s01 = at(0, 1).v + at(1, 0).v, s02 = at(0, 2).v + at(2, 0).v, s12 = at(1, 2).v + at(2, 1).v;
    auto sgn = [](double v) { return v >= 0. ? 1. : -1.; };
    const double g0 = i0 == 0 ? 1. : (i0 == 1 ? sgn(s01) : sgn(s02));
    const double g1 = i0 == 1 ? 1. : (i0 == 0 ? sgn(s01) : sgn(s12));
    const double g2 = i0 == 2 ? 1. : (i0 == 0 ? sgn(s02) : sgn(s12));
    const double wi = i0 == 0 ? w[0].v : (i0 == 1 ? w[1].v : w[2].v);
    const double flip = wi < 0. ? -th : th;
    om[0] = Dual{flip * g0 * a0, 0.};
    om[1] = Dual{flip * g1 * a1, 0.};
    om[2] = Dual{flip * g2 * a2, 0.};
  } else {
    const Dual s = dsqrt(s2);
    Dual th;
    if (c.v > 0.5)
      th = dasin(s);
    else if (c.v < -0.5)
      th = Dual{M_PI, 0.} - dasin(s);
    else
      th = dacos(c);
    const Dual k = th / (2. * s);
    for (int e = 0; e < 3; ++e) om[e] = k * w[e];
  }
  const Dual t2 = om[0] * om[0] + om[1] * om[1] + om[2] * om[2];
  Dual beta;
  if (t2.v < 1e-2) {
    beta = Dual{1. / 12., 0.} + (1. / 720.) * t2 + (1. / 30240.) * (t2 * t2) + (1. / 1209600.) * (t2 * t2 * t2);
  } else {
    const Dual t = dsqrt(t2);
    beta = Dual{1., 0.} / t2 - dsin(t) / (2. * t * (Dual{1., 0.} - dcos(t)));
  }
  // v = (I - 0.5 [w]x + beta [w]x^2) p ; [w]x^2 p = w (w.p) - |w|^2 p
  const Dual wp = om[0] * p[0] + om[1] * p[1] + om[2] * p[2];
  const Dual wxp[3] = {om[1] * p[2] - om[2] * p[1], om[2] * p[0] - om[0] * p[2], om[0] * p[1] - om[1] * p[0]};
  for (int e = 0; e < 3; ++e) {
    const Dual w2p = om[e] * wp - t2 * p[e];
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

// oMf of a frame record d = [joint, R 9, p 3, ...]
MB_HD inline void frame_placement(const Vals& V, const double* d, double* R, double* p) {
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
  if (C.type() == C_FRAME_TRANSLATION) {
    const double* pref = d + 13;
    for (int e = 0; e < 3; ++e) {
      r[e] = pf[e] - pref[e];
      if (Jc) Jc[e] = dp[e];
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
  log6_dual(RD, PD, o);
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
  return t == C_STATE ? nx : (t == C_CONTROL ? nu : (t == C_FRAME_PLACEMENT ? 6 : 3));
}
MB_HD inline const double* cost_weights(const CRec& C, int nx, int nu) { return C.r + C.size() - cost_nr(C, nx, nu); }

// Cost value of the DAM (one thread; kinematics in V): sum of weight * 0.5 r^T W r
// in record (name) order (cost-sum.hxx:89-117).
MB_HD inline double cost_value(const Blk& b, const Vals& V, const double* x, const double* u, int nx, int nu) {
  double total = 0.;
  const double* cr = b.C;
  for (int k = 0; k < b.ncost; ++k) {
    const CRec C{cr};
    const double* w = cost_weights(C, nx, nu);
    double a = 0.;
    if (C.type() == C_STATE) {
      const double* xr = C.d();
      for (int i = 0; i < nx; ++i) {
        const double r = x[i] - xr[i];
        a += w[i] * r * r;
      }
    } else if (C.type() == C_CONTROL) {
      const double* ur = C.d();
      for (int i = 0; i < nu; ++i) {
        const double r = u[i] - ur[i];
        a += w[i] * r * r;
      }
    } else {
      double r[6];
      const int nr = frame_residual(b, V, C, -1, r, nullptr);
      for (int i = 0; i < nr; ++i) a += w[i] * r[i] * r[i];
    }
    total += C.weight() * (0.5 * a);
    cr += C.size();
  }
  return total;
}

// LDS (doubles) of the calc scratch for nj joints: values + [M | b] + small.
__host__ __device__ inline int64_t calc_work_doubles(int nj) {
  return (int64_t)kValsPerJoint * nj + 12 + (int64_t)nj * (nj + 1) + 4 * nj + 8;
}

// model->calc(data, x, u) for the Euler∘FreeFwdDynamics knot (euler.hxx:41-80,
// free-fwddyn.hxx:44-79). Lanes < 64 do the work; every thread of the
// workgroup must call (phases end in barriers). x, u readable by all lanes;
// writes xnext[0..nx) and returns the knot cost. `w`: calc_work_doubles(nj).
template <class X>
MB_HD inline double knot_calc_x(const X& ex, const double* P, int nx, const double* x, const double* u, bool use_u,
                                double* xnext, double* w) {
  const Blk b = parse(P);
  const int nj = b.nj;
  const Vals V{w, nj};
  double* A = w + (int64_t)kValsPerJoint * nj + 12;  // nj x (nj + 1), ld nj
  double* tau = A + (int64_t)nj * (nj + 1);          // nle
  double* ub = tau + nj;                              // u (zero if !use_u)
  double* red = ub + nj;
  int* flag = (int*)(red + 2 * nj + 4);
  ex.run([&](int lane) {
    if (lane < nj) ub[lane] = use_u ? u[lane] : 0.;
    for (int e = lane; e < nj * (nj + 1); e += ex.nt) A[e] = 0.;
    if (lane == 0) value_pass(b, x, x + nj, nullptr, V, tau, true, true);
  });
  ex.run([&](int lane) {
    if (lane < nj) crba_column(b, V, lane, A, nj);
    if (lane == 0) red[0] = cost_value(b, V, x, ub, nx, nj);
    if (lane < nj) A[(int64_t)nj * nj + lane] = ub[lane] - tau[lane];
  });
  const bool ok = gauss_jordan(ex, A, nj, nj + 1, flag);
  const double cc = red[0];
  const double dt = b.dt;
  const double* a = A + (int64_t)nj * nj;
  ex.run([&](int i) {
    if (i >= nj) return;
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
  return knot_calc_x(DevExec{NT}, P, nx, x, u, use_u, xnext, w);
}

// ---------------------------------------------------------------------------
// calcDiff: one 64-thread workgroup per (element, knot).
// ---------------------------------------------------------------------------
struct DiffLayout {
  int64_t vals, A, tang, dtau, J, xu, red, total;
};
__host__ __device__ inline DiffLayout diff_layout(int nj, int nframe) {
  const int L = 2 * nj;
  DiffLayout l;
  l.vals = 0;
  l.A = l.vals + (int64_t)kValsPerJoint * nj + 12;
  l.tang = l.A + (int64_t)nj * 2 * nj;          // [M | I] -> [. | Minv]
  l.dtau = l.tang + (int64_t)18 * nj * L;       // per lane: dv, da, df per joint, [i][c][L]
  l.J = l.dtau + ((int64_t)nj * L > 3 * nj ? (int64_t)nj * L : 3 * nj);  // dtau [i][L] (nle, a first)
  l.xu = l.J + (int64_t)6 * nj * (nframe > 0 ? nframe : 1);  // frame-cost Jacobians [cost][6][nj] + residuals
  l.red = l.xu + 3 * nj + 6 * kMaxFrameCosts + 8;  // x (2nj), u (nj), frame residuals
  l.total = l.red + 8;  // red: flag
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

// model->calcDiff for one knot by one 64-thread workgroup (euler.hxx:83-131,
// free-fwddyn.hxx:82-118, cost-sum.hxx:122-160). Writes full blocks (entries
// beyond nu zero); Lxu is zero (no cost couples x and u). A mass matrix that is
// not positive definite leaves NaN in Fx/Fu, which the backward pass reports
// as backward_error. `w`: diff_layout(nj, nframe).total doubles of LDS.
template <class X>
MB_HD inline void knot_calc_diff_x(const X& ex, const double* P, int nx, int m, const double* xg, const double* ug,
                                   bool use_u, double* w, double* Fx, double* Fu, double* Lxx, double* Lxu,
                                   double* Luu, double* Lx, double* Lu) {
  const Blk b = parse(P);
  const int nj = b.nj, n = nx, L = 2 * nj;
  int nframe = 0;
  {
    const double* cr = b.C;
    for (int k = 0; k < b.ncost; ++k) {
      const CRec C{cr};
      if (C.type() == C_FRAME_PLACEMENT || C.type() == C_FRAME_TRANSLATION) ++nframe;
      cr += C.size();
    }
  }
  const DiffLayout l = diff_layout(nj, nframe);
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
  ex.run([&](int lane) {
    if (lane < nx) x[lane] = xg[lane];
    if (lane < nj) u[lane] = use_u ? ug[lane] : 0.;
    for (int e = lane; e < 2 * nj * nj; e += ex.nt) {
      const int c = e / nj, r = e % nj;
      A[e] = (c == nj + r) ? 1. : 0.;
    }
  });
  // nle -> dtau[0..nj), composite inertias and placements
  ex.run([&](int lane) {
    if (lane == 0) value_pass(b, x, x + nj, nullptr, V, dtau, true, true);
  });
  ex.run([&](int lane) {
    if (lane < nj) crba_column(b, V, lane, A, nj);
  });
  const bool ok = gauss_jordan(ex, A, nj, 2 * nj, flag);
  const double* Minv = A + (int64_t)nj * nj;  // column-major nj x nj
  // a = (M + A)^-1 (tau - nle) -> dtau[nj..2nj)
  ex.run([&](int lane) {
    if (lane >= nj) return;
    double s = 0.;
    for (int k = 0; k < nj; ++k) s += Minv[(int64_t)k * nj + lane] * (u[k] - dtau[k]);
    dtau[nj + lane] = ok ? s : NAN;
  });
  // accelerations and forces at the solved a (the linearisation point of
  // computeABADerivatives); tau lands in red-free scratch dtau[2nj..3nj)
  ex.run([&](int lane) {
    if (lane == 0) value_pass(b, x, x + nj, dtau + nj, V, dtau + 2 * nj, false, false);
  });
  // tangents (lanes < 2 nj) and frame-cost residuals / Jacobian columns (lanes < nj)
  ex.run([&](int lane) {
    if (lane < L) rnea_tangent(b, V, x + nj, lane < nj ? 0 : 1, lane % nj, T, L, lane, dtau);
    if (lane >= nj) return;
    const double* cr = b.C;
    int f = 0;
    for (int k = 0; k < b.ncost; ++k) {
      const CRec C{cr};
      if (C.type() == C_FRAME_PLACEMENT || C.type() == C_FRAME_TRANSLATION) {
        double r[6], Jc[6];
        const int nr = frame_residual(b, V, C, lane, r, Jc);
        for (int e = 0; e < nr; ++e) Jf[((int64_t)f * 6 + e) * nj + lane] = Jc[e];
        if (lane == 0)
          for (int e = 0; e < nr; ++e) rf[6 * f + e] = r[e];
        ++f;
      }
      cr += C.size();
    }
  });
  const double dt = b.dt, dt2 = dt * dt;
  const bool integ = dt != 0.;
  const double sc = integ ? dt : 1.;
  ex.run([&](int lane) {
    // Fx column `lane` (< n): da/dx = -Minv dtau(:, lane)
    if (lane < n) {
      double* col = Fx + (int64_t)lane * n;
      for (int i = 0; i < nj; ++i) {
        double s = 0.;
        for (int k = 0; k < nj; ++k) s += Minv[(int64_t)k * nj + i] * dtau[(int64_t)k * L + lane];
        const double da = ok ? -s : NAN;
        double top, bot;
        if (integ) {
          top = da * dt2 + (lane == nj + i ? dt : 0.) + (lane == i ? 1. : 0.);
          bot = da * dt + (lane == nj + i ? 1. : 0.);
        } else {
          top = lane == i ? 1. : 0.;
          bot = lane == nj + i ? 1. : 0.;
        }
        col[i] = top;
        col[nj + i] = bot;
      }
    }
    // Fu column `lane` (< m): Minv(:, lane) (ActuationModelFull: dtau/du = I)
    if (lane < m) {
      double* col = Fu + (int64_t)lane * n;
      for (int i = 0; i < n; ++i) {
        double f = 0.;
        if (integ && lane < nj) {
          const double mi = ok ? Minv[(int64_t)lane * nj + (i < nj ? i : i - nj)] : NAN;
          f = i < nj ? mi * dt2 : mi * dt;
        }
        col[i] = f;
      }
    }
    // cost derivatives (Gauss-Newton): Lx[lane], Lxx column `lane`
    if (lane < n) {
      const int j = lane;
      double lx = 0.;
      double* col = Lxx + (int64_t)j * n;
      for (int i = 0; i < n; ++i) col[i] = 0.;
      const double* cr = b.C;
      int f = 0;
      for (int k = 0; k < b.ncost; ++k) {
        const CRec C{cr};
        const double wt = C.weight();
        const double* wv = cost_weights(C, nx, nj);
        if (C.type() == C_STATE) {
          lx += wt * wv[j] * (x[j] - C.d()[j]);
          col[j] += wt * wv[j];
        } else if (C.type() == C_FRAME_PLACEMENT || C.type() == C_FRAME_TRANSLATION) {
          const int nr = C.type() == C_FRAME_PLACEMENT ? 6 : 3;
          if (j < nj) {
            const double* Jk = Jf + (int64_t)f * 6 * nj;
            for (int r = 0; r < nr; ++r) lx += wt * Jk[(int64_t)r * nj + j] * wv[r] * rf[6 * f + r];
            for (int i = 0; i < nj; ++i) {
              double s = 0.;
              for (int r = 0; r < nr; ++r) s += Jk[(int64_t)r * nj + i] * wv[r] * Jk[(int64_t)r * nj + j];
              col[i] += wt * s;
            }
          }
          ++f;
        }
        cr += C.size();
      }
      Lx[j] = integ ? sc * lx : lx;
      if (integ)
        for (int i = 0; i < n; ++i) col[i] *= sc;
    }
    // Lu[lane], Luu / Lxu columns `lane` (< m)
    if (lane < m) {
      const int j = lane;
      double lu = 0., luu = 0.;
      if (j < nj) {
        const double* cr = b.C;
        for (int k = 0; k < b.ncost; ++k) {
          const CRec C{cr};
          if (C.type() == C_CONTROL) {
            const double* wv = cost_weights(C, nx, nj);
            lu += C.weight() * wv[j] * (u[j] - C.d()[j]);
            luu += C.weight() * wv[j];
          }
          cr += C.size();
        }
      }
      Lu[j] = integ ? sc * lu : lu;
      double* col = Luu + (int64_t)j * m;
      for (int i = 0; i < m; ++i) col[i] = (i == j) ? (integ ? sc * luu : luu) : 0.;
      double* cx = Lxu + (int64_t)j * n;
      for (int i = 0; i < n; ++i) cx[i] = 0.;
    }
  });
}

__device__ inline void knot_calc_diff(const double* P, int nx, int m, const double* xg, const double* ug, bool use_u,
                                      double* w, double* Fx, double* Fu, double* Lxx, double* Lxu, double* Luu,
                                      double* Lx, double* Lu) {
  knot_calc_diff_x(DevExec{64}, P, nx, m, xg, ug, use_u, w, Fx, Fu, Lxx, Lxu, Luu, Lx, Lu);
}

}  // namespace mb
}  // namespace fddp
