// ORACLE — TEST INFRASTRUCTURE ONLY. C++ restatement of the multibody knots on a
// kinematic tree whose root may be a free-flyer (FDDP_KNOT_EULER_FREEFWD /
// _CONTACTFWD blocks, layout in include/fddp_hip.h), for the CPU baseline of the
// legged-robot configs and as a CPU cross-check of oracle/multibody_np.py:
//   StateMultibody                    multibody/states/multibody.hxx:54-240
//     (pinocchio integrate / difference on SE(3) x R^n, dIntegrate = Jexp6 /
//      Ad(exp6^-1), dDifference = Jlog6, restated)
//   IntegratedActionModelEuler        core/integrator/euler.hxx:41-131
//   ∘ DifferentialActionModelFreeFwdDynamics   multibody/actions/free-fwddyn.hxx:44-118
//   ∘ DifferentialActionModelContactFwdDynamics multibody/actions/contact-fwddyn.hxx:59-160
//     (ActuationModelFloatingBase / Full, ContactModel3D / 6D, LOCAL frame)
//   CostModelSum of State / Control / FramePlacement / FrameTranslation /
//     FrameVelocity / CoMPosition / ContactForce / ContactFrictionCone costs with
//     Quad / WeightedQuad / QuadraticBarrier / WeightedQuadraticBarrier activations
//     (cost-sum.hxx:89-160, multibody/costs/*.hxx, core/activations/*.hpp)
// The rigid-body algorithms (Pinocchio, absent offline) are restated in joint
// frames with multi-dof joints (Featherstone 2008): RNEA (Table 5.1), CRBA
// (Table 6.2) with a Cholesky inverse (pinocchio::forwardDynamics's KKT path),
// and the RNEA derivatives by the linearised recursion along each tangent
// direction (what computeRNEADerivatives returns). Parity is pinned as described in
// oracle/multibody_np.py (tests/test_floating_oracle.py: this port vs that oracle).
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>

#include "multibody_oracle.hpp"

namespace fbo {

using mbo::act_force;
using mbo::act_inv;
using mbo::cr;
using mbo::crf;
using mbo::crm;
using mbo::Dl;
using mbo::inertia6;
using mbo::m6v;
using mbo::mm;
using mbo::mtv;
using mbo::mv;

constexpr int kMaxV = 64;   // dofs
constexpr int kMaxB = 64;   // joints
constexpr int kMaxC = 24;   // contact rows
constexpr int kMaxRows = 96;  // cost residual rows with dense Jacobians
constexpr int kJRec = 27;
enum { J_REVOLUTE = 0, J_FREEFLYER = 1 };
enum {
  C_STATE = 1, C_CONTROL = 2, C_FRAME_PLACEMENT = 3, C_FRAME_TRANSLATION = 4, C_CONTACT_3D = 5, C_CONTACT_6D = 6,
  C_CONTACT_FORCE = 7, C_COM_POSITION = 8, C_FRICTION_CONE = 9, C_FRAME_VELOCITY = 10
};

// ---- SO(3) / SE(3) helpers ---------------------------------------------------
inline void quat_to_R(const double* qv, double* R) {  // Eigen toRotationMatrix, (x y z w), column-major
  const double x = qv[0], y = qv[1], z = qv[2], w = qv[3];
  const double tx = 2 * x, ty = 2 * y, tz = 2 * z, twx = tx * w, twy = ty * w, twz = tz * w;
  const double txx = tx * x, txy = ty * x, txz = tz * x, tyy = ty * y, tyz = tz * y, tzz = tz * z;
  R[0] = 1 - (tyy + tzz), R[3] = txy - twz, R[6] = txz + twy;
  R[1] = txy + twz, R[4] = 1 - (txx + tzz), R[7] = tyz - twx;
  R[2] = txz - twy, R[5] = tyz + twx, R[8] = 1 - (txx + tyy);
}
inline void R_to_quat(const double* R, double* q) {  // Eigen quaternionbase_assign_impl
  auto at = [&](int r, int c) { return R[c * 3 + r]; };
  const double t = at(0, 0) + at(1, 1) + at(2, 2);
  if (t > 0) {
    double s = std::sqrt(t + 1.0);
    q[3] = 0.5 * s;
    s = 0.5 / s;
    q[0] = (at(2, 1) - at(1, 2)) * s;
    q[1] = (at(0, 2) - at(2, 0)) * s;
    q[2] = (at(1, 0) - at(0, 1)) * s;
  } else {
    int i = 0;
    if (at(1, 1) > at(0, 0)) i = 1;
    if (at(2, 2) > at(i, i)) i = 2;
    const int j = (i + 1) % 3, k = (i + 2) % 3;
    double s = std::sqrt(at(i, i) - at(j, j) - at(k, k) + 1.0);
    q[i] = 0.5 * s;
    s = 0.5 / s;
    q[3] = (at(k, j) - at(j, k)) * s;
    q[j] = (at(j, i) + at(i, j)) * s;
    q[k] = (at(k, i) + at(i, k)) * s;
  }
}
// exp6 of (lin, ang) -> (R, p); Taylor branch for t^2 < 1e-8 (multibody_np.exp6)
template <class T>
void exp6(const T* nu, T* R, T* p) {
  using std::cos;
  using std::sin;
  using std::sqrt;
  const T* v = nu;
  const T* w = nu + 3;
  const T t2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  T ct, st_t, a_wxv, a_w;
  if (mbo::val(t2) < 1e-8) {
    ct = T(1.) - t2 * T(0.5) + t2 * t2 * T(1. / 24.);
    st_t = T(1.) - t2 * T(1. / 6.) + t2 * t2 * T(1. / 120.);
    a_wxv = T(0.5) - t2 * T(1. / 24.) + t2 * t2 * T(1. / 720.);
    a_w = T(1. / 6.) - t2 * T(1. / 120.) + t2 * t2 * T(1. / 5040.);
  } else {
    const T t = sqrt(t2);
    ct = cos(t);
    st_t = sin(t) / t;
    a_wxv = (T(1.) - ct) / t2;
    a_w = (T(1.) - st_t) / t2;
  }
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) R[c * 3 + r] = (r == c ? ct : T(0.)) + a_wxv * w[r] * w[c];
  // + st_t [w]x
  R[1] = R[1] + st_t * w[2], R[2] = R[2] - st_t * w[1];
  R[3] = R[3] - st_t * w[2], R[5] = R[5] + st_t * w[0];
  R[6] = R[6] + st_t * w[1], R[7] = R[7] - st_t * w[0];
  const T wv = w[0] * v[0] + w[1] * v[1] + w[2] * v[2];
  const T wxv[3] = {w[1] * v[2] - w[2] * v[1], w[2] * v[0] - w[0] * v[2], w[0] * v[1] - w[1] * v[0]};
  for (int e = 0; e < 3; ++e) p[e] = st_t * v[e] + a_w * wv * w[e] + a_wxv * wxv[e];
}

// ---- robot -------------------------------------------------------------------
struct Robot {
  int nv = 0, nq = 0, nb = 0;
  bool ff = false;
  double g[3];
  const double* arm = nullptr;
  int parent[kMaxB], iv[kMaxB], iq[kMaxB], nvj[kMaxB], type[kMaxB];
  uint64_t anc[kMaxB];  // ancestor-or-self joints (bit per joint)
  const double* rec[kMaxB];
  double I6[kMaxB][36];
  int joint_of[kMaxV];
  void parse(const double* body, int nv_) {
    nv = nv_;
    for (int e = 0; e < 3; ++e) g[e] = body[e];
    arm = body + 3;
    const double* J = arm + nv;
    ff = (int)J[0] == J_FREEFLYER;
    nb = ff ? nv - 5 : nv;
    int v = 0, q = 0;
    for (int i = 0; i < nb; ++i) {
      rec[i] = J + (size_t)kJRec * i;
      type[i] = (int)rec[i][0];
      parent[i] = (int)rec[i][1];
      nvj[i] = type[i] == J_FREEFLYER ? 6 : 1;
      iv[i] = v;
      iq[i] = q;
      for (int k = 0; k < nvj[i]; ++k) joint_of[v + k] = i;
      v += nvj[i];
      q += type[i] == J_FREEFLYER ? 7 : 1;
      anc[i] = (parent[i] >= 0 ? anc[parent[i]] : 0) | (uint64_t(1) << i);
      inertia6(rec[i][17], rec[i] + 18, rec[i] + 21, I6[i]);
    }
    nq = q;
  }
  // column k of the joint-frame motion subspace of joint i
  void S(int i, int k, double* o) const {
    for (int e = 0; e < 6; ++e) o[e] = 0.;
    if (type[i] == J_FREEFLYER)
      o[k] = 1.;
    else
      for (int e = 0; e < 3; ++e) o[3 + e] = rec[i][2 + e];
  }
  // joint velocity S qd_seg (joint frame)
  void vj(int i, const double* qd, double* o) const {
    if (type[i] == J_FREEFLYER) {
      for (int e = 0; e < 6; ++e) o[e] = qd[iv[i] + e];
    } else {
      for (int e = 0; e < 3; ++e) o[e] = 0., o[3 + e] = rec[i][2 + e] * qd[iv[i]];
    }
  }
  void liMi(const double* q, int i, double* R, double* p) const {
    const double* Rpl = rec[i] + 5;
    const double* ppl = rec[i] + 14;
    if (type[i] == J_FREEFLYER) {
      double Rq[9], t[3];
      quat_to_R(q + iq[i] + 3, Rq);
      mm(Rpl, Rq, R);
      mv(Rpl, q + iq[i], t);
      for (int e = 0; e < 3; ++e) p[e] = ppl[e] + t[e];
    } else {
      const double* ax = rec[i] + 2;
      const double qi = q[iq[i]];
      const double s = std::sin(qi), c = std::cos(qi), oc = 1. - c;
      const double Rj[9] = {c + oc * ax[0] * ax[0],         oc * ax[1] * ax[0] + s * ax[2], oc * ax[2] * ax[0] - s * ax[1],
                            oc * ax[0] * ax[1] - s * ax[2], c + oc * ax[1] * ax[1],         oc * ax[2] * ax[1] + s * ax[0],
                            oc * ax[0] * ax[2] + s * ax[1], oc * ax[1] * ax[2] - s * ax[0], c + oc * ax[2] * ax[2]};
      mm(Rpl, Rj, R);
      for (int e = 0; e < 3; ++e) p[e] = ppl[e];
    }
  }
  bool moves(int dof, int joint) const { return (anc[joint] >> joint_of[dof]) & 1u; }
};

struct Kin {
  double R[kMaxB][9], p[kMaxB][3], oR[kMaxB][9], op[kMaxB][3];
};
inline void kinematics(const Robot& rb, const double* q, Kin& K) {
  for (int i = 0; i < rb.nb; ++i) {
    rb.liMi(q, i, K.R[i], K.p[i]);
    const int l = rb.parent[i];
    if (l >= 0) {
      double t[3];
      mm(K.oR[l], K.R[i], K.oR[i]);
      mv(K.oR[l], K.p[i], t);
      for (int e = 0; e < 3; ++e) K.op[i][e] = K.op[l][e] + t[e];
    } else {
      std::memcpy(K.oR[i], K.R[i], sizeof(K.R[i]));
      std::memcpy(K.op[i], K.p[i], sizeof(K.p[i]));
    }
  }
}
// world motion (at the origin) of dof d
inline void world_S(const Robot& rb, const Kin& K, int d, double* o) {
  const int i = rb.joint_of[d];
  double Sl[6], w[3], vl[3];
  rb.S(i, d - rb.iv[i], Sl);
  mv(K.oR[i], Sl + 3, w);
  mv(K.oR[i], Sl, vl);
  double t[3];
  cr(K.op[i], w, t);  // velocity of the origin: v + w x (0 - op) = v + op x w
  for (int e = 0; e < 3; ++e) o[e] = vl[e] + t[e], o[3 + e] = w[e];
}

// ---- RNEA (joint frames) -------------------------------------------------------
struct Rnea {
  double v[kMaxB][6], a[kMaxB][6], F[kMaxB][6], h[kMaxB][6];  // h = I v (body momentum)
};
inline void rnea(const Robot& rb, const Kin& K, const double* qd, const double* qdd, Rnea& Rv, double* tau,
                 const double* fext = nullptr, const double* grav = nullptr) {
  const double* g = grav ? grav : rb.g;
  const double a0[6] = {-g[0], -g[1], -g[2], 0., 0., 0.}, z6[6] = {0., 0., 0., 0., 0., 0.};
  for (int i = 0; i < rb.nb; ++i) {
    const int l = rb.parent[i];
    act_inv(K.R[i], K.p[i], l >= 0 ? Rv.v[l] : z6, Rv.v[i]);
    act_inv(K.R[i], K.p[i], l >= 0 ? Rv.a[l] : a0, Rv.a[i]);
    double VJ[6], AJ[6], t6[6];
    rb.vj(i, qd, VJ);
    rb.vj(i, qdd, AJ);
    for (int e = 0; e < 6; ++e) Rv.v[i][e] += VJ[e];
    crm(Rv.v[i], VJ, t6);
    for (int e = 0; e < 6; ++e) Rv.a[i][e] += AJ[e] + t6[e];
    double Ia[6];
    double* Iv = Rv.h[i];
    m6v(rb.I6[i], Rv.a[i], Ia);
    m6v(rb.I6[i], Rv.v[i], Iv);
    crf(Rv.v[i], Iv, t6);
    for (int e = 0; e < 6; ++e) Rv.F[i][e] = Ia[e] + t6[e] - (fext ? fext[6 * i + e] : 0.);
  }
  for (int i = rb.nb - 1; i >= 0; --i) {
    for (int k = 0; k < rb.nvj[i]; ++k) {
      double S[6];
      rb.S(i, k, S);
      double s = 0.;
      for (int e = 0; e < 6; ++e) s += S[e] * Rv.F[i][e];
      tau[rb.iv[i] + k] = s;
    }
    const int l = rb.parent[i];
    if (l < 0) continue;
    double t6[6];
    act_force(K.R[i], K.p[i], Rv.F[i], t6);
    for (int e = 0; e < 6; ++e) Rv.F[l][e] += t6[e];
  }
}
// d RNEA / d q_d (dir 0) or d qd_d (dir 1) at Rv; tv / ta: the joint-frame velocity /
// acceleration tangents (6 per joint). grav: the gravity of Rv's recursion.
inline void rnea_dir(const Robot& rb, const Kin& K, const Rnea& Rv, const double* qd, int dir, int d, double* dtau,
                     double* tv, double* ta, const double* grav = nullptr) {
  const double* g = grav ? grav : rb.g;
  const double a0[6] = {-g[0], -g[1], -g[2], 0., 0., 0.}, z6[6] = {0., 0., 0., 0., 0., 0.};
  const int j = rb.joint_of[d];
  double Sd[6];
  rb.S(j, d - rb.iv[j], Sd);
  // only the subtree of joint j moves along the direction: the tangents vanish
  // elsewhere, and the backward pass touches the subtree and j's ancestors only
  double dF[kMaxB][6];
  bool nz[kMaxB];
  for (int i = 0; i < rb.nb; ++i) {
    const int l = rb.parent[i];
    double* dv = tv + 6 * i;
    double* da = ta + 6 * i;
    nz[i] = rb.moves(d, i);
    if (!nz[i]) {
      for (int e = 0; e < 6; ++e) dv[e] = da[e] = 0.;
      continue;
    }
    act_inv(K.R[i], K.p[i], l >= 0 ? tv + 6 * l : z6, dv);
    act_inv(K.R[i], K.p[i], l >= 0 ? ta + 6 * l : z6, da);
    double t6[6], u6[6];
    if (i == j && dir == 0) {  // d(X^-1 m)/dq = -S x (X^-1 m)
      act_inv(K.R[i], K.p[i], l >= 0 ? Rv.v[l] : z6, u6);
      crm(Sd, u6, t6);
      for (int e = 0; e < 6; ++e) dv[e] -= t6[e];
      act_inv(K.R[i], K.p[i], l >= 0 ? Rv.a[l] : a0, u6);
      crm(Sd, u6, t6);
      for (int e = 0; e < 6; ++e) da[e] -= t6[e];
    }
    if (i == j && dir == 1)
      for (int e = 0; e < 6; ++e) dv[e] += Sd[e];
    double VJ[6];
    rb.vj(i, qd, VJ);
    crm(dv, VJ, t6);  // d(v x vJ) = dv x vJ (+ v x S on the joint, dir 1)
    for (int e = 0; e < 6; ++e) da[e] += t6[e];
    if (i == j && dir == 1) {
      crm(Rv.v[i], Sd, t6);
      for (int e = 0; e < 6; ++e) da[e] += t6[e];
    }
    double Ida[6], Idv[6];
    const double* Iv = Rv.h[i];
    m6v(rb.I6[i], da, Ida);
    m6v(rb.I6[i], dv, Idv);
    crf(dv, Iv, t6);
    crf(Rv.v[i], Idv, u6);
    for (int e = 0; e < 6; ++e) dF[i][e] = Ida[e] + t6[e] + u6[e];
  }
  for (int i = rb.nb - 1; i >= 0; --i) {
    if (!nz[i]) {
      for (int k = 0; k < rb.nvj[i]; ++k) dtau[rb.iv[i] + k] = 0.;
      continue;
    }
    for (int k = 0; k < rb.nvj[i]; ++k) {
      double S[6];
      rb.S(i, k, S);
      double s = 0.;
      for (int e = 0; e < 6; ++e) s += S[e] * dF[i][e];
      dtau[rb.iv[i] + k] = s;
    }
    const int l = rb.parent[i];
    if (l < 0) continue;
    if (!nz[l]) {  // j's ancestors start accumulating here
      nz[l] = true;
      for (int e = 0; e < 6; ++e) dF[l][e] = 0.;
    }
    double F[6], t6[6];
    std::memcpy(F, dF[i], sizeof(F));
    if (dir == 0 && i == j) {  // d(X^T F)/dq = X^T (S x* F)
      crf(Sd, Rv.F[i], t6);
      for (int e = 0; e < 6; ++e) F[e] += t6[e];
    }
    act_force(K.R[i], K.p[i], F, t6);
    for (int e = 0; e < 6; ++e) dF[l][e] += t6[e];
  }
}
// CRBA + armature; M column-major nv x nv
inline void crba(const Robot& rb, const Kin& K, double* M) {
  const int nv = rb.nv;
  double Ic[kMaxB][36];
  for (int i = 0; i < rb.nb; ++i) std::memcpy(Ic[i], rb.I6[i], sizeof(Ic[i]));
  for (int i = rb.nb - 1; i >= 0; --i) {
    const int l = rb.parent[i];
    if (l < 0) continue;
    double X[36], IX[36], XtIX[36];
    mbo::xmotion(K.R[i], K.p[i], X);
    for (int c = 0; c < 6; ++c) m6v(Ic[i], X + 6 * c, IX + 6 * c);
    for (int c = 0; c < 6; ++c)
      for (int r = 0; r < 6; ++r) {
        double s = 0.;
        for (int k = 0; k < 6; ++k) s += X[r * 6 + k] * IX[c * 6 + k];
        XtIX[c * 6 + r] = s;
      }
    // accumulated into the parent in one contiguous pass: gcc 11 at -march=native on
    // AVX-512 hosts (Zen 5: znver3 + avx512*) vectorised the strided += above with an
    // aligned 32-byte store at a 16-byte-aligned address (the baseline's SIGSEGV)
    for (int e = 0; e < 36; ++e) Ic[l][e] += XtIX[e];
  }
  std::memset(M, 0, sizeof(double) * nv * nv);
  for (int i = 0; i < rb.nb; ++i)
    for (int k = 0; k < rb.nvj[i]; ++k) {
      const int ci = rb.iv[i] + k;
      double S[6], F[6];
      rb.S(i, k, S);
      m6v(Ic[i], S, F);
      for (int k2 = 0; k2 < rb.nvj[i]; ++k2) {
        double S2[6];
        rb.S(i, k2, S2);
        double s = 0.;
        for (int e = 0; e < 6; ++e) s += S2[e] * F[e];
        M[ci * nv + rb.iv[i] + k2] = s + (k2 == k ? rb.arm[ci] : 0.);
      }
      int j = i;
      while (rb.parent[j] >= 0) {
        double t6[6];
        act_force(K.R[j], K.p[j], F, t6);
        std::memcpy(F, t6, sizeof(F));
        j = rb.parent[j];
        for (int k2 = 0; k2 < rb.nvj[j]; ++k2) {
          double S2[6];
          rb.S(j, k2, S2);
          double s = 0.;
          for (int e = 0; e < 6; ++e) s += S2[e] * F[e];
          M[ci * nv + rb.iv[j] + k2] = M[(rb.iv[j] + k2) * nv + ci] = s;
        }
      }
    }
}
// SPD inverse by Cholesky (unit-stride inner loops); false if not positive definite
inline bool spd_inverse(const double* M, int n, double* Minv) {
  static thread_local double L[kMaxV * kMaxV];
  std::memcpy(L, M, sizeof(double) * n * n);  // lower triangle, column-major: L[j*n + i], i >= j
  for (int j = 0; j < n; ++j) {
    double* cj = L + (size_t)j * n;
    for (int k = 0; k < j; ++k) {
      const double* ck = L + (size_t)k * n;
      const double f = ck[j];
      for (int i = j; i < n; ++i) cj[i] -= ck[i] * f;
    }
    if (!(cj[j] > 0.)) return false;
    const double d = std::sqrt(cj[j]);
    const double id = 1. / d;
    cj[j] = d;
    for (int i = j + 1; i < n; ++i) cj[i] *= id;
  }
  for (int c = 0; c < n; ++c) {  // L L^T x = e_c
    double* x = Minv + (size_t)c * n;
    for (int i = 0; i < n; ++i) x[i] = i == c ? 1. : 0.;
    for (int j = 0; j < n; ++j) {  // forward: column-oriented
      const double* cj = L + (size_t)j * n;
      x[j] /= cj[j];
      const double xj = x[j];
      for (int i = j + 1; i < n; ++i) x[i] -= cj[i] * xj;
    }
    for (int i = n - 1; i >= 0; --i) {  // backward with L^T
      const double* ci = L + (size_t)i * n;
      double s = x[i];
      for (int k = i + 1; k < n; ++k) s -= ci[k] * x[k];
      x[i] = s / ci[i];
    }
  }
  return true;
}

// ---- state on SE(3) x R^n ------------------------------------------------------
struct State {
  int nq, nv;
  bool ff;
  void integrate(const double* x, const double* dx, double* out) const {
    int q0 = 0;
    if (ff) {
      double R0[9], Re[9], pe[3], R1[9], qn[4], t[3];
      quat_to_R(x + 3, R0);
      exp6(dx, Re, pe);
      mm(R0, Re, R1);
      mv(R0, pe, t);
      for (int e = 0; e < 3; ++e) out[e] = x[e] + t[e];
      R_to_quat(R1, qn);
      double dt = qn[0] * x[3] + qn[1] * x[4] + qn[2] * x[5] + qn[3] * x[6];
      if (dt < 0)
        for (int e = 0; e < 4; ++e) qn[e] = -qn[e];
      const double n2 = qn[0] * qn[0] + qn[1] * qn[1] + qn[2] * qn[2] + qn[3] * qn[3];
      for (int e = 0; e < 4; ++e) out[3 + e] = qn[e] * ((3 - n2) / 2);
      q0 = 7;
    }
    const int d0 = ff ? 6 : 0;
    for (int i = q0; i < nq; ++i) out[i] = x[i] + dx[d0 + i - q0];
    for (int i = 0; i < nv; ++i) out[nq + i] = x[nq + i] + dx[nv + i];
  }
  void diff(const double* x0, const double* x1, double* out) const {
    int q0 = 0;
    if (ff) {
      double R0[9], R1[9], Rr[9], dp[3], pr[3];
      quat_to_R(x0 + 3, R0);
      quat_to_R(x1 + 3, R1);
      mbo_matTmul(R0, R1, Rr);
      for (int e = 0; e < 3; ++e) dp[e] = x1[e] - x0[e];
      mtv(R0, dp, pr);
      mbo::log6(Rr, pr, out);
      q0 = 7;
    }
    const int d0 = ff ? 6 : 0;
    for (int i = q0; i < nq; ++i) out[d0 + i - q0] = x1[i] - x0[i];
    for (int i = 0; i < nv; ++i) out[nv + i] = x1[nq + i] - x0[nq + i];
  }
  static void mbo_matTmul(const double* A, const double* B, double* O) {
    for (int c = 0; c < 3; ++c) mtv(A, B + 3 * c, O + 3 * c);
  }
};

// ---- activations ---------------------------------------------------------------
struct Act {
  int kind = 0, nr = 0;
  const double* p = nullptr;
  double value2(int i, double r) const {
    if (kind <= 1) return p[i] * r * r;
    const double rl = std::fmin(r - p[i], 0.), ru = std::fmax(r - p[nr + i], 0.);
    const double v = rl * rl + ru * ru;
    return kind == 3 ? p[2 * nr + i] * p[2 * nr + i] * v : v;
  }
  double grad(int i, double r) const {
    if (kind <= 1) return p[i] * r;
    const double g = std::fmin(r - p[i], 0.) + std::fmax(r - p[nr + i], 0.);
    return kind == 3 ? p[2 * nr + i] * p[2 * nr + i] * g : g;
  }
  double hess(int i, double r) const {
    if (kind <= 1) return p[i];
    const double h = (r - p[i] <= 0.) ? 1. : ((r - p[nr + i] >= 0.) ? 1. : 0.);
    return kind == 3 ? p[2 * nr + i] * h : h;
  }
};

// ---- the knot ------------------------------------------------------------------
struct Knot {
  double dt = 0.;
  Robot rb;
  State st;
  int ncost = 0;
  const double* crec[64];
  bool contact = false, enable_force = false, impulse = false;
  int nun = 0, ncon = 0, nc = 0;
  double damping = 0., r_coeff = 0.;
  const double* kk[kMaxC];

  void parse(const double* P) {
    dt = P[0];
    const int nv = (int)P[1];
    ncost = (int)P[2];
    rb.parse(P + 4, nv);
    st = State{rb.nq, rb.nv, rb.ff};
    const double* c = P + 4 + 3 + nv + (size_t)kJRec * rb.nb;
    for (int k = 0; k < ncost; ++k) {
      crec[k] = c;
      c += (int)c[3];
    }
    nun = 0;
    if (c - P < (long)P[3]) {
      contact = true;
      impulse = (int)c[3] == 1;  // [r_coeff, damping, nimpulse, 1] (impulse-fwddyn.hxx)
      nun = impulse ? nv : (int)c[0];
      r_coeff = impulse ? c[0] : 0.;
      damping = c[1];
      ncon = (int)c[2];
      enable_force = (int)c[3] == 2;
      c += 4;
      for (int k = 0; k < ncon; ++k) {
        kk[k] = c;
        nc += (int)c[0] == C_CONTACT_3D ? 3 : 6;
        c += (int)c[3];
      }
    }
  }
  int nu() const { return rb.nv - nun; }

  int cost_nr(const double* rc) const {
    const int t = (int)rc[0];
    if (t == C_CONTACT_FORCE) return (int)rc[5];
    if (t == C_FRICTION_CONE) return (int)rc[6];
    if (t == C_STATE) return 2 * rb.nv;
    if (t == C_CONTROL) return nu();
    return (t == C_FRAME_PLACEMENT || t == C_FRAME_VELOCITY) ? 6 : 3;
  }
  Act act(const double* rc) const {
    Act a;
    a.nr = cost_nr(rc);
    a.kind = (int)rc[2];
    const int np = a.kind <= 1 ? a.nr : (a.kind == 2 ? 2 * a.nr : 3 * a.nr);
    a.p = rc + (int)rc[3] - np;
    return a;
  }
  // oMf of a frame payload [joint, R(9), p(3)]
  void frame(const Kin& K, const double* d, double* Rf, double* pf) const {
    const int j = (int)d[0];
    double t[3];
    mm(K.oR[j], d + 1, Rf);
    mv(K.oR[j], d + 10, t);
    for (int e = 0; e < 3; ++e) pf[e] = K.op[j][e] + t[e];
  }
  // frame placement / translation residual and, for dof dd >= 0, its Jacobian column
  int frame_residual(const Kin& K, const double* d, int type, int dd, double* r, double* Jc) const {
    double Rf[9], pf[3];
    frame(K, d, Rf, pf);
    double dR[9] = {0}, dp[3] = {0};
    const bool sup = dd >= 0 && rb.moves(dd, (int)d[0]);
    if (sup) {
      double S[6], t[3];
      world_S(rb, K, dd, S);
      cr(S + 3, pf, t);
      for (int e = 0; e < 3; ++e) dp[e] = S[e] + t[e];
      for (int c = 0; c < 3; ++c) cr(S + 3, Rf + 3 * c, dR + 3 * c);
    }
    if (type == C_FRAME_TRANSLATION || type == C_CONTACT_3D) {
      for (int e = 0; e < 3; ++e) {
        r[e] = pf[e] - d[13 + e];
        if (Jc) Jc[e] = dp[e];
      }
      return 3;
    }
    double Rr[9], pr[3], dRr[9], dpr[3];
    mm(d + 13, Rf, Rr);
    mv(d + 13, pf, pr);
    for (int e = 0; e < 3; ++e) pr[e] += d[22 + e];
    mm(d + 13, dR, dRr);
    mv(d + 13, dp, dpr);
    Dl RD[9], PD[3], o[6];
    for (int e = 0; e < 9; ++e) RD[e] = Dl(Rr[e], dRr[e]);
    for (int e = 0; e < 3; ++e) PD[e] = Dl(pr[e], dpr[e]);
    mbo::log6(RD, PD, o);
    for (int e = 0; e < 6; ++e) {
      r[e] = o[e].v;
      if (Jc) Jc[e] = sup ? o[e].d : 0.;
    }
    return 6;
  }
  // contact rows: Jc (nc x nv row-major: LOCAL frame Jacobians), a0 at the drift
  void contact_terms(const Kin& K, const Rnea& Rv, double* Jc, double* a0, bool drift = true) const {
    const int nv = rb.nv;
    int row = 0;
    for (int k = 0; k < ncon; ++k) {
      const double* rc = kk[k];
      const double* d = rc + 4;
      const int j = (int)d[0], n = (int)rc[0] == C_CONTACT_3D ? 3 : 6;
      double Rf[9], pf[3];
      frame(K, d, Rf, pf);
      for (int c = 0; c < nv; ++c) {
        double o[6] = {0., 0., 0., 0., 0., 0.};
        if (rb.moves(c, j)) {
          double S[6];
          world_S(rb, K, c, S);
          act_inv(Rf, pf, S, o);
        }
        for (int e = 0; e < n; ++e) Jc[(row + e) * nv + c] = o[e];
      }
      if (!drift) {
        row += n;
        continue;
      }
      double vf[6], af[6], ag[6], gl[3];
      act_inv(d + 1, d + 10, Rv.v[j], vf);
      mtv(K.oR[j], rb.g, gl);  // remove the gravity the recursion carries
      for (int e = 0; e < 6; ++e) ag[e] = Rv.a[j][e] + (e < 3 ? gl[e] : 0.);
      act_inv(d + 1, d + 10, ag, af);
      const double kp = rc[1], kd = rc[2];
      double r[6] = {0., 0., 0., 0., 0., 0.};
      if (kp != 0.) frame_residual(K, d, n == 3 ? C_CONTACT_3D : C_CONTACT_6D, -1, r, nullptr);
      if (n == 3) {
        double wxv[3];
        cr(vf + 3, vf, wxv);
        for (int e = 0; e < 3; ++e) a0[row + e] = af[e] + wxv[e] + kp * r[e] + kd * vf[e];
      } else {
        for (int e = 0; e < 6; ++e) a0[row + e] = af[e] + kp * r[e] + kd * vf[e];
      }
      row += n;
    }
  }
  // da0 along dof c (dir 0: q, 1: v) from the joint tangents tv / ta
  void contact_dir(const Kin& K, const Rnea& Rv, int dir, int c, const double* tv, const double* ta,
                   double* da0) const {
    int row = 0;
    for (int k = 0; k < ncon; ++k) {
      const double* rc = kk[k];
      const double* d = rc + 4;
      const int j = (int)d[0], n = (int)rc[0] == C_CONTACT_3D ? 3 : 6;
      double dv[6], da[6];
      for (int e = 0; e < 6; ++e) dv[e] = tv[6 * j + e], da[e] = ta[6 * j + e];
      const bool sup = rb.moves(c, j);
      if (dir == 0 && sup) {  // gravity tangent: d(R_j^T g)/dq_c = -R_j^T (w_c x g)
        double S[6], wg[3], t[3];
        world_S(rb, K, c, S);
        cr(S + 3, rb.g, wg);
        mtv(K.oR[j], wg, t);
        for (int e = 0; e < 3; ++e) da[e] -= t[e];
      }
      double dvf[6], daf[6], vf[6];
      act_inv(d + 1, d + 10, dv, dvf);
      act_inv(d + 1, d + 10, da, daf);
      act_inv(d + 1, d + 10, Rv.v[j], vf);
      const double kp = rc[1], kd = rc[2];
      double rr[6], Jk[6] = {0., 0., 0., 0., 0., 0.};
      if (kp != 0. && dir == 0 && sup) frame_residual(K, d, n == 3 ? C_CONTACT_3D : C_CONTACT_6D, c, rr, Jk);
      if (n == 3) {
        double t1[3], t2[3];
        cr(dvf + 3, vf, t1);
        cr(vf + 3, dvf, t2);
        for (int e = 0; e < 3; ++e) da0[row + e] = daf[e] + t1[e] + t2[e] + kd * dvf[e] + kp * Jk[e];
      } else {
        for (int e = 0; e < 6; ++e) da0[row + e] = daf[e] + kd * dvf[e] + kp * Jk[e];
      }
      row += n;
    }
  }
  void contact_fext(const double* lam, double* fext) const {
    std::memset(fext, 0, sizeof(double) * 6 * rb.nb);
    int row = 0;
    for (int k = 0; k < ncon; ++k) {
      const double* d = kk[k] + 4;
      const int j = (int)d[0], n = (int)kk[k][0] == C_CONTACT_3D ? 3 : 6;
      double f[6] = {0., 0., 0., 0., 0., 0.}, o[6];
      for (int e = 0; e < n; ++e) f[e] = lam[row + e];
      act_force(d + 1, d + 10, f, o);
      for (int e = 0; e < 6; ++e) fext[6 * j + e] += o[e];
      row += n;
    }
  }
  double com(const Kin& K, double* c, double* mt_out = nullptr) const {
    double m = 0., h[3] = {0., 0., 0.};
    for (int i = 0; i < rb.nb; ++i) {
      const double mi = rb.rec[i][17];
      double t[3];
      mv(K.oR[i], rb.rec[i] + 18, t);
      m += mi;
      for (int e = 0; e < 3; ++e) h[e] += mi * (K.op[i][e] + t[e]);
    }
    for (int e = 0; e < 3; ++e) c[e] = h[e] / m;
    if (mt_out) *mt_out = m;
    return m;
  }
  // dynamics: a (+ lambda, KKT pieces with contacts); false if M or S is not PD
  struct Dyn {
    double a[kMaxV], lam[kMaxC], Mi[kMaxV * kMaxV], Y[kMaxV * kMaxC], Si[kMaxC * kMaxC], Jc[kMaxC * kMaxV];
    Rnea R0;
  };
  bool dynamics(const Kin& K, const double* x, const double* u, Dyn& D) const {
    const int nv = rb.nv, nq = rb.nq;
    static thread_local double M[kMaxV * kMaxV];
    double nle[kMaxV], a0[kMaxC], z[kMaxV], zero[kMaxV] = {0.};
    crba(rb, K, M);
    bool ok = spd_inverse(M, nv, D.Mi);
    rnea(rb, K, x + nq, zero, D.R0, nle);
    for (int i = 0; i < nv; ++i) {
      double s = 0.;
      for (int k = 0; k < nv; ++k) s += D.Mi[k * nv + i] * ((k < nun ? 0. : u[k - nun]) - nle[k]);
      z[i] = s;
    }
    if (nc == 0) {
      std::memcpy(D.a, z, sizeof(double) * nv);
      return ok;
    }
    contact_terms(K, D.R0, D.Jc, a0);
    for (int c = 0; c < nc; ++c)
      for (int i = 0; i < nv; ++i) {
        double s = 0.;
        const double* Jr = D.Jc + c * nv;
        for (int k = 0; k < nv; ++k) s += D.Mi[k * nv + i] * Jr[k];
        D.Y[c * nv + i] = s;
      }
    double S[kMaxC * kMaxC], r[kMaxC];
    for (int c = 0; c < nc; ++c) {
      for (int rr = 0; rr < nc; ++rr) {
        double s = 0.;
        for (int i = 0; i < nv; ++i) s += D.Jc[rr * nv + i] * D.Y[c * nv + i];
        S[c * nc + rr] = s + (rr == c ? damping : 0.);
      }
      double s = 0.;
      for (int i = 0; i < nv; ++i) s += D.Jc[c * nv + i] * z[i];
      r[c] = s + a0[c];
    }
    ok = spd_inverse(S, nc, D.Si) && ok;
    for (int c = 0; c < nc; ++c) {
      double s = 0.;
      for (int k = 0; k < nc; ++k) s += D.Si[k * nc + c] * r[k];
      D.lam[c] = -s;
    }
    for (int i = 0; i < nv; ++i) {
      double s = z[i];
      for (int c = 0; c < nc; ++c) s += D.Y[c * nv + i] * D.lam[c];
      D.a[i] = s;
    }
    return ok;
  }
  // force cost residual row e (lam of the contact rows; inactive: lambda = 0)
  static double force_res(const double* rc, const double* lam, int e) {
    const double* d = rc + 4;
    const int row0 = (int)d[0];
    if ((int)rc[0] == C_CONTACT_FORCE) return (row0 >= 0 ? lam[row0 + e] : 0.) - d[2 + e];
    if (row0 < 0) return 0.;
    const double* A = d + 3 + 3 * e;
    return A[0] * lam[row0] + A[1] * lam[row0 + 1] + A[2] * lam[row0 + 2];
  }
  // the state residual diff(xref, x) (2 nv)
  void state_res(const double* xref, const double* x, double* r) const { st.diff(xref, x, r); }

  double cost_value(const Kin& K, const Rnea& Rv, const double* x, const double* u, const double* lam) const {
    double total = 0.;
    for (int k = 0; k < ncost; ++k) {
      const double* rc = crec[k];
      const int t = (int)rc[0];
      const Act A = act(rc);
      const double* d = rc + 4;
      double a = 0.;
      if (t == C_STATE) {
        double r[2 * kMaxV];
        state_res(d, x, r);
        for (int i = 0; i < A.nr; ++i) a += A.value2(i, r[i]);
      } else if (t == C_CONTROL) {
        for (int i = 0; i < A.nr; ++i) a += A.value2(i, u[i] - d[i]);
      } else if (t == C_CONTACT_FORCE || t == C_FRICTION_CONE) {
        for (int i = 0; i < A.nr; ++i) a += A.value2(i, force_res(rc, lam, i));
      } else if (t == C_COM_POSITION) {
        double c[3];
        com(K, c);
        for (int i = 0; i < 3; ++i) a += A.value2(i, c[i] - d[i]);
      } else if (t == C_FRAME_VELOCITY) {
        double vf[6];
        act_inv(d + 1, d + 10, Rv.v[(int)d[0]], vf);
        for (int i = 0; i < 6; ++i) a += A.value2(i, vf[i] - d[13 + i]);
      } else {
        double r[6];
        const int nr = frame_residual(K, d, t, -1, r, nullptr);
        for (int i = 0; i < nr; ++i) a += A.value2(i, r[i]);
      }
      total += rc[1] * (0.5 * a);
    }
    return total;
  }

  // pinocchio::impulseDynamics by the Schur complement (impulse-fwddyn.hxx:53-86):
  // [M Jc^T; Jc -damping I] [v+; -Lambda] = [M v; -r Jc v]
  bool impulse_solve(const Kin& K, const double* x, double* M, Dyn& D, double* vp) const {
    const int nv = rb.nv, nq = rb.nq;
    const double* v = x + nq;
    double a0[kMaxC];
    crba(rb, K, M);
    bool ok = spd_inverse(M, nv, D.Mi);
    contact_terms(K, D.R0, D.Jc, a0, false);
    for (int c = 0; c < nc; ++c)
      for (int i = 0; i < nv; ++i) {
        double s = 0.;
        for (int k = 0; k < nv; ++k) s += D.Mi[k * nv + i] * D.Jc[c * nv + k];
        D.Y[c * nv + i] = s;
      }
    double S[kMaxC * kMaxC], Jv[kMaxC];
    for (int c = 0; c < nc; ++c) {
      for (int rr = 0; rr < nc; ++rr) {
        double s = 0.;
        for (int i = 0; i < nv; ++i) s += D.Jc[rr * nv + i] * D.Y[c * nv + i];
        S[c * nc + rr] = s + (rr == c ? damping : 0.);
      }
      double s = 0.;
      for (int i = 0; i < nv; ++i) s += D.Jc[c * nv + i] * v[i];
      Jv[c] = (1. + r_coeff) * s;
    }
    ok = spd_inverse(S, nc, D.Si) && ok;
    for (int c = 0; c < nc; ++c) {
      double s = 0.;
      for (int k = 0; k < nc; ++k) s += D.Si[k * nc + c] * Jv[k];
      D.lam[c] = -s;
    }
    for (int i = 0; i < nv; ++i) {
      double s = v[i];
      for (int c = 0; c < nc; ++c) s += D.Y[c * nv + i] * D.lam[c];
      vp[i] = ok ? s : NAN;
    }
    return ok;
  }

  void calc(const double* x, const double* u, double* xnext, double* cost) const {
    const int nv = rb.nv, nq = rb.nq;
    Kin K;
    kinematics(rb, x, K);
    static thread_local Dyn D;
    if (impulse) {  // xnext = (q, v+), cost = costs(x) (impulse-fwddyn.hxx:53-86)
      static thread_local double M[kMaxV * kMaxV];
      double vp[kMaxV];
      impulse_solve(K, x, M, D, vp);
      for (int i = 0; i < nq; ++i) xnext[i] = x[i];
      for (int i = 0; i < nv; ++i) xnext[nq + i] = vp[i];
      *cost = cost_value(K, D.R0, x, u, D.lam);
      return;
    }
    const bool ok = dynamics(K, x, u, D);
    if (!ok)
      for (int i = 0; i < nv; ++i) D.a[i] = NAN;
    const double cc = cost_value(K, D.R0, x, u, D.lam);
    if (dt != 0.) {
      double dx[2 * kMaxV];
      for (int i = 0; i < nv; ++i) dx[i] = x[nq + i] * dt + D.a[i] * dt * dt, dx[nv + i] = D.a[i] * dt;
      st.integrate(x, dx, xnext);
      *cost = dt * cc;
    } else {
      for (int i = 0; i < nq + nv; ++i) xnext[i] = x[i];
      *cost = cc;
    }
  }

  // impulse-fwddyn.hxx:89-127: Fx = [[I, 0], [-G dtau_dq - H dv0_dq, G M]] with G, H the
  // KKT-inverse blocks, dtau_dq = d/dq [RNEA(q, 0, v+ - v) - Jc^T Lambda] without gravity
  // (Lambda fixed in the contact frames) and dv0_dq = d/dq (Jc v+)
  bool impulse_fx(const Kin& K, const double* x, Dyn& D, double* H, Rnea& Rv, double* Fx) const {
    const int nv = rb.nv, nq = rb.nq, n = 2 * nv;
    static thread_local double M[kMaxV * kMaxV], fext[6 * kMaxB], dtau[kMaxV * kMaxV], dv0[kMaxC * kMaxV];
    double vp[kMaxV], dv[kMaxV], zero[kMaxV] = {0.}, tau[kMaxV], tv[6 * kMaxB], ta[6 * kMaxB];
    const double g0[3] = {0., 0., 0.};
    const bool ok = impulse_solve(K, x, M, D, vp);
    double* G = D.Mi;
    for (int c = 0; c < nc; ++c)
      for (int i = 0; i < nv; ++i) {
        double s = 0.;
        for (int k = 0; k < nc; ++k) s += D.Y[k * nv + i] * D.Si[c * nc + k];
        H[c * nv + i] = s;
      }
    for (int c = 0; c < nv; ++c)
      for (int i = 0; i < nv; ++i) {
        double s = 0.;
        for (int k = 0; k < nc; ++k) s += H[k * nv + i] * D.Y[k * nv + c];
        G[c * nv + i] -= s;
      }
    contact_fext(D.lam, fext);
    for (int i = 0; i < nv; ++i) dv[i] = vp[i] - x[nq + i];
    Rnea R1;
    rnea(rb, K, zero, dv, Rv, tau, fext, g0);
    rnea(rb, K, vp, zero, R1, tau);  // joint velocities at v+
    for (int c = 0; c < nv; ++c) {
      double col[kMaxV];
      rnea_dir(rb, K, Rv, zero, 0, c, col, tv, ta, g0);
      for (int k = 0; k < nv; ++k) dtau[k * nv + c] = col[k];
      rnea_dir(rb, K, R1, vp, 0, c, col, tv, ta);
      int row = 0;
      for (int q = 0; q < ncon; ++q) {  // LOCAL frame velocity tangent, linear rows for 3D
        const double* d = kk[q] + 4;
        const int j = (int)d[0], nr = (int)kk[q][0] == C_CONTACT_3D ? 3 : 6;
        double o[6];
        act_inv(d + 1, d + 10, tv + 6 * j, o);
        for (int e = 0; e < nr; ++e) dv0[(row + e) * nv + c] = o[e];
        row += nr;
      }
    }
    for (int c = 0; c < n; ++c)
      for (int i = 0; i < n; ++i) {
        double f;
        if (i < nv) {
          f = c == i ? 1. : 0.;
        } else if (c < nv) {
          const int r = i - nv;
          double s = 0.;
          for (int k = 0; k < nv; ++k) s += G[k * nv + r] * dtau[k * nv + c];
          for (int k = 0; k < nc; ++k) s += H[k * nv + r] * dv0[k * nv + c];
          f = ok ? -s : NAN;
        } else {
          const int r = i - nv, cc = c - nv;
          double s = 0.;
          for (int k = 0; k < nv; ++k) s += G[k * nv + r] * M[cc * nv + k];
          f = ok ? s : NAN;
        }
        Fx[(size_t)c * n + i] = f;
      }
    return ok;
  }

  // euler.hxx:83-131; blocks column-major, n = 2 nv rows, m = nu_max columns
  bool calc_diff(const double* x, const double* u, int m, double* Fx, double* Fu, double* Lxx, double* Lxu,
                 double* Luu, double* Lx, double* Lu) const {
    const int nv = rb.nv, nq = rb.nq, n = 2 * nv, L = 2 * nv, nuk = nu();
    Kin K;
    kinematics(rb, x, K);
    static thread_local Dyn D;
    // Kinv blocks: H = Y S^-1 (nv x nc), G = Minv - H Y^T (in place of Minv)
    static thread_local double H[kMaxV * kMaxC], fext[6 * kMaxB], dtau[kMaxV * 2 * kMaxV], da0[kMaxC * 2 * kMaxV];
    static thread_local double da[kMaxV * 2 * kMaxV], tv[6 * kMaxB], ta[6 * kMaxB], dfx[kMaxC * 2 * kMaxV],
        dfu[kMaxC * kMaxV], tvs_[2 * kMaxV * 6 * kMaxB];
    Rnea Rv;
    bool ok;
    if (impulse) {
      ok = impulse_fx(K, x, D, H, Rv, Fx);
    } else {
      ok = dynamics(K, x, u, D);
      double* G = D.Mi;
      if (nc > 0) {
        for (int c = 0; c < nc; ++c)
          for (int i = 0; i < nv; ++i) {
            double s = 0.;
            for (int k = 0; k < nc; ++k) s += D.Y[k * nv + i] * D.Si[c * nc + k];
            H[c * nv + i] = s;
          }
        for (int c = 0; c < nv; ++c)
          for (int i = 0; i < nv; ++i) {
            double s = 0.;
            for (int k = 0; k < nc; ++k) s += H[k * nv + i] * D.Y[k * nv + c];
            G[c * nv + i] -= s;
          }
        contact_fext(D.lam, fext);
      }
      double tau[kMaxV];
      rnea(rb, K, x + nq, D.a, Rv, tau, nc > 0 ? fext : nullptr);
      // tangent directions: dtau/dx [k][L] (row k, column c), da0/dx, frame-velocity tangents
      for (int c = 0; c < L; ++c) {
        double dt_[kMaxV];
        rnea_dir(rb, K, Rv, x + nq, c < nv ? 0 : 1, c % nv, dt_, tv, ta);
        for (int k = 0; k < nv; ++k) dtau[k * L + c] = dt_[k];
        if (nc > 0) {
          double d0[kMaxC];
          contact_dir(K, Rv, c < nv ? 0 : 1, c % nv, tv, ta, d0);
          for (int k = 0; k < nc; ++k) da0[k * L + c] = d0[k];
        }
        // joint-velocity tangents, kept for the frame-velocity Jacobians
        std::memcpy(tvs_ + (size_t)c * 6 * kMaxB, tv, sizeof(double) * 6 * rb.nb);
      }
      for (int r = 0; r < nv; ++r) {  // da/dx = -(G dtau + H da0), row axpys
        double* row = da + r * L;
        for (int c = 0; c < L; ++c) row[c] = 0.;
        for (int k = 0; k < nv; ++k) {
          const double g = G[k * nv + r];
          const double* tr = dtau + k * L;
          for (int c = 0; c < L; ++c) row[c] += g * tr[c];
        }
        for (int k = 0; k < nc; ++k) {
          const double h = H[k * nv + r];
          const double* tr = da0 + k * L;
          for (int c = 0; c < L; ++c) row[c] += h * tr[c];
        }
        for (int c = 0; c < L; ++c) row[c] = ok ? -row[c] : NAN;
      }
      if (enable_force && nc > 0) {  // d lambda / dx (Kinv bottom-left H^T), d lambda / du
        for (int k = 0; k < nc; ++k)
          for (int c = 0; c < L; ++c) {
            double s = 0.;
            for (int i = 0; i < nv; ++i) s += H[k * nv + i] * dtau[i * L + c];
            for (int m2 = 0; m2 < nc; ++m2) s -= D.Si[m2 * nc + k] * da0[m2 * L + c];
            dfx[k * L + c] = s;
          }
        for (int k = 0; k < nc; ++k)
          for (int c = 0; c < nv; ++c) dfu[k * nv + c] = c < nuk ? -H[k * nv + nun + c] : 0.;
      }
      // Euler assembly (euler.hxx:100-112) with dIntegrate on the free-flyer
      const double dt2 = dt * dt;
      const bool integ = dt != 0.;
      double Je[36], Ai[36];
      const bool ffe = rb.ff && integ;
      if (ffe) ff_jacobians(x, D.a, Je, Ai);
      for (int c = 0; c < n; ++c)
        for (int i = 0; i < n; ++i) {
          double f;
          if (!integ) {
            f = c == i ? 1. : 0.;
          } else if (i < nv && ffe && i < 6) {
            double s = c < 6 ? Ai[c * 6 + i] : 0.;
            for (int r = 0; r < 6; ++r) s += Je[r * 6 + i] * (da[r * L + c] * dt2 + (c == nv + r ? dt : 0.));
            f = s;
          } else if (i < nv) {
            f = da[i * L + c] * dt2 + (c == nv + i ? dt : 0.) + (c == i ? 1. : 0.);
          } else {
            f = da[(i - nv) * L + c] * dt + (c == i ? 1. : 0.);
          }
          Fx[(size_t)c * n + i] = f;
        }
      for (int c = 0; c < m; ++c)
        for (int i = 0; i < n; ++i) {
          double f = 0.;
          if (integ && c < nuk) {
            if (i < nv && ffe && i < 6) {
              double s = 0.;
              for (int r = 0; r < 6; ++r) s += Je[r * 6 + i] * G[(nun + c) * nv + r];
              f = ok ? s * dt2 : NAN;
            } else {
              const double mi = ok ? G[(nun + c) * nv + (i < nv ? i : i - nv)] : NAN;
              f = i < nv ? mi * dt2 : mi * dt;
            }
          }
          Fu[(size_t)c * n + i] = f;
        }
    }
    // costs: stacked residual rows over (x, u) and diagonal terms (cost-sum.hxx:122-160)
    std::memset(Lxx, 0, sizeof(double) * n * n);
    if (m > 0) {  // impulse knots have no control blocks (null pointers)
      std::memset(Lxu, 0, sizeof(double) * n * m);
      std::memset(Luu, 0, sizeof(double) * m * m);
      std::memset(Lu, 0, sizeof(double) * m);
    }
    std::memset(Lx, 0, sizeof(double) * n);
    static thread_local double R[kMaxRows * 3 * kMaxV];
    const int ld = L + nuk;
    for (int k = 0; k < ncost; ++k) {
      const double* rc = crec[k];
      const int t = (int)rc[0];
      const Act A = act(rc);
      const double* d = rc + 4;
      const double wt = rc[1];
      int nr = 0;
      double res[6];
      if (t == C_STATE) {
        double r[2 * kMaxV];
        state_res(d, x, r);
        const int i0 = rb.ff ? 6 : 0;
        if (rb.ff) {  // Jlog6 block (dDifference second argument)
          double Jl[36];
          state_jlog6(d, x, Jl);
          for (int e = 0; e < 6; ++e) {
            res[e] = r[e];
            for (int c = 0; c < ld; ++c) R[e * ld + c] = c < 6 ? Jl[c * 6 + e] : 0.;
          }
          nr = 6;
        }
        for (int i = i0; i < n; ++i) {
          Lx[i] += wt * A.grad(i, r[i]);
          Lxx[(size_t)i * n + i] += wt * A.hess(i, r[i]);
        }
        // the free-flyer rows below use activation rows 0..5
      } else if (t == C_CONTROL) {
        for (int i = 0; i < nuk; ++i) {
          Lu[i] += wt * A.grad(i, u[i] - d[i]);
          Luu[(size_t)i * m + i] += wt * A.hess(i, u[i] - d[i]);
        }
      } else if (t == C_CONTACT_FORCE || t == C_FRICTION_CONE) {
        if (enable_force && nc > 0 && (int)d[0] >= 0) {
          nr = A.nr;
          for (int e = 0; e < nr; ++e) {
            res[e] = force_res(rc, D.lam, e);
            for (int c = 0; c < ld; ++c) {
              double dl[3];
              const int row0 = (int)d[0];
              auto col = [&](int kr) { return c < L ? dfx[kr * L + c] : dfu[kr * nv + (c - L)]; };
              if (t == C_CONTACT_FORCE) {
                R[e * ld + c] = col(row0 + e);
              } else {
                for (int q = 0; q < 3; ++q) dl[q] = col(row0 + q);
                const double* Am = d + 3 + 3 * e;
                R[e * ld + c] = Am[0] * dl[0] + Am[1] * dl[1] + Am[2] * dl[2];
              }
            }
          }
        }
      } else if (t == C_COM_POSITION) {
        double cm[3], mt;
        com(K, cm, &mt);
        for (int e = 0; e < 3; ++e) res[e] = cm[e] - d[e];
        for (int c = 0; c < ld; ++c)
          for (int e = 0; e < 3; ++e) R[e * ld + c] = 0.;
        for (int c = 0; c < nv; ++c) {  // sum over the bodies moved by dof c
          double S[6], acc[3] = {0., 0., 0.};
          world_S(rb, K, c, S);
          for (int i = 0; i < rb.nb; ++i) {
            if (!rb.moves(c, i)) continue;
            const double mi = rb.rec[i][17];
            double t3[3], pc[3], wxp[3];
            mv(K.oR[i], rb.rec[i] + 18, t3);
            for (int e = 0; e < 3; ++e) pc[e] = K.op[i][e] + t3[e];
            cr(S + 3, pc, wxp);
            for (int e = 0; e < 3; ++e) acc[e] += mi * (S[e] + wxp[e]);
          }
          for (int e = 0; e < 3; ++e) R[e * ld + c] = acc[e] / mt;
        }
        nr = 3;
      } else if (t == C_FRAME_VELOCITY) {
        const int j = (int)d[0];
        double vf[6];
        act_inv(d + 1, d + 10, Rv.v[j], vf);
        for (int e = 0; e < 6; ++e) res[e] = vf[e] - d[13 + e];
        for (int c = 0; c < ld; ++c) {
          double o[6] = {0., 0., 0., 0., 0., 0.};
          if (c < L) act_inv(d + 1, d + 10, tvs_ + (size_t)c * 6 * kMaxB + 6 * j, o);
          for (int e = 0; e < 6; ++e) R[e * ld + c] = o[e];
        }
        nr = 6;
      } else {  // frame placement / translation
        double J[kMaxV][6];
        for (int c = 0; c < nv; ++c) nr = frame_residual(K, d, t, c, res, J[c]);
        for (int c = 0; c < ld; ++c)
          for (int e = 0; e < nr; ++e) R[e * ld + c] = c < nv ? J[c][e] : 0.;
      }
      // Gauss-Newton from the rows: L += wt R^T Arr R, wt R^T Ar
      for (int e = 0; e < nr; ++e) {
        const double h = wt * A.hess(e, res[e]), gr = wt * A.grad(e, res[e]);
        const double* Re = R + e * ld;
        for (int c = 0; c < L; ++c) Lx[c] += Re[c] * gr;
        for (int c = 0; c < nuk; ++c) Lu[c] += Re[L + c] * gr;
        for (int j = 0; j < ld; ++j) {
          const double hj = h * Re[j];
          if (hj == 0.) continue;
          if (j < L) {
            double* col = Lxx + (size_t)j * n;
            for (int i = 0; i < L; ++i) col[i] += Re[i] * hj;
          } else {
            double* colxu = Lxu + (size_t)(j - L) * n;
            for (int i = 0; i < L; ++i) colxu[i] += Re[i] * hj;
            double* coluu = Luu + (size_t)(j - L) * m;
            for (int i = 0; i < nuk; ++i) coluu[i] += Re[L + i] * hj;
          }
        }
      }
    }
    if (dt != 0.) {
      for (int i = 0; i < n; ++i) Lx[i] *= dt;
      for (int i = 0; i < m; ++i) Lu[i] *= dt;
      for (int i = 0; i < n * n; ++i) Lxx[i] *= dt;
      for (int i = 0; i < n * m; ++i) Lxu[i] *= dt;
      for (int i = 0; i < m * m; ++i) Luu[i] *= dt;
    }
    return ok;
  }

  // Jexp6(dq) (col-major 6x6) and Ad(exp6(dq)^-1) for dq = v dt + a dt^2 on the free-flyer
  void ff_jacobians(const double* x, const double* a, double* Je, double* Ai) const {
    const int nq = rb.nq;
    double dq[6], R[9], p[3];
    for (int e = 0; e < 6; ++e) dq[e] = x[nq + e] * dt + a[e] * dt * dt;
    exp6(dq, R, p);
    for (int k = 0; k < 6; ++k) {  // column k: log6(exp6(dq)^-1 exp6(dq + eps e_k)) / eps
      Dl D[6], RD[9], PD[3];
      for (int e = 0; e < 6; ++e) D[e] = Dl(dq[e], e == k ? 1. : 0.);
      exp6(D, RD, PD);
      Dl RR[9], PP[3], o[6];
      for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) {  // R^T RD
          Dl s(0., 0.);
          for (int q = 0; q < 3; ++q) s = s + Dl(R[r * 3 + q], 0.) * RD[c * 3 + q];
          RR[c * 3 + r] = s;
        }
      for (int r = 0; r < 3; ++r) {  // R^T (PD - p)
        Dl s(0., 0.);
        for (int q = 0; q < 3; ++q) s = s + Dl(R[r * 3 + q], 0.) * (PD[q] - Dl(p[q], 0.));
        PP[r] = s;
      }
      mbo::log6(RR, PP, o);
      for (int e = 0; e < 6; ++e) Je[k * 6 + e] = o[e].d;
    }
    for (int i = 0; i < 36; ++i) Ai[i] = 0.;
    for (int c = 0; c < 3; ++c)
      for (int r = 0; r < 3; ++r) {
        Ai[c * 6 + r] = R[r * 3 + c];
        Ai[(c + 3) * 6 + r + 3] = R[r * 3 + c];
      }
    for (int c = 0; c < 3; ++c) {  // -R^T [p]x
      const double e3[3] = {c == 0 ? 1. : 0., c == 1 ? 1. : 0., c == 2 ? 1. : 0.};
      double t[3], o[3];
      cr(p, e3, t);
      mtv(R, t, o);
      for (int r = 0; r < 3; ++r) Ai[(c + 3) * 6 + r] = -o[r];
    }
  }
  // Jlog6 of log6(Mref^-1 M) along the tangent of M (col-major 6x6): column k is the
  // derivative along M exp(eps e_k)
  void state_jlog6(const double* xref, const double* x, double* Jl) const {
    double R0[9], R1[9], Rr[9], dp[3], pr[3];
    quat_to_R(xref + 3, R0);
    quat_to_R(x + 3, R1);
    State::mbo_matTmul(R0, R1, Rr);
    for (int e = 0; e < 3; ++e) dp[e] = x[e] - xref[e];
    mtv(R0, dp, pr);
    for (int k = 0; k < 6; ++k) {
      double dRr[9] = {0}, dpr[3] = {0};
      if (k < 3) {  // translation along R1 e_k: pr += R0^T R1 e_k
        for (int e = 0; e < 3; ++e) dpr[e] = Rr[k * 3 + e];
      } else {  // rotation: Rr [e_k]x
        const double w[3] = {k == 3 ? 1. : 0., k == 4 ? 1. : 0., k == 5 ? 1. : 0.};
        for (int c = 0; c < 3; ++c) {
          const double ec[3] = {c == 0 ? 1. : 0., c == 1 ? 1. : 0., c == 2 ? 1. : 0.};
          double wxe[3];
          cr(w, ec, wxe);
          mv(Rr, wxe, dRr + 3 * c);
        }
      }
      Dl RD[9], PD[3], o[6];
      for (int e = 0; e < 9; ++e) RD[e] = Dl(Rr[e], dRr[e]);
      for (int e = 0; e < 3; ++e) PD[e] = Dl(pr[e], dpr[e]);
      mbo::log6(RD, PD, o);
      for (int e = 0; e < 6; ++e) Jl[k * 6 + e] = o[e].d;
    }
  }
};

}  // namespace fbo
