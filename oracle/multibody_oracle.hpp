// ORACLE — TEST INFRASTRUCTURE ONLY. C++ restatement of the multibody knot
// (FDDP_KNOT_EULER_FREEFWD, layout in include/fddp_hip.h) for the CPU
// baseline and as a second CPU cross-check of oracle/multibody_np.py:
//   IntegratedActionModelEuler        core/integrator/euler.hxx:41-131
//   ∘ DifferentialActionModelFreeFwdDynamics  multibody/actions/free-fwddyn.hxx:44-118
//     calc: a = ABA(q, v, tau) (free-fwddyn.hxx:64; Featherstone Table 7.1, the
//           algorithm pinocchio::aba implements), armature added to D
//     calcDiff: da/dx = -M^-1 dRNEA/dx at (q, v, a) (what
//           pinocchio::computeABADerivatives returns, free-fwddyn.hxx:102-107),
//           dRNEA by the linearised recursion in joint frames, M by CRBA and
//           its inverse by Cholesky; Fu = M^-1 (ActuationModelFull)
//   CostModelSum of State / Control / FramePlacement / FrameTranslation costs
//     (cost-sum.hxx:89-160, state.hxx:130-169, control.hxx:56-87,
//      frame-placement.hxx:45-80, frame-translation.hxx:50-81); the
//      FramePlacement Jacobian Jlog6(rMf) fJf is the local frame Jacobian pushed
//      through log6 in dual numbers (pinocchio::log6 restated).
// Pinocchio (third-party, absent offline) is restated from its published
// algorithms; multibody parity is pinned as described in oracle/multibody_np.py.
#pragma once

#include <cmath>
#include <cstring>

namespace mbo {

constexpr int kMaxJ = 32;
constexpr int kJRec = 27;  // [type, parent, axis(3), R(9), p(3), mass, CoM(3), I(6)]
enum { C_STATE = 1, C_CONTROL = 2, C_FRAME_PLACEMENT = 3, C_FRAME_TRANSLATION = 4 };

// 3x3 column-major helpers
inline void mv(const double* R, const double* v, double* o) {
  const double x = R[0] * v[0] + R[3] * v[1] + R[6] * v[2], y = R[1] * v[0] + R[4] * v[1] + R[7] * v[2],
               z = R[2] * v[0] + R[5] * v[1] + R[8] * v[2];
  o[0] = x, o[1] = y, o[2] = z;
}
inline void mtv(const double* R, const double* v, double* o) {
  const double x = R[0] * v[0] + R[1] * v[1] + R[2] * v[2], y = R[3] * v[0] + R[4] * v[1] + R[5] * v[2],
               z = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
  o[0] = x, o[1] = y, o[2] = z;
}
inline void mm(const double* A, const double* B, double* O) {
  for (int c = 0; c < 3; ++c) mv(A, B + 3 * c, O + 3 * c);
}
inline void cr(const double* a, const double* b, double* o) {
  const double x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
  o[0] = x, o[1] = y, o[2] = z;
}

// spatial algebra, (linear, angular); X: liMi = (R, p) child in parent
inline void act_inv(const double* R, const double* p, const double* m, double* o) {  // motion parent -> child
  double t[3];
  cr(p, m + 3, t);
  const double l[3] = {m[0] - t[0], m[1] - t[1], m[2] - t[2]};
  double a[3], b[3];
  mtv(R, l, a);
  mtv(R, m + 3, b);
  for (int e = 0; e < 3; ++e) o[e] = a[e], o[3 + e] = b[e];
}
inline void act_force(const double* R, const double* p, const double* f, double* o) {  // force child -> parent
  double a[3], b[3], t[3];
  mv(R, f, a);
  mv(R, f + 3, b);
  cr(p, a, t);
  for (int e = 0; e < 3; ++e) o[e] = a[e], o[3 + e] = b[e] + t[e];
}
inline void crm(const double* m, const double* n, double* o) {  // m x n (motion)
  double a[3], b[3], c[3];
  cr(m + 3, n, a);
  cr(m, n + 3, b);
  cr(m + 3, n + 3, c);
  for (int e = 0; e < 3; ++e) o[e] = a[e] + b[e], o[3 + e] = c[e];
}
inline void crf(const double* m, const double* f, double* o) {  // m x* f
  double a[3], b[3], c[3];
  cr(m + 3, f, a);
  cr(m + 3, f + 3, b);
  cr(m, f, c);
  for (int e = 0; e < 3; ++e) o[e] = a[e], o[3 + e] = b[e] + c[e];
}
// 6x6 spatial inertia (lin, ang) about the joint origin from (m, c, Ic)
inline void inertia6(double m, const double* c, const double* I, double* M6) {
  double C[9] = {0., c[2], -c[1], -c[2], 0., c[0], c[1], -c[0], 0.};  // [c]x column-major
  std::memset(M6, 0, 36 * sizeof(double));
  const double Ic[9] = {I[0], I[3], I[4], I[3], I[1], I[5], I[4], I[5], I[2]};
  double CC[9];
  mm(C, C, CC);
  for (int r = 0; r < 3; ++r)
    for (int cc = 0; cc < 3; ++cc) {
      M6[cc * 6 + r] = r == cc ? m : 0.;
      M6[(cc + 3) * 6 + r] = -m * C[cc * 3 + r];
      M6[cc * 6 + r + 3] = m * C[cc * 3 + r];
      M6[(cc + 3) * 6 + r + 3] = Ic[cc * 3 + r] - m * CC[cc * 3 + r];
    }
}
inline void m6v(const double* M, const double* v, double* o) {
  for (int r = 0; r < 6; ++r) {
    double s = 0.;
    for (int c = 0; c < 6; ++c) s += M[c * 6 + r] * v[c];
    o[r] = s;
  }
}
// 6x6 motion transform child <- parent (column-major) of liMi = (R, p)
inline void xmotion(const double* R, const double* p, double* X) {
  for (int c = 0; c < 6; ++c) {
    double e[6] = {0., 0., 0., 0., 0., 0.};
    e[c] = 1.;
    act_inv(R, p, e, X + 6 * c);
  }
}

struct Robot {
  int nj = 0;
  double g[3];
  const double* arm = nullptr;
  int parent[kMaxJ];
  const double* rec[kMaxJ];
  double I6[kMaxJ][36];
  void parse(const double* body, int n) {
    nj = n;
    for (int e = 0; e < 3; ++e) g[e] = body[e];
    arm = body + 3;
    const double* J = arm + nj;
    for (int i = 0; i < nj; ++i) {
      rec[i] = J + (size_t)kJRec * i;
      parent[i] = (int)rec[i][1];
      inertia6(rec[i][17], rec[i] + 18, rec[i] + 21, I6[i]);
    }
  }
  const double* axis(int i) const { return rec[i] + 2; }
  void liMi(const double* q, int i, double* R, double* p) const {
    const double* ax = axis(i);
    const double s = std::sin(q[i]), c = std::cos(q[i]), oc = 1. - c;
    const double Rj[9] = {c + oc * ax[0] * ax[0],         oc * ax[1] * ax[0] + s * ax[2], oc * ax[2] * ax[0] - s * ax[1],
                          oc * ax[0] * ax[1] - s * ax[2], c + oc * ax[1] * ax[1],         oc * ax[2] * ax[1] + s * ax[0],
                          oc * ax[0] * ax[2] + s * ax[1], oc * ax[1] * ax[2] - s * ax[0], c + oc * ax[2] * ax[2]};
    mm(rec[i] + 5, Rj, R);
    for (int e = 0; e < 3; ++e) p[e] = rec[i][14 + e];
  }
};

struct Kin {  // per-joint placements
  double R[kMaxJ][9], p[kMaxJ][3], oR[kMaxJ][9], op[kMaxJ][3];
};

inline void kinematics(const Robot& rb, const double* q, Kin& K) {
  for (int i = 0; i < rb.nj; ++i) {
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

// ABA (Featherstone Table 7.1), armature added to D
inline void aba(const Robot& rb, const Kin& K, const double* qd, const double* tau, double* qdd) {
  const int nj = rb.nj;
  double v[kMaxJ][6], c[kMaxJ][6], IA[kMaxJ][36], pA[kMaxJ][6], U[kMaxJ][6], D[kMaxJ], u[kMaxJ], X[kMaxJ][36];
  for (int i = 0; i < nj; ++i) {
    const int l = rb.parent[i];
    xmotion(K.R[i], K.p[i], X[i]);
    double vp[6] = {0., 0., 0., 0., 0., 0.};
    if (l >= 0) act_inv(K.R[i], K.p[i], v[l], vp);
    const double* ax = rb.axis(i);
    const double S[6] = {0., 0., 0., ax[0] * qd[i], ax[1] * qd[i], ax[2] * qd[i]};
    for (int e = 0; e < 6; ++e) v[i][e] = vp[e] + S[e];
    crm(v[i], S, c[i]);
    std::memcpy(IA[i], rb.I6[i], sizeof(IA[i]));
    double Iv[6];
    m6v(rb.I6[i], v[i], Iv);
    crf(v[i], Iv, pA[i]);
  }
  for (int i = nj - 1; i >= 0; --i) {
    const double* ax = rb.axis(i);
    for (int r = 0; r < 6; ++r) U[i][r] = IA[i][18 + r] * ax[0] + IA[i][24 + r] * ax[1] + IA[i][30 + r] * ax[2];
    D[i] = ax[0] * U[i][3] + ax[1] * U[i][4] + ax[2] * U[i][5] + rb.arm[i];
    u[i] = tau[i] - (ax[0] * pA[i][3] + ax[1] * pA[i][4] + ax[2] * pA[i][5]);
    const int l = rb.parent[i];
    if (l < 0) continue;
    double Ia[36], pa[6], t6[6];
    for (int c2 = 0; c2 < 6; ++c2)
      for (int r = 0; r < 6; ++r) Ia[c2 * 6 + r] = IA[i][c2 * 6 + r] - U[i][r] * U[i][c2] / D[i];
    m6v(Ia, c[i], t6);
    for (int e = 0; e < 6; ++e) pa[e] = pA[i][e] + t6[e] + U[i][e] * (u[i] / D[i]);
    // IA[l] += X^T Ia X ; pA[l] += X^T pa
    double IaX[36];
    for (int c2 = 0; c2 < 6; ++c2) m6v(Ia, X[i] + 6 * c2, IaX + 6 * c2);
    for (int c2 = 0; c2 < 6; ++c2)
      for (int r = 0; r < 6; ++r) {
        double s = 0.;
        for (int k = 0; k < 6; ++k) s += X[i][r * 6 + k] * IaX[c2 * 6 + k];
        IA[l][c2 * 6 + r] += s;
      }
    for (int r = 0; r < 6; ++r) {
      double s = 0.;
      for (int k = 0; k < 6; ++k) s += X[i][r * 6 + k] * pa[k];
      pA[l][r] += s;
    }
  }
  double a[kMaxJ][6];
  const double a0[6] = {-rb.g[0], -rb.g[1], -rb.g[2], 0., 0., 0.};
  for (int i = 0; i < nj; ++i) {
    const int l = rb.parent[i];
    double ai[6];
    act_inv(K.R[i], K.p[i], l >= 0 ? a[l] : a0, ai);
    for (int e = 0; e < 6; ++e) ai[e] += c[i][e];
    double s = 0.;
    for (int e = 0; e < 6; ++e) s += U[i][e] * ai[e];
    qdd[i] = (u[i] - s) / D[i];
    const double* ax = rb.axis(i);
    for (int e = 0; e < 3; ++e) ai[3 + e] += ax[e] * qdd[i];
    std::memcpy(a[i], ai, sizeof(ai));
  }
}

// RNEA values (joint frames) at (q, qd, qdd): v, a, accumulated F
struct Rnea {
  double v[kMaxJ][6], a[kMaxJ][6], F[kMaxJ][6];
};
// fext (may be null): external forces in the joint frames (pinocchio's fext)
inline void rnea(const Robot& rb, const Kin& K, const double* qd, const double* qdd, Rnea& Rv, double* tau,
                 const double* fext = nullptr) {
  const int nj = rb.nj;
  const double a0[6] = {-rb.g[0], -rb.g[1], -rb.g[2], 0., 0., 0.}, z6[6] = {0., 0., 0., 0., 0., 0.};
  for (int i = 0; i < nj; ++i) {
    const int l = rb.parent[i];
    const double* ax = rb.axis(i);
    act_inv(K.R[i], K.p[i], l >= 0 ? Rv.v[l] : z6, Rv.v[i]);
    act_inv(K.R[i], K.p[i], l >= 0 ? Rv.a[l] : a0, Rv.a[i]);
    const double S[6] = {0., 0., 0., ax[0] * qd[i], ax[1] * qd[i], ax[2] * qd[i]};
    for (int e = 0; e < 6; ++e) Rv.v[i][e] += S[e];
    double t6[6];
    crm(Rv.v[i], S, t6);
    for (int e = 0; e < 3; ++e) Rv.a[i][3 + e] += ax[e] * qdd[i];
    for (int e = 0; e < 6; ++e) Rv.a[i][e] += t6[e];
    double Ia[6], Iv[6];
    m6v(rb.I6[i], Rv.a[i], Ia);
    m6v(rb.I6[i], Rv.v[i], Iv);
    crf(Rv.v[i], Iv, t6);
    for (int e = 0; e < 6; ++e) Rv.F[i][e] = Ia[e] + t6[e] - (fext ? fext[6 * i + e] : 0.);
  }
  for (int i = nj - 1; i >= 0; --i) {
    const double* ax = rb.axis(i);
    tau[i] = ax[0] * Rv.F[i][3] + ax[1] * Rv.F[i][4] + ax[2] * Rv.F[i][5];
    const int l = rb.parent[i];
    if (l < 0) continue;
    double t6[6];
    act_force(K.R[i], K.p[i], Rv.F[i], t6);
    for (int e = 0; e < 6; ++e) Rv.F[l][e] += t6[e];
  }
}

// dRNEA/dq_j (dir 0) or dRNEA/dqd_j (dir 1) at the values in Rv -> dtau
// (tv / ta, may be null: the joint velocity / acceleration tangents, 6 per joint)
inline void rnea_dir(const Robot& rb, const Kin& K, const Rnea& Rv, const double* qd, int dir, int j, double* dtau,
                     double* tv = nullptr, double* ta = nullptr) {
  const int nj = rb.nj;
  const double a0[6] = {-rb.g[0], -rb.g[1], -rb.g[2], 0., 0., 0.}, z6[6] = {0., 0., 0., 0., 0., 0.};
  double dv[kMaxJ][6], da[kMaxJ][6], dF[kMaxJ][6];
  for (int i = 0; i < nj; ++i) {
    const int l = rb.parent[i];
    const double* ax = rb.axis(i);
    const double S[6] = {0., 0., 0., ax[0], ax[1], ax[2]};
    act_inv(K.R[i], K.p[i], l >= 0 ? dv[l] : z6, dv[i]);
    act_inv(K.R[i], K.p[i], l >= 0 ? da[l] : z6, da[i]);
    double t6[6], u6[6];
    if (i == j && dir == 0) {  // d(X^-1 m)/dq = -S x (X^-1 m)
      act_inv(K.R[i], K.p[i], l >= 0 ? Rv.v[l] : z6, u6);
      crm(S, u6, t6);
      for (int e = 0; e < 6; ++e) dv[i][e] -= t6[e];
      act_inv(K.R[i], K.p[i], l >= 0 ? Rv.a[l] : a0, u6);
      crm(S, u6, t6);
      for (int e = 0; e < 6; ++e) da[i][e] -= t6[e];
    }
    if (i == j && dir == 1)
      for (int e = 0; e < 6; ++e) dv[i][e] += S[e];
    const double Sw[6] = {0., 0., 0., ax[0] * qd[i], ax[1] * qd[i], ax[2] * qd[i]};
    crm(dv[i], Sw, t6);
    for (int e = 0; e < 6; ++e) da[i][e] += t6[e];
    if (i == j && dir == 1) {
      crm(Rv.v[i], S, t6);
      for (int e = 0; e < 6; ++e) da[i][e] += t6[e];
    }
    double Ida[6], Iv[6], Idv[6];
    m6v(rb.I6[i], da[i], Ida);
    m6v(rb.I6[i], Rv.v[i], Iv);
    m6v(rb.I6[i], dv[i], Idv);
    crf(dv[i], Iv, t6);
    crf(Rv.v[i], Idv, u6);
    for (int e = 0; e < 6; ++e) dF[i][e] = Ida[e] + t6[e] + u6[e];
    if (tv)
      for (int e = 0; e < 6; ++e) tv[6 * i + e] = dv[i][e], ta[6 * i + e] = da[i][e];
  }
  for (int i = nj - 1; i >= 0; --i) {
    const double* ax = rb.axis(i);
    dtau[i] = ax[0] * dF[i][3] + ax[1] * dF[i][4] + ax[2] * dF[i][5];
    const int l = rb.parent[i];
    if (l < 0) continue;
    double F[6], t6[6];
    std::memcpy(F, dF[i], sizeof(F));
    if (dir == 0 && i == j) {  // d(X F)/dq = X (S x* F)
      const double S[6] = {0., 0., 0., ax[0], ax[1], ax[2]};
      crf(S, Rv.F[i], t6);
      for (int e = 0; e < 6; ++e) F[e] += t6[e];
    }
    act_force(K.R[i], K.p[i], F, t6);
    for (int e = 0; e < 6; ++e) dF[l][e] += t6[e];
  }
}

// CRBA (Featherstone Table 6.2) + armature; M column-major nj x nj
inline void crba(const Robot& rb, const Kin& K, double* M) {
  const int nj = rb.nj;
  double Ic[kMaxJ][36], X[kMaxJ][36];
  for (int i = 0; i < nj; ++i) {
    std::memcpy(Ic[i], rb.I6[i], sizeof(Ic[i]));
    xmotion(K.R[i], K.p[i], X[i]);
  }
  for (int i = nj - 1; i >= 0; --i) {
    const int l = rb.parent[i];
    if (l < 0) continue;
    double IX[36];
    for (int c = 0; c < 6; ++c) m6v(Ic[i], X[i] + 6 * c, IX + 6 * c);
    for (int c = 0; c < 6; ++c)
      for (int r = 0; r < 6; ++r) {
        double s = 0.;
        for (int k = 0; k < 6; ++k) s += X[i][r * 6 + k] * IX[c * 6 + k];
        Ic[l][c * 6 + r] += s;
      }
  }
  std::memset(M, 0, sizeof(double) * nj * nj);
  for (int i = 0; i < nj; ++i) {
    const double* ax = rb.axis(i);
    double F[6];
    for (int r = 0; r < 6; ++r) F[r] = Ic[i][18 + r] * ax[0] + Ic[i][24 + r] * ax[1] + Ic[i][30 + r] * ax[2];
    M[i * nj + i] = ax[0] * F[3] + ax[1] * F[4] + ax[2] * F[5] + rb.arm[i];
    int j = i;
    while (rb.parent[j] >= 0) {
      double t6[6];
      act_force(K.R[j], K.p[j], F, t6);
      std::memcpy(F, t6, sizeof(F));
      j = rb.parent[j];
      const double* aj = rb.axis(j);
      M[i * nj + j] = M[j * nj + i] = aj[0] * F[3] + aj[1] * F[4] + aj[2] * F[5];
    }
  }
}

// Minv by Cholesky (M SPD); false if not positive definite
inline bool spd_inverse(const double* M, int n, double* Minv) {
  double L[kMaxJ * kMaxJ];
  for (int j = 0; j < n; ++j) {
    double d = M[j * n + j];
    for (int k = 0; k < j; ++k) d -= L[k * n + j] * L[k * n + j];
    if (!(d > 0.)) return false;
    d = std::sqrt(d);
    L[j * n + j] = d;
    for (int i = j + 1; i < n; ++i) {
      double s = M[j * n + i];
      for (int k = 0; k < j; ++k) s -= L[k * n + i] * L[k * n + j];
      L[j * n + i] = s / d;
    }
  }
  for (int c = 0; c < n; ++c) {  // solve L L^T x = e_c
    double y[kMaxJ];
    for (int i = 0; i < n; ++i) {
      double s = (i == c) ? 1. : 0.;
      for (int k = 0; k < i; ++k) s -= L[k * n + i] * y[k];
      y[i] = s / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
      double s = y[i];
      for (int k = i + 1; k < n; ++k) s -= L[i * n + k] * Minv[c * n + k];
      Minv[c * n + i] = s / L[i * n + i];
    }
  }
  return true;
}

// ---- log6 (pinocchio::log6 restated), templated for dual numbers ----------
struct Dl {
  double v, d;
  Dl(double a = 0., double b = 0.) : v(a), d(b) {}
};
inline Dl operator+(Dl a, Dl b) { return {a.v + b.v, a.d + b.d}; }
inline Dl operator-(Dl a, Dl b) { return {a.v - b.v, a.d - b.d}; }
inline Dl operator*(Dl a, Dl b) { return {a.v * b.v, a.d * b.v + a.v * b.d}; }
inline Dl operator/(Dl a, Dl b) { return {a.v / b.v, (a.d * b.v - a.v * b.d) / (b.v * b.v)}; }
inline Dl sqrt(Dl a) {
  const double s = std::sqrt(a.v);
  return {s, a.d / (2. * s)};
}
inline Dl asin(Dl a) { return {std::asin(a.v), a.d / std::sqrt(1. - a.v * a.v)}; }
inline Dl acos(Dl a) { return {std::acos(a.v), -a.d / std::sqrt(1. - a.v * a.v)}; }
inline Dl sin(Dl a) { return {std::sin(a.v), a.d * std::cos(a.v)}; }
inline Dl cos(Dl a) { return {std::cos(a.v), -a.d * std::sin(a.v)}; }
inline double val(Dl a) { return a.v; }
inline double val(double a) { return a; }

template <class T>
void log6(const T* R, const T* p, T* out) {
  using std::acos;
  using std::asin;
  using std::cos;
  using std::sin;
  using std::sqrt;
  auto at = [&](int r, int c) { return R[c * 3 + r]; };
  const T tr = at(0, 0) + at(1, 1) + at(2, 2);
  const T c = T(0.5) * (tr - T(1.));
  const T w[3] = {at(2, 1) - at(1, 2), at(0, 2) - at(2, 0), at(1, 0) - at(0, 1)};
  const T s2 = T(0.25) * (w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  T om[3];
  if (val(s2) < 1e-8 && val(c) > 0.) {
    const T k = T(0.5) * (T(1.) + s2 * T(1. / 6.) + s2 * s2 * T(3. / 40.) + s2 * s2 * s2 * T(5. / 112.));
    for (int e = 0; e < 3; ++e) om[e] = k * w[e];
  } else if (val(s2) < 1e-8) {  // near pi (value only)
    const double cv = val(c) < -1. ? -1. : val(c), th = std::acos(cv);
    double ax[3];
    int i0 = 0;
    for (int e = 0; e < 3; ++e) {
      const double t = (val(at(e, e)) - cv) / (1. - cv);
      ax[e] = t > 0. ? std::sqrt(t) : 0.;
      if (ax[e] > ax[i0]) i0 = e;
    }
    for (int e = 0; e < 3; ++e) {
      const double sg = e == i0 ? 1. : ((val(at(i0, e)) + val(at(e, i0))) >= 0. ? 1. : -1.);
      om[e] = T((val(w[i0]) < 0. ? -th : th) * sg * ax[e]);
    }
  } else {
    const T s = sqrt(s2);
    T th;
    if (val(c) > 0.5)
      th = asin(s);
    else if (val(c) < -0.5)
      th = T(M_PI) - asin(s);
    else
      th = acos(c);
    const T k = th / (T(2.) * s);
    for (int e = 0; e < 3; ++e) om[e] = k * w[e];
  }
  const T t2 = om[0] * om[0] + om[1] * om[1] + om[2] * om[2];
  T beta;
  if (val(t2) < 1e-2) {
    beta = T(1. / 12.) + t2 * T(1. / 720.) + t2 * t2 * T(1. / 30240.) + t2 * t2 * t2 * T(1. / 1209600.);
  } else {
    const T t = sqrt(t2);
    beta = T(1.) / t2 - sin(t) / (T(2.) * t * (T(1.) - cos(t)));
  }
  const T wp = om[0] * p[0] + om[1] * p[1] + om[2] * p[2];
  const T wxp[3] = {om[1] * p[2] - om[2] * p[1], om[2] * p[0] - om[0] * p[2], om[0] * p[1] - om[1] * p[0]};
  for (int e = 0; e < 3; ++e) {
    out[e] = p[e] - T(0.5) * wxp[e] + beta * (om[e] * wp - t2 * p[e]);
    out[3 + e] = om[e];
  }
}

// frame cost residual (and d r / d q_j for joint j >= 0 in the frame's support)
inline int frame_residual(const Robot& rb, const Kin& K, const double* d, int type, int j, double* r, double* Jc) {
  const int fj = (int)d[0];
  double Rf[9], pf[3], t[3];
  mm(K.oR[fj], d + 1, Rf);
  mv(K.oR[fj], d + 10, t);
  for (int e = 0; e < 3; ++e) pf[e] = K.op[fj][e] + t[e];
  double dR[9] = {0}, dp[3] = {0};
  bool sup = false;
  if (j >= 0) {
    for (int i = fj; i >= 0; i = rb.parent[i])
      if (i == j) sup = true;
    if (sup) {
      double w[3], dd[3];
      mv(K.oR[j], rb.axis(j), w);
      for (int e = 0; e < 3; ++e) dd[e] = pf[e] - K.op[j][e];
      cr(w, dd, dp);
      for (int c = 0; c < 3; ++c) cr(w, Rf + 3 * c, dR + 3 * c);
    }
  }
  if (type == C_FRAME_TRANSLATION) {
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
  log6(RD, PD, o);
  for (int e = 0; e < 6; ++e) {
    r[e] = o[e].v;
    if (Jc) Jc[e] = sup ? o[e].d : 0.;
  }
  return 6;
}

struct Costs {  // record pointers in name order
  int n = 0;
  const double* rec[64];
};
inline const double* cost_w(const double* rc, int nr) { return rc + (int)rc[3] - nr; }
inline int cost_nr(const double* rc, int nx, int nu) {
  const int t = (int)rc[0];
  if (t == 7) return (int)rc[5];
  return t == C_STATE ? nx : (t == C_CONTROL ? nu : (t == C_FRAME_PLACEMENT ? 6 : 3));
}

// The knot: parse the block, calc, calcDiff (outputs column-major, n = 2 nj, m = nj)
struct Knot {
  double dt = 0.;
  Robot rb;
  Costs cs;
  // contact section (Euler ∘ ContactFwdDynamics; contact-fwddyn.hxx:59-160)
  int nun = 0, ncon = 0, nc = 0;
  bool contact = false;
  double damping = 0.;
  const double* crec[kMaxJ];
  void parse(const double* P) {
    dt = P[0];
    const int nj = (int)P[1];
    cs.n = (int)P[2];
    rb.parse(P + 4, nj);
    const double* c = P + 4 + 3 + nj + (size_t)kJRec * nj;
    for (int k = 0; k < cs.n; ++k) {
      cs.rec[k] = c;
      c += (int)c[3];
    }
    if (c - P < (long)P[3]) {  // [nun, damping, ncontact, 0] + records
      contact = true;
      nun = (int)c[0];
      damping = c[1];
      ncon = (int)c[2];
      c += 4;
      for (int k = 0; k < ncon; ++k) {
        crec[k] = c;
        nc += (int)c[0] == 5 ? 3 : 6;
        c += (int)c[3];
      }
    }
  }
  int nu() const { return rb.nj - nun; }
  // LOCAL frame Jacobians stacked (nc x nj, row-major) and a0 at the drift
  // (Rv from RNEA(q, v, 0): joint-frame v, gravity-including a)
  void contact_terms(const Kin& K, const Rnea& Rv, double* Jc, double* a0) const {
    const int nj = rb.nj;
    int row = 0;
    for (int k = 0; k < ncon; ++k) {
      const double* rc = crec[k];
      const double* d = rc + 4;
      const int j = (int)d[0], n = (int)rc[0] == 5 ? 3 : 6;
      for (int c = 0; c < nj; ++c) {  // S_c moved from joint c to the frame
        bool sup = false;
        for (int i = j; i >= 0; i = rb.parent[i]) sup |= i == c;
        double o[6] = {0., 0., 0., 0., 0., 0.};
        if (sup) {  // X_{f <- c} S_c = actInv(oMf) oMc S_c
          double w[3], ow[3], Rf[9], pf[3], t[3], Sw[6];
          mv(K.oR[c], rb.axis(c), w);
          cr(K.op[c], w, ow);  // world motion at the origin: (op x w, w)
          mm(K.oR[j], d + 1, Rf);
          mv(K.oR[j], d + 10, t);
          for (int e = 0; e < 3; ++e) pf[e] = K.op[j][e] + t[e], Sw[e] = ow[e], Sw[3 + e] = w[e];
          act_inv(Rf, pf, Sw, o);
        }
        for (int e = 0; e < n; ++e) Jc[(row + e) * nj + c] = o[e];
      }
      double vf[6], af[6], ag[6], gl[3];
      act_inv(d + 1, d + 10, Rv.v[j], vf);
      mtv(K.oR[j], rb.g, gl);  // remove the gravity RNEA carries: a + (R^T g, 0)
      for (int e = 0; e < 6; ++e) ag[e] = Rv.a[j][e] + (e < 3 ? gl[e] : 0.);
      act_inv(d + 1, d + 10, ag, af);
      const double kp = rc[1], kd = rc[2];
      double r[6] = {0., 0., 0., 0., 0., 0.};
      if (kp != 0.) frame_residual(rb, K, d, n == 3 ? C_FRAME_TRANSLATION : C_FRAME_PLACEMENT, -1, r, nullptr);
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
  // forwardDynamics by the Schur complement: a, lambda; Y = Minv Jc^T (nj x nc),
  // Sinv (nc x nc). false if M or S is not positive definite.
  bool contact_solve(const Kin& K, const double* x, const double* u, double* a, double* lam, double* Jc, double* Mi,
                     double* Y, double* Si, Rnea& Rv) const {
    const int nj = rb.nj;
    double M[kMaxJ * kMaxJ], nle[kMaxJ], a0[kMaxJ], z6[kMaxJ] = {0.};
    crba(rb, K, M);
    bool ok = spd_inverse(M, nj, Mi);
    rnea(rb, K, x + nj, z6, Rv, nle);
    contact_terms(K, Rv, Jc, a0);
    double z[kMaxJ];
    for (int i = 0; i < nj; ++i) {
      double s = 0.;
      for (int k = 0; k < nj; ++k) s += Mi[k * nj + i] * ((k < nun ? 0. : u[k - nun]) - nle[k]);
      z[i] = s;
    }
    for (int c = 0; c < nc; ++c)
      for (int i = 0; i < nj; ++i) {
        double s = 0.;
        for (int k = 0; k < nj; ++k) s += Mi[k * nj + i] * Jc[c * nj + k];
        Y[c * nj + i] = s;
      }
    double S[kMaxJ * kMaxJ], r[kMaxJ];
    for (int c = 0; c < nc; ++c) {
      for (int rr = 0; rr < nc; ++rr) {
        double s = 0.;
        for (int i = 0; i < nj; ++i) s += Jc[rr * nj + i] * Y[c * nj + i];
        S[c * nc + rr] = s + (rr == c ? damping : 0.);
      }
      double s = 0.;
      for (int i = 0; i < nj; ++i) s += Jc[c * nj + i] * z[i];
      r[c] = s + a0[c];
    }
    if (nc > 0) ok = spd_inverse(S, nc, Si) && ok;
    for (int c = 0; c < nc; ++c) {
      double s = 0.;
      for (int k = 0; k < nc; ++k) s += Si[k * nc + c] * r[k];
      lam[c] = -s;
    }
    for (int i = 0; i < nj; ++i) {
      double s = z[i];
      for (int c = 0; c < nc; ++c) s += Y[c * nj + i] * lam[c];
      a[i] = s;
    }
    return ok;
  }
  // da0/dx along q_c (dir 0) / v_c (dir 1) from the joint tangents tv / ta
  // (contact-3d.hxx:46-71, contact-6d.hxx:48-66)
  void contact_dir(const Kin& K, const Rnea& Rv, int dir, int c, const double* tv, const double* ta,
                   double* da0) const {
    int row = 0;
    for (int k = 0; k < ncon; ++k) {
      const double* rc = crec[k];
      const double* d = rc + 4;
      const int j = (int)d[0], n = (int)rc[0] == 5 ? 3 : 6;
      double dv[6], da[6];
      for (int e = 0; e < 6; ++e) dv[e] = tv[6 * j + e], da[e] = ta[6 * j + e];
      bool sup = false;
      for (int i = j; i >= 0; i = rb.parent[i]) sup |= i == c;
      if (dir == 0 && sup) {  // gravity tangent: d(-R_j^T g)/dq_c = R_j^T (w_c x g)
        double wc[3], wg[3], t[3];
        mv(K.oR[c], rb.axis(c), wc);
        cr(wc, rb.g, wg);
        mtv(K.oR[j], wg, t);
        for (int e = 0; e < 3; ++e) da[e] -= t[e];
      }
      double dvf[6], daf[6], vf[6];
      act_inv(d + 1, d + 10, dv, dvf);
      act_inv(d + 1, d + 10, da, daf);
      act_inv(d + 1, d + 10, Rv.v[j], vf);
      const double kp = rc[1], kd = rc[2];
      double rr[6], Jk[6] = {0., 0., 0., 0., 0., 0.};
      if (kp != 0. && dir == 0 && sup)
        frame_residual(rb, K, d, n == 3 ? C_FRAME_TRANSLATION : C_FRAME_PLACEMENT, c, rr, Jk);
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
  // joint-frame external forces of the multipliers (updateForce: jMf.act(lambda))
  void contact_fext(const double* lam, double* fext) const {
    std::memset(fext, 0, sizeof(double) * 6 * rb.nj);
    int row = 0;
    for (int k = 0; k < ncon; ++k) {
      const double* d = crec[k] + 4;
      const int j = (int)d[0], n = (int)crec[k][0] == 5 ? 3 : 6;
      double f[6] = {0., 0., 0., 0., 0., 0.}, o[6];
      for (int e = 0; e < n; ++e) f[e] = lam[row + e];
      act_force(d + 1, d + 10, f, o);
      for (int e = 0; e < 6; ++e) fext[6 * j + e] += o[e];
      row += n;
    }
  }
  double cost_c(const Kin& K, const double* x, const double* u) const {
    const int nj = rb.nj, nx = 2 * nj;
    double total = 0.;
    for (int k = 0; k < cs.n; ++k) {
      const double* rc = cs.rec[k];
      const int type = (int)rc[0], nr = cost_nr(rc, nx, nu());
      const double* w = cost_w(rc, nr);
      const double* d = rc + 4;
      double r[6], a = 0.;
      if (type == C_STATE) {
        for (int i = 0; i < nx; ++i) a += w[i] * (x[i] - d[i]) * (x[i] - d[i]);
      } else if (type == C_CONTROL) {
        for (int i = 0; i < nu(); ++i) a += w[i] * (u[i] - d[i]) * (u[i] - d[i]);
      } else if (type == 7) {  // CostModelContactForce: not restated in this port (numpy oracle only)
        a = NAN;
      } else {
        frame_residual(rb, K, d, type, -1, r, nullptr);
        for (int i = 0; i < nr; ++i) a += w[i] * r[i] * r[i];
      }
      total += rc[1] * (0.5 * a);
    }
    return total;
  }
  // euler.hxx:41-80
  void calc(const double* x, const double* u, double* xnext, double* cost) const {
    const int nj = rb.nj;
    Kin K;
    kinematics(rb, x, K);
    double qdd[kMaxJ];
    if (contact) {
      double lam[kMaxJ], Jc[kMaxJ * kMaxJ], Mi[kMaxJ * kMaxJ], Y[kMaxJ * kMaxJ], Si[kMaxJ * kMaxJ];
      Rnea Rv;
      if (!contact_solve(K, x, u, qdd, lam, Jc, Mi, Y, Si, Rv))
        for (int i = 0; i < nj; ++i) qdd[i] = NAN;
    } else {
      aba(rb, K, x + nj, u, qdd);
    }
    const double cc = cost_c(K, x, u);
    if (dt != 0.) {
      for (int i = 0; i < nj; ++i) {
        xnext[i] = x[i] + (x[nj + i] * dt + qdd[i] * dt * dt);
        xnext[nj + i] = x[nj + i] + qdd[i] * dt;
      }
      *cost = dt * cc;
    } else {
      for (int i = 0; i < 2 * nj; ++i) xnext[i] = x[i];
      *cost = cc;
    }
  }
  // euler.hxx:83-131; Luu ld = m (nu_max), other blocks ld = n
  bool calc_diff(const double* x, const double* u, int m, double* Fx, double* Fu, double* Lxx, double* Lxu,
                 double* Luu, double* Lx, double* Lu) const {
    const int nj = rb.nj, n = 2 * nj;
    Kin K;
    kinematics(rb, x, K);
    double qdd[kMaxJ], M[kMaxJ * kMaxJ], Mi[kMaxJ * kMaxJ], tau[kMaxJ];
    double Jc[kMaxJ * kMaxJ], Y[kMaxJ * kMaxJ], Si[kMaxJ * kMaxJ], H[kMaxJ * kMaxJ], lam[kMaxJ], fext[6 * kMaxJ];
    bool ok;
    if (contact) {  // contact-fwddyn.hxx:107-140: Kinv blocks G = Minv - H Y^T, H = Y S^-1
      Rnea R0;
      ok = contact_solve(K, x, u, qdd, lam, Jc, Mi, Y, Si, R0);
      contact_fext(lam, fext);
      for (int c = 0; c < nc; ++c)
        for (int i = 0; i < nj; ++i) {
          double s = 0.;
          for (int k = 0; k < nc; ++k) s += Y[k * nj + i] * Si[c * nc + k];
          H[c * nj + i] = s;
        }
      for (int c = 0; c < nj; ++c)
        for (int i = 0; i < nj; ++i) {
          double s = 0.;
          for (int k = 0; k < nc; ++k) s += H[k * nj + i] * Y[k * nj + c];
          Mi[c * nj + i] -= s;
        }
    } else {
      aba(rb, K, x + nj, u, qdd);  // computeABADerivatives evaluates ABA first
      crba(rb, K, M);
      ok = spd_inverse(M, nj, Mi);
    }
    Rnea Rv;
    rnea(rb, K, x + nj, qdd, Rv, tau, contact ? fext : nullptr);
    std::memset(Fx, 0, sizeof(double) * n * n);
    std::memset(Fu, 0, sizeof(double) * n * m);
    const double dt2 = dt * dt;
    for (int c = 0; c < n; ++c) {  // da/dx column c
      double dt_[kMaxJ], da[kMaxJ], tv[6 * kMaxJ], ta[6 * kMaxJ], da0[kMaxJ];
      rnea_dir(rb, K, Rv, x + nj, c < nj ? 0 : 1, c % nj, dt_, tv, ta);
      if (contact) contact_dir(K, Rv, c < nj ? 0 : 1, c % nj, tv, ta, da0);
      for (int i = 0; i < nj; ++i) {
        double s = 0.;
        for (int k = 0; k < nj; ++k) s += Mi[k * nj + i] * dt_[k];
        if (contact)
          for (int k = 0; k < nc; ++k) s += H[k * nj + i] * da0[k];
        da[i] = ok ? -s : NAN;
      }
      for (int i = 0; i < nj; ++i) {
        if (dt != 0.) {
          Fx[c * n + i] = da[i] * dt2 + (c == nj + i ? dt : 0.) + (c == i ? 1. : 0.);
          Fx[c * n + nj + i] = da[i] * dt + (c == nj + i ? 1. : 0.);
        } else {
          Fx[c * n + i] = c == i ? 1. : 0.;
          Fx[c * n + nj + i] = c == nj + i ? 1. : 0.;
        }
      }
    }
    if (dt != 0.)
      for (int c = 0; c < nu(); ++c)
        for (int i = 0; i < nj; ++i) {
          Fu[c * n + i] = (ok ? Mi[(nun + c) * nj + i] : NAN) * dt2;
          Fu[c * n + nj + i] = (ok ? Mi[(nun + c) * nj + i] : NAN) * dt;
        }
    // cost derivatives: Gauss-Newton, cost-sum.hxx:122-160
    std::memset(Lxx, 0, sizeof(double) * n * n);
    std::memset(Lxu, 0, sizeof(double) * n * m);
    std::memset(Luu, 0, sizeof(double) * m * m);
    std::memset(Lx, 0, sizeof(double) * n);
    std::memset(Lu, 0, sizeof(double) * m);
    for (int k = 0; k < cs.n; ++k) {
      const double* rc = cs.rec[k];
      const int type = (int)rc[0], nr = cost_nr(rc, n, nu());
      const double* w = cost_w(rc, nr);
      const double* d = rc + 4;
      const double wt = rc[1];
      if (type == C_STATE) {
        for (int i = 0; i < n; ++i) {
          Lx[i] += wt * w[i] * (x[i] - d[i]);
          Lxx[i * n + i] += wt * w[i];
        }
      } else if (type == 7) {
        for (int i = 0; i < n; ++i) Lx[i] = NAN;
      } else if (type == C_CONTROL) {
        for (int i = 0; i < nu(); ++i) {
          Lu[i] += wt * w[i] * (u[i] - d[i]);
          Luu[i * m + i] += wt * w[i];
        }
      } else {
        double r[6], J[kMaxJ][6];
        for (int j = 0; j < nj; ++j) frame_residual(rb, K, d, type, j, r, J[j]);
        for (int j = 0; j < nj; ++j) {
          for (int e = 0; e < nr; ++e) Lx[j] += wt * J[j][e] * w[e] * r[e];
          for (int i = 0; i < nj; ++i) {
            double s = 0.;
            for (int e = 0; e < nr; ++e) s += J[i][e] * w[e] * J[j][e];
            Lxx[j * n + i] += wt * s;
          }
        }
      }
    }
    if (dt != 0.) {
      for (int i = 0; i < n; ++i) Lx[i] *= dt;
      for (int i = 0; i < m; ++i) Lu[i] *= dt;
      for (int i = 0; i < n * n; ++i) Lxx[i] *= dt;
      for (int i = 0; i < m * m; ++i) Luu[i] *= dt;
    }
    return ok;
  }
};

}  // namespace mbo
