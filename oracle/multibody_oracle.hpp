// ORACLE — TEST INFRASTRUCTURE ONLY. Spatial-algebra helpers of the C++ multibody
// restatement (oracle/floating_oracle.hpp, which holds the knots): 3x3 / 6D
// operations in Pinocchio's (linear, angular) convention and pinocchio::log6,
// templated so the frame-residual Jacobians come out of dual numbers.
// Pinocchio (third-party, absent offline) is restated from its published
// algorithms; parity is pinned as described in oracle/multibody_np.py.
#pragma once

#include <cmath>
#include <cstring>

namespace mbo {

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

}  // namespace mbo
