// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference hot path (Crocoddyl 1.4.0 fork at
// /root/reference): ShootingProblem::calc/calcDiff + SolverDDP/SolverFDDP.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// load this library, and only as the checker / the reported CPU baseline.
// The product (crocoddyl_amd + libfddp_hip.so) never links or calls it.
//
// Parity pinning: the reference cannot be built here (no Eigen/Boost/
// Pinocchio, empty cmake submodule) nor imported (no compiled extension),
// see SURVEY.md §8c. This restatement is pinned by the reference's own test
// designs, re-run in tests/: FDDP == dense KKT Newton solve at 1e-9
// (unittest/test_solvers.cpp:65-110), the closed-form one-step Riccati
// (unittest/python/test_solvers.py:217-271), analytic vs finite-difference
// derivatives (unittest/test_actions.cpp:70-110), and an independent numpy
// restatement (oracle/fddp_np.py) at 1e-9 (unittest/bindings/test_solvers.py).
//
// Every routine follows the reference's operation sequence; each cites the
// file:line it restates. Dense blocks are column-major as Eigen stores them.
// Parallelism: OpenMP over batch elements (mode 2) or over knots inside
// calc/calcDiff as the reference's WITH_MULTITHREADING build (mode 1,
// shooting.hxx:143-145,176-178).
// ============================================================================
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <limits>
#include <string>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/fddp_hip.h"
#include "floating_oracle.hpp"
#include "multibody_oracle.hpp"

namespace oracle {

typedef std::vector<double> Vec;

struct Mat {
  int r = 0, c = 0;
  Vec a;
  void resize(int rr, int cc) {
    r = rr;
    c = cc;
    a.assign((size_t)rr * cc, 0.0);
  }
  double& operator()(int i, int j) { return a[(size_t)j * r + i]; }
  double operator()(int i, int j) const { return a[(size_t)j * r + i]; }
};

// raiseIfNaN — src/core/solver-base.cpp:175-181
static inline bool raiseIfNaN(double v) { return std::isnan(v) || std::isinf(v) || v >= 1e30; }

// Eigen lpNorm<Infinity>
static inline double normInf(const Vec& v) {
  double m = 0.;
  for (double x : v) {
    double ax = std::fabs(x);
    if (std::isnan(ax)) return ax;
    if (ax > m) m = ax;
  }
  return m;
}
static inline double dot(const double* a, const double* b, int n) {
  double s = 0.;
  for (int i = 0; i < n; ++i) s += a[i] * b[i];
  return s;
}
// y = A x, A (r x c) col-major with leading dimension r
static inline void gemv(const double* A, int r, int c, const double* x, double* y) {
  for (int i = 0; i < r; ++i) y[i] = 0.;
  for (int j = 0; j < c; ++j) {
    const double xj = x[j];
    for (int i = 0; i < r; ++i) y[i] += A[(size_t)j * r + i] * xj;
  }
}
// y = A^T x
static inline void gemvT(const double* A, int r, int c, const double* x, double* y) {
  for (int j = 0; j < c; ++j) y[j] = dot(A + (size_t)j * r, x, r);
}
// sum_j K(i, j) dx_j of the forward pass's feedback term (fddp.cpp:199 K_[t] * dx_[t]):
// one chain in j order, as Eigen's column-major GEMV accumulates a row, and as the
// device's rollout (fddp_kernels.hpp fwd_trial). Built without reassociation: with
// -fassociative-math gcc would split this reduction over vector lanes (two partial sums).
#if defined(__GNUC__) && !defined(__clang__)
__attribute__((optimize("no-associative-math")))
#endif
static double gain_row_dot(const double* K, int ld, int i, const double* dx, int n) {
  double s = 0.;
#if defined(__clang__)
#pragma clang loop vectorize(disable)
#endif
  for (int j = 0; j < n; ++j) s = std::fma(K[(size_t)j * ld + i], dx[j], s);
  return s;
}

// ---------------------------------------------------------------------------
// Knot models. One ActionData per knot (core/action-base.hpp:101-142).
// ---------------------------------------------------------------------------
struct Data {
  double cost = 0.;
  Vec xnext;
  Mat Fx, Fu, Lxx, Lxu, Luu;
  Vec Lx, Lu;
  // IntegratedActionModelEuler extras (core/integrator/euler.hpp): dx and
  // the differential data (xout, cost, Fx nv x nx, Fu nv x nu, L*)
  Vec dx, xout;
  double cost_c = 0.;
  Mat dFx, dFu, dLxx, dLxu, dLuu;
  Vec dLx, dLu;
};

struct Model {
  int kind = 0;
  int nx = 0, ndx = 0, nu = 0;
  const double* p = nullptr;  // this element's parameter block
};

// createData — action-base.hpp:109-129 (+ unicycle.hpp:79, diff-lqr.hpp data ctor)
static void createData(const Model& m, Data& d) {
  d.cost = 0.;
  d.xnext.assign(m.nx, 0.);
  d.Fx.resize(m.ndx, m.ndx);
  d.Fu.resize(m.ndx, m.nu);
  d.Lxx.resize(m.ndx, m.ndx);
  d.Lxu.resize(m.ndx, m.nu);
  d.Luu.resize(m.nu, m.nu);
  d.Lx.assign(m.ndx, 0.);
  d.Lu.assign(m.nu, 0.);
  if (m.kind == FDDP_KNOT_UNICYCLE) {
    for (int i = 0; i < m.ndx; ++i) d.Fx(i, i) = 1.;  // unicycle.hpp:79
  }
  if (m.kind == FDDP_KNOT_EULER_DIFFLQR) {
    const int nv = m.nx / 2;
    d.dx.assign(m.ndx, 0.);
    d.xout.assign(nv, 0.);
    d.dFx.resize(nv, m.ndx);
    d.dFu.resize(nv, m.nu);
    d.dLxx.resize(m.ndx, m.ndx);
    d.dLxu.resize(m.ndx, m.nu);
    d.dLuu.resize(m.nu, m.nu);
    d.dLx.assign(m.ndx, 0.);
    d.dLu.assign(m.nu, 0.);
  }
}

// Parameter-block views (layouts declared in include/fddp_hip.h)
struct LQRView {
  bool drift_free;
  const double *Fx, *Fu, *f0, *Lxx, *Lxu, *Luu, *lx, *lu;
  LQRView(const double* p, int nx, int nu) {
    drift_free = p[0] != 0.;
    const double* q = p + FDDP_PARAM_HEADER;
    Fx = q;
    q += (size_t)nx * nx;
    Fu = q;
    q += (size_t)nx * nu;
    f0 = q;
    q += nx;
    Lxx = q;
    q += (size_t)nx * nx;
    Lxu = q;
    q += (size_t)nx * nu;
    Luu = q;
    q += (size_t)nu * nu;
    lx = q;
    q += nx;
    lu = q;
  }
};
struct DiffLQRView {
  double dt;
  bool drift_free;
  const double *Fq, *Fv, *Fu, *f0, *Lxx, *Lxu, *Luu, *lx, *lu;
  DiffLQRView(const double* p, int nx, int nu) {
    const int nq = nx / 2;
    dt = p[0];
    drift_free = p[1] != 0.;
    const double* q = p + FDDP_PARAM_HEADER;
    Fq = q;
    q += (size_t)nq * nq;
    Fv = q;
    q += (size_t)nq * nq;
    Fu = q;
    q += (size_t)nq * nu;
    f0 = q;
    q += nq;
    Lxx = q;
    q += (size_t)nx * nx;
    Lxu = q;
    q += (size_t)nx * nu;
    Luu = q;
    q += (size_t)nu * nu;
    lx = q;
    q += nx;
    lu = q;
  }
};

// quadratic cost shared by LQR and DiffLQR:
// 0.5 x.Lxx x + 0.5 u.Luu u + x.Lxu u + lx.x + lu.u   (lqr.hxx:47-48, diff-lqr.hxx:54-55)
static double lqCost(const double* Lxx, const double* Lxu, const double* Luu, const double* lx, const double* lu,
                     const double* x, const double* u, int nx, int nu) {
  Vec t1(nx), t2(nu), t3(nx);
  gemv(Lxx, nx, nx, x, t1.data());
  gemv(Luu, nu, nu, u, t2.data());
  gemv(Lxu, nx, nu, u, t3.data());
  return 0.5 * dot(x, t1.data(), nx) + 0.5 * dot(u, t2.data(), nu) + dot(x, t3.data(), nx) + dot(lx, x, nx) +
         dot(lu, u, nu);
}
// Lx = lx + Lxx x + Lxu u ; Lu = lu + Lxu^T x + Luu u   (lqr.hxx:63-64, diff-lqr.hxx:71-72)
static void lqGrad(const double* Lxx, const double* Lxu, const double* Luu, const double* lx, const double* lu,
                   const double* x, const double* u, int nx, int nu, double* Lx, double* Lu) {
  Vec a(nx), b(nx), c(nu), e(nu);
  gemv(Lxx, nx, nx, x, a.data());
  gemv(Lxu, nx, nu, u, b.data());
  for (int i = 0; i < nx; ++i) Lx[i] = lx[i] + a[i] + b[i];
  gemvT(Lxu, nx, nu, x, c.data());
  gemv(Luu, nu, nu, u, e.data());
  for (int i = 0; i < nu; ++i) Lu[i] = lu[i] + c[i] + e[i];
}

// model->calc(data, x, u) ; u == nullptr => calc(data, x) with unone_ = 0 (action-base.hxx:28-31)
static void calc(const Model& m, Data& d, const double* x, const double* u_in) {
  Vec zeros(m.nu > 0 ? m.nu : 1, 0.);
  const double* u = u_in ? u_in : zeros.data();
  switch (m.kind) {
    case FDDP_KNOT_LQR: {  // lqr.hxx:30-49
      LQRView P(m.p, m.nx, m.nu);
      Vec a(m.nx), b(m.nx);
      gemv(P.Fx, m.nx, m.nx, x, a.data());
      gemv(P.Fu, m.nx, m.nu, u, b.data());
      for (int i = 0; i < m.nx; ++i) d.xnext[i] = P.drift_free ? a[i] + b[i] : a[i] + b[i] + P.f0[i];
      d.cost = lqCost(P.Lxx, P.Lxu, P.Luu, P.lx, P.lu, x, u, m.nx, m.nu);
      break;
    }
    case FDDP_KNOT_UNICYCLE: {  // unicycle.hxx:22-40
      const double dt = m.p[0], wx = m.p[1], wu = m.p[2];
      const double c = std::cos(x[2]), s = std::sin(x[2]);
      d.xnext[0] = x[0] + c * u[0] * dt;
      d.xnext[1] = x[1] + s * u[0] * dt;
      d.xnext[2] = x[2] + u[1] * dt;
      double r[5] = {wx * x[0], wx * x[1], wx * x[2], wu * u[0], wu * u[1]};
      d.cost = 0.5 * dot(r, r, 5);
      break;
    }
    case FDDP_KNOT_EULER_DIFFLQR: {  // euler.hxx:41-80 around diff-lqr.hxx:34-56
      DiffLQRView P(m.p, m.nx, m.nu);
      const int nq = m.nx / 2, nv = nq;
      const double* q = x;
      const double* v = x + nq;
      Vec a1(nv), a2(nv), a3(nv);
      gemv(P.Fq, nq, nq, q, a1.data());
      gemv(P.Fv, nv, nv, v, a2.data());
      gemv(P.Fu, nq, m.nu, u, a3.data());
      for (int i = 0; i < nv; ++i) d.xout[i] = P.drift_free ? a1[i] + a2[i] + a3[i] : a1[i] + a2[i] + a3[i] + P.f0[i];
      d.cost_c = lqCost(P.Lxx, P.Lxu, P.Luu, P.lx, P.lu, x, u, m.nx, m.nu);
      const double dt = P.dt, dt2 = dt * dt;
      if (dt != 0.) {  // enable_integration_ (euler.hxx:32-34)
        for (int i = 0; i < nv; ++i) {
          d.dx[i] = v[i] * dt + d.xout[i] * dt2;
          d.dx[nv + i] = d.xout[i] * dt;
        }
        for (int i = 0; i < m.nx; ++i) d.xnext[i] = x[i] + d.dx[i];  // StateVector::integrate
        d.cost = dt * d.cost_c;
      } else {
        for (int i = 0; i < m.ndx; ++i) d.dx[i] = 0.;
        for (int i = 0; i < m.nx; ++i) d.xnext[i] = x[i];
        d.cost = d.cost_c;
      }
      break;
    }
    case FDDP_KNOT_EULER_FREEFWD:     // euler.hxx:41-80 around free-fwddyn.hxx:44-79 (multibody_oracle.hpp)
    case FDDP_KNOT_EULER_CONTACTFWD:  // ... or contact-fwddyn.hxx:59-104
    case FDDP_KNOT_IMPULSEFWD: {      // impulse-fwddyn.hxx:53-86
      fbo::Knot k;  // (floating_oracle.hpp: any root, every cost type)
      k.parse(m.p);
      k.calc(x, u, d.xnext.data(), &d.cost);
      break;
    }
  }
}

static void calcDiff(const Model& m, Data& d, const double* x, const double* u_in) {
  Vec zeros(m.nu > 0 ? m.nu : 1, 0.);
  const double* u = u_in ? u_in : zeros.data();
  switch (m.kind) {
    case FDDP_KNOT_LQR: {  // lqr.hxx:51-70
      LQRView P(m.p, m.nx, m.nu);
      lqGrad(P.Lxx, P.Lxu, P.Luu, P.lx, P.lu, x, u, m.nx, m.nu, d.Lx.data(), d.Lu.data());
      std::memcpy(d.Fx.a.data(), P.Fx, sizeof(double) * m.nx * m.nx);
      std::memcpy(d.Fu.a.data(), P.Fu, sizeof(double) * m.nx * m.nu);
      std::memcpy(d.Lxx.a.data(), P.Lxx, sizeof(double) * m.nx * m.nx);
      std::memcpy(d.Lxu.a.data(), P.Lxu, sizeof(double) * m.nx * m.nu);
      std::memcpy(d.Luu.a.data(), P.Luu, sizeof(double) * m.nu * m.nu);
      break;
    }
    case FDDP_KNOT_UNICYCLE: {  // unicycle.hxx:43-73
      const double dt = m.p[0], wx = m.p[1], wu = m.p[2];
      const double w_x = wx * wx, w_u = wu * wu;
      for (int i = 0; i < 3; ++i) d.Lx[i] = x[i] * w_x;
      for (int i = 0; i < 2; ++i) d.Lu[i] = u[i] * w_u;
      for (int i = 0; i < 3; ++i) d.Lxx(i, i) = w_x;
      for (int i = 0; i < 2; ++i) d.Luu(i, i) = w_u;
      const double c = std::cos(x[2]), s = std::sin(x[2]);
      d.Fx(0, 2) = -s * u[0] * dt;
      d.Fx(1, 2) = c * u[0] * dt;
      d.Fu(0, 0) = c * dt;
      d.Fu(1, 0) = s * dt;
      d.Fu(2, 1) = dt;
      break;
    }
    case FDDP_KNOT_EULER_DIFFLQR: {  // euler.hxx:83-131 around diff-lqr.hxx:59-79
      DiffLQRView P(m.p, m.nx, m.nu);
      const int nq = m.nx / 2, nv = nq, nx = m.nx, nu = m.nu;
      lqGrad(P.Lxx, P.Lxu, P.Luu, P.lx, P.lu, x, u, nx, nu, d.dLx.data(), d.dLu.data());
      for (int j = 0; j < nq; ++j)
        for (int i = 0; i < nv; ++i) {
          d.dFx(i, j) = P.Fq[(size_t)j * nq + i];
          d.dFx(i, nq + j) = P.Fv[(size_t)j * nv + i];
        }
      std::memcpy(d.dFu.a.data(), P.Fu, sizeof(double) * nv * nu);
      std::memcpy(d.dLxx.a.data(), P.Lxx, sizeof(double) * nx * nx);
      std::memcpy(d.dLxu.a.data(), P.Lxu, sizeof(double) * nx * nu);
      std::memcpy(d.dLuu.a.data(), P.Luu, sizeof(double) * nu * nu);
      const double dt = P.dt, dt2 = dt * dt;
      if (dt != 0.) {
        for (int j = 0; j < nx; ++j)
          for (int i = 0; i < nv; ++i) {
            d.Fx(i, j) = d.dFx(i, j) * dt2;       // topRows = da_dx * dt^2
            d.Fx(nv + i, j) = d.dFx(i, j) * dt;   // bottomRows = da_dx * dt
          }
        for (int i = 0; i < nv; ++i) d.Fx(i, nv + i) += dt;  // topRightCorner diag += dt
        for (int j = 0; j < nu; ++j)
          for (int i = 0; i < nv; ++i) {
            d.Fu(i, j) = d.dFu(i, j) * dt2;
            d.Fu(nv + i, j) = d.dFu(i, j) * dt;
          }
        // JintegrateTransport: no-op (euclidean.hxx:139-147); Jintegrate(first, addto): diag += 1 (:91)
        for (int i = 0; i < nx; ++i) d.Fx(i, i) += 1.;
        for (int i = 0; i < nx; ++i) d.Lx[i] = dt * d.dLx[i];
        for (int i = 0; i < nu; ++i) d.Lu[i] = dt * d.dLu[i];
        for (size_t i = 0; i < d.Lxx.a.size(); ++i) d.Lxx.a[i] = dt * d.dLxx.a[i];
        for (size_t i = 0; i < d.Lxu.a.size(); ++i) d.Lxu.a[i] = dt * d.dLxu.a[i];
        for (size_t i = 0; i < d.Luu.a.size(); ++i) d.Luu.a[i] = dt * d.dLuu.a[i];
      } else {
        // Jintegrate(x, dx, Fx, Fx) both/setto: diagonal = 1 (euclidean.hxx:78-111)
        for (int i = 0; i < nx; ++i) d.Fx(i, i) = 1.;
        std::fill(d.Fu.a.begin(), d.Fu.a.end(), 0.);
        d.Lx = d.dLx;
        d.Lu = d.dLu;
        d.Lxx.a = d.dLxx.a;
        d.Lxu.a = d.dLxu.a;
        d.Luu.a = d.dLuu.a;
      }
      break;
    }
    case FDDP_KNOT_EULER_FREEFWD:     // euler.hxx:83-131 around free-fwddyn.hxx:82-118 (multibody_oracle.hpp)
    case FDDP_KNOT_EULER_CONTACTFWD:  // ... or contact-fwddyn.hxx:107-160
    case FDDP_KNOT_IMPULSEFWD: {      // impulse-fwddyn.hxx:89-127
      fbo::Knot k;
      k.parse(m.p);
      k.calc_diff(x, u, m.nu, d.Fx.a.data(), d.Fu.a.data(), d.Lxx.a.data(), d.Lxu.a.data(), d.Luu.a.data(),
                  d.Lx.data(), d.Lu.data());
      break;
    }
  }
}

// ---------------------------------------------------------------------------
// ShootingProblem (core/optctrl/shooting.hxx) for one batch element.
// ---------------------------------------------------------------------------
struct Problem {
  int T = 0, nx = 0, ndx = 0, nu_max = 0;
  Vec x0;
  std::vector<Model> models;  // T running + terminal
  std::vector<Data> datas;
  double cost = 0.;
  int omp_knots = 0;  // reference WITH_MULTITHREADING
  // StateMultibody on SE(3) x R^n when nx != ndx (multibody.hxx:54-91), else StateVector
  fbo::State st{0, 0, false};
  bool manifold() const { return nx != ndx; }
  void diff(const double* x0, const double* x1, double* out) const {  // state->diff(x0, x1)
    if (manifold()) return st.diff(x0, x1, out);
    for (int i = 0; i < ndx; ++i) out[i] = x1[i] - x0[i];
  }
  void integrate(const double* x, const double* dx, double* out) const {  // state->integrate(x, dx)
    if (manifold()) return st.integrate(x, dx, out);
    for (int i = 0; i < nx; ++i) out[i] = x[i] + dx[i];
  }

  // shooting.hxx:133-161
  double calc(const std::vector<Vec>& xs, const std::vector<Vec>& us) {
#pragma omp parallel for if (omp_knots)
    for (int i = 0; i < T; ++i) {
      if (models[i].nu != 0)
        oracle::calc(models[i], datas[i], xs[i].data(), us[i].data());
      else
        oracle::calc(models[i], datas[i], xs[i].data(), nullptr);
    }
    oracle::calc(models[T], datas[T], xs[T].data(), nullptr);
    cost = 0.;
    for (int i = 0; i < T; ++i) cost += datas[i].cost;
    cost += datas[T].cost;
    return cost;
  }
  // shooting.hxx:164-195
  double calcDiff(const std::vector<Vec>& xs, const std::vector<Vec>& us) {
#pragma omp parallel for if (omp_knots)
    for (int i = 0; i < T; ++i) {
      if (models[i].nu != 0)
        oracle::calcDiff(models[i], datas[i], xs[i].data(), us[i].data());
      else
        oracle::calcDiff(models[i], datas[i], xs[i].data(), nullptr);
    }
    oracle::calcDiff(models[T], datas[T], xs[T].data(), nullptr);
    cost = 0.;
    for (int i = 0; i < T; ++i) cost += datas[i].cost;
    cost += datas[T].cost;
    return cost;
  }
};

constexpr int kMaxN = 256;  // largest ndx the backward's column accumulators hold

struct TraceRec {
  double cost, stop, d0, d1, xreg, ureg, steplength, is_feasible;
};


// ---------------------------------------------------------------------------
// Eigen LLT (lower) of a dense SPD matrix; false = NumericalIssue (a pivot
// <= 0 or NaN), as Eigen::LLT::info() reports it.
// ---------------------------------------------------------------------------
static bool llt(const Mat& A, Mat& L) {
  const int n = A.r;
  L.resize(n, n);
  for (int j = 0; j < n; ++j) {
    double s = A(j, j);
    for (int kk = 0; kk < j; ++kk) s -= L(j, kk) * L(j, kk);
    if (!(s > 0.)) return false;
    const double ljj = std::sqrt(s);
    L(j, j) = ljj;
    for (int i = j + 1; i < n; ++i) {
      double v = A(i, j);
      for (int kk = 0; kk < j; ++kk) v -= L(i, kk) * L(j, kk);
      L(i, j) = v / ljj;
    }
  }
  return true;
}
// L L^T y = b in place (LLT::solveInPlace)
static void llt_solve(const Mat& L, double* b) {
  const int n = L.r;
  for (int i = 0; i < n; ++i) {
    double v = b[i];
    for (int kk = 0; kk < i; ++kk) v -= L(i, kk) * b[kk];
    b[i] = v / L(i, i);
  }
  for (int i = n - 1; i >= 0; --i) {
    double v = b[i];
    for (int kk = i + 1; kk < n; ++kk) v -= L(kk, i) * b[kk];
    b[i] = v / L(i, i);
  }
}

// ---------------------------------------------------------------------------
// BoxQP — projected Newton for  min 0.5 x'Hx + q'x  s.t. lb <= x <= ub
// (src/core/solvers/box-qp.cpp:14-182, include/.../box-qp.hpp:29-206).
// ---------------------------------------------------------------------------
struct BoxQPSolution {  // box-qp.hpp:29-53
  Mat Hff_inv;
  Vec x;
  std::vector<int> free_idx, clamped_idx;
};

struct BoxQP {
  int nx = 0, maxiter = 100;
  double th_acceptstep = 0.1, th_grad = 1e-9, reg = 1e-9;
  std::vector<double> alphas;
  BoxQPSolution sol;
  std::vector<int> inv_idx;  // the free set sol.Hff_inv was factorised on (harness)
  int iters = 0;  // Newton iterations run by the last solve (diagnostic)

  // box-qp.cpp:14-46 (alphas 2^-k, k = 0..9)
  void init(int n, int mi, double ta, double tg, double rg) {
    nx = n;
    maxiter = mi;
    th_acceptstep = ta;
    th_grad = tg;
    reg = rg;
    alphas.resize(10);
    for (int k = 0; k < 10; ++k) alphas[k] = 1. / std::pow(2., (double)k);
  }

  // box-qp.cpp:51-182. Returns false where the reference throws
  // "backward_error" (the LLT of the free Hessian failed).
  bool solve(const Mat& H, const double* q, const double* lb, const double* ub, const double* xinit) {
    const int n = nx;
    Vec x(n), g(n), Hx(n), dx(n), xnew(n), Hxn(n);
    inv_idx.clear();
    for (int i = 0; i < n; ++i) x[i] = std::max(std::min(xinit[i], ub[i]), lb[i]);  // :89-91
    iters = 0;
    for (int k = 0; k < maxiter; ++k) {
      sol.clamped_idx.clear();
      sol.free_idx.clear();
      gemv(H.a.data(), n, n, x.data(), Hx.data());  // g = q + H x (:97-99)
      for (int i = 0; i < n; ++i) g[i] = q[i] + Hx[i];
      for (int j = 0; j < n; ++j) {  // :100-110
        if ((x[j] == lb[j] && g[j] > 0.) || (x[j] == ub[j] && g[j] < 0.))
          sol.clamped_idx.push_back(j);
        else
          sol.free_idx.push_back(j);
      }
      const int nf = (int)sol.free_idx.size(), nc = (int)sol.clamped_idx.size();
      if (normInf(g) <= th_grad || nf == 0) {  // :113-135
        if (k == 0) {
          Mat Hff, L;
          Hff.resize(nf, nf);
          for (int i = 0; i < nf; ++i)
            for (int j = 0; j < nf; ++j) Hff(i, j) = H(sol.free_idx[i], sol.free_idx[j]);
          if (reg != 0.)
            for (int i = 0; i < nf; ++i) Hff(i, i) += reg;
          if (!llt(Hff, L)) return false;
          sol.Hff_inv.resize(nf, nf);
          for (int j = 0; j < nf; ++j) {
            sol.Hff_inv(j, j) = 1.;
            llt_solve(L, &sol.Hff_inv.a[(size_t)j * nf]);
          }
          inv_idx = sol.free_idx;
        }
        sol.x = x;
        return true;
      }
      ++iters;
      // Newton step on the free subspace (:138-175)
      Mat Hff, Hfc, L;
      Hff.resize(nf, nf);
      Hfc.resize(nf, nc);
      Vec qf(nf), xf(nf), xc(nc), dxf(nf);
      for (int i = 0; i < nf; ++i) {
        const int fi = sol.free_idx[i];
        qf[i] = q[fi];
        xf[i] = x[fi];
        for (int j = 0; j < nf; ++j) Hff(i, j) = H(fi, sol.free_idx[j]);
        for (int j = 0; j < nc; ++j) {
          const int cj = sol.clamped_idx[j];
          xc[j] = x[cj];
          Hfc(i, j) = H(fi, cj);
        }
      }
      if (reg != 0.)
        for (int i = 0; i < nf; ++i) Hff(i, i) += reg;
      if (!llt(Hff, L)) return false;
      sol.Hff_inv.resize(nf, nf);
      for (int j = 0; j < nf; ++j) {
        sol.Hff_inv(j, j) = 1.;
        llt_solve(L, &sol.Hff_inv.a[(size_t)j * nf]);
      }
      inv_idx = sol.free_idx;
      for (int i = 0; i < nf; ++i) dxf[i] = -qf[i];
      if (nc != 0)
        for (int i = 0; i < nf; ++i) {
          double s = 0.;
          for (int j = 0; j < nc; ++j) s += Hfc(i, j) * xc[j];
          dxf[i] -= s;
        }
      llt_solve(L, dxf.data());
      for (int i = 0; i < nf; ++i) dxf[i] -= xf[i];
      std::fill(dx.begin(), dx.end(), 0.);
      for (int i = 0; i < nf; ++i) dx[sol.free_idx[i]] = dxf[i];
      // line search (:178-189)
      const double fold = 0.5 * dot(x.data(), Hx.data(), n) + dot(q, x.data(), n);
      for (double a : alphas) {
        for (int i = 0; i < n; ++i) xnew[i] = std::max(std::min(x[i] + a * dx[i], ub[i]), lb[i]);
        gemv(H.a.data(), n, n, xnew.data(), Hxn.data());
        const double fnew = 0.5 * dot(xnew.data(), Hxn.data(), n) + dot(q, xnew.data(), n);
        double gd = 0.;
        for (int i = 0; i < n; ++i) gd += g[i] * (x[i] - xnew[i]);
        if (fold - fnew > th_acceptstep * gd) {
          x = xnew;
          break;
        }
      }
    }
    sol.x = x;
    return true;
  }
};

// ---------------------------------------------------------------------------
// SolverDDP / SolverFDDP (src/core/solvers/ddp.cpp, fddp.cpp) for one element.
// ---------------------------------------------------------------------------
struct Solver {
  Problem* P = nullptr;
  fddp_params prm;
  // SolverAbstract state (solver-base.cpp:14-38)
  std::vector<Vec> xs, us;
  bool is_feasible = false;
  double cost = 0., stop = 0., xreg = NAN, ureg = NAN, steplength = 1., dV = 0., dVexp = 0.;
  double d[2] = {0., 0.};
  int iter = 0;
  // SolverDDP state (ddp.cpp:328-384)
  std::vector<Mat> Vxx, Qxx, Qxu, Quu, K, FuTVxx;
  std::vector<Vec> Vx, Qx, Qu, k, fs, xs_try, us_try, dx, Quuk;
  Mat FxTVxx;
  Vec fTVxx, xnext;
  double cost_try = 0.;
  bool was_feasible = false;
  // SolverFDDP
  double dg = 0., dq = 0., dv = 0.;
  // SolverBoxFDDP (box-fddp.cpp:15-47): limits per knot, qp_, Quu_inv_
  bool box = false;
  std::vector<Vec> ulb, uub;      // [T][nu_max] (-inf / +inf = none)
  std::vector<char> haslim;       // has_control_limits per running knot
  std::vector<Mat> Quu_inv;
  BoxQP qp;
  // bookkeeping for the harness
  int status = FDDP_STATUS_RUNNING;
  int n_iter_run = 0;
  std::vector<TraceRec> trace;
  // phase timers (CLOCK_MONOTONIC, as core/utils/timer.hpp:16-40): seconds spent in
  // the iteration-0 calc, calcDiff + gaps, the backward pass, the forward passes
  double ph[4] = {0., 0., 0., 0.};
  static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }

  void init(Problem* prob, const fddp_params& p) {
    P = prob;
    prm = p;
    const int T = P->T, ndx = P->ndx, nu = P->nu_max, nx = P->nx;
    xs.assign(T + 1, Vec(nx, 0.));
    us.assign(T, Vec(nu, 0.));
    Vxx.resize(T + 1);
    Vx.resize(T + 1);
    Qxx.resize(T);
    Qxu.resize(T);
    Quu.resize(T);
    Qx.resize(T);
    Qu.resize(T);
    K.resize(T);
    k.resize(T);
    fs.resize(T + 1);
    xs_try.resize(T + 1);
    us_try.resize(T);
    dx.resize(T + 1);
    FuTVxx.resize(T);
    Quuk.resize(T);
    for (int t = 0; t < T; ++t) {
      const int nut = P->models[t].nu;
      Vxx[t].resize(ndx, ndx);
      Vx[t].assign(ndx, 0.);
      Qxx[t].resize(ndx, ndx);
      Qxu[t].resize(ndx, nut);
      Quu[t].resize(nut, nut);
      Qx[t].assign(ndx, 0.);
      Qu[t].assign(nut, 0.);
      K[t].resize(nut, ndx);
      k[t].assign(nut, 0.);
      fs[t].assign(ndx, 0.);
      xs_try[t] = (t == 0) ? P->x0 : Vec(nx, 0.);
      us_try[t].assign(nu, 0.);
      dx[t].assign(ndx, 0.);
      FuTVxx[t].resize(nut, ndx);
      Quuk[t].assign(nut, 0.);
    }
    Vxx[T].resize(ndx, ndx);
    Vx[T].assign(ndx, 0.);
    xs_try[T].assign(nx, 0.);
    fs[T].assign(ndx, 0.);
    dx[T].assign(ndx, 0.);
    FxTVxx.resize(ndx, ndx);
    fTVxx.assign(ndx, 0.);
    xnext.assign(nx, 0.);
    // SolverBoxFDDP: qp_(runningModels[0]->nu, 100, 0.1, 1e-5, 0.) (box-fddp.cpp:16)
    qp.init(P->models[0].nu, 100, 0.1, 1e-5, 0.);
    Quu_inv.resize(T);
    for (int t = 0; t < T; ++t) Quu_inv[t].resize(nu, nu);
    ulb.assign(T, Vec(nu, -INFINITY));
    uub.assign(T, Vec(nu, INFINITY));
    haslim.assign(T, 0);
  }

  // per-knot buffers after the model at knot t changed (fddp_set_knots):
  // sized by the new nu as Eigen's resizing assignments leave them; k keeps
  // its first entries (the box QP's warm start reads them)
  void resize_knot(int t, int nut) {
    const int ndx = P->ndx;
    if (Quu[t].r == nut) return;
    Qxu[t].resize(ndx, nut);
    Quu[t].resize(nut, nut);
    K[t].resize(nut, ndx);
    FuTVxx[t].resize(nut, ndx);
    Qu[t].assign(nut, 0.);
    Quuk[t].assign(nut, 0.);
    k[t].resize(nut, 0.);
  }

  // solver-base.cpp:42-67 (xs_warm / us_warm may be null => zeros)
  void setCandidate(const double* xs_warm, const double* us_warm, bool feasible) {
    const int T = P->T, nx = P->nx, nu = P->nu_max;
    for (int t = 0; t <= T; ++t)
      for (int i = 0; i < nx; ++i) xs[t][i] = xs_warm ? xs_warm[(size_t)t * nx + i] : 0.;
    if (!xs_warm && P->manifold())  // state->zero(): the neutral configuration
      for (int t = 0; t <= T; ++t) xs[t][6] = 1.;
    for (int t = 0; t < T; ++t)
      for (int i = 0; i < nu; ++i) us[t][i] = us_warm ? us_warm[(size_t)t * nu + i] : 0.;
    is_feasible = feasible;
  }
  void setCandidateTry(bool feasible) {
    for (int t = 0; t <= P->T; ++t) xs[t] = xs_try[t];
    for (int t = 0; t < P->T; ++t) us[t] = us_try[t];
    is_feasible = feasible;
  }

  // ddp.cpp:157-178
  double calcDiff() {
    const double t0 = now();
    if (iter == 0) P->calc(xs, us);
    const double t1 = now();
    cost = P->calcDiff(xs, us);
    const int T = P->T, ndx = P->ndx;
    if (!is_feasible) {
      P->diff(xs[0].data(), P->x0.data(), fs[0].data());  // diff(xs[0], x0)
      for (int t = 0; t < T; ++t) P->diff(xs[t + 1].data(), P->datas[t].xnext.data(), fs[t + 1].data());
      (void)ndx;
    } else if (!was_feasible) {
      for (auto& f : fs) std::fill(f.begin(), f.end(), 0.);
    }
    ph[0] += t1 - t0;
    ph[1] += now() - t1;
    return cost;
  }

  // SolverBoxFDDP::computeGains (box-fddp.cpp:48-79)
  bool computeGainsBox(int t) {
    const int nu = P->models[t].nu;
    if (nu <= 0) return true;
    if (!haslim[t] || !is_feasible) return computeGainsDDP(t);  // vanilla DDP gains
    // qp_ has runningModels[0]->nu variables; BoxQP::solve throws on any other
    // size (box-qp.cpp:53-72) and solve() catches every exception as a
    // backward_error (fddp.cpp:37-38)
    if (nu != qp.nx) return false;
    const int n = P->ndx;
    Vec dlb(nu), dub(nu);
    for (int i = 0; i < nu; ++i) {
      dlb[i] = ulb[t][i] - us[t][i];
      dub[i] = uub[t][i] - us[t][i];
    }
    if (!qp.solve(Quu[t], Qu[t].data(), dlb.data(), dub.data(), k[t].data())) return false;
    const BoxQPSolution& sol = qp.sol;
    // Quu_inv(free_i, free_j) = Hff_inv(i, j). Hff_inv is the one of the last
    // Newton iteration; when the QP converges at k > 0 the free set may have
    // changed since, and the reference then indexes Hff_inv by position
    // (beyond its size is out of bounds in Eigen: taken as 0 here).
    Mat& Qi = Quu_inv[t];
    std::fill(Qi.a.begin(), Qi.a.end(), 0.);
    const int nf = (int)sol.free_idx.size(), ni = sol.Hff_inv.r;
    for (int i = 0; i < nf; ++i)
      for (int j = 0; j < nf; ++j) Qi(sol.free_idx[i], sol.free_idx[j]) = (i < ni && j < ni) ? sol.Hff_inv(i, j) : 0.;
    for (int j = 0; j < n; ++j)  // K = Quu_inv Qxu^T
      for (int i = 0; i < nu; ++i) {
        double s = 0.;
        for (int l = 0; l < nu; ++l) s += Qi(i, l) * Qxu[t](j, l);
        K[t](i, j) = s;
      }
    for (int i = 0; i < nu; ++i) k[t][i] = -sol.x[i];
    for (int c : sol.clamped_idx) Qu[t][c] = 0.;
    return true;
  }
  bool computeGains(int t) { return box ? computeGainsBox(t) : computeGainsDDP(t); }

  // ddp.cpp:298-310 — Eigen LLT (lower) + solveInPlace
  bool computeGainsDDP(int t) {
    const int nu = P->models[t].nu;
    if (nu <= 0) return true;
    const int n = P->ndx;
    Mat L;
    L.resize(nu, nu);
    const Mat& A = Quu[t];
    for (int j = 0; j < nu; ++j) {
      double s = A(j, j);
      for (int kk = 0; kk < j; ++kk) s -= L(j, kk) * L(j, kk);
      if (!(s > 0.)) return false;  // Eigen: NumericalIssue when pivot <= 0
      const double ljj = std::sqrt(s);
      L(j, j) = ljj;
      for (int i = j + 1; i < nu; ++i) {
        double v = A(i, j);
        for (int kk = 0; kk < j; ++kk) v -= L(i, kk) * L(j, kk);
        L(i, j) = v / ljj;
      }
    }
    auto solve = [&](double* b) {  // L L^T y = b
      for (int i = 0; i < nu; ++i) {
        double v = b[i];
        for (int kk = 0; kk < i; ++kk) v -= L(i, kk) * b[kk];
        b[i] = v / L(i, i);
      }
      for (int i = nu - 1; i >= 0; --i) {
        double v = b[i];
        for (int kk = i + 1; kk < nu; ++kk) v -= L(kk, i) * b[kk];
        b[i] = v / L(i, i);
      }
    };
    // K = Qxu^T ; solveInPlace
    for (int j = 0; j < n; ++j) {
      for (int i = 0; i < nu; ++i) K[t](i, j) = Qxu[t](j, i);
      solve(&K[t].a[(size_t)j * nu]);
    }
    k[t] = Qu[t];
    solve(k[t].data());
    return true;
  }

  // ddp.cpp:180-253 ; returns false on backward_error
  bool backwardPass() {
    const int T = P->T, n = P->ndx;
    const Data& dT = P->datas[T];
    Vxx[T].a = dT.Lxx.a;
    Vx[T] = dT.Lx;
    if (!std::isnan(xreg))
      for (int i = 0; i < n; ++i) Vxx[T](i, i) += xreg;
    if (!is_feasible) {
      Vec tmp(n);
      gemv(Vxx[T].a.data(), n, n, fs[T].data(), tmp.data());
      for (int i = 0; i < n; ++i) Vx[T][i] += tmp[i];
    }
    for (int t = T - 1; t >= 0; --t) {
      const Data& d = P->datas[t];
      const Mat& Vxx_p = Vxx[t + 1];
      const Vec& Vx_p = Vx[t + 1];
      const int nu = P->models[t].nu;
      Qxx[t].a = d.Lxx.a;
      Qx[t] = d.Lx;
      // FxTVxx = Fx^T Vxx'
      for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) FxTVxx(i, j) = dot(&d.Fx.a[(size_t)i * n], &Vxx_p.a[(size_t)j * n], n);
      // Qxx += FxTVxx Fx (column axpys: the same summation order per entry)
      for (int j = 0; j < n; ++j) {
        double* q = &Qxx[t].a[(size_t)j * n];
        double acc[kMaxN];
        for (int i = 0; i < n; ++i) acc[i] = 0.;
        for (int kk = 0; kk < n; ++kk) {
          const double f = d.Fx(kk, j);
          const double* c = &FxTVxx.a[(size_t)kk * n];
          for (int i = 0; i < n; ++i) acc[i] += c[i] * f;
        }
        for (int i = 0; i < n; ++i) q[i] += acc[i];
      }
      // Qx += Fx^T Vx'
      {
        Vec tmp(n);
        gemvT(d.Fx.a.data(), n, n, Vx_p.data(), tmp.data());
        for (int i = 0; i < n; ++i) Qx[t][i] += tmp[i];
      }
      if (nu != 0) {
        Qxu[t].a = d.Lxu.a;
        Quu[t].a = d.Luu.a;
        Qu[t] = d.Lu;
        for (int j = 0; j < n; ++j)
          for (int i = 0; i < nu; ++i) FuTVxx[t](i, j) = dot(&d.Fu.a[(size_t)i * n], &Vxx_p.a[(size_t)j * n], n);
        for (int j = 0; j < nu; ++j) {
          double acc[kMaxN];
          for (int i = 0; i < n; ++i) acc[i] = 0.;
          for (int kk = 0; kk < n; ++kk) {
            const double f = d.Fu(kk, j);
            const double* c = &FxTVxx.a[(size_t)kk * n];
            for (int i = 0; i < n; ++i) acc[i] += c[i] * f;
          }
          for (int i = 0; i < n; ++i) Qxu[t](i, j) += acc[i];
        }
        for (int j = 0; j < nu; ++j) {
          double acc[kMaxN];
          for (int i = 0; i < nu; ++i) acc[i] = 0.;
          for (int kk = 0; kk < n; ++kk) {
            const double f = d.Fu(kk, j);
            const double* c = &FuTVxx[t].a[(size_t)kk * nu];
            for (int i = 0; i < nu; ++i) acc[i] += c[i] * f;
          }
          for (int i = 0; i < nu; ++i) Quu[t](i, j) += acc[i];
        }
        Vec tmp(nu);
        gemvT(d.Fu.a.data(), n, nu, Vx_p.data(), tmp.data());
        for (int i = 0; i < nu; ++i) Qu[t][i] += tmp[i];
        if (!std::isnan(ureg))
          for (int i = 0; i < nu; ++i) Quu[t](i, i) += ureg;
      }
      if (!computeGains(t)) return false;
      Vx[t] = Qx[t];
      Vxx[t].a = Qxx[t].a;
      if (nu != 0) {
        if (std::isnan(ureg)) {
          for (int i = 0; i < n; ++i) Vx[t][i] -= dot(&K[t].a[(size_t)i * nu], Qu[t].data(), nu);
        } else {
          gemv(Quu[t].a.data(), nu, nu, k[t].data(), Quuk[t].data());
          for (int i = 0; i < n; ++i) Vx[t][i] += dot(&K[t].a[(size_t)i * nu], Quuk[t].data(), nu);
          for (int i = 0; i < n; ++i) Vx[t][i] -= 2 * dot(&K[t].a[(size_t)i * nu], Qu[t].data(), nu);
        }
        for (int j = 0; j < n; ++j) {
          double acc[kMaxN];
          for (int i = 0; i < n; ++i) acc[i] = 0.;
          for (int kk = 0; kk < nu; ++kk) {
            const double f = K[t](kk, j);
            const double* c = &Qxu[t].a[(size_t)kk * n];
            for (int i = 0; i < n; ++i) acc[i] += c[i] * f;
          }
          for (int i = 0; i < n; ++i) Vxx[t](i, j) -= acc[i];
        }
      }
      // Vxx = 0.5 (Vxx + Vxx^T)
      {
        Mat S;
        S.resize(n, n);
        for (int j = 0; j < n; ++j)
          for (int i = 0; i < n; ++i) S(i, j) = 0.5 * (Vxx[t](i, j) + Vxx[t](j, i));
        Vxx[t].a = S.a;
      }
      if (!std::isnan(xreg))
        for (int i = 0; i < n; ++i) Vxx[t](i, i) += xreg;
      if (!is_feasible) {
        Vec tmp(n);
        gemv(Vxx[t].a.data(), n, n, fs[t].data(), tmp.data());
        for (int i = 0; i < n; ++i) Vx[t][i] += tmp[i];
      }
      if (raiseIfNaN(normInf(Vx[t]))) return false;
      if (raiseIfNaN(normInf(Vxx[t].a))) return false;
    }
    return true;
  }

  // ddp.cpp:120-125 ; false on backward_error
  bool computeDirection(bool recalc) {
    if (recalc) calcDiff();
    const double t0 = now();
    const bool ok = backwardPass();
    ph[2] += now() - t0;
    return ok;
  }

  // fddp.cpp:149-225 ; false on forward_error
  bool forwardPass(double alpha) {
    const int T = P->T, n = P->ndx;
    cost_try = 0.;
    xnext = P->x0;
    for (int t = 0; t < T; ++t) {
      const Model& m = P->models[t];
      Data& d = P->datas[t];
      if (is_feasible || alpha == 1) {
        xs_try[t] = xnext;
      } else {
        for (int i = 0; i < n; ++i) dx[t][i] = fs[t][i] * (alpha - 1);  // integrate(xnext, fs (alpha - 1))
        P->integrate(xnext.data(), dx[t].data(), xs_try[t].data());
      }
      P->diff(xs[t].data(), xs_try[t].data(), dx[t].data());  // diff(xs, xs_try)
      if (m.nu != 0) {
        for (int i = 0; i < m.nu; ++i) {
          const double v = std::fma(-k[t][i], alpha, us[t][i]);  // us - k alpha (contracted, as the device)
          us_try[t][i] = v - gain_row_dot(K[t].a.data(), K[t].r, i, dx[t].data(), n);
          // SolverBoxFDDP::forwardPass clamps (box-fddp.cpp:100-102):
          // cwiseMax(u_lb).cwiseMin(u_ub)
          if (box && haslim[t]) us_try[t][i] = std::min(std::max(us_try[t][i], ulb[t][i]), uub[t][i]);
        }
        oracle::calc(m, d, xs_try[t].data(), us_try[t].data());
      } else {
        oracle::calc(m, d, xs_try[t].data(), nullptr);
      }
      xnext = d.xnext;
      cost_try += d.cost;
      if (raiseIfNaN(cost_try)) return false;
      if (raiseIfNaN(normInf(xnext))) return false;
    }
    const Model& m = P->models[T];
    Data& d = P->datas[T];
    if (is_feasible || alpha == 1) {
      xs_try[T] = xnext;
    } else {
      for (int i = 0; i < n; ++i) dx[T][i] = fs[T][i] * (alpha - 1);
      P->integrate(xnext.data(), dx[T].data(), xs_try[T].data());
    }
    oracle::calc(m, d, xs_try[T].data(), nullptr);
    cost_try += d.cost;
    if (raiseIfNaN(cost_try)) return false;
    return true;
  }
  bool tryStep(double alpha, double* dVout) {
    const double t0 = now();
    const bool ok = forwardPass(alpha);
    ph[3] += now() - t0;
    if (!ok) return false;
    *dVout = cost - cost_try;
    return true;
  }

  // fddp.cpp:107-124
  void expectedImprovement() {
    dv = 0.;
    const int T = P->T, n = P->ndx;
    if (!is_feasible) {
      P->diff(xs_try[T].data(), xs[T].data(), dx[T].data());  // diff(xs_try, xs)
      gemv(Vxx[T].a.data(), n, n, dx[T].data(), fTVxx.data());
      dv -= dot(fs[T].data(), fTVxx.data(), n);
      for (int t = 0; t < T; ++t) {
        P->diff(xs_try[t].data(), xs[t].data(), dx[t].data());
        gemv(Vxx[t].a.data(), n, n, dx[t].data(), fTVxx.data());
        dv -= dot(fs[t].data(), fTVxx.data(), n);
      }
    }
    d[0] = dg + dv;
    d[1] = dq - 2 * dv;
  }
  // fddp.cpp:126-147
  void updateExpectedImprovement() {
    dg = 0.;
    dq = 0.;
    const int T = P->T, n = P->ndx;
    if (!is_feasible) {
      dg -= dot(Vx[T].data(), fs[T].data(), n);
      gemv(Vxx[T].a.data(), n, n, fs[T].data(), fTVxx.data());
      dq += dot(fs[T].data(), fTVxx.data(), n);
    }
    for (int t = 0; t < T; ++t) {
      const int nu = P->models[t].nu;
      if (nu != 0) {
        dg += dot(Qu[t].data(), k[t].data(), nu);
        dq -= dot(k[t].data(), Quuk[t].data(), nu);
      }
      if (!is_feasible) {
        dg -= dot(Vx[t].data(), fs[t].data(), n);
        gemv(Vxx[t].a.data(), n, n, fs[t].data(), fTVxx.data());
        dq += dot(fs[t].data(), fTVxx.data(), n);
      }
    }
  }
  // ddp.cpp:132-142
  double stoppingCriteria() {
    stop = 0.;
    for (int t = 0; t < P->T; ++t)
      if (P->models[t].nu != 0) stop += dot(Qu[t].data(), Qu[t].data(), P->models[t].nu);
    return stop;
  }
  // ddp.cpp:312-326
  void increaseRegularization() {
    xreg *= prm.regfactor;
    if (xreg > prm.regmax) xreg = prm.regmax;
    ureg = xreg;
  }
  void decreaseRegularization() {
    xreg /= prm.regfactor;
    if (xreg < prm.regmin) xreg = prm.regmin;
    ureg = xreg;
  }

  // fddp.cpp:19-105 (from the current candidate; setCandidate done by caller)
  bool solve(int maxiter, bool feasible, double reginit) {
    xs_try[0] = P->x0;
    is_feasible = feasible;
    if (std::isnan(reginit)) {
      xreg = prm.regmin;
      ureg = prm.regmin;
    } else {
      xreg = reginit;
      ureg = reginit;
    }
    was_feasible = false;
    status = FDDP_STATUS_RUNNING;
    n_iter_run = 0;
    trace.clear();
    bool recalcDiff = true;
    for (iter = 0; iter < maxiter; ++iter) {
      ++n_iter_run;
      while (true) {
        if (!computeDirection(recalcDiff)) {
          recalcDiff = false;
          increaseRegularization();
          if (xreg == prm.regmax) {
            status = FDDP_STATUS_REGMAX;
            return false;
          }
          continue;
        }
        break;
      }
      updateExpectedImprovement();
      recalcDiff = false;
      for (int a = 0; a < prm.n_alphas; ++a) {
        steplength = prm.alphas[a];
        double dVt;
        if (!tryStep(steplength, &dVt)) continue;
        dV = dVt;
        expectedImprovement();
        dVexp = steplength * (d[0] + 0.5 * steplength * d[1]);
        if (dVexp >= 0) {
          if (d[0] < prm.th_grad || dV > prm.th_acceptstep * dVexp) {
            was_feasible = is_feasible;
            setCandidateTry(was_feasible || steplength == 1);
            cost = cost_try;
            recalcDiff = true;
            break;
          }
        } else {
          if (dV > prm.th_acceptnegstep * dVexp) {
            was_feasible = is_feasible;
            setCandidateTry(was_feasible || steplength == 1);
            cost = cost_try;
            recalcDiff = true;
            break;
          }
        }
      }
      if (steplength > prm.th_stepdec) decreaseRegularization();
      if (steplength <= prm.th_stepinc) {
        increaseRegularization();
        if (xreg == prm.regmax) {
          status = FDDP_STATUS_REGMAX;
          return false;
        }
      }
      stoppingCriteria();
      trace.push_back({cost, stop, d[0], d[1], xreg, ureg, steplength, is_feasible ? 1. : 0.});
      if (was_feasible && stop < prm.th_stop) {
        status = FDDP_STATUS_CONVERGED;
        return true;
      }
    }
    return false;
  }
};

}  // namespace oracle

// ============================================================================
// C ABI mirroring include/fddp_hip.h with an `oracle_` prefix.
// ============================================================================
using namespace oracle;

struct oracle_handle {
  fddp_dims dims;
  std::vector<fddp_knot_desc> knots;
  std::vector<double> params;
  std::vector<Problem> problems;
  std::vector<Solver> solvers;
  fddp_params prm;
  int mode = 2;  // 1: OpenMP over knots (reference), 2: OpenMP over batch elements
  int nthreads = 1;
};

static thread_local std::string g_err;
extern "C" void oracle_default_params(fddp_params* p);

extern "C" {

const char* oracle_last_error(void) { return g_err.c_str(); }

static void bind_models(oracle_handle* h) {
  const fddp_dims& D = h->dims;
  for (int b = 0; b < D.B; ++b) {
    Problem& P = h->problems[b];
    for (int t = 0; t <= D.T; ++t) {
      const fddp_knot_desc& kd = h->knots[t];
      P.models[t].p = h->params.data() + kd.param_offset + (int64_t)b * kd.param_stride;
    }
  }
}

int oracle_create(const fddp_dims* dims, const fddp_knot_desc* knots, const double* params, int64_t n_params,
                  oracle_handle** out) {
  if (!dims || !knots || !params || !out || dims->T < 1 || dims->B < 1 || dims->nx < 1 || dims->ndx > kMaxN || dims->nu_max > kMaxN ||
      (dims->nx != dims->ndx && (dims->nx != dims->ndx + 1 || dims->ndx % 2 || dims->ndx < 12))) {
    g_err = "oracle_create: invalid argument";
    return FDDP_ERR_INVALID_ARG;
  }
  if (dims->nx != dims->ndx)
    for (int t = 0; t <= dims->T; ++t)
      if (knots[t].kind < FDDP_KNOT_EULER_FREEFWD || knots[t].kind > FDDP_KNOT_IMPULSEFWD) {
        g_err = "oracle_create: free-flyer states are restated for the multibody knots only";
        return FDDP_ERR_INVALID_ARG;
      }
  auto* h = new oracle_handle();
  h->dims = *dims;
  h->knots.assign(knots, knots + dims->T + 1);
  h->params.assign(params, params + n_params);
  oracle_default_params(&h->prm);
  h->problems.resize(dims->B);
  h->solvers.resize(dims->B);
  for (int b = 0; b < dims->B; ++b) {
    Problem& P = h->problems[b];
    P.T = dims->T;
    P.nx = dims->nx;
    P.ndx = dims->ndx;
    P.nu_max = dims->nu_max;
    P.x0.assign(dims->nx, 0.);
    P.st = fbo::State{dims->nx - dims->ndx / 2, dims->ndx / 2, dims->nx != dims->ndx};
    P.models.resize(dims->T + 1);
    P.datas.resize(dims->T + 1);
    for (int t = 0; t <= dims->T; ++t) {
      Model& m = P.models[t];
      m.kind = knots[t].kind;
      m.nx = dims->nx;
      m.ndx = dims->ndx;
      m.nu = knots[t].nu;
    }
  }
  bind_models(h);
  for (int b = 0; b < dims->B; ++b) {
    Problem& P = h->problems[b];
    for (int t = 0; t <= dims->T; ++t) createData(P.models[t], P.datas[t]);
    h->solvers[b].init(&P, h->prm);
  }
  *out = h;
  return FDDP_OK;
}

void oracle_destroy(oracle_handle* h) { delete h; }

int oracle_set_threading(oracle_handle* h, int mode, int nthreads) {
  h->mode = mode;
  h->nthreads = nthreads > 0 ? nthreads : 1;
  for (auto& P : h->problems) P.omp_knots = (mode == 1 && h->nthreads > 1) ? 1 : 0;
#ifdef _OPENMP
  omp_set_num_threads(h->nthreads);
#endif
  return FDDP_OK;
}

int oracle_set_x0(oracle_handle* h, const double* x0) {
  for (int b = 0; b < h->dims.B; ++b)
    for (int i = 0; i < h->dims.nx; ++i) h->problems[b].x0[i] = x0[(size_t)b * h->dims.nx + i];
  return FDDP_OK;
}

int oracle_set_params(oracle_handle* h, const fddp_params* p) {
  h->prm = *p;
  for (auto& s : h->solvers) s.prm = *p;
  return FDDP_OK;
}

int oracle_set_candidate(oracle_handle* h, const double* xs, const double* us, int is_feasible) {
  const fddp_dims& D = h->dims;
  const size_t sx = (size_t)(D.T + 1) * D.nx, su = (size_t)D.T * D.nu_max;
  for (int b = 0; b < D.B; ++b)
    h->solvers[b].setCandidate(xs ? xs + b * sx : nullptr, us ? us + b * su : nullptr, is_feasible != 0);
  return FDDP_OK;
}

static void fill_result(const Solver& s, fddp_result* r) {
  r->status = s.status;
  r->iter = s.iter;
  r->is_feasible = s.is_feasible;
  r->n_iter_run = s.n_iter_run;
  r->cost = s.cost;
  r->stop = s.stop;
  r->xreg = s.xreg;
  r->ureg = s.ureg;
  r->steplength = s.steplength;
  r->dV = s.dV;
  r->dVexp = s.dVexp;
  r->d0 = s.d[0];
  r->d1 = s.d[1];
}

int oracle_solve(oracle_handle* h, int maxiter, int is_feasible, double reg_init, fddp_result* out) {
  const int B = h->dims.B;
  if (h->mode == 2) {
#pragma omp parallel for schedule(dynamic, 1) num_threads(h->nthreads)
    for (int b = 0; b < B; ++b) h->solvers[b].solve(maxiter, is_feasible != 0, reg_init);
  } else {
    for (int b = 0; b < B; ++b) h->solvers[b].solve(maxiter, is_feasible != 0, reg_init);
  }
  if (out)
    for (int b = 0; b < B; ++b) fill_result(h->solvers[b], &out[b]);
  return FDDP_OK;
}

// Phase times summed over the elements (seconds of thread time): the iteration-0 calc,
// calcDiff + gaps, the backward passes, the forward passes (line-search trials);
// reset != 0 zeroes them afterwards.
int oracle_get_phase_times(oracle_handle* h, double* out, int reset) {
  for (int i = 0; i < 4; ++i) out[i] = 0.;
  for (auto& s : h->solvers)
    for (int i = 0; i < 4; ++i) {
      out[i] += s.ph[i];
      if (reset) s.ph[i] = 0.;
    }
  return FDDP_OK;
}

int oracle_get_results(oracle_handle* h, fddp_result* out) {
  for (int b = 0; b < h->dims.B; ++b) fill_result(h->solvers[b], &out[b]);
  return FDDP_OK;
}

int oracle_get_xs(oracle_handle* h, double* out) {
  const fddp_dims& D = h->dims;
  for (int b = 0; b < D.B; ++b)
    for (int t = 0; t <= D.T; ++t)
      std::memcpy(out + ((size_t)b * (D.T + 1) + t) * D.nx, h->solvers[b].xs[t].data(), sizeof(double) * D.nx);
  return FDDP_OK;
}
int oracle_get_us(oracle_handle* h, double* out) {
  const fddp_dims& D = h->dims;
  for (int b = 0; b < D.B; ++b)
    for (int t = 0; t < D.T; ++t)
      std::memcpy(out + ((size_t)b * D.T + t) * D.nu_max, h->solvers[b].us[t].data(), sizeof(double) * D.nu_max);
  return FDDP_OK;
}
int oracle_get_xs_try(oracle_handle* h, double* out) {
  const fddp_dims& D = h->dims;
  for (int b = 0; b < D.B; ++b)
    for (int t = 0; t <= D.T; ++t)
      std::memcpy(out + ((size_t)b * (D.T + 1) + t) * D.nx, h->solvers[b].xs_try[t].data(), sizeof(double) * D.nx);
  return FDDP_OK;
}
int oracle_get_us_try(oracle_handle* h, double* out) {
  const fddp_dims& D = h->dims;
  for (int b = 0; b < D.B; ++b)
    for (int t = 0; t < D.T; ++t)
      std::memcpy(out + ((size_t)b * D.T + t) * D.nu_max, h->solvers[b].us_try[t].data(), sizeof(double) * D.nu_max);
  return FDDP_OK;
}

int oracle_problem_calc(oracle_handle* h, double* cost) {
  for (int b = 0; b < h->dims.B; ++b) {
    Solver& s = h->solvers[b];
    double c = h->problems[b].calc(s.xs, s.us);
    if (cost) cost[b] = c;
  }
  return FDDP_OK;
}
int oracle_problem_calc_diff(oracle_handle* h, double* cost) {
  for (int b = 0; b < h->dims.B; ++b) {
    Solver& s = h->solvers[b];
    double c = h->problems[b].calcDiff(s.xs, s.us);
    if (cost) cost[b] = c;
  }
  return FDDP_OK;
}
// Solver state for the step API (iter_ == 0, regularisation as set).
int oracle_set_solver_state(oracle_handle* h, int iter, double xreg, double ureg, int was_feasible) {
  for (auto& s : h->solvers) {
    s.iter = iter;
    s.xreg = xreg;
    s.ureg = ureg;
    s.was_feasible = was_feasible != 0;
  }
  return FDDP_OK;
}
int oracle_compute_direction(oracle_handle* h, int recalc, int32_t* status) {
  for (int b = 0; b < h->dims.B; ++b) {
    bool ok = h->solvers[b].computeDirection(recalc != 0);
    if (status) status[b] = ok ? 0 : 1;
  }
  return FDDP_OK;
}
// SolverDDP::calcDiff (ddp.cpp:157-178)
int oracle_calc_diff(oracle_handle* h, double* cost) {
  for (int b = 0; b < h->dims.B; ++b) {
    const double c = h->solvers[b].calcDiff();
    if (cost) cost[b] = c;
  }
  return FDDP_OK;
}
// SolverDDP::backwardPass (ddp.cpp:180-253)
int oracle_backward_pass(oracle_handle* h, int32_t* status) {
  for (int b = 0; b < h->dims.B; ++b) {
    const bool ok = h->solvers[b].backwardPass();
    if (status) status[b] = ok ? 0 : 1;
  }
  return FDDP_OK;
}
// SolverFDDP::forwardPass (fddp.cpp:149-225)
int oracle_forward_pass(oracle_handle* h, double alpha, double* cost_try, int32_t* status) {
  if (alpha > 1. || alpha < 0.) {  // fddp.cpp:150-153
    g_err = "invalid step length, value is between 0. to 1.";
    return FDDP_ERR_INVALID_ARG;
  }
  for (int b = 0; b < h->dims.B; ++b) {
    const bool ok = h->solvers[b].forwardPass(alpha);
    if (cost_try) cost_try[b] = h->solvers[b].cost_try;
    if (status) status[b] = ok ? 0 : 1;
  }
  return FDDP_OK;
}
int oracle_update_expected_improvement(oracle_handle* h) {
  for (auto& s : h->solvers) s.updateExpectedImprovement();
  return FDDP_OK;
}
int oracle_try_step(oracle_handle* h, double alpha, double* dV, int32_t* status) {
  for (int b = 0; b < h->dims.B; ++b) {
    double v = NAN;
    bool ok = h->solvers[b].tryStep(alpha, &v);
    if (dV) dV[b] = v;
    if (status) status[b] = ok ? 0 : 1;
  }
  return FDDP_OK;
}
int oracle_expected_improvement(oracle_handle* h, double* d) {
  for (int b = 0; b < h->dims.B; ++b) {
    h->solvers[b].expectedImprovement();
    if (d) {
      d[2 * b] = h->solvers[b].d[0];
      d[2 * b + 1] = h->solvers[b].d[1];
    }
  }
  return FDDP_OK;
}
int oracle_stopping_criteria(oracle_handle* h, double* stop) {
  for (int b = 0; b < h->dims.B; ++b) {
    double s = h->solvers[b].stoppingCriteria();
    if (stop) stop[b] = s;
  }
  return FDDP_OK;
}

// Same `which` codes as fddp_get_quantity.
int oracle_get_quantity(oracle_handle* h, int which, double* out) {
  const fddp_dims& D = h->dims;
  const int n = D.ndx, m = D.nu_max, T = D.T;
  size_t per = 0;
  int nk = 0;
  switch (which) {
    case FDDP_Q_FX: case FDDP_Q_LXX: per = (size_t)n * n; nk = T + 1; break;
    case FDDP_Q_FU: case FDDP_Q_LXU: per = (size_t)n * m; nk = T + 1; break;
    case FDDP_Q_LUU: per = (size_t)m * m; nk = T + 1; break;
    case FDDP_Q_LX: per = n; nk = T + 1; break;
    case FDDP_Q_LU: per = m; nk = T + 1; break;
    case FDDP_Q_XNEXT: per = D.nx; nk = T; break;
    case FDDP_Q_FS: per = n; nk = T + 1; break;
    case FDDP_Q_K: per = (size_t)m * n; nk = T; break;
    case FDDP_Q_KV: per = m; nk = T; break;
    case FDDP_Q_VXX: per = (size_t)n * n; nk = T + 1; break;
    case FDDP_Q_VX: per = n; nk = T + 1; break;
    case FDDP_Q_QXX: per = (size_t)n * n; nk = T; break;
    case FDDP_Q_QXU: per = (size_t)n * m; nk = T; break;
    case FDDP_Q_QUU: per = (size_t)m * m; nk = T; break;
    case FDDP_Q_QX: per = n; nk = T; break;
    case FDDP_Q_QU: per = m; nk = T; break;
    default: g_err = "bad quantity"; return FDDP_ERR_INVALID_ARG;
  }
  std::memset(out, 0, sizeof(double) * per * nk * D.B);
  for (int b = 0; b < D.B; ++b) {
    const Solver& s = h->solvers[b];
    const Problem& P = h->problems[b];
    for (int t = 0; t < nk; ++t) {
      double* o = out + ((size_t)b * nk + t) * per;
      const int nut = P.models[t].nu;
      auto put = [&](const Vec& v) { std::memcpy(o, v.data(), sizeof(double) * std::min(per, v.size())); };
      switch (which) {
        case FDDP_Q_FX: put(P.datas[t].Fx.a); break;
        case FDDP_Q_FU: put(P.datas[t].Fu.a); break;  // ndx x nu_t, col-major (stride ndx)
        case FDDP_Q_LXX: put(P.datas[t].Lxx.a); break;
        case FDDP_Q_LXU: put(P.datas[t].Lxu.a); break;
        case FDDP_Q_LUU:  // nu_t x nu_t placed with leading dimension nu_max
          for (int j = 0; j < nut; ++j)
            for (int i = 0; i < nut; ++i) o[(size_t)j * m + i] = P.datas[t].Luu(i, j);
          break;
        case FDDP_Q_LX: put(P.datas[t].Lx); break;
        case FDDP_Q_LU: put(P.datas[t].Lu); break;
        case FDDP_Q_XNEXT: put(P.datas[t].xnext); break;
        case FDDP_Q_FS: put(s.fs[t]); break;
        case FDDP_Q_K:  // nu_t x ndx placed with leading dimension nu_max
          for (int j = 0; j < n; ++j)
            for (int i = 0; i < nut; ++i) o[(size_t)j * m + i] = s.K[t](i, j);
          break;
        case FDDP_Q_KV: put(s.k[t]); break;
        case FDDP_Q_VXX: put(s.Vxx[t].a); break;
        case FDDP_Q_VX: put(s.Vx[t]); break;
        case FDDP_Q_QXX: put(s.Qxx[t].a); break;
        case FDDP_Q_QXU: put(s.Qxu[t].a); break;
        case FDDP_Q_QUU:
          for (int j = 0; j < nut; ++j)
            for (int i = 0; i < nut; ++i) o[(size_t)j * m + i] = s.Quu[t](i, j);
          break;
        case FDDP_Q_QX: put(s.Qx[t]); break;
        case FDDP_Q_QU: put(s.Qu[t]); break;
      }
    }
  }
  return FDDP_OK;
}

// Per-iteration trace of element b: n records of 8 doubles
// (cost, stop, d0, d1, xreg, ureg, steplength, is_feasible) — the columns of
// CallbackVerbose (src/core/utils/callbacks.cpp:13-67).
int oracle_get_trace(oracle_handle* h, int b, double* out, int maxn) {
  const auto& tr = h->solvers[b].trace;
  int n = std::min<int>((int)tr.size(), maxn);
  for (int i = 0; i < n; ++i) std::memcpy(out + 8 * i, &tr[i], sizeof(TraceRec));
  return n;
}

// MPC shift, same semantics as fddp_mpc_shift.
int oracle_mpc_shift(oracle_handle* h) {
  const fddp_dims& D = h->dims;
  for (int b = 0; b < D.B; ++b) {
    Solver& s = h->solvers[b];
    h->problems[b].x0 = s.xs[1];
    for (int t = 0; t < D.T; ++t) s.xs[t] = s.xs[t + 1];
    for (int t = 0; t + 1 < D.T; ++t) s.us[t] = s.us[t + 1];
  }
  return FDDP_OK;
}


// New knot sequence + parameter pool, same contract as fddp_set_knots:
// models are rebound and their datas recreated (createData); solver state,
// trajectories and gains are kept.
int oracle_set_knots(oracle_handle* h, const fddp_knot_desc* knots, const double* params, int64_t n_params) {
  const fddp_dims& D = h->dims;
  h->knots.assign(knots, knots + D.T + 1);
  h->params.assign(params, params + n_params);
  for (int b = 0; b < D.B; ++b) {
    Problem& P = h->problems[b];
    for (int t = 0; t <= D.T; ++t) {
      Model& m = P.models[t];
      m.kind = knots[t].kind;
      m.nu = knots[t].nu;
    }
  }
  bind_models(h);
  for (int b = 0; b < D.B; ++b) {
    Problem& P = h->problems[b];
    for (int t = 0; t <= D.T; ++t) createData(P.models[t], P.datas[t]);
    for (int t = 0; t < D.T; ++t) h->solvers[b].resize_knot(t, knots[t].nu);
  }
  return FDDP_OK;
}

// SolverBoxFDDP / SolverFDDP selection (fddp_set_solver_kind).
int oracle_set_solver_kind(oracle_handle* h, int kind) {
  for (auto& s : h->solvers) s.box = kind == FDDP_SOLVER_BOXFDDP;
  return FDDP_OK;
}
// Control limits (fddp_set_control_limits): B*T*nu_max each, or both NULL.
int oracle_set_control_limits(oracle_handle* h, const double* lb, const double* ub) {
  const fddp_dims& D = h->dims;
  for (int b = 0; b < D.B; ++b) {
    Solver& s = h->solvers[b];
    for (int t = 0; t < D.T; ++t) {
      const int nu = h->problems[b].models[t].nu;
      bool anylb = false, anyub = false;
      for (int i = 0; i < D.nu_max; ++i) {
        const size_t e = ((size_t)b * D.T + t) * D.nu_max + i;
        s.ulb[t][i] = lb ? lb[e] : -INFINITY;
        s.uub[t][i] = ub ? ub[e] : INFINITY;
        if (i < nu) {  // update_has_control_limits (action-base.hxx:142-144)
          anylb = anylb || std::isfinite(s.ulb[t][i]);
          anyub = anyub || std::isfinite(s.uub[t][i]);
        }
      }
      s.haslim[t] = (anylb && anyub) ? 1 : 0;
    }
  }
  return FDDP_OK;
}
// SolverBoxFDDP::get_Quu_inv, same layout as FDDP_Q_QUU_INV.
int oracle_get_quu_inv(oracle_handle* h, double* out) {
  const fddp_dims& D = h->dims;
  const int m = D.nu_max;
  for (int b = 0; b < D.B; ++b)
    for (int t = 0; t < D.T; ++t)
      std::memcpy(out + ((size_t)b * D.T + t) * m * m, h->solvers[b].Quu_inv[t].a.data(), sizeof(double) * m * m);
  return FDDP_OK;
}
// Batched BoxQP, same contract as fddp_boxqp_solve.
int oracle_boxqp_solve(int B, int nx, const double* H, const double* q, const double* lb, const double* ub,
                       const double* xinit, const fddp_boxqp_params* p, double* x, uint64_t* free_mask,
                       uint64_t* inv_mask, double* Hff_inv, int32_t* status, int32_t* iters) {
  if (B < 0 || nx < 1 || nx > 64 || !H || !q || !lb || !ub || !xinit || !p) {
    g_err = "oracle_boxqp_solve: invalid argument";
    return FDDP_ERR_INVALID_ARG;
  }
  for (int b = 0; b < B; ++b) {
    BoxQP qp;
    qp.init(nx, p->maxiter, p->th_acceptstep, p->th_grad, p->reg);
    qp.alphas.assign(p->alphas, p->alphas + p->n_alphas);
    Mat Hm;
    Hm.resize(nx, nx);
    std::memcpy(Hm.a.data(), H + (size_t)b * nx * nx, sizeof(double) * nx * nx);
    const size_t o = (size_t)b * nx;
    const bool ok = qp.solve(Hm, q + o, lb + o, ub + o, xinit + o);
    if (status) status[b] = ok ? 0 : 1;
    if (iters) iters[b] = qp.iters;
    if (x) std::memcpy(x + o, qp.sol.x.data(), sizeof(double) * std::min<size_t>(nx, qp.sol.x.size()));
    uint64_t fm = 0;
    for (int i : qp.sol.free_idx) fm |= 1ull << i;
    if (free_mask) free_mask[b] = fm;
    // Hff_inv embedded at the indices of the free set it was factorised on
    const int ni = qp.sol.Hff_inv.r;
    uint64_t im = 0;
    for (int i : qp.inv_idx) im |= 1ull << i;
    if (inv_mask) inv_mask[b] = im;
    if (Hff_inv) {
      double* Ho = Hff_inv + (size_t)b * nx * nx;
      std::memset(Ho, 0, sizeof(double) * nx * nx);
      for (int j = 0; j < ni; ++j)
        for (int i = 0; i < ni; ++i) Ho[(size_t)qp.inv_idx[j] * nx + qp.inv_idx[i]] = qp.sol.Hff_inv(i, j);
    }
  }
  return FDDP_OK;
}

// Reference defaults (ddp.cpp:15-37, fddp.cpp:14-15, solver-base.cpp:24-25).
void oracle_default_params(fddp_params* p) {
  p->th_acceptstep = 0.1;
  p->th_stop = 1e-9;
  p->th_grad = 1e-12;
  p->th_stepdec = 0.5;
  p->th_stepinc = 0.01;
  p->th_acceptnegstep = 2.;
  p->regfactor = 10.;
  p->regmin = 1e-9;
  p->regmax = 1e9;
  p->n_alphas = 10;
  p->pad_ = 0;
  for (int i = 0; i < 16; ++i) p->alphas[i] = i < 10 ? 1. / std::pow(2., (double)i) : 0.;
}

}  // extern "C"
