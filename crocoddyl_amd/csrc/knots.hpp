// Knot models on the device: calc / calcDiff of one knot by one workgroup.
//
// Each routine is the device restatement of a reference ActionModel:
//   LQR        include/crocoddyl/core/actions/lqr.hxx:30-70
//   Unicycle   include/crocoddyl/core/actions/unicycle.hxx:22-73
//   Euler∘DiffLQR  include/crocoddyl/core/integrator/euler.hxx:41-131 around
//              include/crocoddyl/core/actions/diff-lqr.hxx:34-79 (Euclidean state,
//              so JintegrateTransport is a no-op and Jintegrate adds I,
//              core/states/euclidean.hxx:74-147).
//   Euler∘FreeFwdDynamics  multibody.hpp (multibody/actions/free-fwddyn.hxx)
// Parameter-block layouts are declared in include/fddp_hip.h.
//
// Threads split the rows of every matrix-vector product (column-major blocks:
// consecutive threads read consecutive addresses of one column), and the
// scalar cost is a workgroup reduction of per-row terms.
#pragma once

#include "fddp_device.hpp"
#include "multibody.hpp"

namespace fddp {

struct LQRBlk {
  bool drift_free;
  const double *Fx, *Fu, *f0, *Lxx, *Lxu, *Luu, *lx, *lu;
  __device__ LQRBlk(const double* p, int nx, int nu) {
    drift_free = p[0] != 0.;
    const double* q = p + FDDP_PARAM_HEADER;
    Fx = q; q += (int64_t)nx * nx;
    Fu = q; q += (int64_t)nx * nu;
    f0 = q; q += nx;
    Lxx = q; q += (int64_t)nx * nx;
    Lxu = q; q += (int64_t)nx * nu;
    Luu = q; q += (int64_t)nu * nu;
    lx = q; q += nx;
    lu = q;
  }
};

struct DLQRBlk {
  double dt;
  bool drift_free;
  const double *Fq, *Fv, *Fu, *f0, *Lxx, *Lxu, *Luu, *lx, *lu;
  __device__ DLQRBlk(const double* p, int nx, int nu) {
    const int nq = nx / 2;
    dt = p[0];
    drift_free = p[1] != 0.;
    const double* q = p + FDDP_PARAM_HEADER;
    Fq = q; q += (int64_t)nq * nq;
    Fv = q; q += (int64_t)nq * nq;
    Fu = q; q += (int64_t)nq * nu;
    f0 = q; q += nq;
    Lxx = q; q += (int64_t)nx * nx;
    Lxu = q; q += (int64_t)nx * nu;
    Luu = q; q += (int64_t)nu * nu;
    lx = q; q += nx;
    lu = q;
  }
};

// Per-row quadratic-cost terms of 0.5 x.Lxx x + 0.5 u.Luu u + x.Lxu u + lx.x + lu.u
// (lqr.hxx:47-48 / diff-lqr.hxx:54-55); t[0..4] accumulate the five dot products.
__device__ inline void lq_cost_rows(const double* Lxx, const double* Lxu, const double* Luu, const double* lx,
                                    const double* lu, const double* x, const double* u, bool use_u, int nx, int nu,
                                    int NT, double (&t)[5]) {
  for (int i = threadIdx.x; i < nx; i += NT) {
    double s1 = 0.;
    for (int j = 0; j < nx; ++j) s1 += Lxx[(int64_t)j * nx + i] * x[j];
    t[0] += x[i] * s1;
    if (use_u) {
      double s3 = 0.;
      for (int j = 0; j < nu; ++j) s3 += Lxu[(int64_t)j * nx + i] * u[j];
      t[2] += x[i] * s3;
    }
    t[3] += lx[i] * x[i];
  }
  if (use_u) {
    for (int i = threadIdx.x; i < nu; i += NT) {
      double s2 = 0.;
      for (int j = 0; j < nu; ++j) s2 += Luu[(int64_t)j * nu + i] * u[j];
      t[1] += u[i] * s2;
      t[4] += lu[i] * u[i];
    }
  }
}

__device__ inline double lq_cost_total(const double (&t)[5]) {
  return 0.5 * t[0] + 0.5 * t[1] + t[2] + t[3] + t[4];
}

// model->calc(data, x, u) (use_u) or model->calc(data, x) with unone_ = 0
// (action-base.hxx:28-31). x, u: readable by every thread (LDS or global).
// Writes xnext[0..nx) and returns the knot cost in every thread.
// `red`: LDS scratch of >= 5*NT/64 doubles; `mbw`: LDS scratch of
// mb::calc_work_doubles(nj) for multibody knots. Contains barriers: call uniformly.
// MB: the caller guarantees every knot is a multibody kind (the dense kinds are not
// compiled in, which keeps the rollout's register budget for the multibody calc).
template <int NT, bool MB = false>
__device__ __forceinline__ double knot_calc(const fddp_knot_desc& kd, const double* P, int nx, const double* x, const double* u,
                            bool use_u, double* xnext, double* red, double* mbw) {
  const int nu = kd.nu;
  use_u = use_u && nu > 0;
  // multibody blocks are always staged in LDS (fddp_create checks the budget), as are
  // the trial state / control / next state and the scratch of every caller
  if (MB || is_mb_kind(kd.kind))
    return mb::knot_calc<NT>(lds_ptr(P), nx, lds_ptr(x), lds_ptr(u), use_u, lds_ptr(xnext), lds_ptr(mbw));
  double t[5] = {0., 0., 0., 0., 0.};
  if (kd.kind == FDDP_KNOT_LQR) {
    LQRBlk Pm(P, nx, nu);
    for (int i = threadIdx.x; i < nx; i += NT) {
      double a = 0., b = 0.;
      for (int j = 0; j < nx; ++j) a += Pm.Fx[(int64_t)j * nx + i] * x[j];
      if (use_u)
        for (int j = 0; j < nu; ++j) b += Pm.Fu[(int64_t)j * nx + i] * u[j];
      xnext[i] = Pm.drift_free ? a + b : a + b + Pm.f0[i];
    }
    lq_cost_rows(Pm.Lxx, Pm.Lxu, Pm.Luu, Pm.lx, Pm.lu, x, u, use_u, nx, nu, NT, t);
    wg_sums<NT, 5>(t, red);
    return lq_cost_total(t);
  } else if (kd.kind == FDDP_KNOT_EULER_DIFFLQR) {
    DLQRBlk Pm(P, nx, nu);
    const int nq = nx / 2, nv = nq;
    const double dt = Pm.dt, dt2 = dt * dt;
    for (int i = threadIdx.x; i < nv; i += NT) {
      double a1 = 0., a2 = 0., a3 = 0.;
      for (int j = 0; j < nq; ++j) a1 += Pm.Fq[(int64_t)j * nq + i] * x[j];
      for (int j = 0; j < nv; ++j) a2 += Pm.Fv[(int64_t)j * nv + i] * x[nq + j];
      if (use_u)
        for (int j = 0; j < nu; ++j) a3 += Pm.Fu[(int64_t)j * nq + i] * u[j];
      const double a = Pm.drift_free ? a1 + a2 + a3 : a1 + a2 + a3 + Pm.f0[i];
      if (dt != 0.) {
        const double dq = x[nq + i] * dt + a * dt2;  // v*dt + a*dt^2 (euler.hxx:66)
        const double dv = a * dt;                    // a*dt (euler.hxx:67)
        xnext[i] = x[i] + dq;
        xnext[nq + i] = x[nq + i] + dv;
      } else {
        xnext[i] = x[i];
        xnext[nq + i] = x[nq + i];
      }
    }
    lq_cost_rows(Pm.Lxx, Pm.Lxu, Pm.Luu, Pm.lx, Pm.lu, x, u, use_u, nx, nu, NT, t);
    wg_sums<NT, 5>(t, red);
    const double cc = lq_cost_total(t);
    return dt != 0. ? dt * cc : cc;
  } else {  // FDDP_KNOT_UNICYCLE
    const double dt = P[0], wx = P[1], wu = P[2];
    if (threadIdx.x == 0) {
      const double u0 = use_u ? u[0] : 0., u1 = use_u ? u[1] : 0.;
      const double c = cos(x[2]), s = sin(x[2]);
      xnext[0] = x[0] + c * u0 * dt;
      xnext[1] = x[1] + s * u0 * dt;
      xnext[2] = x[2] + u1 * dt;
      const double r0 = wx * x[0], r1 = wx * x[1], r2 = wx * x[2], r3 = wu * u0, r4 = wu * u1;
      red[0] = 0.5 * (r0 * r0 + r1 * r1 + r2 * r2 + r3 * r3 + r4 * r4);
    }
    __syncthreads();
    const double c = red[0];
    __syncthreads();
    return c;
  }
}

// Output pointers of one knot's derivative blocks (ActionData members).
struct KnotDiffOut {
  double *Fx, *Fu, *Lxx, *Lxu, *Luu, *Lx, *Lu;
};

// model->calcDiff(data, x, u) / calcDiff(data, x). Writes full blocks (entries
// beyond the knot's nu are zero); Luu has leading dimension m = nu_max.
// Multibody knots are differentiated by mb_calc_diff_kernel (one workgroup
// per knot) instead.
template <int NT>
__device__ __forceinline__ void knot_calc_diff(const fddp_knot_desc& kd, const double* P, int nx, int m, const double* x,
                               const double* u, bool use_u, const KnotDiffOut& o) {
  const int n = nx;
  const int nu = kd.nu;
  use_u = use_u && nu > 0;
  const int tid = threadIdx.x;
  if (is_mb_kind(kd.kind)) return;
  if (kd.kind == FDDP_KNOT_LQR) {  // lqr.hxx:51-70
    LQRBlk Pm(P, nx, nu);
    for (int i = tid; i < n; i += NT) {
      double a = 0., b = 0.;
      for (int j = 0; j < n; ++j) a += Pm.Lxx[(int64_t)j * n + i] * x[j];
      if (use_u)
        for (int j = 0; j < nu; ++j) b += Pm.Lxu[(int64_t)j * n + i] * u[j];
      o.Lx[i] = Pm.lx[i] + a + b;
    }
    for (int i = tid; i < m; i += NT) {
      double v = 0.;
      if (i < nu) {
        double a = 0., b = 0.;
        for (int j = 0; j < n; ++j) a += Pm.Lxu[(int64_t)i * n + j] * x[j];
        if (use_u)
          for (int j = 0; j < nu; ++j) b += Pm.Luu[(int64_t)j * nu + i] * u[j];
        v = Pm.lu[i] + a + b;
      }
      o.Lu[i] = v;
    }
    for (int64_t e = tid; e < (int64_t)n * n; e += NT) {
      o.Fx[e] = Pm.Fx[e];
      o.Lxx[e] = Pm.Lxx[e];
    }
    for (int64_t e = tid; e < (int64_t)n * m; e += NT) {
      const bool in = e < (int64_t)n * nu;
      o.Fu[e] = in ? Pm.Fu[e] : 0.;
      o.Lxu[e] = in ? Pm.Lxu[e] : 0.;
    }
    for (int64_t e = tid; e < (int64_t)m * m; e += NT) {
      const int i = (int)(e % m), j = (int)(e / m);
      o.Luu[e] = (i < nu && j < nu) ? Pm.Luu[(int64_t)j * nu + i] : 0.;
    }
  } else if (kd.kind == FDDP_KNOT_EULER_DIFFLQR) {  // euler.hxx:83-131, diff-lqr.hxx:59-79
    DLQRBlk Pm(P, nx, nu);
    const int nq = n / 2, nv = nq;
    const double dt = Pm.dt, dt2 = dt * dt;
    const bool integ = dt != 0.;
    const double sc = integ ? dt : 1.;
    for (int i = tid; i < n; i += NT) {
      double a = 0., b = 0.;
      for (int j = 0; j < n; ++j) a += Pm.Lxx[(int64_t)j * n + i] * x[j];
      if (use_u)
        for (int j = 0; j < nu; ++j) b += Pm.Lxu[(int64_t)j * n + i] * u[j];
      const double lx = Pm.lx[i] + a + b;
      o.Lx[i] = integ ? sc * lx : lx;
    }
    for (int i = tid; i < m; i += NT) {
      double v = 0.;
      if (i < nu) {
        double a = 0., b = 0.;
        for (int j = 0; j < n; ++j) a += Pm.Lxu[(int64_t)i * n + j] * x[j];
        if (use_u)
          for (int j = 0; j < nu; ++j) b += Pm.Luu[(int64_t)j * nu + i] * u[j];
        const double lu = Pm.lu[i] + a + b;
        v = integ ? sc * lu : lu;
      }
      o.Lu[i] = v;
    }
    for (int64_t e = tid; e < (int64_t)n * n; e += NT) {
      const int i = (int)(e % n), j = (int)(e / n);
      double f;
      if (integ) {
        const int r = i < nv ? i : i - nv;
        const double da = j < nq ? Pm.Fq[(int64_t)j * nq + r] : Pm.Fv[(int64_t)(j - nq) * nv + r];
        f = i < nv ? da * dt2 : da * dt;
        if (i < nv && j == nv + i) f += dt;  // topRightCorner(nv,nv).diagonal() += dt
        if (i == j) f += 1.;                 // Jintegrate(first, addto)
      } else {
        f = (i == j) ? 1. : 0.;              // Jintegrate(x, dx, Fx, Fx): diagonal = 1
      }
      o.Fx[e] = f;
      o.Lxx[e] = integ ? sc * Pm.Lxx[e] : Pm.Lxx[e];
    }
    for (int64_t e = tid; e < (int64_t)n * m; e += NT) {
      const int i = (int)(e % n), j = (int)(e / n);
      double f = 0., l = 0.;
      if (j < nu) {
        if (integ) {
          const int r = i < nv ? i : i - nv;
          const double da = Pm.Fu[(int64_t)j * nq + r];
          f = i < nv ? da * dt2 : da * dt;
          l = sc * Pm.Lxu[e];
        } else {
          l = Pm.Lxu[e];
        }
      }
      o.Fu[e] = f;
      o.Lxu[e] = l;
    }
    for (int64_t e = tid; e < (int64_t)m * m; e += NT) {
      const int i = (int)(e % m), j = (int)(e / m);
      double l = 0.;
      if (i < nu && j < nu) {
        const double c = Pm.Luu[(int64_t)j * nu + i];
        l = integ ? sc * c : c;
      }
      o.Luu[e] = l;
    }
  } else {  // FDDP_KNOT_UNICYCLE, unicycle.hxx:43-73 (Fx = I initially, unicycle.hpp:79)
    const double dt = P[0], wx = P[1], wu = P[2];
    const double w_x = wx * wx, w_u = wu * wu;
    const double u0 = use_u ? u[0] : 0., u1 = use_u ? u[1] : 0.;
    const double c = cos(x[2]), s = sin(x[2]);
    for (int64_t e = tid; e < (int64_t)n * n; e += NT) {
      const int i = (int)(e % n), j = (int)(e / n);
      double f = (i == j) ? 1. : 0.;
      if (i == 0 && j == 2) f = -s * u0 * dt;
      if (i == 1 && j == 2) f = c * u0 * dt;
      o.Fx[e] = f;
      o.Lxx[e] = (i == j) ? w_x : 0.;
    }
    for (int64_t e = tid; e < (int64_t)n * m; e += NT) {
      const int i = (int)(e % n), j = (int)(e / n);
      double f = 0.;
      if (i == 0 && j == 0) f = c * dt;
      if (i == 1 && j == 0) f = s * dt;
      if (i == 2 && j == 1) f = dt;
      o.Fu[e] = f;
      o.Lxu[e] = 0.;
    }
    for (int64_t e = tid; e < (int64_t)m * m; e += NT) {
      const int i = (int)(e % m), j = (int)(e / m);
      o.Luu[e] = (i == j && i < 2) ? w_u : 0.;
    }
    for (int i = tid; i < n; i += NT) o.Lx[i] = x[i] * w_x;
    for (int i = tid; i < m; i += NT) o.Lu[i] = i == 0 ? u0 * w_u : (i == 1 ? u1 * w_u : 0.);
  }
}

}  // namespace fddp
