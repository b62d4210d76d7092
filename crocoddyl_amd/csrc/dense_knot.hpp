// Dense knot kinds (ActionModelLQR, Euler∘DifferentialActionModelLQR) as
// seen by the fast path: parameter views, the thread -> (row, segment) map of
// the segmented products, and the per-entry formulas of their derivative
// blocks (lqr.hxx:52-70; euler.hxx:83-131 with diff-lqr.hxx:59-80).
#pragma once

#include "knots.hpp"

namespace fddp {

struct DenseKnot {
  bool dlqr, integ, drift_free;
  double dt, sc;  // Euler step; cost / derivative scale (dt when integrating)
  int nr;         // dynamics rows: nx (LQR) or nq (Euler∘DiffLQR)
  const double *F, *f0, *Lxx, *Lxu, *Luu, *lx, *lu;
  __device__ DenseKnot(int kind, const double* P, int nx, int nu) {
    if (kind == FDDP_KNOT_LQR) {
      LQRBlk Bk(P, nx, nu);
      dlqr = false;
      integ = false;
      dt = 0.;
      sc = 1.;
      drift_free = Bk.drift_free;
      nr = nx;
      F = Bk.Fx;
      f0 = Bk.f0;
      Lxx = Bk.Lxx;
      Lxu = Bk.Lxu;
      Luu = Bk.Luu;
      lx = Bk.lx;
      lu = Bk.lu;
    } else {
      DLQRBlk Bk(P, nx, nu);
      dlqr = true;
      dt = Bk.dt;
      integ = dt != 0.;
      sc = integ ? dt : 1.;
      drift_free = Bk.drift_free;
      nr = nx / 2;
      F = Bk.Fq;
      f0 = Bk.f0;
      Lxx = Bk.Lxx;
      Lxu = Bk.Lxu;
      Luu = Bk.Luu;
      lx = Bk.lx;
      lu = Bk.lu;
    }
  }
};

__device__ __forceinline__ bool dense_kind(int kind) { return kind == FDDP_KNOT_LQR || kind == FDDP_KNOT_EULER_DIFFLQR; }

// Thread -> (row i, column segment g) of a rows-row product; G segments.
struct RowSeg {
  int i, g, G;
  bool on;
  __device__ RowSeg(int rows, int nt, int tid) {
    G = rows > 0 ? nt / rows : 1;
    if (G < 1) G = 1;
    i = rows > 0 ? tid % rows : 0;
    g = rows > 0 ? tid / rows : 0;
    on = rows > 0 && g < G;
  }
};

// sum_{j = j0, j0+G, ... < cols} A[j*lda + i] * v[j], four accumulators.
__device__ __forceinline__ double seg_dot(const double* A, int lda, int i, int j0, int G, int cols, const double* v) {
  double a0 = 0., a1 = 0., a2 = 0., a3 = 0.;
  int j = j0;
  for (; j + 3 * G < cols; j += 4 * G) {
    a0 = fma(A[j * lda + i], v[j], a0);
    a1 = fma(A[(j + G) * lda + i], v[j + G], a1);
    a2 = fma(A[(j + 2 * G) * lda + i], v[j + 2 * G], a2);
    a3 = fma(A[(j + 3 * G) * lda + i], v[j + 3 * G], a3);
  }
  for (; j < cols; j += G) a0 = fma(A[j * lda + i], v[j], a0);
  return (a0 + a1) + (a2 + a3);
}
// Transposed: sum_j A[i*lda + j] * v[j] (row i of A^T = column i of A).
__device__ __forceinline__ double seg_dot_t(const double* A, int lda, int i, int j0, int G, int cols, const double* v) {
  const double* a = A + i * lda;
  double a0 = 0., a1 = 0., a2 = 0., a3 = 0.;
  int j = j0;
  for (; j + 3 * G < cols; j += 4 * G) {
    a0 = fma(a[j], v[j], a0);
    a1 = fma(a[j + G], v[j + G], a1);
    a2 = fma(a[j + 2 * G], v[j + 2 * G], a2);
    a3 = fma(a[j + 3 * G], v[j + 3 * G], a3);
  }
  for (; j < cols; j += G) a0 = fma(a[j], v[j], a0);
  return (a0 + a1) + (a2 + a3);
}

// Streams one knot's derivative blocks out: thread -> (row pair, column
// segment), 16-byte stores (n even; odd n falls back to 8-byte stores). The
// per-row factors of the Euler integration are per-thread constants; each
// column is a coalesced store across consecutive row pairs.
__device__ __forceinline__ void dense_fx_rows(const DenseKnot& K, int n, int i, int& ldf, int& ri, int& jd, double& a) {
  ldf = n;
  ri = i;
  jd = -1;
  a = 1.;
  if (K.dlqr) {
    const int nv = n / 2;
    ldf = nv;
    ri = i < nv ? i : i - nv;
    a = K.integ ? (i < nv ? K.dt * K.dt : K.dt) : 0.;
    jd = (K.integ && i < nv) ? nv + i : -1;
  }
}
__device__ __forceinline__ double dense_fx_at(const DenseKnot& K, int n, int i, int j, int ldf, int ri, int jd, double a) {
  double f = K.dlqr ? (K.integ ? a * K.F[j * ldf + ri] : 0.) : K.F[j * n + i];
  if (j == jd) f += K.dt;
  if (K.dlqr && j == i) f += 1.;
  return f;
}
__device__ __forceinline__ double dense_fu_at(const DenseKnot& K, int n, int nu, int i, int j, int ldf, int ri, double a) {
  if (j >= nu) return 0.;
  return K.dlqr ? (K.integ ? a * K.F[(n + j) * ldf + ri] : 0.) : K.F[(n + j) * n + i];
}


}  // namespace fddp
