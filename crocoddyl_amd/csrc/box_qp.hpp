// Box QP on one wave: BoxQP::solve (src/core/solvers/box-qp.cpp:51-182),
// projected Newton for  min 0.5 x'Hx + q'x  s.t.  lb <= x <= ub,  restated
// for gfx950 with one decision variable per lane (nx <= 64).
//
// Per Newton iteration: g = q + Hx (one LDS GEMV: H column j at lane-
// consecutive addresses, x_j broadcast), the free / clamped split and the
// convergence test as wave ballots, the free-Hessian inverse by a masked
// symmetric sweep (caller-supplied: the register sweep of the MFMA Riccati
// kernel or the LDS sweep below), the Newton direction as two more GEMVs, and
// the projected line search over the alphas (one GEMV + two wave sums per
// trial). Every branch is taken on a ballot or on lane 0's sum, so the wave
// stays uniform.
//
// Same results as the reference, with three exact shortcuts:
//  - an iteration whose line search accepts no alpha leaves x unchanged, so
//    every later iteration repeats it bit for bit until maxiter: the loop
//    stops there with the state the reference returns after maxiter;
//  - Hff_inv is kept embedded in an nx x nx matrix (zero off the free set), and
//    an iteration on the free set of the previous one reuses it (and the
//    accepted trial's H x) instead of recomputing the same values.
// When the QP converges at k > 0 the reference returns the previous
// iteration's Hff_inv with the new free_idx, and SolverBoxFDDP scatters it
// by position (box-fddp.cpp:64-69); `remap` reproduces that scatter by
// inverting the previous free Hessian relabelled onto the new free indices.
#pragma once

#include "fddp_device.hpp"

namespace fddp {

// Position of the p-th (0-based) set bit of v.
__device__ __forceinline__ int select_bit(uint64_t v, int p) {
  int pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const int c = __popcll(v & ((1ull << w) - 1));
    if (p >= c) {
      v >>= w;
      pos += w;
      p -= c;
    }
  }
  return pos;
}

// Index map of a masked inverse. Entry (i, j) of the matrix that is inverted
// is H(sig(i), sig(j)) (+ reg on the diagonal) for i, j in `used`, the
// identity elsewhere; the result is kept on out x out and zero elsewhere.
// Plain: used = out = fsol = finv, sig = id. Remap: the free Hessian of finv,
// its p-th free index relabelled to the p-th index of fsol (then to the
// indices outside fsol, in order, when finv is the larger set).
struct InvMap {
  uint64_t fsol, finv;
  int nsol, ninv, m;
  bool remap;
  double reg;
  __device__ static InvMap plain(uint64_t f, int m, double reg) {
    InvMap r;
    r.fsol = r.finv = f;
    r.nsol = r.ninv = __popcll(f);
    r.m = m;
    r.remap = false;
    r.reg = reg;
    return r;
  }
  __device__ static InvMap remapped(uint64_t fsol, uint64_t finv, int m, double reg) {
    InvMap r;
    r.fsol = fsol;
    r.finv = finv;
    r.nsol = __popcll(fsol);
    r.ninv = __popcll(finv);
    r.m = m;
    r.remap = true;
    r.reg = reg;
    return r;
  }
  __device__ int rank(int i) const {
    const uint64_t below = (1ull << i) - 1;
    return ((fsol >> i) & 1) ? __popcll(fsol & below) : nsol + __popcll(~fsol & below);
  }
  __device__ bool used(int i) const {
    if (i >= m) return false;
    return remap ? rank(i) < ninv : ((finv >> i) & 1) != 0;
  }
  __device__ bool out(int i) const {
    if (i >= m) return false;
    return remap ? (((fsol >> i) & 1) && rank(i) < ninv) : ((fsol >> i) & 1) != 0;
  }
  __device__ int sig(int i) const { return remap ? select_bit(finv, rank(i)) : i; }
  // entry (i, j) of the matrix to invert; H column-major with leading dimension ld
  __device__ double load(const double* H, int ld, int i, int j) const {
    if (used(i) && used(j)) {
      double v = H[sig(j) * ld + sig(i)];
      if (i == j) v += reg;
      return v;
    }
    return i == j ? 1. : 0.;
  }
};

// Masked inverse by the symmetric sweep on one wave, any m <= 64, working
// in LDS: lane j owns column j of A (ld lda). Pivot k is the k-th Schur
// complement, so `pivot <= 0` is Eigen LLT's failure. Row k is published
// through rb (64 doubles) and read back as column k (the sweep keeps A
// exactly symmetric: every update uses the commutative product rb_i rb_j).
// Returns true if a pivot was not positive. Used by the generic Riccati
// sweep and the standalone box-QP kernel.
__device__ inline bool wave_sweep_inverse_lds(const double* H, int ldh, double* A, int lda, double* rb, int m,
                                              const InvMap& mp, int lane) {
  const bool valid = lane < m;
  if (valid)
    for (int i = 0; i < m; ++i) A[lane * lda + i] = mp.load(H, ldh, i, lane);
  bool bad = false;
  for (int k = 0; k < m; ++k) {
    asm volatile("" ::: "memory");
    if (valid) rb[lane] = A[lane * lda + k];  // A(k, j) = A(j, k)
    asm volatile("" ::: "memory");
    const double d = rb[k];
    bad |= !(d > 0.);
    const double dinv = 1. / d;
    if (valid) {
      double* col = A + lane * lda;
      const double akj = rb[lane];
      if (lane == k) {
        for (int i = 0; i < m; ++i) col[i] = i == k ? -dinv : rb[i] * dinv;
      } else {
        for (int i = 0; i < m; ++i) col[i] = i == k ? akj * dinv : fma(-(rb[i] * akj), dinv, col[i]);
      }
    }
    asm volatile("" ::: "memory");
  }
  if (valid)
    for (int i = 0; i < m; ++i) A[lane * lda + i] = (mp.out(i) && mp.out(lane)) ? -A[lane * lda + i] : 0.;
  asm volatile("" ::: "memory");
  return bad;
}

// std::min / std::max semantics (NaN propagation as in the reference)
__device__ __forceinline__ double std_min(double a, double b) { return (b < a) ? b : a; }
__device__ __forceinline__ double std_max(double a, double b) { return (a < b) ? b : a; }

// The box QP. Called by all 64 lanes of one wave. H (m x m, ld ldh) and Qi
// (ld ldq) in LDS; vb: 64 doubles of LDS scratch (may alias the inverse's
// row buffer: the two are never live together). Per lane (lane < m): q, lb,
// ub; x: in xinit, out the solution. inv(const InvMap&) writes the masked
// inverse into Qi and returns true on a failed pivot. Returns false where the
// reference throws "backward_error". free_sol: the free set of the solution
// (free_idx); free_inv: the set Hff_inv was factorised on. With remap, Qi is
// left holding the Quu_inv that SolverBoxFDDP assembles; without, the
// embedded Hff_inv of free_inv.
template <class Inv>
__device__ __forceinline__ bool box_qp_wave(const double* H, int ldh, double* Qi, int ldq, double* vb, int m,
                                            int lane, double q, double lb, double ub, double& x, const BoxQPCfg& c,
                                            Inv&& inv, bool remap, uint64_t& free_sol, uint64_t& free_inv,
                                            int& iters) {
  const bool valid = lane < m;
  auto matvec = [&](const double* A, int lda, double v) {
    asm volatile("" ::: "memory");
    vb[lane] = valid ? v : 0.;
    asm volatile("" ::: "memory");
    double s0 = 0., s1 = 0.;
    if (valid) {
      int j = 0;
      // eight columns' loads issued before their FMAs (one LDS round trip per eight);
      // the even / odd chains as below, so the sums are the same
      for (; j + 8 <= m; j += 8) {
        double a[8], x[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          a[q] = A[(j + q) * lda + lane];
          x[q] = vb[j + q];
        }
#pragma unroll
        for (int q = 0; q < 8; q += 2) {
          s0 = fma(a[q], x[q], s0);
          s1 = fma(a[q + 1], x[q + 1], s1);
        }
      }
      for (; j + 1 < m; j += 2) {
        s0 = fma(A[j * lda + lane], vb[j], s0);
        s1 = fma(A[(j + 1) * lda + lane], vb[j + 1], s1);
      }
      if (j < m) s0 = fma(A[j * lda + lane], vb[j], s0);
    }
    asm volatile("" ::: "memory");
    return s0 + s1;
  };
  auto zero_qi = [&]() {
    for (int e = lane; e < m * m; e += 64) Qi[(e / m) * ldq + e % m] = 0.;
    asm volatile("" ::: "memory");
  };
  // lane 0's value of a wave-uniform decision (butterfly sums may differ in
  // the last bit between lanes)
  auto uniform = [](bool p) { return (__ballot(p) & 1ull) != 0; };
  x = valid ? std_max(std_min(x, ub), lb) : 0.;  // feasible warm start (:89-91)
  free_inv = 0;
  free_sol = 0;
  iters = 0;
  uint64_t fr = 0;
  // Qi holds the plain inverse of free_inv from the last Newton step (an iteration on the
  // same free set reuses it: the reference refactorises the same matrix to the same bits);
  // H x of an accepted trial is the next iteration's H x
  bool qi_plain = false, have_hx = false;
  double Hx = 0.;
  for (int k = 0; k < c.maxiter; ++k) {
    if (!have_hx) Hx = matvec(H, ldh, x);
    have_hx = false;
    const double g = q + Hx;
    const bool clamped = valid && ((x == lb && g > 0.) || (x == ub && g < 0.));
    fr = __ballot(valid && !clamped);
    const bool gbig = __ballot(valid && !(fabs(g) <= c.th_grad)) != 0;
    if (!gbig || fr == 0) {  // converged (:113-135)
      if (k == 0) {
        if (inv(InvMap::plain(fr, m, c.reg))) return false;
        free_inv = fr;
      } else if (remap && fr != free_inv) {
        if (fr == 0)
          zero_qi();
        else
          (void)inv(InvMap::remapped(fr, free_inv, m, c.reg));  // factorised before: cannot fail in exact arithmetic
      }
      free_sol = fr;
      return true;
    }
    ++iters;
    // Newton step on the free subspace (:138-175)
    if (!(qi_plain && fr == free_inv) && inv(InvMap::plain(fr, m, c.reg))) return false;
    free_inv = fr;
    qi_plain = true;
    const bool isfree = valid && ((fr >> lane) & 1);
    const double Hxc = matvec(H, ldh, clamped ? x : 0.);
    const double rf = isfree ? (-q - Hxc) : 0.;
    const double sol = matvec(Qi, ldq, rf);
    const double dx = isfree ? sol - x : 0.;
    // projected line search (:178-189)
    const double fold = wave_sum(valid ? x * (0.5 * Hx) + q * x : 0.);
    bool accepted = false;
    for (int a = 0; a < c.n_alphas; ++a) {
      const double al = c.alphas[a];
      const double xn = valid ? std_max(std_min(x + al * dx, ub), lb) : 0.;
      const double Hxn = matvec(H, ldh, xn);
      const double fnew = wave_sum(valid ? xn * (0.5 * Hxn) + q * xn : 0.);
      const double gd = wave_sum(valid ? g * (x - xn) : 0.);
      if (uniform(fold - fnew > c.th_acceptstep * gd)) {
        x = xn;
        Hx = Hxn;
        have_hx = true;
        accepted = true;
        break;
      }
    }
    if (!accepted) break;  // a fixed point: the remaining iterations repeat this one
  }
  free_sol = fr;
  if (c.maxiter <= 0) zero_qi();
  return true;
}

}  // namespace fddp
