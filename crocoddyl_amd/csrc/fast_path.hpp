// Fast path of ShootingProblem::calc / calcDiff and of the FDDP forward
// rollout for the dense knot kinds (ActionModelLQR, Euler∘DifferentialLQR),
// used when every knot is one of them and ndx, nu_max <= NT.
//
// Same arithmetic as knot_calc / knot_calc_diff (knots.hpp) and fwd_trial
// (fddp_kernels.hpp), reorganised for latency: on gfx950 a dependent f64 FMA
// takes 32 cycles, so a row-per-thread dot product of length n is a 32n-cycle
// chain. Every matrix-vector product here splits each row over G = NT / rows
// column segments (thread -> row i, segment g; consecutive threads read
// consecutive rows of a column, conflict-free in LDS and coalesced in HBM),
// four independent accumulators per segment, and one LDS reduction. The knot
// cost is reduced from per-thread partials (wave shuffles + one LDS slot per
// wave), and the forward pass defers its NaN checks to the end of the trial
// (a trial that raises at knot t fails exactly as if it had stopped there).
//
// The dynamics of both kinds are one product with a contiguous block of the
// parameter pool: LQR [Fx | Fu] (ld nx) times [x; u], Euler∘DiffLQR
// [Fq | Fv | Fu] (ld nq) times [q; v; u]; the cost rows are [Lxx | Lxu]
// (ld nx) times [x; u] and the u rows Lxu^T x + Luu u.
#pragma once

#include "fddp_kernels.hpp"
#include "bwd_mfma.hpp"  // Stamp

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

// Per-thread partials of one dense knot at (x, u) = xu[0..nx), xu[nx..nx+nu):
//   dyn : dynamics row partial (-> pdyn[g*nr + i])
//   lx  : (Lxx x + Lxu u) row partial (-> plx[g*nx + i]) when want_lx
//   lu  : (Lxu^T x + Luu u) row partial (-> plu[g*nu + i]) when want_lu
// Returns this thread's share of the unscaled knot cost
//   0.5 x.Lxx x + 0.5 u.Luu u + x.Lxu u + lx.x + lu.u   (lqr.hxx:47-48).
template <int NT>
__device__ __forceinline__ double dense_partials(const DenseKnot& K, int nx, int nu, bool use_u, const double* xu,
                                                 bool want_dyn, bool want_lx, bool want_lu, bool want_cost,
                                                 double* pdyn, double* plx, double* plu, int tid) {
  const double* x = xu;
  const double* u = xu + nx;
  const int nuu = use_u ? nu : 0;
  double cost = 0.;
  if (want_dyn) {
    const RowSeg r(K.nr, NT, tid);
    if (r.on) pdyn[r.g * K.nr + r.i] = seg_dot(K.F, K.nr, r.i, r.g, r.G, nx + nuu, xu);
  }
  if (want_lx || want_cost) {
    const RowSeg r(nx, NT, tid);
    if (r.on) {
      const double sx = seg_dot(K.Lxx, nx, r.i, r.g, r.G, nx, x);
      const double su = nuu > 0 ? seg_dot(K.Lxu, nx, r.i, r.g, r.G, nuu, u) : 0.;
      if (want_lx) plx[r.g * nx + r.i] = sx + su;
      if (want_cost) {
        cost = x[r.i] * (0.5 * sx + su);
        if (r.g == 0) cost = fma(K.lx[r.i], x[r.i], cost);
      }
    }
  }
  if ((want_lu || want_cost) && nu > 0) {
    const RowSeg r(nu, NT, tid);
    if (r.on) {
      const double a = seg_dot_t(K.Lxu, nx, r.i, r.g, r.G, nx, x);
      const double bb = nuu > 0 ? seg_dot(K.Luu, nu, r.i, r.g, r.G, nuu, u) : 0.;
      if (want_lu) plu[r.g * nu + r.i] = a + bb;
      if (want_cost && nuu > 0) {
        cost = fma(0.5 * u[r.i], bb, cost);
        if (r.g == 0) cost = fma(K.lu[r.i], u[r.i], cost);
      }
    }
  }
  return cost;
}

// Sum of the G partials of row i.
__device__ __forceinline__ double seg_sum(const double* p, int rows, int i, int nt) {
  int G = nt / rows;
  if (G < 1) G = 1;
  double s = 0.;
  for (int g = 0; g < G; ++g) s += p[g * rows + i];
  return s;
}

// xnext rows i < nr from the reduced dynamics sum (lqr.hxx:38-44,
// euler.hxx:60-70 with diff-lqr.hxx:36-44). Writes xnext[i] (and [nq + i]).
__device__ __forceinline__ void dense_xnext(const DenseKnot& K, int nx, int i, double a, const double* x, double* xn) {
  if (!K.drift_free) a += K.f0[i];
  if (!K.dlqr) {
    xn[i] = a;
    return;
  }
  const int nq = nx / 2;
  if (K.integ) {
    const double dt = K.dt, dt2 = dt * dt;
    const double dq = x[nq + i] * dt + a * dt2;  // v*dt + a*dt^2 (euler.hxx:66)
    const double dv = a * dt;                    // a*dt (euler.hxx:67)
    xn[i] = x[i] + dq;
    xn[nq + i] = x[nq + i] + dv;
  } else {
    xn[i] = x[i];
    xn[nq + i] = x[nq + i];
  }
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

template <int NT>
__device__ __forceinline__ void dense_write_blocks(const DenseKnot& K, int n, int m, int nu, const KnotDiffOut& o,
                                                   int part, int tid) {
  const bool scale = K.dlqr && K.integ;
  const double sc = scale ? K.sc : 1.;
  const bool wide = (n & 1) == 0;
  const int rows = wide ? n / 2 : n;  // row pairs (or rows)
  const RowSeg r(rows, NT, tid);
  const int i0 = wide ? 2 * r.i : r.i;
  int ldf0, ri0, jd0, ldf1, ri1, jd1;
  double a0, a1;
  dense_fx_rows(K, n, i0, ldf0, ri0, jd0, a0);
  dense_fx_rows(K, n, i0 + 1, ldf1, ri1, jd1, a1);
  if ((part & 1) && r.on) {  // Fx, Lxx
    for (int j = r.g; j < n; j += r.G) {
      const int e = j * n + i0;
      if (wide) {
        double2 f, l;
        f.x = dense_fx_at(K, n, i0, j, ldf0, ri0, jd0, a0);
        f.y = dense_fx_at(K, n, i0 + 1, j, ldf1, ri1, jd1, a1);
        l.x = sc * K.Lxx[e];
        l.y = sc * K.Lxx[e + 1];
        *reinterpret_cast<double2*>(o.Fx + e) = f;
        *reinterpret_cast<double2*>(o.Lxx + e) = l;
      } else {
        o.Fx[e] = dense_fx_at(K, n, i0, j, ldf0, ri0, jd0, a0);
        o.Lxx[e] = sc * K.Lxx[e];
      }
    }
  }
  if (part & 2) {  // Fu, Lxu, Luu
    for (int j = r.g; r.on && j < m; j += r.G) {
      const int e = j * n + i0;
      const bool in = j < nu;
      if (wide) {
        double2 f, l;
        f.x = dense_fu_at(K, n, nu, i0, j, ldf0, ri0, a0);
        f.y = dense_fu_at(K, n, nu, i0 + 1, j, ldf1, ri1, a1);
        l.x = in ? sc * K.Lxu[e] : 0.;
        l.y = in ? sc * K.Lxu[e + 1] : 0.;
        *reinterpret_cast<double2*>(o.Fu + e) = f;
        *reinterpret_cast<double2*>(o.Lxu + e) = l;
      } else {
        o.Fu[e] = dense_fu_at(K, n, nu, i0, j, ldf0, ri0, a0);
        o.Lxu[e] = in ? sc * K.Lxu[e] : 0.;
      }
    }
    // Luu (m x m): row pairs of m when m is even
    const bool wu = (m & 1) == 0;
    const RowSeg r2(wu ? m / 2 : m, NT, tid);
    if (r2.on) {
      const int u0 = wu ? 2 * r2.i : r2.i;
      for (int j = r2.g; j < m; j += r2.G) {
        const double v0 = (u0 < nu && j < nu) ? sc * K.Luu[j * nu + u0] : 0.;
        if (wu) {
          double2 v;
          v.x = v0;
          v.y = (u0 + 1 < nu && j < nu) ? sc * K.Luu[j * nu + u0 + 1] : 0.;
          *reinterpret_cast<double2*>(o.Luu + j * m + u0) = v;
        } else {
          o.Luu[j * m + u0] = v0;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// ShootingProblem::calc (shooting.hxx:133-161) and/or calcDiff (164-195) with
// the gaps of SolverDDP::calcDiff (ddp.cpp:160-176), fused: one workgroup per
// element walks its knots with the parameter block LDS-resident. Elements
// selected by sel_calc get xnext and the knot costs, those selected by
// sel_diff the derivative blocks (+ gaps when `gaps`).
// The derivative blocks (140 KB per knot at C5) dominate: they are written
// by every wave with 16-byte stores (a wave's store throughput is bounded by
// its outstanding stores, so bytes per store and waves per CU both count),
// half of them before the LDS-bound partial sums so that they drain while
// those run.
// ---------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(NT) void calc_fused_kernel(Dev D, int sel_calc, int sel_diff, int gaps, int64_t pcap) {
  const int b = blockIdx.x;
  const ElemState s = D.st[b];  // by value: a reference would re-load it from HBM after every store
  const bool do_calc = sel_calc >= 0 && selected(s, sel_calc);
  const bool do_diff = sel_diff >= 0 && selected(s, sel_diff);
  if (!do_calc && !do_diff) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* pl = sm;                 // pcap
  double* xu = pl + pcap;          // sX + sM
  double* xn = xu + D.sX + D.sM;   // sX
  double* pdyn = xn + D.sX;        // NT
  double* plx = pdyn + NT;         // NT
  double* plu = plx + NT;          // NT
  double* red = plu + NT;          // 16
  const int c = s.cur, nx = D.nx, n = D.n, m = D.m, T = D.T, tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const double* cached = nullptr;
  Stamp stamp(D.stamps ? D.stamps + (int64_t)D.B * 64 + ((int64_t)b * 8 + wid) * 8 : nullptr);
  // x and u of knots t+1..t+PD are in flight in registers while knot t
  // computes (a rotating window; thread i holds x_i, u_i; nx, m <= NT here)
  constexpr int PD = 4;
  double px[PD], pu[PD];
  auto fetch = [&](int t, double& x_, double& u_) {
    x_ = (t <= T && tid < nx) ? D.xs[c][D.knot(b, t) * D.sX + tid] : 0.;
    u_ = (t < T && tid < m) ? D.us[c][D.run(b, t) * D.sM + tid] : 0.;
  };
#pragma unroll
  for (int q = 0; q < PD; ++q) fetch(q, px[q], pu[q]);
  for (int t = 0; t <= T; ++t) {
    const fddp_knot_desc kd = D.knots[t];
    const double* P = stage_params<NT>(D.pblock(b, t), block_doubles_dev(kd.kind, nx, kd.nu), pl, pcap, cached);
    const int64_t kk = D.knot(b, t);
    const bool running = t < T;
    const int nu = kd.nu;
    const bool use_u = running && nu > 0;
    if (tid < nx) xu[tid] = px[0];
    if (use_u && tid < nu) xu[nx + tid] = pu[0];
#pragma unroll
    for (int q = 0; q + 1 < PD; ++q) {
      px[q] = px[q + 1];
      pu[q] = pu[q + 1];
    }
    fetch(t + PD, px[PD - 1], pu[PD - 1]);
    stamp.mark(0);
    __syncthreads();
    stamp.mark(1);
    const DenseKnot K(kd.kind, P, nx, nu);
    const bool want_dyn = do_calc && running;
    KnotDiffOut o;
    o.Fx = D.Fx + kk * D.sNN;
    o.Fu = D.Fu + kk * D.sNM;
    o.Lxx = D.Lxx + kk * D.sNN;
    o.Lxu = D.Lxu + kk * D.sNM;
    o.Luu = D.Luu + kk * D.sMM;
    if (do_diff) dense_write_blocks<NT>(K, n, m, nu, o, 1, tid);
    double cp = dense_partials<NT>(K, nx, nu, use_u, xu, want_dyn, do_diff, do_diff, do_calc, pdyn, plx, plu, tid);
    if (do_calc) {
      cp = wave_sum(cp);
      if (lane == 0) red[wid] = cp;
    }
    stamp.mark(2);
    __syncthreads();
    stamp.mark(3);
    // reductions spread over the waves: xnext rows from thread 0, Lu rows
    // from 64, Lx rows from 128 (NT = 512 here), the cost on thread NT - 1
    constexpr int TLU = NT >= 256 ? 64 : 0, TLX = NT >= 256 ? 128 : 0, TC = NT - 1;
    if (want_dyn) {
      for (int i = tid; i < K.nr; i += NT) dense_xnext(K, nx, i, seg_sum(pdyn, K.nr, i, NT), xu, xn);
    }
    if (do_calc && tid == TC) {
      double cst = 0.;
      for (int w = 0; w < NT / 64; ++w) cst += red[w];
      cst = K.dlqr && K.integ ? K.dt * cst : cst;
      D.kcost[c][kk] = cst;
    }
    if (do_diff) {
      const bool scale = K.dlqr && K.integ;
      double* Lx = D.Lx + kk * D.sN;
      double* Lu = D.Lu + kk * D.sM;
      for (int i = tid - TLX; i >= 0 && i < n; i += NT) {
        const double l = K.lx[i] + seg_sum(plx, nx, i, NT);
        Lx[i] = scale ? K.sc * l : l;
      }
      for (int i = tid - TLU; i >= 0 && i < m; i += NT) {
        double v = 0.;
        if (i < nu) {
          const double l = K.lu[i] + seg_sum(plu, nu, i, NT);
          v = scale ? K.sc * l : l;
        }
        Lu[i] = v;
      }
      stamp.mark(4);
      dense_write_blocks<NT>(K, n, m, nu, o, 2, tid);
    }
    stamp.mark(5);
    __syncthreads();  // xn complete
    stamp.mark(6);
    if (want_dyn) {
      double* xo = D.xnext[c] + D.run(b, t) * D.sX;
      if (tid < nx) xo[tid] = xn[tid];
    }
    if (do_diff && gaps) {
      if (!s.is_feasible) {
        // fs[0] = diff(xs[0], x0) = x0 - xs[0]; fs[t+1] = diff(xs[t+1], data[t].xnext)
        if (t == 0 && tid < n) {
          double* f = D.fs + D.knot(b, 0) * D.sN;
          const double* x0 = D.x0 + (int64_t)b * D.sX;
          f[tid] = x0[tid] - xu[tid];
        }
        if (running && tid < n) {  // px[0] holds xs[t+1][tid] now
          double* f = D.fs + D.knot(b, t + 1) * D.sN;
          const double* xng = D.xnext[c] + D.run(b, t) * D.sX;
          f[tid] = (want_dyn ? xn[tid] : xng[tid]) - px[0];
        }
      } else if (!s.was_feasible && tid < n) {  // closing the gaps
        D.fs[kk * D.sN + tid] = 0.;
      }
    }
    __syncthreads();
    stamp.mark(7);
  }
  stamp.flush();
}

// ---------------------------------------------------------------------------
// One forward trial (fwd_trial) with the dense-knot arithmetic above. Per
// knot: us_try = us - alpha k - K dx (segmented product with K read once from
// HBM; next knot's K, k, us, xs, fs, Vxx fs are prefetched into registers),
// then the dynamics and cost partials, then xnext. Knot costs go to kcost;
// the in-order running sum and the NaN checks run once at the end.
// ---------------------------------------------------------------------------
template <int NT, bool FAST>
__device__ __forceinline__ bool fwd_trial_fast(const Dev& D, int b, const ElemState& s, double alpha, double* xu,
                                               double* dxv, double* xn, double* pa, double* pdyn, double* red,
                                               int* flag, double& cost_try, double& dv, double* pl, int64_t pcap,
                                               const double*& cached) {
  const int n = D.n, nx = D.nx, m = D.m, T = D.T, tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  constexpr int NW = NT / 64;
  const int c = s.cur, o = 1 - c;
  const bool feas = s.is_feasible != 0;
  const bool full = feas || alpha == 1.;
  const double* x0 = D.x0 + (int64_t)b * D.sX;
  if (tid < nx) xn[tid] = x0[tid];
  bool bad = false;
  // this thread's share of K dx: row rk.i of K (m x n, ld m), columns
  // rk.g + s * rk.G, held in registers one knot ahead when they fit
  const RowSeg rk(m, NT, tid);
  constexpr int KMAX = 16;
  const int kcols = rk.on ? (n - rk.g + rk.G - 1) / rk.G : 0;
  const bool kreg = (n + rk.G - 1) / rk.G <= KMAX;
  // knots t+1..t+PD in flight in registers (rotating window; deeper windows
  // measured slower: register pressure)
  constexpr int PD = 1;
  double pK[PD][KMAX];
  double pxs[PD], pfs[PD], pvf[PD], pus[PD], pkv[PD];
  auto fetch = [&](int t, int q) {
    pxs[q] = pfs[q] = pvf[q] = pus[q] = pkv[q] = 0.;
    if (t > T) return;
    const int64_t kk = D.knot(b, t);
    if (tid < nx) {
      pxs[q] = D.xs[c][kk * D.sX + tid];
      pfs[q] = D.fs[kk * D.sN + tid];
      pvf[q] = feas ? 0. : D.Vxxfs[kk * D.sN + tid];
    }
    if (t < T) {
      const int64_t rr = D.run(b, t);
      if (tid < m) {
        pus[q] = D.us[c][rr * D.sM + tid];
        pkv[q] = D.k[rr * D.sM + tid];
      }
      if (kreg) {
        const double* Kt = D.K + rr * D.sNM;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) pK[q][j] = j < kcols ? Kt[(rk.g + j * rk.G) * m + rk.i] : 0.;
      }
    }
  };
#pragma unroll
  for (int q = 0; q < PD; ++q) fetch(q, q);
  __syncthreads();
  for (int t = 0; t <= T; ++t) {
    const int64_t kk = D.knot(b, t);
    const bool running = t < T;
    const fddp_knot_desc kd = D.knots[t];
    const int nu = kd.nu;
    const double cxs = pxs[0], cfs = pfs[0], cvf = pvf[0], cus = pus[0], ckv = pkv[0];
    double cK[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; ++j) cK[j] = pK[0][j];
#pragma unroll
    for (int q = 0; q + 1 < PD; ++q) {
      pxs[q] = pxs[q + 1];
      pfs[q] = pfs[q + 1];
      pvf[q] = pvf[q + 1];
      pus[q] = pus[q + 1];
      pkv[q] = pkv[q + 1];
#pragma unroll
      for (int j = 0; j < KMAX; ++j) pK[q][j] = pK[q + 1][j];
    }
    fetch(t + PD, PD - 1);
    // xs_try[t] = xnext  or  integrate(xnext, fs[t] * (alpha - 1)); dx = xs_try - xs
    double pd = 0.;
    if (tid < nx) {
      const double v = full ? xn[tid] : xn[tid] + cfs * (alpha - 1);
      xu[tid] = v;
      D.xs[o][kk * D.sX + tid] = v;
      const double dxi = v - cxs;
      dxv[tid] = dxi;
      if (!feas) pd = dxi * cvf;  // -fs^T Vxx diff(xs_try, xs)
    }
    if (!feas) {
      pd = wave_sum(pd);
      if (lane == 0) red[8 + wid] = pd;
    }
    const double* P = stage_params<NT>(D.pblock(b, t), block_doubles_dev(kd.kind, nx, nu), pl, pcap, cached);
    __syncthreads();
    if (running) {
      // us_try = us - k * alpha - K * dx
      if (rk.on) {
        double a;
        if (kreg) {
          double a0 = 0., a1 = 0.;
#pragma unroll
          for (int q = 0; q < KMAX; q += 2) {
            if (q < kcols) a0 = fma(cK[q], dxv[rk.g + q * rk.G], a0);
            if (q + 1 < kcols) a1 = fma(cK[q + 1], dxv[rk.g + (q + 1) * rk.G], a1);
          }
          a = a0 + a1;
        } else {
          a = seg_dot(D.K + D.run(b, t) * D.sNM, m, rk.i, rk.g, rk.G, n, dxv);
        }
        pa[rk.g * m + rk.i] = a;
      }
      __syncthreads();
      if (tid < m) {
        double v = 0.;
        if (tid < nu) v = (cus - ckv * alpha) - seg_sum(pa, m, tid, NT);
        xu[nx + tid] = v;
        D.us[o][D.run(b, t) * D.sM + tid] = v;
      }
      __syncthreads();
    }
    const DenseKnot K(kd.kind, P, nx, nu);
    double cp = dense_partials<NT>(K, nx, nu, running && nu > 0, xu, running, false, false, true, pdyn, nullptr,
                                   nullptr, tid);
    cp = wave_sum(cp);
    if (lane == 0) red[wid] = cp;
    __syncthreads();
    if (running) {
      for (int i = tid; i < K.nr; i += NT) dense_xnext(K, nx, i, seg_sum(pdyn, K.nr, i, NT), xu, xn);
    }
    if (tid == 0) {
      double cst = 0., p2 = 0.;
      for (int w = 0; w < NW; ++w) {
        cst += red[w];
        p2 += red[8 + w];
      }
      D.kcost[o][kk] = K.dlqr && K.integ ? K.dt * cst : cst;
      D.dvp[kk] = feas ? 0. : p2;
    }
    __syncthreads();  // xn complete; red / pa / pdyn free
    if (running && tid < nx) {
      D.xnext[o][D.run(b, t) * D.sX + tid] = xn[tid];
      bad |= bad_entry(xn[tid]);
    }
  }
  // cost_try in knot order with raiseIfNaN on every partial sum (fddp.cpp:
  // 189-196); dv: terminal first, then t = 0..T-1 (fddp.cpp:110-119)
  __syncthreads();
  if (tid == 0) {
    const double* kc = D.kcost[o] + D.knot(b, 0);
    double ct = 0.;
    bool nan = false;
    for (int t = 0; t <= T; ++t) {
      ct += kc[t];
      nan |= raise_if_nan(ct);
    }
    double acc = 0.;
    if (!feas) {
      const double* dvp = D.dvp + D.knot(b, 0);
      acc += dvp[T];
      for (int t = 0; t < T; ++t) acc += dvp[t];
    }
    red[0] = ct;
    red[1] = acc;
    bad |= nan;
  }
  const bool any_bad = wg_any(bad, flag);
  cost_try = red[0];
  dv = red[1];
  __syncthreads();
  return !any_bad;
}

}  // namespace fddp
