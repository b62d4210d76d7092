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
#include "dense_knot.hpp"
#include "bwd_mfma.hpp"  // Stamp

namespace fddp {

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
// element, the parameter block LDS-resident. Elements selected by sel_calc
// get xnext and the knot costs, those selected by sel_diff the derivative
// blocks, Lx, Lu (+ gaps when `gaps`).
// Knots that share one parameter block (the reference's std::vector(T, model)
// shares one model over the running knots; host-computed segments) go in
// tiles of 8: the per-knot matrix-vector products of a tile become one small
// matrix product, [Lxx | Lxu] [x; u], [Lxu^T | Luu] [x; u] and F [x; u]
// (F = [Fx | Fu] or [Fq | Fv | Fu]) with one output row per lane and 8 knot
// columns in flight (8 independent FMA chains, operands broadcast from LDS);
// Lx, Lu, xnext, gaps and knot costs are written straight from registers.
// The 140 KB of derivative blocks per knot (C5) are the bulk: dedicated
// waves stream them with 16-byte stores and never load from global memory.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void dense_xnext2(const DenseKnot& K, int nx, int i, double a, double xi, double vi,
                                             double& o0, double& o1) {  // dense_xnext for one row pair
  if (!K.drift_free) a += K.f0[i];
  if (!K.dlqr) {
    o0 = a;
    return;
  }
  if (K.integ) {
    const double dt = K.dt, dt2 = dt * dt;
    const double dq = vi * dt + a * dt2;  // v*dt + a*dt^2 (euler.hxx:66)
    const double dv = a * dt;             // a*dt (euler.hxx:67)
    o0 = xi + dq;
    o1 = vi + dv;
  } else {
    o0 = xi;
    o1 = vi;
  }
}

constexpr int kCalcKT = 16;  // knots per compute tile (the MFMA N dimension)
constexpr int kCalcKP = 18;  // xu columns: the tile's knots + x of the next knot, padded even

// LDS doubles of calc_tiled_kernel besides the parameter block
__host__ __device__ inline int64_t calc_tiled_lds(int64_t sX, int64_t sM) {
  return (sX + sM) * kCalcKP + 8 * 16 + 16;
}

// (knot_desc_s: fddp_device.hpp)
__device__ __forceinline__ int segend_s(const Dev& D, int t) {
  typedef __attribute__((address_space(4))) const int* cptr;
  return ((cptr)D.segend)[t];
}

// Parameter block -> LDS by LDS-DMA (no register round trip: every chunk of
// the block is in flight at once). The fast path guarantees size <= the LDS
// reserve (fddp_create); callers then read the block through the LDS pointer
// itself, so that the compiler emits LDS reads: a flat read (pointer of
// unknown address space) also waits on vmcnt, i.e. for every global store
// still in flight.
template <int NT>
__device__ __forceinline__ void stage_params_batched(const double* g, int64_t size, double* lds, const double*& cached) {
  if (g == cached) return;
  __syncthreads();
  if ((reinterpret_cast<uintptr_t>(g) & 15) == 0) {
    dma_vec<NT / 64>(lds, g, (int)size, threadIdx.x >> 6, threadIdx.x & 63);
    dma_barrier();
  } else {
    for (int64_t e = threadIdx.x; e < size; e += NT) lds[e] = g[e];
    __syncthreads();
  }
  cached = g;
}

// One compute tile (knots t0..t0+nt-1, nt <= 16, one parameter block) on the
// workgroup's fp64 matrix cores: the stacked products
//   R1 = [Lxx x | Lxu u]   (Lx, cost)      rows i < nx
//   R2 = [Lxu^T x | Luu u] (Lu, cost)      rows j < nu
//   R3 = F [x; u]          (xnext, gaps)   rows i < nr   (calc only)
// for the tile's 16 knot columns, in 16-row blocks spread over the waves
// (v_mfma_f64_16x16x4: A = parameter rows from LDS, B = xu[k][knot] from
// LDS; accumulator register r of lane (q, c) = row q + 4r of knot column c).
// The x and u parts of R1 / R2 accumulate separately (the cost uses
// 0.5 x.Lxx x + x.Lxu u). Outputs are written from the accumulators; knot
// costs are reduced through `red` ([8 waves][16]).
template <int NT>
__device__ __forceinline__ void calc_tile_mfma(const Dev& D, const DenseKnot& K, const ElemState& s, int b, int t0,
                                               int nt, int nu, bool do_calc, bool do_diff, int gaps, double* xu,
                                               double* red, int tid) {
  constexpr int KP = kCalcKP, NW = NT / 64;
  const int c_ = s.cur, nx = D.nx, n = D.n, m = D.m, T = D.T;
  const int lane = tid & 63, wid = tid >> 6, q = lane >> 4, cc = lane & 15;
  const bool running = t0 < T;
  const int nuu = running ? nu : 0, nk = nx + nuu;
  // xu: x of knots t0..t0+nt (the last for the gaps; none after the terminal
  // knot), u of t0..t0+nt-1; entry e -> (column tt, row k), rows fastest
  {
    const int cnt = nk * nt + (t0 + nt <= T ? nx : 0);
    constexpr int U = 4;
    for (int base = 0; base < cnt; base += NT * U) {
      double r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e0 = base + NT * u + tid, e = e0 < cnt ? e0 : cnt - 1;
        const int tt = e / nk, k = e - tt * nk;
        r[u] = k < nx ? D.xs[c_][D.knot(b, t0 + tt) * D.sX + k] : D.us[c_][D.run(b, t0 + tt) * D.sM + k - nx];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = base + NT * u + tid;
        if (e < cnt) {
          const int tt = e / nk, k = e - tt * nk;
          xu[k * KP + tt] = r[u];
        }
      }
    }
  }
  __syncthreads();
  const bool scale = K.dlqr && K.integ;
  const bool want_dyn = do_calc && running;
  const bool infeas_gaps = do_diff && gaps && !s.is_feasible;
  const int nb1 = (nx + 15) >> 4, nb2 = nu > 0 ? (nu + 15) >> 4 : 0, nb3 = want_dyn ? (K.nr + 15) >> 4 : 0;
  const int nq = nx / 2;
  const bool col_ok = cc < nt;
  const int t = t0 + cc;
  double cp = 0.;  // this lane's share of knot cc's cost
  for (int rb = wid; rb < nb1 + nb2 + nb3; rb += NW) {
    f64x4 a1 = {0., 0., 0., 0.}, a2 = {0., 0., 0., 0.};
    if (rb < nb1) {  // R1 rows r0 + c: Lxx (x part) and Lxu (u part)
      const int r0 = 16 * rb, ra = r0 + cc;
      for (int k0 = 0; k0 < nx; k0 += 4) {
        const int k = k0 + q;
        const double av = (ra < nx && k < nx) ? K.Lxx[k * nx + ra] : 0.;
        const double bv = k < nx ? xu[k * KP + cc] : 0.;
        a1 = mfma4(av, bv, a1);
      }
      for (int k0 = 0; k0 < nuu; k0 += 4) {
        const int k = k0 + q;
        const double av = (ra < nx && k < nuu) ? K.Lxu[k * nx + ra] : 0.;
        const double bv = k < nuu ? xu[(nx + k) * KP + cc] : 0.;
        a2 = mfma4(av, bv, a2);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = r0 + q + 4 * r;
        if (col_ok && i < nx) {
          const double xi = xu[i * KP + cc];
          if (do_diff) {
            const double l = K.lx[i] + (a1[r] + a2[r]);
            D.Lx[D.knot(b, t) * D.sN + i] = scale ? K.sc * l : l;
          }
          cp += fma(K.lx[i], xi, xi * (0.5 * a1[r] + a2[r]));
        }
      }
    } else if (rb < nb1 + nb2) {  // R2 rows: Lxu^T (x part) and Luu (u part)
      const int r0 = 16 * (rb - nb1), ra = r0 + cc;
      for (int k0 = 0; k0 < nx; k0 += 4) {
        const int k = k0 + q;
        const double av = (ra < nu && k < nx) ? K.Lxu[ra * nx + k] : 0.;
        const double bv = k < nx ? xu[k * KP + cc] : 0.;
        a1 = mfma4(av, bv, a1);
      }
      for (int k0 = 0; k0 < nuu; k0 += 4) {
        const int k = k0 + q;
        const double av = (ra < nu && k < nuu) ? K.Luu[k * nu + ra] : 0.;
        const double bv = k < nuu ? xu[(nx + k) * KP + cc] : 0.;
        a2 = mfma4(av, bv, a2);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = r0 + q + 4 * r;
        if (col_ok && j < nu) {
          if (do_diff) {
            const double l = K.lu[j] + (a1[r] + a2[r]);
            D.Lu[D.knot(b, t) * D.sM + j] = scale ? K.sc * l : l;
          }
          if (nuu > 0) {
            const double uj = xu[(nx + j) * KP + cc];
            cp += fma(K.lu[j], uj, 0.5 * uj * a2[r]);
          }
        }
      }
    } else {  // R3 rows of F [x; u]: xnext (+ the gaps fs[t+1] = xnext - xs[t+1])
      const int r0 = 16 * (rb - nb1 - nb2), ra = r0 + cc;
      for (int k0 = 0; k0 < nk; k0 += 4) {
        const int k = k0 + q;
        const double av = (ra < K.nr && k < nk) ? K.F[k * K.nr + ra] : 0.;
        const double bv = k < nk ? xu[k * KP + cc] : 0.;
        a1 = mfma4(av, bv, a1);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = r0 + q + 4 * r;
        if (col_ok && i < K.nr) {
          double* xo = D.xnext[c_] + D.run(b, t) * D.sX;
          double* f = D.fs + D.knot(b, t + 1) * D.sN;
          double o0, o1 = 0.;
          dense_xnext2(K, nx, i, a1[r], xu[i * KP + cc], K.dlqr ? xu[(nq + i) * KP + cc] : 0., o0, o1);
          xo[i] = o0;
          if (infeas_gaps) f[i] = o0 - xu[i * KP + cc + 1];
          if (K.dlqr) {
            xo[nq + i] = o1;
            if (infeas_gaps) f[nq + i] = o1 - xu[(nq + i) * KP + cc + 1];
          }
        }
      }
    }
  }
  if (do_calc) {
    cp += __shfl_xor(cp, 16, 64);
    cp += __shfl_xor(cp, 32, 64);
    if (q == 0) red[wid * 16 + cc] = cp;
  }
  __syncthreads();
  if (do_calc && tid < nt) {
    double cst = 0.;
    for (int w = 0; w < NW; ++w) cst += red[w * 16 + tid];
    D.kcost[c_][D.knot(b, t0 + tid)] = scale ? K.dt * cst : cst;
  }
  if (do_diff && m > nu) {  // Lu rows nu..m-1 of the padded block
    for (int e = tid; e < nt * (m - nu); e += NT) {
      const int tt = e / (m - nu), j = nu + e - tt * (m - nu);
      D.Lu[D.knot(b, t0 + tt) * D.sM + j] = 0.;
    }
  }
  if (do_diff && gaps) {
    if (!s.is_feasible) {
      // fs[0] = diff(xs[0], x0) = x0 - xs[0]; fs[t+1] = diff(xs[t+1], data[t].xnext)
      if (t0 == 0)
        for (int i = tid; i < n; i += NT) D.fs[D.knot(b, 0) * D.sN + i] = D.x0[(int64_t)b * D.sX + i] - xu[i * KP];
      if (running && !want_dyn)  // xnext of the current candidate (computed by an earlier calc)
        for (int e = tid; e < nt * n; e += NT) {
          const int tt = e / n, i = e - tt * n;
          D.fs[D.knot(b, t0 + tt + 1) * D.sN + i] = D.xnext[c_][D.run(b, t0 + tt) * D.sX + i] - xu[i * KP + tt + 1];
        }
    } else if (!s.was_feasible) {  // closing the gaps
      for (int e = tid; e < nt * n; e += NT) {
        const int tt = e / n, i = e - tt * n;
        D.fs[D.knot(b, t0 + tt) * D.sN + i] = 0.;
      }
    }
  }
  __syncthreads();  // xu / red free for the next tile
}

// The derivative blocks of knots [ts, te) (one parameter block, so the same
// values at every knot): each thread computes its 16-byte units of a block
// once (unit u = doubles 2u, 2u+1 of the column-major block: rows 2p, 2p+1 of
// column j) and then only stores them, knot after knot. Same values as
// dense_write_blocks. Needs n and m even (callers check).
// A: 0 Lxx, 1 Fx, 2 Fu, 3 Lxu, 4 Luu.
template <int A>
__device__ __forceinline__ double2 block_unit(const DenseKnot& K, int n, int nu, double sc, int i0, int j) {
  double2 w;
  if constexpr (A == 0) {
    w.x = sc * K.Lxx[j * n + i0];
    w.y = sc * K.Lxx[j * n + i0 + 1];
  } else if constexpr (A == 1 || A == 2) {
    int ldf0, ri0, jd0, ldf1, ri1, jd1;
    double a0, a1;
    dense_fx_rows(K, n, i0, ldf0, ri0, jd0, a0);
    dense_fx_rows(K, n, i0 + 1, ldf1, ri1, jd1, a1);
    if constexpr (A == 1) {
      w.x = dense_fx_at(K, n, i0, j, ldf0, ri0, jd0, a0);
      w.y = dense_fx_at(K, n, i0 + 1, j, ldf1, ri1, jd1, a1);
    } else {
      w.x = dense_fu_at(K, n, nu, i0, j, ldf0, ri0, a0);
      w.y = dense_fu_at(K, n, nu, i0 + 1, j, ldf1, ri1, a1);
    }
  } else if constexpr (A == 3) {
    const bool in = j < nu;
    w.x = in ? sc * K.Lxu[j * n + i0] : 0.;
    w.y = in ? sc * K.Lxu[j * n + i0 + 1] : 0.;
  } else {
    w.x = (i0 < nu && j < nu) ? sc * K.Luu[j * nu + i0] : 0.;
    w.y = (i0 + 1 < nu && j < nu) ? sc * K.Luu[j * nu + i0 + 1] : 0.;
  }
  return w;
}

template <int A, int NB>
__device__ __forceinline__ void write_block_segment(const Dev& D, const DenseKnot& K, int b, int ts, int te, int nu,
                                                    double sc, int ptid) {
  constexpr int UK = 8;  // units per thread in flight
  const int n = D.n, m = D.m;
  double* const base = A == 0 ? D.Lxx : A == 1 ? D.Fx : A == 2 ? D.Fu : A == 3 ? D.Lxu : D.Luu;
  const int64_t stride = A <= 1 ? D.sNN : A <= 3 ? D.sNM : D.sMM;
  const int nrow = A <= 3 ? n : m, ncol = A <= 1 ? n : m;
  const int np = nrow / 2, units = np * ncol;
  for (int u0 = 0; u0 < units; u0 += UK * NB) {
    double2 v[UK];
#pragma unroll
    for (int k = 0; k < UK; ++k) {
      const int u = u0 + k * NB + ptid, uc = u < units ? u : units - 1;
      const int j = uc / np, i0 = 2 * (uc - j * np);
      v[k] = block_unit<A>(K, n, nu, sc, i0, j);
    }
    for (int t = ts; t < te; ++t) {
      double2* dst = reinterpret_cast<double2*>(base + D.knot(b, t) * stride);
#pragma unroll
      for (int k = 0; k < UK; ++k) {
        const int u = u0 + k * NB + ptid;
        if (u < units) dst[u] = v[k];
      }
    }
  }
}

template <int NB>
__device__ __forceinline__ void write_blocks_segment(const Dev& D, const DenseKnot& K, int b, int ts, int te, int nu,
                                                     int ptid) {
  const double sc = (K.dlqr && K.integ) ? K.sc : 1.;
  write_block_segment<0, NB>(D, K, b, ts, te, nu, sc, ptid);
  write_block_segment<1, NB>(D, K, b, ts, te, nu, sc, ptid);
  write_block_segment<2, NB>(D, K, b, ts, te, nu, sc, ptid);
  write_block_segment<3, NB>(D, K, b, ts, te, nu, sc, ptid);
  write_block_segment<4, NB>(D, K, b, ts, te, nu, sc, ptid);
}

// Per segment: the compute tiles (calc_tile_mfma, the whole workgroup), then
// every wave streams its share of the derivative blocks (params in LDS ->
// registers -> global; the block writer loads nothing from global memory, so
// its stores never wait, and no compute load queues behind them).
template <int NT>
__global__ __launch_bounds__(NT) void calc_tiled_kernel(Dev D, int sel_calc, int sel_diff, int gaps, int64_t pcap) {
  constexpr int KT = kCalcKT, KP = kCalcKP;
  const int b = blockIdx.x;
  const ElemState s = D.st[b];  // by value: a reference would re-load it from HBM after every store
  const bool do_calc = sel_calc >= 0 && selected(s, sel_calc);
  const bool do_diff = sel_diff >= 0 && selected(s, sel_diff);
  if (!do_calc && !do_diff) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int nx = D.nx, n = D.n, m = D.m, T = D.T, tid = threadIdx.x;
  const int wid = tid >> 6;
  double* pl = sm;
  double* xu = pl + pcap;                   // [nx + m][KP]
  double* red = xu + (D.sX + D.sM) * KP;    // [8][16]
  const double* cached = nullptr;
  Stamp stamp(D.stamps ? D.stamps + (int64_t)D.B * 64 + ((int64_t)b * 8 + wid) * 8 : nullptr);
  for (int ts = 0; ts <= T;) {
    const int te = segend_s(D, ts);  // knots [ts, te) share knot desc and parameter block
    const fddp_knot_desc kd = knot_desc_s(D, ts);
    const int nu = kd.nu;
    stage_params_batched<NT>(D.params + kd.param_offset + (int64_t)b * kd.param_stride,
                             block_doubles_dev(kd.kind, nx, nu), pl, cached);
    stamp.mark(0);
    const DenseKnot K(kd.kind, pl, nx, nu);
    for (int t0 = ts; t0 < te; t0 += KT) {
      const int nt = te - t0 < KT ? te - t0 : KT;
      calc_tile_mfma<NT>(D, K, s, b, t0, nt, nu, do_calc, do_diff, gaps, xu, red, tid);
    }
    stamp.mark(1);
    if (do_diff && (n & 1) == 0 && (m & 1) == 0) {
      write_blocks_segment<NT>(D, K, b, ts, te, nu, tid);
    } else if (do_diff) {
      for (int t = ts; t < te; ++t) {
        const int64_t kk = D.knot(b, t);
        KnotDiffOut o;
        o.Fx = D.Fx + kk * D.sNN;
        o.Fu = D.Fu + kk * D.sNM;
        o.Lxx = D.Lxx + kk * D.sNN;
        o.Lxu = D.Lxu + kk * D.sNM;
        o.Luu = D.Luu + kk * D.sMM;
        dense_write_blocks<NT>(K, n, m, nu, o, 3, tid);
      }
    }
    stamp.mark(5);
    ts = te;
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
  // knots t+1..t+PD in flight in registers (rotating window). Two knots ahead: C2's knot
  // 13.5k -> 12.6k cycles (phase stamps, wave 0), rollout 0.60 -> 0.57 ms, at 256 VGPRs
  // and 2 spills; deeper windows measured slower (register pressure)
#ifndef FDDP_FAST_PD
#define FDDP_FAST_PD 2
#endif
  constexpr int PD = FDDP_FAST_PD;
  double pK[PD][KMAX];
  double pxs[PD], pfs[PD], pvf[PD], pus[PD], pkv[PD], plb[PD], pub[PD];
  auto fetch = [&](int t, int q) {
    pxs[q] = pfs[q] = pvf[q] = pus[q] = pkv[q] = 0.;
    plb[q] = -INFINITY;  // no limits: the clamp below is an exact no-op
    pub[q] = INFINITY;
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
        if (D.box_knot(b, t)) {
          plb[q] = D.ulb[rr * D.sM + tid];
          pub[q] = D.uub[rr * D.sM + tid];
        }
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
  // (diagnostic phase timer, FDDP_STAMPS=1 on the stamps build: per wave, summed)
  Stamp stamp(D.stamps && wid == 0 ? D.stamps + (int64_t)D.B * 128 + (int64_t)b * 8 : nullptr);  // (wave 0's)
  __syncthreads();
  for (int t = 0; t <= T; ++t) {
    const int64_t kk = D.knot(b, t);
    const bool running = t < T;
    const fddp_knot_desc kd = knot_desc_s(D, t);  // scalar loads: no wait behind the prefetches
    const int nu = kd.nu;
    const double cxs = pxs[0], cfs = pfs[0], cvf = pvf[0], cus = pus[0], ckv = pkv[0], clb = plb[0], cub = pub[0];
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
      plb[q] = plb[q + 1];
      pub[q] = pub[q + 1];
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
    stamp.mark(0);
    stage_params_batched<NT>(D.params + kd.param_offset + (int64_t)b * kd.param_stride, block_doubles_dev(kd.kind, nx, nu), pl, cached);
    const double* P = pl;
    __syncthreads();
    stamp.mark(1);
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
        // SolverBoxFDDP::forwardPass clamp (box-fddp.cpp:100-102); +-inf when unlimited
        if (D.box && tid < nu) v = std_min(std_max(v, clb), cub);
        xu[nx + tid] = v;
        D.us[o][D.run(b, t) * D.sM + tid] = v;
      }
      __syncthreads();
    }
    stamp.mark(2);
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
    stamp.mark(3);
    if (running && tid < nx) {
      D.xnext[o][D.run(b, t) * D.sX + tid] = xn[tid];
      bad |= bad_entry(xn[tid]);
    }
    stamp.mark(4);
  }
  stamp.flush();
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
