// Backward Riccati sweep on the fp64 matrix cores (v_mfma_f64_16x16x4_f64).
//
// Same computation as bwd_sweep (SolverDDP::backwardPass + computeGains,
// src/core/solvers/ddp.cpp:180-253, 298-310), reorganised for gfx950:
//
//   Z  = [Fx | Fu]                 (n x (n+m), streamed from HBM per knot)
//   G  = Vxx' Z                    (MFMA; Vxx' LDS-resident)
//   H  = G^T Z + [Lxx Lxu; . Luu]  = [[Qxx, Qxu], [Qux, Quu]]   (MFMA; the G
//        accumulators are the A operands of H with no data movement:
//        accumulator register r holds rows 4r..4r+3 of a 16-row block, which
//        is exactly the k-slice of one 16x16x4 step; Vxx' is symmetric so
//        G^T = Z^T Vxx' = Fx^T Vxx' as the reference forms it)
//   Quu^-1 from a Cholesky factorisation (wave 0, overlapped with the Qxx /
//        Qxu tiles of waves 1-3); a pivot <= 0 is the reference's LLT failure
//   K  = Quu^-1 Qxu^T, k = Quu^-1 Qu (MFMA / VALU)
//   Vxx = Qxx - Qxu K (+ xreg I), written symmetric (upper tile mirrored)
//   Vx  = Qx + K^T Quu k - 2 K^T Qu (+ Vxx fs)
//
// One workgroup (4 waves, one per SIMD) per batch element; the element's
// horizon is swept serially. n and m are padded to 16-multiples (NTL, MTL
// tiles); padded rows/cols are kept exactly zero.
// MFMA fragment maps (MI355X guide, f64 16x16x4): A[i=lane&15][k=lane>>4],
// B[k=lane>>4][j=lane&15], C/D col=lane&15, row=(lane>>4)+4*reg.
#pragma once

#include "fddp_device.hpp"

namespace fddp {

typedef double f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f64x4 mfma4(double a, double b, f64x4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// Column blocks of Z owned by each wave (computed on the host, LPT).
struct BwdSched {
  int32_t nown[4];
  int32_t blk[4][4];
  int32_t jstart[4][4];
};

template <int NTL, int MTL>
struct MfmaCfg {
  static constexpr int NP = 16 * NTL;
  static constexpr int MP = 16 * MTL;
  static constexpr int JT = NTL + MTL;
  // leading dimensions = 16 (mod 32) doubles: the two 16-lane halves of a
  // ds_read_b64 fragment read land on disjoint bank halves
  static constexpr int LDV = (NP % 32 == 0) ? NP + 16 : NP;
  static constexpr int LDQ = (MP % 32 == 0) ? MP + 16 : MP;
  static constexpr int NQXX = NTL * (NTL + 1) / 2;
  static constexpr int MAXOWN = (MTL > (NTL + 2) / 3) ? MTL : (NTL + 2) / 3;
  static_assert(MP <= 64, "u block must fit one wave for the factorisation");
  // LDS carve (doubles)
  static constexpr int oV = 0;
  static constexpr int oQxx = oV + LDV * NP;
  static constexpr int oQxu = oQxx + NQXX * 256;
  static constexpr int oQuu = oQxu + LDV * MP;
  static constexpr int oQi = oQuu + LDQ * MP;
  static constexpr int oKT = oQi + LDQ * MP;  // also the Cholesky factor during phase 1
  static constexpr int oVec = oKT + (LDV * MP > LDQ * MP ? LDV * MP : LDQ * MP);
  static constexpr int oVx = oVec;
  static constexpr int oQx = oVx + NP;
  static constexpr int oFs = oQx + NP;
  static constexpr int oVf = oFs + NP;
  static constexpr int oQu = oVf + NP;
  static constexpr int oKv = oQu + MP;
  static constexpr int oQuuk = oKv + MP;
  static constexpr int oCol = oQuuk + MP;
  static constexpr int oDinv = oCol + MP;
  static constexpr int oRed = oDinv + MP;
  static constexpr int oFlag = oRed + 64;
  static constexpr int total = oFlag + 2;
  static constexpr size_t bytes = sizeof(double) * total;
};

template <int NTL, int MTL>
__device__ __forceinline__ double zfrag(const double* __restrict__ Fx, const double* __restrict__ Fu, int n, int m,
                                        int s, int j, int q, int c) {
  const int row = 4 * s + q;
  if (j < NTL) {
    const int col = 16 * j + c;
    return (row < n && col < n) ? Fx[(int64_t)col * n + row] : 0.;
  }
  const int col = 16 * (j - NTL) + c;
  return (row < n && col < m) ? Fu[(int64_t)col * n + row] : 0.;
}

// Diagnostic phase timer (FDDP_STAMPS=1): per wave, cycles spent per phase.
struct Stamp {
  unsigned long long* out;
  unsigned long long t0;
  __device__ Stamp(unsigned long long* o) : out(o), t0(o ? __builtin_amdgcn_s_memtime() : 0) {}
  __device__ __forceinline__ void mark(int ph) {
    if (out) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if ((threadIdx.x & 63) == 0) out[ph] += t - t0;
      t0 = t;
    }
  }
};

template <int NTL, int MTL>
__device__ __forceinline__ bool bwd_sweep_mfma(const Dev& D, int b, bool feas, double xreg, double ureg, double* sm,
                               const BwdSched& sch) {
  using Cfg = MfmaCfg<NTL, MTL>;
  constexpr int NP = Cfg::NP, MP = Cfg::MP, JT = Cfg::JT, LDV = Cfg::LDV, LDQ = Cfg::LDQ, MAXOWN = Cfg::MAXOWN;
  double* V = sm + Cfg::oV;
  double* Qxx = sm + Cfg::oQxx;
  double* Qxu = sm + Cfg::oQxu;
  double* Quu = sm + Cfg::oQuu;
  double* Qi = sm + Cfg::oQi;
  double* KT = sm + Cfg::oKT;
  double* Lm = sm + Cfg::oKT;
  double* vx = sm + Cfg::oVx;
  double* qx = sm + Cfg::oQx;
  double* fsv = sm + Cfg::oFs;
  double* qu = sm + Cfg::oQu;
  double* kv = sm + Cfg::oKv;
  double* quuk = sm + Cfg::oQuuk;
  double* colbuf = sm + Cfg::oCol;
  double* dinv = sm + Cfg::oDinv;
  double* red = sm + Cfg::oRed;
  int* flag = (int*)(sm + Cfg::oFlag);

  const int n = D.n, m = D.m, T = D.T, tid = threadIdx.x;
  const int wid = tid >> 6, lane = tid & 63, q = lane >> 4, c = lane & 15;
  const bool xr = !isnan(xreg), ur = !isnan(ureg);
  Stamp stamp(D.stamps ? D.stamps + ((int64_t)b * 4 + wid) * 8 : nullptr);

  // ---- terminal: Vxx = Lxx_T (+ xreg I), Vx = Lx_T (+ Vxx fs_T) ------------
  {
    const int64_t kk = D.knot(b, T);
    const double* Lxx = D.Lxx + kk * D.sNN;
    const double* Lx = D.Lx + kk * D.sN;
    const double* fs = D.fs + kk * D.sN;
    // stored transposed so that G = V Z uses Lxx_T itself (it may be asymmetric)
    for (int e = tid; e < NP * NP; e += 256) {
      const int i = e % NP, j = e / NP;
      double v = (i < n && j < n) ? Lxx[(int64_t)i * n + j] : 0.;
      if (xr && i == j && i < n) v += xreg;
      V[j * LDV + i] = v;
    }
    for (int i = tid; i < NP; i += 256) fsv[i] = i < n ? fs[i] : 0.;
    __syncthreads();
    double pv[2] = {0., 0.};
    for (int i = tid; i < NP; i += 256) {
      double v = i < n ? Lx[i] : 0.;
      if (!feas && i < n) {
        double a = 0.;
        for (int j = 0; j < n; ++j) a += Lxx[(int64_t)j * n + i] * fsv[j];
        if (xr) a += xreg * fsv[i];
        D.Vxxfs[kk * D.sN + i] = a;
        v += a;
        pv[0] += v * fsv[i];
        pv[1] += fsv[i] * a;
      }
      vx[i] = v;
    }
    wg_sums<256, 2>(pv, red);
    if (tid == 0) {
      double* p = D.part + kk * 8;
      p[0] = 0.; p[1] = 0.; p[2] = pv[0]; p[3] = pv[1]; p[4] = 0.;
    }
    if (D.dVxx) {
      for (int e = tid; e < n * n; e += 256) {
        const int i = e % n, j = e / n;
        D.dVxx[kk * D.sNN + e] = Lxx[e] + ((xr && i == j) ? xreg : 0.);
      }
      for (int i = tid; i < n; i += 256) D.dVx[kk * D.sN + i] = vx[i];
    }
  }

  for (int t = T - 1; t >= 0; --t) {
    const int64_t kk = D.knot(b, t);
    const int64_t rr = D.run(b, t);
    const double* Fx = D.Fx + kk * D.sNN;
    const double* Fu = D.Fu + kk * D.sNM;
    const double* Lxx = D.Lxx + kk * D.sNN;
    const double* Lxu = D.Lxu + kk * D.sNM;
    const double* Luu = D.Luu + kk * D.sMM;
    __syncthreads();
    stamp.mark(7);
    // ---- phase 0: fs, Qx = Lx + Fx^T Vx', Qu = Lu + Fu^T Vx' -----------------
    {
      const double* fs = D.fs + kk * D.sN;
      const double* Lx = D.Lx + kk * D.sN;
      const double* Lu = D.Lu + kk * D.sM;
      for (int i = tid; i < NP; i += 256) fsv[i] = i < n ? fs[i] : 0.;
      for (int o = tid; o < NP + MP; o += 256) {
        if (o < NP) {
          double a = 0.;
          if (o < n) {
            const double* col = Fx + (int64_t)o * n;
            for (int k2 = 0; k2 < n; ++k2) a += col[k2] * vx[k2];
            a = Lx[o] + a;
          }
          qx[o] = a;
        } else {
          const int u = o - NP;
          double a = 0.;
          if (u < m) {
            const double* col = Fu + (int64_t)u * n;
            for (int k2 = 0; k2 < n; ++k2) a += col[k2] * vx[k2];
            a = Lu[u] + a;
          }
          qu[u] = a;
        }
      }
      if (tid == 0) *flag = 0;
    }
    stamp.mark(0);
    __syncthreads();
    stamp.mark(1);
    // ---- phase 1: G = V Z_i, H(i, j) = G_i^T Z_j + L(i, j) per owned block ---
    {
      const int nown = sch.nown[wid];
      int ib[MAXOWN], js[MAXOWN];
#pragma unroll
      for (int o = 0; o < MAXOWN; ++o) {
        ib[o] = o < nown ? sch.blk[wid][o] : 0;
        js[o] = o < nown ? sch.jstart[wid][o] : JT;
      }
      // Initial accumulator of H(i, j): the cost block (symmetric part of Lxx
      // for Qxx, which the reference reaches through its Vxx symmetrisation;
      // Lxu for Qxu; Luu + ureg I for Quu).
      auto linit = [&](f64x4(&acc)[MAXOWN], int j) {
#pragma unroll
        for (int o = 0; o < MAXOWN; ++o) {
          acc[o] = f64x4{0., 0., 0., 0.};
          if (o < nown && j >= js[o]) {
            const int i = ib[o];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int R = 16 * i + q + 4 * r, C = 16 * j + c;
              double v = 0.;
              if (j < NTL) {
                if (R < n && C < n) v = 0.5 * (Lxx[(int64_t)C * n + R] + Lxx[(int64_t)R * n + C]);
              } else if (i < NTL) {
                const int Cu = C - NP;
                if (R < n && Cu < m) v = Lxu[(int64_t)Cu * n + R];
              } else {
                const int Ru = R - NP, Cu = C - NP;
                if (Ru < m && Cu < m) {
                  v = Luu[(int64_t)Cu * m + Ru];
                  if (ur && Ru == Cu) v += ureg;
                }
              }
              acc[o][r] = v;
            }
          }
        }
      };
      int jmin = JT;
#pragma unroll
      for (int o = 0; o < MAXOWN; ++o) jmin = js[o] < jmin ? js[o] : jmin;
      // Issue every global load of the G phase and of the first H column at
      // once: the fragments are independent, so one memory latency is exposed
      // per batch instead of one per k-step.
      double zg[MAXOWN][4 * NTL];
#pragma unroll
      for (int o = 0; o < MAXOWN; ++o)
#pragma unroll
        for (int s2 = 0; s2 < 4 * NTL; ++s2) zg[o][s2] = o < nown ? zfrag<NTL, MTL>(Fx, Fu, n, m, s2, ib[o], q, c) : 0.;
      double zc[4 * NTL];
      f64x4 ac[MAXOWN];
      if (jmin < JT) {
#pragma unroll
        for (int s2 = 0; s2 < 4 * NTL; ++s2) zc[s2] = zfrag<NTL, MTL>(Fx, Fu, n, m, s2, jmin, q, c);
        linit(ac, jmin);
      }
      f64x4 G[MAXOWN][NTL];
#pragma unroll
      for (int o = 0; o < MAXOWN; ++o)
#pragma unroll
        for (int a = 0; a < NTL; ++a) G[o][a] = f64x4{0., 0., 0., 0.};
      if (nown > 0) {
#pragma unroll
        for (int s = 0; s < 4 * NTL; ++s) {
          double vf[NTL];
#pragma unroll
          for (int a = 0; a < NTL; ++a) vf[a] = V[(4 * s + q) * LDV + 16 * a + c];
#pragma unroll
          for (int o = 0; o < MAXOWN; ++o) {
            if (o < nown) {
#pragma unroll
              for (int a = 0; a < NTL; ++a) G[o][a] = mfma4(vf[a], zg[o][s], G[o][a]);
            }
          }
        }
      }
      // H columns, double-buffered: column j+1's fragments and cost block are
      // in flight while column j's MFMAs run.
      for (int j = jmin; j < JT; ++j) {
        const bool more = j + 1 < JT;
        double zn[4 * NTL];
        f64x4 an[MAXOWN];
        if (more) {
#pragma unroll
          for (int s2 = 0; s2 < 4 * NTL; ++s2) zn[s2] = zfrag<NTL, MTL>(Fx, Fu, n, m, s2, j + 1, q, c);
          linit(an, j + 1);
        }
#pragma unroll
        for (int s = 0; s < 4 * NTL; ++s) {
#pragma unroll
          for (int o = 0; o < MAXOWN; ++o)
            if (o < nown && j >= js[o]) ac[o] = mfma4(G[o][s >> 2][s & 3], zc[s], ac[o]);
        }
#pragma unroll
        for (int o = 0; o < MAXOWN; ++o) {
          if (o < nown && j >= js[o]) {
            const int i = ib[o];
            if (j < NTL) {
              const int tq = i * NTL - (i * (i - 1)) / 2 + (j - i);
#pragma unroll
              for (int r = 0; r < 4; ++r) Qxx[tq * 256 + r * 64 + lane] = ac[o][r];
            } else if (i < NTL) {
#pragma unroll
              for (int r = 0; r < 4; ++r) Qxu[(16 * (j - NTL) + c) * LDV + 16 * i + q + 4 * r] = ac[o][r];
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r) Quu[(16 * (j - NTL) + c) * LDQ + 16 * (i - NTL) + q + 4 * r] = ac[o][r];
            }
          }
        }
        if (more) {
#pragma unroll
          for (int s2 = 0; s2 < 4 * NTL; ++s2) zc[s2] = zn[s2];
#pragma unroll
          for (int o = 0; o < MAXOWN; ++o) ac[o] = an[o];
        }
      }
      // ---- wave 0: Quu^-1 by in-place Gauss-Jordan (overlaps waves 1-3) ------
      // Without pivoting on an SPD matrix the k-th pivot equals L(k,k)^2 of its
      // Cholesky factor, so `pivot <= 0` is exactly Eigen LLT's failure
      // (ddp.cpp:300-304). Lane l owns column j = l % MP and RPL rows
      // i = (l / MP) * RPL + r of the MP x MP matrix; row k / column k are
      // broadcast through LDS at each step.
      if (wid == 0) {
        constexpr int RPL = MP * MP / 64;
        static_assert(MP * MP % 64 == 0 && 64 % MP == 0, "Gauss-Jordan lane layout");
        const int jc = lane % MP, h = lane / MP;
        double* rowbuf = dinv;  // MP doubles
        __builtin_amdgcn_s_waitcnt(0xc07f);  // this wave's Quu stores have landed
        __builtin_amdgcn_wave_barrier();
        double A[RPL];
#pragma unroll
        for (int r = 0; r < RPL; ++r) A[r] = Quu[jc * LDQ + h * RPL + r];
        bool bad = false;
        for (int k = 0; k < m; ++k) {
          const int hk = k / RPL, rk = k % RPL;
          // column k (before elimination) and the pivot
#pragma unroll
          for (int r = 0; r < RPL; ++r)
            if (jc == k) colbuf[h * RPL + r] = A[r];
          __builtin_amdgcn_s_waitcnt(0xc07f);
          __builtin_amdgcn_wave_barrier();
          const double p = colbuf[k];
          if (!(p > 0.)) bad = true;
          const double pinv = 1. / p;
          // row k scaled by 1/p (A(k,k) <- 1 first, so it becomes 1/p)
#pragma unroll
          for (int r = 0; r < RPL; ++r) {
            if (h == hk && r == rk) {
              const double v = (jc == k ? 1. : A[r]) * pinv;
              A[r] = v;
              rowbuf[jc] = v;
            }
          }
          __builtin_amdgcn_s_waitcnt(0xc07f);
          __builtin_amdgcn_wave_barrier();
          const double rkj = rowbuf[jc];
#pragma unroll
          for (int r = 0; r < RPL; ++r) {
            const int i = h * RPL + r;
            if (i != k) {
              const double f = colbuf[i];
              A[r] = (jc == k ? 0. : A[r]) - f * rkj;
            }
          }
          __builtin_amdgcn_s_waitcnt(0xc07f);
          __builtin_amdgcn_wave_barrier();
        }
        // Quu^-1 is symmetric: store (i, j) at (j, i) (conflict-free rows)
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
          const int i = h * RPL + r;
          Qi[i * LDQ + jc] = (i < m && jc < m) ? A[r] : 0.;
        }
        if (bad && lane == 0) *flag = 1;
      }
    }
    stamp.mark(2);
    __syncthreads();
    stamp.mark(3);
    if (*flag) return false;
    // ---- phase 2: K = Quu^-1 Qxu^T (MFMA), k = Quu^-1 Qu ------------------------
    for (int jt = wid; jt < NTL; jt += 4) {
      f64x4 acc[MTL];
#pragma unroll
      for (int it = 0; it < MTL; ++it) acc[it] = f64x4{0., 0., 0., 0.};
#pragma unroll
      for (int s = 0; s < 4 * MTL; ++s) {
        const double bq = Qxu[(4 * s + q) * LDV + 16 * jt + c];
#pragma unroll
        for (int it = 0; it < MTL; ++it) acc[it] = mfma4(Qi[(4 * s + q) * LDQ + 16 * it + c], bq, acc[it]);
      }
      double* Kg = D.K + rr * D.sNM;
      const int C = 16 * jt + c;
#pragma unroll
      for (int it = 0; it < MTL; ++it)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int R = 16 * it + q + 4 * r;
          KT[R * LDV + C] = acc[it][r];
          if (R < m && C < n) Kg[(int64_t)C * m + R] = acc[it][r];
        }
    }
    for (int i = tid; i < MP; i += 256) {
      double a = 0.;
      if (i < m)
        for (int k2 = 0; k2 < m; ++k2) a += Qi[k2 * LDQ + i] * qu[k2];
      kv[i] = a;
      if (i < m) D.k[rr * D.sM + i] = a;
    }
    stamp.mark(4);
    __syncthreads();
    // ---- phase 2b: Quuk = Quu k ; Vxx = Qxx - Qxu K (+ xreg I), symmetric ------
    for (int i = tid; i < MP; i += 256) {
      double a = 0.;
      if (i < m)
        for (int k2 = 0; k2 < m; ++k2) a += Quu[k2 * LDQ + i] * kv[k2];
      quuk[i] = a;
    }
    {
      bool bad = false;
      for (int u = wid; u < Cfg::NQXX; u += 4) {
        int i = 0, rem = u;
        while (rem >= NTL - i) {
          rem -= NTL - i;
          ++i;
        }
        const int j = i + rem;
        f64x4 acc;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = Qxx[u * 256 + r * 64 + lane];
#pragma unroll
        for (int s = 0; s < 4 * MTL; ++s)
          acc = mfma4(-Qxu[(4 * s + q) * LDV + 16 * i + c], KT[(4 * s + q) * LDV + 16 * j + c], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int R = 16 * i + q + 4 * r, C = 16 * j + c;
          double v = acc[r];
          if (xr && R == C && R < n) v += xreg;
          if (i < j || R <= C) {
            V[C * LDV + R] = v;
            V[R * LDV + C] = v;
            if (R < n && C < n) bad |= bad_entry(v);
          }
        }
      }
      if (bad) *flag = 1;
    }
    stamp.mark(5);
    __syncthreads();
    // ---- phase 3: Vx, Vxx fs, checks, reduction terms, stores ----------------
    {
      bool bad = false;
      double pv[5] = {0., 0., 0., 0., 0.};
      for (int i = tid; i < NP; i += 256) {
        double v = 0.;
        if (i < n) {
          double a = 0., c2 = 0.;
          for (int k2 = 0; k2 < m; ++k2) {
            const double kt = KT[k2 * LDV + i];
            a += kt * quuk[k2];
            c2 += kt * qu[k2];
          }
          v = ur ? (qx[i] + a) - 2 * c2 : qx[i] - c2;
          if (!feas) {
            double f = 0.;
            for (int j = 0; j < n; ++j) f += V[j * LDV + i] * fsv[j];
            D.Vxxfs[kk * D.sN + i] = f;
            v += f;
            pv[2] += v * fsv[i];
            pv[3] += fsv[i] * f;
          }
          bad |= bad_entry(v);
        }
        vx[i] = v;
      }
      for (int i = tid; i < m; i += 256) {
        pv[0] += qu[i] * kv[i];
        pv[1] += kv[i] * quuk[i];
        pv[4] += qu[i] * qu[i];
      }
      if (bad) *flag = 1;
      wg_sums<256, 5>(pv, red);
      if (tid == 0) {
        double* p = D.part + kk * 8;
        for (int j = 0; j < 5; ++j) p[j] = pv[j];
      }
      if (D.dQxx) {
        for (int e = tid; e < n * n; e += 256) {
          const int R = e % n, C = e / n;
          const int lo = R < C ? R : C, hi = R < C ? C : R;
          const int i = lo / 16, j = hi / 16;
          // Qxx tile (i, j) element (lo, hi) in accumulator order
          const int tq = i * NTL - (i * (i - 1)) / 2 + (j - i);
          const int rl = lo - 16 * i, cl = hi - 16 * j;
          double v;
          if (i == j) {
            const int rr2 = R - 16 * i, cc2 = C - 16 * j;
            v = Qxx[tq * 256 + (rr2 >> 2) * 64 + (rr2 & 3) * 16 + cc2];
          } else {
            v = Qxx[tq * 256 + (rl >> 2) * 64 + (rl & 3) * 16 + cl];
          }
          D.dQxx[rr * D.sNN + e] = v;
          D.dVxx[kk * D.sNN + e] = V[C * LDV + R];
        }
        for (int e = tid; e < n * m; e += 256) D.dQxu[rr * D.sNM + e] = Qxu[(e / n) * LDV + e % n];
        for (int e = tid; e < m * m; e += 256) D.dQuu[rr * D.sMM + e] = Quu[(e / m) * LDQ + e % m];
        for (int i = tid; i < n; i += 256) {
          D.dQx[rr * D.sN + i] = qx[i];
          D.dVx[kk * D.sN + i] = vx[i];
        }
        for (int i = tid; i < m; i += 256) D.dQu[rr * D.sM + i] = qu[i];
      }
    }
    stamp.mark(6);
    __syncthreads();
    if (*flag) return false;
  }
  return true;
}

template <int NTL, int MTL>
__global__ __launch_bounds__(256) void backward_mfma_kernel(Dev D, Prm prm, int mode, BwdSched sch) {
  const int b = blockIdx.x;
  ElemState* st = D.st + b;
  if (mode == 0 && !st->active) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  using Cfg = MfmaCfg<NTL, MTL>;
  int* flag = (int*)(sm + Cfg::oFlag);
  const bool feas = st->is_feasible != 0;
  double xreg = st->xreg, ureg = st->ureg;
  bool ok;
  for (;;) {
    ok = bwd_sweep_mfma<NTL, MTL>(D, b, feas, xreg, ureg, sm, sch);
    __syncthreads();
    if (ok || mode == 1) break;
    xreg *= prm.regfactor;  // increaseRegularization (ddp.cpp:312-318)
    if (xreg > prm.regmax) xreg = prm.regmax;
    ureg = xreg;
    if (xreg == prm.regmax) break;
  }
  (void)flag;
  if (threadIdx.x == 0) {
    st->xreg = xreg;
    st->ureg = ureg;
    st->bwd_fail = ok ? 0 : 1;
    if (!ok && mode == 0) {
      st->status = FDDP_STATUS_REGMAX;
      st->active = 0;
      st->n_iter_run += 1;
    }
    if (ok) {
      const double* p = D.part + D.knot(b, 0) * 8;
      const int T = D.T;
      double dg = 0., dq = 0., stop = 0.;
      if (!feas) {
        dg -= p[T * 8 + 2];
        dq += p[T * 8 + 3];
      }
      for (int t = 0; t < T; ++t) {
        dg += p[t * 8 + 0];
        dq -= p[t * 8 + 1];
        stop += p[t * 8 + 4];
        if (!feas) {
          dg -= p[t * 8 + 2];
          dq += p[t * 8 + 3];
        }
      }
      st->dg = dg;
      st->dq = dq;
      st->stop = stop;
    }
  }
}

}  // namespace fddp
