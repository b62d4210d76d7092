// Backward Riccati sweep for small knots (n = ndx <= 16, m = nu_max <= 16): one wave
// per batch element, no workgroup barrier.
//
// The same computation as bwd_sweep (fddp_kernels.hpp; SolverDDP::backwardPass +
// computeGains, src/core/solvers/ddp.cpp:180-253, 298-310), for the sizes where the
// 4/8-wave MFMA sweep (bwd_mfma.hpp) spends its knot on barriers and LDS-DMA waits
// (the C3 arm, n = 14, m = 7: 16 x 16 tiles mostly padding). Here:
//  - one 64-lane wave owns an element; its LDS area is private, so the phases are
//    ordered by wave-local fences (wave_sync), never by s_barrier;
//  - the next knot's Fx, Fu, Lxx, Lxu, Luu, Lx, Lu, fs are loaded into registers while
//    the current knot is swept (one HBM round trip per knot, hidden), and stored to LDS
//    at the top of the next iteration;
//  - every product is an fp64 VALU dot product over k in increasing order (as the
//    generic sweep's wg_gemm), one output entry per lane per pass (gfx950 runs f64 on
//    the vector unit at the matrix-core rate; at these sizes the tiles would be padding);
//  - Quu is factorised by Cholesky (the reference's LLT; a pivot <= 0 is its
//    backward_error), K and k by the two triangular solves, one right-hand side per lane.
// Several waves (elements) share a workgroup (kWavesPerWg) so a CU holds many elements.
#pragma once

#include "fddp_device.hpp"

namespace fddp {

constexpr int kBwdWaveMax = 16;  // n, m bound of this variant
constexpr int kWavesPerWg = 4;   // elements per workgroup (one per wave)

// LDS doubles per wave: 7 matrices, the operand block (5 matrices + 3 vectors), 5 vectors
__host__ __device__ constexpr int bwd_wave_doubles() {
  return 12 * kBwdWaveMax * kBwdWaveMax + 8 * kBwdWaveMax + 8;
}
// registers of the next knot's operands per lane (ceil(total / 64))
constexpr int kBwdWavePre = (4 * kBwdWaveMax * kBwdWaveMax + kBwdWaveMax * kBwdWaveMax + 3 * kBwdWaveMax + 63) / 64;

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double wave_sum64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// The knot's operands in one flat index space: Fx (n n) | Fu (n m) | Lxx (n n) |
// Lxu (n m) | Luu (m m) | Lx (n) | Lu (m) | fs (n); `pre` holds entries lane + 64 r.
struct WaveKnot {
  int n, m, o1, o2, o3, o4, o5, o6, o7, tot;
  __device__ WaveKnot(int n_, int m_) : n(n_), m(m_) {
    o1 = n * n;
    o2 = o1 + n * m;
    o3 = o2 + n * n;
    o4 = o3 + n * m;
    o5 = o4 + m * m;
    o6 = o5 + n;
    o7 = o6 + m;
    tot = o7 + n;
  }
  __device__ double load(const Dev& D, int64_t kk, int e) const {
    if (e < o1) return D.Fx[kk * D.sNN + e];
    if (e < o2) return D.Fu[kk * D.sNM + (e - o1)];
    if (e < o3) return D.Lxx[kk * D.sNN + (e - o2)];
    if (e < o4) return D.Lxu[kk * D.sNM + (e - o3)];
    if (e < o5) return D.Luu[kk * D.sMM + (e - o4)];
    if (e < o6) return D.Lx[kk * D.sN + (e - o5)];
    if (e < o7) return D.Lu[kk * D.sM + (e - o6)];
    return D.fs[kk * D.sN + (e - o7)];
  }
};

// one element's sweep on the calling wave; false on backward_error
__device__ __forceinline__ bool bwd_sweep_wave(const Dev& D, int b, bool feas, double xreg, double ureg, double* w) {
  const int n = D.n, m = D.m, T = D.T, lane = threadIdx.x & 63;
  const bool xr = !isnan(xreg), ur = !isnan(ureg);
  constexpr int NN = kBwdWaveMax * kBwdWaveMax;
  double* V = w;             // Vxx' then Qxx, then Vxx (n x n, ld n)
  double* A = V + NN;        // Fx^T Vxx' (n x n)
  double* BU = A + NN;       // Fu^T Vxx' (nu x n, ld m)
  double* Qxu = BU + NN;     // n x nu, ld n
  double* Quu = Qxu + NN;    // nu x nu, ld m
  double* Lc = Quu + NN;     // Cholesky factor (lower), ld m
  double* Km = Lc + NN;      // K (nu x n, ld m)
  double* op = Km + NN;      // the knot's operands (WaveKnot order): Fx | Fu | Lxx | Lxu | Luu | Lx | Lu | fs
  // vectors after the operand block (at most 5 NN + 3 kBwdWaveMax doubles)
  double* vec = op + 5 * NN + 3 * kBwdWaveMax;
  double* vxv = vec;                    // Vx
  double* qx = vxv + kBwdWaveMax;
  double* qu = qx + kBwdWaveMax;
  double* kv = qu + kBwdWaveMax;
  double* quuk = kv + kBwdWaveMax;
  int* flag = (int*)(quuk + kBwdWaveMax);
  const WaveKnot kn(n, m);
  double pre[kBwdWavePre];
  auto fetch = [&](int t) {  // knot t's operands into registers
    const int64_t kk = D.knot(b, t);
#pragma unroll
    for (int r = 0; r < kBwdWavePre; ++r) {
      const int e = lane + 64 * r;
      pre[r] = e < kn.tot ? kn.load(D, kk, e) : 0.;
    }
  };
  auto stage = [&]() {  // registers -> LDS
#pragma unroll
    for (int r = 0; r < kBwdWavePre; ++r) {
      const int e = lane + 64 * r;
      if (e < kn.tot) op[e] = pre[r];
    }
  };
  const double* Fx = op;
  const double* Fu = op + kn.o1;
  const double* Lxx = op + kn.o2;
  const double* Lxu = op + kn.o3;
  const double* Luu = op + kn.o4;
  const double* Lx = op + kn.o5;
  const double* Lu = op + kn.o6;
  const double* fs = op + kn.o7;
  if (lane == 0) *flag = 0;
  // terminal: Vxx = Lxx_T (+ xreg I), Vx = Lx_T (+ Vxx fs_T)
  fetch(T);
  stage();
  if (T > 0) fetch(T - 1);
  wave_sync();
  {
    const int64_t kk = D.knot(b, T);
    for (int e = lane; e < n * n; e += 64) {
      const int i = e % n, j = e / n;
      V[e] = (xr && i == j) ? Lxx[e] + xreg : Lxx[e];
    }
    wave_sync();
    double p2 = 0., p3 = 0.;
    if (lane < n) {
      double v = Lx[lane];
      if (!feas) {
        double a = 0.;
        for (int j = 0; j < n; ++j) a += V[j * n + lane] * fs[j];
        D.Vxxfs[kk * D.sN + lane] = a;
        v += a;
        p2 = v * fs[lane];
        p3 = fs[lane] * a;
      }
      vxv[lane] = v;
    }
    p2 = wave_sum64(p2);
    p3 = wave_sum64(p3);
    if (lane == 0) {
      double* p = D.part + kk * 8;
      p[0] = 0.;
      p[1] = 0.;
      p[2] = p2;
      p[3] = p3;
      p[4] = 0.;
    }
    if (D.dVxx) {
      for (int e = lane; e < n * n; e += 64) D.dVxx[kk * D.sNN + e] = V[e];
      if (lane < n) D.dVx[kk * D.sN + lane] = vxv[lane];
    }
    wave_sync();
  }
  for (int t = T - 1; t >= 0; --t) {
    const int64_t kk = D.knot(b, t);
    const int nu = D.knots[t].nu;
    stage();  // knot t's operands (fetched during the previous knot)
    if (t > 0) fetch(t - 1);
    wave_sync();
    // A = Fx^T Vxx', BU = Fu^T Vxx' ; Qx = Lx + Fx^T Vx', Qu = Lu + Fu^T Vx'
    for (int e = lane; e < n * n + nu * n; e += 64) {
      const bool ux = e >= n * n;
      const int f = ux ? e - n * n : e;
      const int i = ux ? f % nu : f % n, j = ux ? f / nu : f / n;
      const double* c = ux ? Fu + i * n : Fx + i * n;
      double a = 0.;
      for (int k2 = 0; k2 < n; ++k2) a += c[k2] * V[j * n + k2];
      if (ux)
        BU[j * m + i] = a;
      else
        A[j * n + i] = a;
    }
    if (lane < n + nu) {
      const bool ux = lane >= n;
      const int i = ux ? lane - n : lane;
      const double* c = ux ? Fu + i * n : Fx + i * n;
      double a = 0.;
      for (int k2 = 0; k2 < n; ++k2) a += c[k2] * vxv[k2];
      if (ux)
        qu[i] = Lu[i] + a;
      else
        qx[i] = Lx[i] + a;
    }
    wave_sync();
    // Qxx = Lxx + A Fx (into V), Qxu = Lxu + A Fu, Quu = Luu + BU Fu (+ ureg I)
    for (int e = lane; e < n * n + n * nu + nu * nu; e += 64) {
      double a = 0.;
      if (e < n * n) {
        const int i = e % n, j = e / n;
        for (int k2 = 0; k2 < n; ++k2) a += A[k2 * n + i] * Fx[j * n + k2];
        V[e] = Lxx[e] + a;
      } else if (e < n * n + n * nu) {
        const int f = e - n * n, i = f % n, j = f / n;
        for (int k2 = 0; k2 < n; ++k2) a += A[k2 * n + i] * Fu[j * n + k2];
        Qxu[j * n + i] = Lxu[j * n + i] + a;
      } else {
        const int f = e - n * n - n * nu, i = f % nu, j = f / nu;
        for (int k2 = 0; k2 < n; ++k2) a += BU[k2 * m + i] * Fu[j * n + k2];
        double v = Luu[j * m + i] + a;
        if (ur && i == j) v += ureg;
        Quu[j * m + i] = v;
      }
    }
    wave_sync();
    if (D.dQxx) {
      const int64_t r = D.run(b, t);
      for (int e = lane; e < n * n; e += 64) D.dQxx[r * D.sNN + e] = V[e];
      if (lane < n) D.dQx[r * D.sN + lane] = qx[lane];
      for (int e = lane; e < n * m; e += 64) D.dQxu[r * D.sNM + e] = (e / n < nu) ? Qxu[e] : 0.;
      for (int e = lane; e < m * m; e += 64) D.dQuu[r * D.sMM + e] = (e % m < nu && e / m < nu) ? Quu[(e / m) * m + e % m] : 0.;
      if (lane < m) D.dQu[r * D.sM + lane] = lane < nu ? qu[lane] : 0.;
    }
    if (nu) {
      // Cholesky (lower) of Quu, column by column; Eigen's LLT fails on a pivot <= 0
      for (int j = 0; j < nu; ++j) {
        if (lane == 0) {
          double sd = Quu[j * m + j];
          for (int k2 = 0; k2 < j; ++k2) sd -= Lc[k2 * m + j] * Lc[k2 * m + j];
          if (!(sd > 0.)) *flag = 1;
          Lc[j * m + j] = sqrt(sd);
        }
        wave_sync();
        const double ljj = Lc[j * m + j];
        const int i = j + 1 + lane;
        if (i < nu) {
          double v = Quu[j * m + i];
          for (int k2 = 0; k2 < j; ++k2) v -= Lc[k2 * m + i] * Lc[k2 * m + j];
          Lc[j * m + i] = v / ljj;
        }
        wave_sync();
      }
      if (*flag) return false;
      // K = Quu^-1 Qxu^T (Km, nu x n, ld m), k = Quu^-1 Qu: one right-hand side per lane
      if (lane <= n) {
        double* y = lane < n ? Km + lane * m : kv;
        for (int i = 0; i < nu; ++i) {
          double v = lane < n ? Qxu[i * n + lane] : qu[i];
          for (int k2 = 0; k2 < i; ++k2) v -= Lc[k2 * m + i] * y[k2];
          y[i] = v / Lc[i * m + i];
        }
        for (int i = nu - 1; i >= 0; --i) {
          double v = y[i];
          for (int k2 = i + 1; k2 < nu; ++k2) v -= Lc[i * m + k2] * y[k2];
          y[i] = v / Lc[i * m + i];
        }
      }
      wave_sync();
      // store K, k ; Quuk = Quu k
      {
        const int64_t r = D.run(b, t);
        double* Kg = D.K + r * D.sNM;
        for (int e = lane; e < m * n; e += 64) Kg[e] = (e % m < nu) ? Km[e] : 0.;
        if (lane < m) D.k[r * D.sM + lane] = lane < nu ? kv[lane] : 0.;
        if (lane < nu) {
          double a = 0.;
          for (int k2 = 0; k2 < nu; ++k2) a += Quu[k2 * m + lane] * kv[k2];
          quuk[lane] = a;
        }
      }
      wave_sync();
      // Vx = Qx + K^T Quuk - 2 K^T Qu (or Qx - K^T Qu without ureg); Vxx = Qxx - Qxu K
      if (lane < n) {
        const double* Kc = Km + lane * m;
        if (ur) {
          double a = 0., c = 0.;
          for (int k2 = 0; k2 < nu; ++k2) a += Kc[k2] * quuk[k2];
          for (int k2 = 0; k2 < nu; ++k2) c += Kc[k2] * qu[k2];
          vxv[lane] = (qx[lane] + a) - 2 * c;
        } else {
          double c = 0.;
          for (int k2 = 0; k2 < nu; ++k2) c += Kc[k2] * qu[k2];
          vxv[lane] = qx[lane] - c;
        }
      }
      double vn[(kBwdWaveMax * kBwdWaveMax + 63) / 64];
#pragma unroll
      for (int r = 0; r < (kBwdWaveMax * kBwdWaveMax + 63) / 64; ++r) {
        const int e = lane + 64 * r;
        if (e < n * n) {
          const int i = e % n, j = e / n;
          double a = 0.;
          for (int k2 = 0; k2 < nu; ++k2) a += Qxu[k2 * n + i] * Km[j * m + k2];
          vn[r] = V[e] - a;
        }
      }
      wave_sync();  // every lane has read V before it is overwritten
#pragma unroll
      for (int r = 0; r < (kBwdWaveMax * kBwdWaveMax + 63) / 64; ++r) {
        const int e = lane + 64 * r;
        if (e < n * n) V[e] = vn[r];
      }
    } else {
      if (lane < n) vxv[lane] = qx[lane];
      const int64_t r = D.run(b, t);
      for (int e = lane; e < m * n; e += 64) D.K[r * D.sNM + e] = 0.;
      if (lane < m) D.k[r * D.sM + lane] = 0.;
    }
    wave_sync();
    // Vxx = 0.5 (Vxx + Vxx^T) (+ xreg I): entries (i < j) by their lane pairs
    {
      double sv[(kBwdWaveMax * kBwdWaveMax + 63) / 64];
#pragma unroll
      for (int r = 0; r < (kBwdWaveMax * kBwdWaveMax + 63) / 64; ++r) {
        const int e = lane + 64 * r;
        if (e < n * n) {
          const int i = e % n, j = e / n;
          sv[r] = i == j ? (xr ? V[e] + xreg : V[e]) : 0.5 * (V[j * n + i] + V[i * n + j]);
        }
      }
      wave_sync();
#pragma unroll
      for (int r = 0; r < (kBwdWaveMax * kBwdWaveMax + 63) / 64; ++r) {
        const int e = lane + 64 * r;
        if (e < n * n) V[e] = sv[r];
      }
    }
    wave_sync();
    // Vx += Vxx fs (infeasible), NaN checks, reduction terms
    bool bad = false;
    double pv[5] = {0., 0., 0., 0., 0.};
    if (lane < n) {
      double v = vxv[lane];
      if (!feas) {
        double a = 0.;
        for (int j = 0; j < n; ++j) a += V[j * n + lane] * fs[j];
        D.Vxxfs[kk * D.sN + lane] = a;
        v += a;
        vxv[lane] = v;
        pv[2] = v * fs[lane];
        pv[3] = fs[lane] * a;
      }
      bad |= bad_entry(v);
    }
    for (int e = lane; e < n * n; e += 64) bad |= bad_entry(V[e]);
    if (lane < nu) {
      pv[0] = qu[lane] * kv[lane];
      pv[1] = kv[lane] * quuk[lane];
      pv[4] = qu[lane] * qu[lane];
    }
#pragma unroll
    for (int j = 0; j < 5; ++j) pv[j] = wave_sum64(pv[j]);
    if (lane == 0) {
      double* p = D.part + kk * 8;
      for (int j = 0; j < 5; ++j) p[j] = pv[j];
    }
    if (D.dVxx) {
      for (int e = lane; e < n * n; e += 64) D.dVxx[kk * D.sNN + e] = V[e];
      if (lane < n) D.dVx[kk * D.sN + lane] = vxv[lane];
    }
    if (__any(bad)) return false;
    wave_sync();
  }
  return true;
}

// One element per wave, kWavesPerWg elements per workgroup. The in-kernel retry loop and
// the reductions of the generic backward_kernel (fddp_kernels.hpp).
__global__ __launch_bounds__(64 * kWavesPerWg) void backward_wave_kernel(Dev D, Prm prm, int mode) {
  const int b = blockIdx.x * kWavesPerWg + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= D.B) return;
  ElemState* st = D.st + b;
  if (mode == 0 && !st->active) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* w = sm + (int64_t)(threadIdx.x >> 6) * bwd_wave_doubles();
  const bool feas = st->is_feasible != 0;
  double xreg = st->xreg, ureg = st->ureg;
  bool ok;
  for (;;) {
    ok = bwd_sweep_wave(D, b, feas, xreg, ureg, w);
    wave_sync();
    if (ok || mode == 1) break;
    xreg *= prm.regfactor;  // increaseRegularization (ddp.cpp:312-318)
    if (xreg > prm.regmax) xreg = prm.regmax;
    ureg = xreg;
    if (xreg == prm.regmax) break;
  }
  if (lane == 0) {
    st->xreg = xreg;
    st->ureg = ureg;
    st->bwd_fail = ok ? 0 : 1;
    if (!ok && mode == 0) {  // solve() returns false inside this loop body (fddp.cpp:41-43)
      st->status = FDDP_STATUS_REGMAX;
      st->active = 0;
      st->n_iter_run += 1;
    }
    if (ok) {
      // updateExpectedImprovement (fddp.cpp:126-147) and stoppingCriteria, in knot order
      const double* p = D.part + D.knot(b, 0) * 8;
      const int T = D.T;
      double dg = 0., dq = 0., stop = 0.;
      if (!feas) {
        dg -= p[T * 8 + 2];
        dq += p[T * 8 + 3];
      }
      for (int t = 0; t < T; ++t) {
        if (D.knots[t].nu != 0) {
          dg += p[t * 8 + 0];
          dq -= p[t * 8 + 1];
          stop += p[t * 8 + 4];
        }
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
