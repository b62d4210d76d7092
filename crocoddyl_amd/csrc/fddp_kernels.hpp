// libfddp_hip kernels (generic sizes). One workgroup per knot for the
// ShootingProblem fan-out, one workgroup per batch element for the serial
// Riccati sweep and the line-searched rollout.
#pragma once

#include "fddp_device.hpp"
#include "box_qp.hpp"
#include "knots.hpp"

namespace fddp {

// Non-template kernels are compiled in one translation unit each: FDDP_TU_MAIN
// (fddp_hip.hip) or FDDP_TU_MB = the multibody variant (k_mb.hip, ktab.hpp).

// Doubles in a knot's parameter block (layouts in include/fddp_hip.h); the
// multibody block carries its size in its header (g: the block).
__device__ inline int64_t block_doubles_dev(int kind, int nx, int nu, const double* g = nullptr) {
  if (is_mb_kind(kind)) return (int64_t)g[3];
  if (kind == FDDP_KNOT_LQR) return FDDP_PARAM_HEADER + 2LL * nx * nx + 2LL * nx * nu + (int64_t)nu * nu + 2LL * nx + nu;
  if (kind == FDDP_KNOT_UNICYCLE) return FDDP_PARAM_HEADER;
  const int64_t nq = nx / 2;
  return FDDP_PARAM_HEADER + 2 * nq * nq + nq * nu + nq + (int64_t)nx * nx + (int64_t)nx * nu + (int64_t)nu * nu + nx +
         nu;
}

// StateMultibody with a free-flyer root (nx = ndx + 1: x = (p, quat xyzw, q_rest, v)),
// otherwise a Euclidean state (StateVector, or StateMultibody over revolute joints).
// diff(x0, x1) / integrate(x, dx) (multibody.hxx:54-91, euclidean.hxx:28-61) over the
// threads of a workgroup; thread `first` (0 by default) does the free-flyer's SE(3)
// part, so two differences of one phase can run their logs on different waves. out
// may not alias the inputs. No barrier inside.
template <int NT>
__device__ __forceinline__ void state_diff_wg(const Dev& D, const double* x0, const double* x1, double* out,
                                              int first = 0) {
  const int n = D.n;
  if (D.nx == n) {
    for (int i = threadIdx.x; i < n; i += NT) out[i] = x1[i] - x0[i];
    return;
  }
  const int nv = n / 2, nq = D.nx - nv;
  for (int i = ((int)threadIdx.x + NT - first) % NT; i < n; i += NT) {
    if (i < 6) {
      if (i == 0) mb::ff_difference(x0, x1, out);
    } else if (i < nv) {
      out[i] = x1[i + 1] - x0[i + 1];
    } else {
      out[i] = x1[nq + i - nv] - x0[nq + i - nv];
    }
  }
}
// integrate(x, s * dx)
template <int NT>
__device__ __forceinline__ void state_integrate_wg(const Dev& D, const double* x, const double* dx, double s,
                                                   double* out) {
  const int n = D.n;
  if (D.nx == n) {
    for (int i = threadIdx.x; i < n; i += NT) out[i] = x[i] + dx[i] * s;
    return;
  }
  const int nv = n / 2, nq = D.nx - nv;
  for (int i = threadIdx.x; i < n; i += NT) {
    if (i < 6) {
      if (i == 0) {
        double d6[6];
        for (int e = 0; e < 6; ++e) d6[e] = dx[e] * s;
        mb::ff_integrate(x, d6, out);
      }
    } else if (i < nv) {
      out[i + 1] = x[i + 1] + dx[i] * s;
    } else {
      out[nq + i - nv] = x[nq + i - nv] + dx[i] * s;
    }
  }
}

// Keep one knot parameter block resident in LDS across consecutive knots that
// share it (a reference model object shared by several knots, or one
// element's perturbed model used at every t). Returns the pointer to read the
// block from (LDS copy, or global when it does not fit `cap` doubles).
// Contains barriers when it (re)stages: call uniformly.
template <int NT>
__device__ inline const double* stage_params(const double* g, int64_t size, double* lds, int64_t cap,
                                             const double*& cached) {
  if (g == cached) return lds;
  if (size > cap) return g;
  __syncthreads();
  const int64_t n2 = size & ~int64_t(1);
  const bool al = ((reinterpret_cast<uintptr_t>(g) & 15) == 0);
  if (al) {
    const double2* s2 = reinterpret_cast<const double2*>(g);
    double2* d2 = reinterpret_cast<double2*>(lds);
    for (int64_t e = threadIdx.x; e < n2 / 2; e += NT) d2[e] = s2[e];
    for (int64_t e = n2 + threadIdx.x; e < size; e += NT) lds[e] = g[e];
  } else {
    for (int64_t e = threadIdx.x; e < size; e += NT) lds[e] = g[e];
  }
  __syncthreads();
  cached = g;
  return lds;
}

// ---------------------------------------------------------------------------
// Workgroup GEMM: C = C0 + sgn * op(A) op(B), column-major, 2x2 register tiles.
// TA: A is stored K x M (use A^T).  TB: B is stored N x K (use B^T).
// C0 may alias C (each output reads its own C0 entry before writing it).
// C0 == nullptr means zero.
// ---------------------------------------------------------------------------
template <int NT, bool TA, bool TB>
__device__ __forceinline__ void wg_gemm(int M, int N, int K, const double* __restrict__ A, int lda, const double* __restrict__ Bm,
                        int ldb, const double* C0, int ldc0, double* C, int ldc, double sgn) {
  const int mt = (M + 1) >> 1, ntl = (N + 1) >> 1;
  for (int tile = threadIdx.x; tile < mt * ntl; tile += NT) {
    const int i0 = (tile % mt) * 2, j0 = (tile / mt) * 2;
    const bool ok1 = i0 + 1 < M, okj = j0 + 1 < N;
    const int i1 = ok1 ? i0 + 1 : i0, j1 = okj ? j0 + 1 : j0;
    double c00 = 0., c01 = 0., c10 = 0., c11 = 0.;
    for (int k = 0; k < K; ++k) {
      const double a0 = TA ? A[(int64_t)i0 * lda + k] : A[(int64_t)k * lda + i0];
      const double a1 = TA ? A[(int64_t)i1 * lda + k] : A[(int64_t)k * lda + i1];
      const double b0 = TB ? Bm[(int64_t)k * ldb + j0] : Bm[(int64_t)j0 * ldb + k];
      const double b1 = TB ? Bm[(int64_t)k * ldb + j1] : Bm[(int64_t)j1 * ldb + k];
      c00 += a0 * b0;
      c01 += a0 * b1;
      c10 += a1 * b0;
      c11 += a1 * b1;
    }
    auto put = [&](int i, int j, double c) {
      const double base = C0 ? C0[(int64_t)j * ldc0 + i] : 0.;
      C[(int64_t)j * ldc + i] = base + sgn * c;
    };
    put(i0, j0, c00);
    if (okj) put(i0, j1, c01);
    if (ok1) put(i1, j0, c10);
    if (ok1 && okj) put(i1, j1, c11);
  }
}

// ---------------------------------------------------------------------------
// ShootingProblem::calc (shooting.hxx:133-161): one workgroup per element
// walks its T+1 knots (independent knots; the loop only lets the element's
// parameter block stay in LDS). Writes data[t].xnext and data[t].cost of
// trajectory cur.
// ---------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(NT) void calc_kernel(Dev D, int sel, int64_t pcap, int skip_mb) {
  const int b = blockIdx.x;
  const ElemState s = D.st[b];  // by value: a reference would re-load it from HBM after every store
  if (!selected(s, sel)) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* pl = sm;               // pcap
  double* x = pl + pcap;         // sX
  double* u = x + D.sX;          // sM
  double* xn = u + D.sM;         // sX
  double* red = xn + D.sX;       // 5*NT/64
  double* mbw = red + 5 * (NT / kWave) + 16;  // multibody calc scratch (D.mbw)
  const int c = s.cur;
  const double* cached = nullptr;
  for (int t = 0; t <= D.T; ++t) {
    const fddp_knot_desc kd = D.knots[t];
    if (skip_mb && is_mb_kind(kd.kind)) continue;  // computed by mb_knot_kernel
    const double* P = stage_params<NT>(D.pblock(b, t), block_doubles_dev(kd.kind, D.nx, kd.nu, D.pblock(b, t)), pl, pcap, cached);
    const double* xg = D.xs[c] + D.knot(b, t) * D.sX;
    for (int i = threadIdx.x; i < D.nx; i += NT) x[i] = xg[i];
    const bool running = t < D.T;
    if (running) {
      const double* ug = D.us[c] + D.run(b, t) * D.sM;
      for (int i = threadIdx.x; i < D.m; i += NT) u[i] = ug[i];
    }
    __syncthreads();
    const double cost = knot_calc<NT>(kd, P, D.nx, x, u, running, xn, red, mbw);
    if (running) {
      double* xo = D.xnext[c] + D.run(b, t) * D.sX;
      for (int i = threadIdx.x; i < D.nx; i += NT) xo[i] = xn[i];
    }
    if (threadIdx.x == 0) D.kcost[c][D.knot(b, t)] = cost;
    __syncthreads();
  }
}

// cost_ = sum of data[t].cost in knot order, terminal last (shooting.hxx:155-160).
#if defined(FDDP_TU_MAIN)
__global__ void cost_sum_kernel(Dev D, int sel, double* out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= D.B) return;
  ElemState& s = D.st[b];
  if (!selected(s, sel)) return;
  const double* kc = D.kcost[s.cur] + D.knot(b, 0);
  // in knot order (shooting.hxx:133-161), the loads of 16 knots issued before their adds
  // (a load per add made this one-thread-per-element sum 45 us at C2)
  double c = 0.;
  int t = 0;
  for (; t + 16 <= D.T + 1; t += 16) {
    double v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = kc[t + q];
#pragma unroll
    for (int q = 0; q < 16; ++q) c += v[q];
  }
  for (; t <= D.T; ++t) c += kc[t];
  s.cost = c;
  if (out) out[b] = c;
}
#endif


// ---------------------------------------------------------------------------
// ShootingProblem::calcDiff (shooting.hxx:164-195) fused with the gap
// computation of SolverDDP::calcDiff (ddp.cpp:160-176). One workgroup per
// element walks its knots with the parameter block LDS-resident; the
// derivative blocks stream out with coalesced stores (HBM-write bound).
// ---------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(NT) void calc_diff_kernel(Dev D, int sel, int gaps, int64_t pcap) {
  const int b = blockIdx.x;
  const ElemState s = D.st[b];  // by value: a reference would re-load it from HBM after every store
  if (!selected(s, sel)) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* pl = sm;
  double* x = pl + pcap;
  double* u = x + D.sX;
  const int c = s.cur;
  const double* cached = nullptr;
  for (int t = 0; t <= D.T; ++t) {
    const fddp_knot_desc kd = D.knots[t];
    const double* P = stage_params<NT>(D.pblock(b, t), block_doubles_dev(kd.kind, D.nx, kd.nu, D.pblock(b, t)), pl, pcap, cached);
    const int64_t kk = D.knot(b, t);
    const double* xg = D.xs[c] + kk * D.sX;
    for (int i = threadIdx.x; i < D.nx; i += NT) x[i] = xg[i];
    const bool running = t < D.T;
    if (running) {
      const double* ug = D.us[c] + D.run(b, t) * D.sM;
      for (int i = threadIdx.x; i < D.m; i += NT) u[i] = ug[i];
    }
    __syncthreads();
    KnotDiffOut o;
    o.Fx = D.Fx + kk * D.sNN;
    o.Fu = D.Fu + kk * D.sNM;
    o.Lxx = D.Lxx + kk * D.sNN;
    o.Lxu = D.Lxu + kk * D.sNM;
    o.Luu = D.Luu + kk * D.sMM;
    o.Lx = D.Lx + kk * D.sN;
    o.Lu = D.Lu + kk * D.sM;
    knot_calc_diff<NT>(kd, P, D.nx, D.m, x, u, running, o);
    if (gaps) {
      if (!s.is_feasible) {
        // fs[0] = diff(xs[0], x0) = x0 - xs[0]; fs[t+1] = diff(xs[t+1], data[t].xnext)
        if (t == 0) state_diff_wg<NT>(D, x, D.x0 + (int64_t)b * D.sX, D.fs + D.knot(b, 0) * D.sN);
        if (running)
          state_diff_wg<NT>(D, D.xs[c] + D.knot(b, t + 1) * D.sX, D.xnext[c] + D.run(b, t) * D.sX,
                            D.fs + D.knot(b, t + 1) * D.sN);
      } else if (!s.was_feasible) {  // closing the gaps
        double* f = D.fs + kk * D.sN;
        for (int i = threadIdx.x; i < D.n; i += NT) f[i] = 0.;
      }
    }
    __syncthreads();
  }
}

// Multibody knots (multibody.hpp), knot-parallel: one mb::kMbDiffNT-thread workgroup per
// (knot t = blockIdx.x, element b = blockIdx.y); knots of other kinds return.
// calc (xnext, knot cost) for elements selected by sel_calc and calcDiff
// (derivative blocks) for those selected by sel_diff (-1: none), fused: the
// calcDiff evaluates the dynamics the calc needs anyway. The gaps of these
// knots are written by calc_diff_kernel as for any knot.
template <int NT, int SP = 0>
__device__ __forceinline__ void mb_knot_body(const Dev& D, int sel_calc, int sel_diff) {
  const int t = blockIdx.x, b = blockIdx.y;
  const fddp_knot_desc kd = D.knots[t];
  if (!is_mb_kind(kd.kind)) return;
  const ElemState s = D.st[b];
  const bool do_calc = sel_calc >= 0 && selected(s, sel_calc);
  const bool do_diff = sel_diff >= 0 && selected(s, sel_diff);
  if (!do_calc && !do_diff) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int c = s.cur;
  const int64_t kk = D.knot(b, t);
  const bool running = t < D.T;
  const double* xg = D.xs[c] + kk * D.sX;
  const double* ug = running ? D.us[c] + D.run(b, t) * D.sM : nullptr;
  double* xn = (do_calc && running) ? D.xnext[c] + D.run(b, t) * D.sX : nullptr;
  double* cost = do_calc ? D.kcost[c] + kk : nullptr;
  // the parameter block is read in every phase: stage it in LDS (D.mbp doubles, after the work area)
  const double* Pg = D.pblock(b, t);
  double* P = sm + D.mbd;
  // this thread's x / u entries loaded beside the parameter block (the knot's first
  // phase stores them: one global round trip fewer on its critical path)
  double xu[2] = {0., 0.};
  const bool pre = D.nx <= NT;
  if (pre) {
    if ((int)threadIdx.x < D.nx) xu[0] = xg[threadIdx.x];
    if (ug && (int)threadIdx.x < D.m) xu[1] = ug[threadIdx.x];
  }
  const int psz = (int)Pg[3];
  for (int e = threadIdx.x; e < psz; e += NT) P[e] = Pg[e];
  __syncthreads();
  if (do_diff)
    mb::knot_calc_diff<NT, SP>(P, D.nx, D.m, xg, ug, running && kd.nu > 0, sm, D.Fx + kk * D.sNN, D.Fu + kk * D.sNM,
                       D.Lxx + kk * D.sNN, D.Lxu + kk * D.sNM, D.Luu + kk * D.sMM, D.Lx + kk * D.sN,
                       D.Lu + kk * D.sM, xn, cost, pre ? xu : nullptr, D.mbspill);
  else
    mb::knot_calc_diff<NT, SP>(P, D.nx, D.m, xg, ug, running && kd.nu > 0, sm, nullptr, nullptr, nullptr, nullptr, nullptr,
                       nullptr, nullptr, xn, cost, pre ? xu : nullptr, D.mbspill);
}
// Two register budgets of the same kernel: 2 waves/EU (256 VGPRs, a few spills) lets two
// workgroups share a CU where the LDS plan allows it (<= 80 KB: the trot, the arm); when
// the plan leaves room for one workgroup per CU anyway (Talos: ~140 KB) the 1-wave/EU
// build gets the whole register file (VGPRs + AGPRs) and nothing spills.
#if defined(FDDP_TU_MB) && FDDP_TU_MB == 0
__global__ __launch_bounds__(mb::kMbDiffNT) __attribute__((amdgpu_waves_per_eu(2))) void mb_knot_kernel(Dev D, int sel_calc, int sel_diff) {
  mb_knot_body<mb::kMbDiffNT>(D, sel_calc, sel_diff);
}
#endif

#if defined(FDDP_TU_MB) && FDDP_TU_MB == 1
__global__ __launch_bounds__(mb::kMbDiffNT) __attribute__((amdgpu_waves_per_eu(1, 1))) void mb_knot_kernel_w1(Dev D, int sel_calc,
                                                                                                   int sel_diff) {
  mb_knot_body<mb::kMbDiffNT>(D, sel_calc, sel_diff);
}
#endif

// Two waves per (knot, element) workgroup, for the small trees (the arm: nv = 7), whose
// phases leave most lanes of four waves idle: four workgroups per CU under the same
// register budget.
#if defined(FDDP_TU_MB) && FDDP_TU_MB == 2
#ifndef FDDP_X2_WPE
#define FDDP_X2_WPE 3
#endif
__global__ __launch_bounds__(mb::kMbDiffNT / 2) __attribute__((amdgpu_waves_per_eu(FDDP_X2_WPE))) void mb_knot_kernel_x2(Dev D, int sel_calc, int sel_diff) {
  mb_knot_body<mb::kMbDiffNT / 2>(D, sel_calc, sel_diff);
}
#endif

// The spilled plan (multibody.hpp diff_spill: the large trees, whose all-LDS plan leaves
// room for one workgroup per CU): two 256-thread workgroups per CU.
#if defined(FDDP_TU_MB) && FDDP_TU_MB == 4
__global__ __launch_bounds__(mb::kMbDiffNT) __attribute__((amdgpu_waves_per_eu(2))) void mb_knot_kernel_s2(Dev D, int sel_calc, int sel_diff) {
  mb_knot_body<mb::kMbDiffNT, 1>(D, sel_calc, sel_diff);
}
#endif

// Eight waves per (knot, element) workgroup: one workgroup per CU on the large LDS plans
// still puts two waves on every SIMD, and the phases' independent work (Gauss-Jordan
// slabs, MFMA tiles, the output blocks) spreads over twice the waves.
#if defined(FDDP_TU_MB) && FDDP_TU_MB == 3
__global__ __launch_bounds__(2 * mb::kMbDiffNT) void mb_knot_kernel_x8(Dev D, int sel_calc, int sel_diff) {
  mb_knot_body<2 * mb::kMbDiffNT>(D, sel_calc, sel_diff);
}
#endif


// ---------------------------------------------------------------------------
// Backward Riccati sweep — SolverDDP::backwardPass + computeGains
// (ddp.cpp:180-253, 298-310), one workgroup per element, V_xx carried in LDS.
// mode 0 (solve): on backward_error raise the regularisation and redo the
// sweep without calcDiff, as SolverFDDP::solve does (fddp.cpp:35-48).
// mode 1 (step API): one sweep with the element's current xreg/ureg.
// Outputs K, k, Vxx*fs per knot and the per-element reductions of
// updateExpectedImprovement (fddp.cpp:126-147) and stoppingCriteria
// (ddp.cpp:132-142), summed in the reference's order.
// ---------------------------------------------------------------------------
struct BwdSmem {
  double *V, *A, *BU, *Qxu, *Quu, *L, *vx, *qx, *qu, *kv, *quuk, *fsv, *vf, *red;
  int* flag;
  // gwork != null: FxT Vxx' (A) and FuT Vxx' (BU) live in this element's
  // global workspace instead of LDS (large n, m).
  __device__ BwdSmem(double* sm, int n, int m, double* gwork) {
    V = sm;
    double* next = V + n * n;
    if (gwork) {
      A = gwork;
      BU = gwork + n * n;
    } else {
      A = next;
      BU = A + n * n;
      next = BU + pad2(m * n);
    }
    Qxu = next;
    Quu = Qxu + pad2(n * m);
    L = Quu + pad2(m * m);
    vx = L + pad2(m * m);
    qx = vx + pad2(n);
    qu = qx + pad2(n);
    kv = qu + pad2(m);
    quuk = kv + pad2(m);
    fsv = quuk + pad2(m);
    vf = fsv + pad2(n);
    red = vf + pad2(n);
    flag = (int*)(red + 64);
  }
  __host__ static size_t bytes(int n, int m, bool global_work) {
    const size_t work = global_work ? 0 : (size_t)(n * n + pad2(m * n));
    return sizeof(double) * (n * n + work + pad2(n * m) + 2 * pad2(m * m) + 4 * pad2(n) + 3 * pad2(m) + 64 + 2);
  }
  __host__ __device__ static int64_t work_doubles(int n, int m) { return (int64_t)n * n + pad2(m * n); }
};

// SolverBoxFDDP::computeGains (box-fddp.cpp:48-79) on wave 0 of the generic
// sweep: the box QP (box_qp.hpp) with the LDS sweep inverse; Quu_inv into
// Qi (ld m), k = -x into kv and D.k, Qu zeroed on the clamped set. False
// where the reference raises backward_error.
__device__ inline bool box_gains_generic(const Dev& D, BwdSmem& S, double* Qi, int b, int t, int cur, int lane) {
  const int nu = D.knots[t].nu, m = D.m;
  if (nu != D.knots[0].nu) return false;  // qp_ has runningModels[0]->nu variables (box-fddp.cpp:16)
  const int64_t rr = D.run(b, t);
  const bool valid = lane < nu;
  double q = 0., lb = 0., ub = 0., x = 0.;
  if (valid) {
    const double u = D.us[cur][rr * D.sM + lane];
    q = S.qu[lane];
    lb = D.ulb[rr * D.sM + lane] - u;
    ub = D.uub[rr * D.sM + lane] - u;
    x = D.k[rr * D.sM + lane];
  }
  uint64_t fsol, finv;
  int iters;
  auto inv = [&](const InvMap& mp) { return wave_sweep_inverse_lds(S.Quu, m, Qi, m, S.red, nu, mp, lane); };
  if (!box_qp_wave(S.Quu, m, Qi, m, S.red, nu, lane, q, lb, ub, x, D.boxcfg, inv, true, fsol, finv, iters))
    return false;
  if (valid) {
    S.kv[lane] = -x;
    if (!((fsol >> lane) & 1)) S.qu[lane] = 0.;
  }
  if (D.dQuuInv)
    for (int e = lane; e < nu * nu; e += 64) D.dQuuInv[rr * D.sMM + (e / nu) * m + e % nu] = Qi[(e / nu) * m + e % nu];
  return true;
}

template <int NT>
__device__ __forceinline__ bool bwd_sweep(const Dev& D, int b, bool feas, double xreg, double ureg, int cur,
                                          BwdSmem& S) {
  const int n = D.n, m = D.m, T = D.T, tid = threadIdx.x;
  const bool xr = !isnan(xreg), ur = !isnan(ureg);
  // terminal: Vxx = Lxx_T (+ xreg I), Vx = Lx_T (+ Vxx fs_T)
  {
    const int64_t kk = D.knot(b, T);
    const double* Lxx = D.Lxx + kk * D.sNN;
    const double* Lx = D.Lx + kk * D.sN;
    for (int e = tid; e < n * n; e += NT) {
      const int i = e % n, j = e / n;
      S.V[e] = (xr && i == j) ? Lxx[e] + xreg : Lxx[e];
    }
    const double* fs = D.fs + kk * D.sN;
    for (int i = tid; i < n; i += NT) S.fsv[i] = fs[i];
    __syncthreads();
    double pv[2] = {0., 0.};
    for (int i = tid; i < n; i += NT) {
      double v = Lx[i];
      if (!feas) {
        double a = 0.;
        for (int j = 0; j < n; ++j) a += S.V[j * n + i] * S.fsv[j];
        S.vf[i] = a;
        D.Vxxfs[kk * D.sN + i] = a;
        v += a;
        pv[0] += v * S.fsv[i];   // Vx_T . fs_T
        pv[1] += S.fsv[i] * a;   // fs_T . Vxx_T fs_T
      }
      S.vx[i] = v;
    }
    wg_sums<NT, 2>(pv, S.red);
    if (tid == 0) {
      double* p = D.part + kk * 8;
      p[0] = 0.; p[1] = 0.; p[2] = pv[0]; p[3] = pv[1]; p[4] = 0.;
    }
    if (D.dVxx) {
      for (int e = tid; e < n * n; e += NT) D.dVxx[kk * D.sNN + e] = S.V[e];
      for (int i = tid; i < n; i += NT) D.dVx[kk * D.sN + i] = S.vx[i];
    }
  }
  for (int t = T - 1; t >= 0; --t) {
    const int64_t kk = D.knot(b, t);
    const int nu = D.knots[t].nu;
    const double* Fx = D.Fx + kk * D.sNN;
    const double* Fu = D.Fu + kk * D.sNM;
    __syncthreads();
    // FxTVxx = Fx^T Vxx' ; FuTVxx = Fu^T Vxx'
    wg_gemm<NT, true, false>(n, n, n, Fx, n, S.V, n, nullptr, 0, S.A, n, 1.);
    if (nu) wg_gemm<NT, true, false>(nu, n, n, Fu, n, S.V, n, nullptr, 0, S.BU, m, 1.);
    // Qx = Lx + Fx^T Vx' ; Qu = Lu + Fu^T Vx'
    {
      const double* Lx = D.Lx + kk * D.sN;
      const double* Lu = D.Lu + kk * D.sM;
      for (int i = tid; i < n; i += NT) {
        double a = 0.;
        for (int k2 = 0; k2 < n; ++k2) a += Fx[(int64_t)i * n + k2] * S.vx[k2];
        S.qx[i] = Lx[i] + a;
      }
      for (int i = tid; i < nu; i += NT) {
        double a = 0.;
        for (int k2 = 0; k2 < n; ++k2) a += Fu[(int64_t)i * n + k2] * S.vx[k2];
        S.qu[i] = Lu[i] + a;
      }
      const double* fs = D.fs + kk * D.sN;
      for (int i = tid; i < n; i += NT) S.fsv[i] = fs[i];
    }
    __syncthreads();
    // Qxx = Lxx + FxTVxx Fx (into V) ; Qxu = Lxu + FxTVxx Fu ; Quu = Luu + FuTVxx Fu (+ ureg I)
    wg_gemm<NT, false, false>(n, n, n, S.A, n, Fx, n, D.Lxx + kk * D.sNN, n, S.V, n, 1.);
    if (nu) {
      wg_gemm<NT, false, false>(n, nu, n, S.A, n, Fu, n, D.Lxu + kk * D.sNM, n, S.Qxu, n, 1.);
      wg_gemm<NT, false, false>(nu, nu, n, S.BU, m, Fu, n, D.Luu + kk * D.sMM, m, S.Quu, m, 1.);
    }
    __syncthreads();
    if (nu && ur)
      for (int i = tid; i < nu; i += NT) S.Quu[i * m + i] += ureg;
    if (D.dQxx) {
      const int64_t r = D.run(b, t);
      for (int e = tid; e < n * n; e += NT) D.dQxx[r * D.sNN + e] = S.V[e];
      for (int i = tid; i < n; i += NT) D.dQx[r * D.sN + i] = S.qx[i];
      for (int e = tid; e < n * m; e += NT) D.dQxu[r * D.sNM + e] = (e / n < nu) ? S.Qxu[e] : 0.;
      for (int e = tid; e < m * m; e += NT) D.dQuu[r * D.sMM + e] = (e % m < nu && e / m < nu) ? S.Quu[e] : 0.;
      for (int i = tid; i < m; i += NT) D.dQu[r * D.sM + i] = i < nu ? S.qu[i] : 0.;
    }
    __syncthreads();
    if (nu && feas && D.box_knot(b, t)) {
      // box QP gains; K = Quu_inv Qxu^T (S.A, nu x n, ld m)
      if (tid < 64 && !box_gains_generic(D, S, S.L, b, t, cur, tid) && tid == 0) *S.flag = 1;
      __syncthreads();
      if (*S.flag) return false;
      for (int e = tid; e < nu * n; e += NT) {
        const int i = e % nu, j = e / nu;
        double a = 0.;
        for (int l = 0; l < nu; ++l) a += S.L[l * m + i] * S.Qxu[l * n + j];
        S.A[j * m + i] = a;
      }
      __syncthreads();
    } else if (nu) {
      // Cholesky (lower) of Quu — Eigen LLT fails on a pivot <= 0
      for (int j = 0; j < nu; ++j) {
        if (tid == 0) {
          double sd = S.Quu[j * m + j];
          for (int k2 = 0; k2 < j; ++k2) sd -= S.L[k2 * m + j] * S.L[k2 * m + j];
          if (!(sd > 0.)) *S.flag = 1;
          S.L[j * m + j] = sqrt(sd);
        }
        __syncthreads();
        const double ljj = S.L[j * m + j];
        for (int i = j + 1 + tid; i < nu; i += NT) {
          double v = S.Quu[j * m + i];
          for (int k2 = 0; k2 < j; ++k2) v -= S.L[k2 * m + i] * S.L[k2 * m + j];
          S.L[j * m + i] = v / ljj;
        }
        __syncthreads();
      }
      if (*S.flag) return false;
      // K = Quu^-1 Qxu^T (K in S.A, nu x n, ld m) ; k = Quu^-1 Qu
      for (int j = tid; j <= n; j += NT) {
        double* y = (j < n) ? S.A + j * m : S.kv;
        for (int i = 0; i < nu; ++i) {
          double v = (j < n) ? S.Qxu[i * n + j] : S.qu[i];
          for (int k2 = 0; k2 < i; ++k2) v -= S.L[k2 * m + i] * y[k2];
          y[i] = v / S.L[i * m + i];
        }
        for (int i = nu - 1; i >= 0; --i) {
          double v = y[i];
          for (int k2 = i + 1; k2 < nu; ++k2) v -= S.L[i * m + k2] * y[k2];
          y[i] = v / S.L[i * m + i];
        }
      }
      __syncthreads();
    }
    if (nu) {
      // store K, k ; Quuk = Quu k
      {
        const int64_t r = D.run(b, t);
        double* Kg = D.K + r * D.sNM;
        for (int e = tid; e < m * n; e += NT) Kg[e] = (e % m < nu) ? S.A[e] : 0.;
        double* kg = D.k + r * D.sM;
        for (int i = tid; i < m; i += NT) kg[i] = i < nu ? S.kv[i] : 0.;
        for (int i = tid; i < nu; i += NT) {
          double a = 0.;
          for (int k2 = 0; k2 < nu; ++k2) a += S.Quu[k2 * m + i] * S.kv[k2];
          S.quuk[i] = a;
        }
      }
      __syncthreads();
      // Vx = Qx + K^T Quuk - 2 K^T Qu   (or Qx - K^T Qu without ureg)
      for (int i = tid; i < n; i += NT) {
        const double* Kc = S.A + i * m;
        if (ur) {
          double a = 0., c = 0.;
          for (int k2 = 0; k2 < nu; ++k2) a += Kc[k2] * S.quuk[k2];
          for (int k2 = 0; k2 < nu; ++k2) c += Kc[k2] * S.qu[k2];
          S.vx[i] = (S.qx[i] + a) - 2 * c;
        } else {
          double c = 0.;
          for (int k2 = 0; k2 < nu; ++k2) c += Kc[k2] * S.qu[k2];
          S.vx[i] = S.qx[i] - c;
        }
      }
      // Vxx = Qxx - Qxu K
      wg_gemm<NT, false, false>(n, n, nu, S.Qxu, n, S.A, m, S.V, n, S.V, n, -1.);
    } else {
      for (int i = tid; i < n; i += NT) S.vx[i] = S.qx[i];
    }
    __syncthreads();
    // Vxx = 0.5 (Vxx + Vxx^T) (+ xreg I)
    for (int e = tid; e < n * n; e += NT) {
      const int i = e % n, j = e / n;
      if (i < j) {
        const double s2 = 0.5 * (S.V[j * n + i] + S.V[i * n + j]);
        S.V[j * n + i] = s2;
        S.V[i * n + j] = s2;
      } else if (i == j && xr) {
        S.V[e] += xreg;
      }
    }
    __syncthreads();
    // Vx += Vxx fs (infeasible), NaN checks, reduction terms
    bool bad = false;
    double pv[5] = {0., 0., 0., 0., 0.};
    for (int i = tid; i < n; i += NT) {
      double v = S.vx[i];
      if (!feas) {
        double a = 0.;
        for (int j = 0; j < n; ++j) a += S.V[j * n + i] * S.fsv[j];
        D.Vxxfs[kk * D.sN + i] = a;
        v += a;
        S.vx[i] = v;
        pv[2] += v * S.fsv[i];
        pv[3] += S.fsv[i] * a;
      }
      bad |= bad_entry(v);
    }
    for (int e = tid; e < n * n; e += NT) bad |= bad_entry(S.V[e]);
    for (int i = tid; i < nu; i += NT) {
      pv[0] += S.qu[i] * S.kv[i];    // Qu . k
      pv[1] += S.kv[i] * S.quuk[i];  // k . Quuk
      pv[4] += S.qu[i] * S.qu[i];    // |Qu|^2
    }
    if (bad) *S.flag = 1;
    wg_sums<NT, 5>(pv, S.red);
    if (tid == 0) {
      double* p = D.part + kk * 8;
      for (int j = 0; j < 5; ++j) p[j] = pv[j];
    }
    if (D.dVxx) {
      for (int e = tid; e < n * n; e += NT) D.dVxx[kk * D.sNN + e] = S.V[e];
      for (int i = tid; i < n; i += NT) D.dVx[kk * D.sN + i] = S.vx[i];
    }
    if (*S.flag) return false;
  }
  return true;
}

template <int NT>
__global__ __launch_bounds__(NT) void backward_kernel(Dev D, Prm prm, int mode) {
  const int b = blockIdx.x;
  ElemState* st = D.st + b;
  if (mode == 0 && !st->active) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  BwdSmem S(sm, D.n, D.m, D.bwork ? D.bwork + (int64_t)b * BwdSmem::work_doubles(D.n, D.m) : nullptr);
  const bool feas = st->is_feasible != 0;
  double xreg = st->xreg, ureg = st->ureg;
  bool ok;
  int tries = 0;
  const int max_tries = reg_retry_bound(prm, xreg);
  for (;;) {
    if (threadIdx.x == 0) *S.flag = 0;
    __syncthreads();
    ok = bwd_sweep<NT>(D, b, feas, xreg, ureg, st->cur, S);
    __syncthreads();
    if (ok || mode == 1) break;
    // increaseRegularization (ddp.cpp:312-318); abort at regmax (fddp.cpp:41-43)
    xreg *= prm.regfactor;
    if (xreg > prm.regmax) xreg = prm.regmax;
    ureg = xreg;
    // (as the reference: at regmax; a NaN / zero xreg never reaches it: the bound
    // reg_retry_bound makes every wave of the workgroup leave the loop)
    if (!(xreg < prm.regmax) || ++tries >= max_tries) break;
  }
  if (threadIdx.x == 0) {
    st->xreg = xreg;
    st->ureg = ureg;
    st->bwd_fail = ok ? 0 : 1;
    if (!ok && mode == 0) {  // solve() returns false inside this loop body
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

// ---------------------------------------------------------------------------
// Forward pass — SolverFDDP::forwardPass (fddp.cpp:149-225) + the line search
// and bookkeeping of SolverFDDP::solve (fddp.cpp:49-103). One workgroup per
// element rolls the horizon out serially; trials are written into the other
// trajectory buffer and accepted by flipping `cur` (no copy).
// mode 0: full line search + regularisation/convergence update (solve).
// mode 1: a single trial at `alpha` (tryStep), storing cost_try, dV and dv.
// ---------------------------------------------------------------------------
// Where a trial writes xs_try / us_try / xnext / knot costs / dv terms: slot 0 is the
// other trajectory buffer (accepted by flipping cur), slots > 0 the parallel copies.
struct TrialOut {
  double *xs, *us, *xnext, *kcost, *dvp;
  __device__ TrialOut(const Dev& D, int o, int slot) {
    if (slot == 0) {
      xs = D.xs[o], us = D.us[o], xnext = D.xnext[o], kcost = D.kcost[o], dvp = D.dvp;
    } else {
      const int64_t B = D.B, K1 = D.T + 1, K0 = D.T, q = slot - 1;
      xs = D.pxs + q * B * K1 * D.sX, us = D.pus + q * B * K0 * D.sM, xnext = D.pxnext + q * B * K0 * D.sX;
      kcost = D.pkcost + q * B * K1, dvp = D.pdvp + q * B * K1;
    }
  }
};

// A store of the rollout's trial trajectories / per-knot terms (HBM) through a global
// pointer: a flat store would make the wave's next LDS access wait for it.
__device__ __forceinline__ void gstore(double* p, double v) { *(__attribute__((address_space(1))) double*)p = v; }

// sum_j K(i, j) dx_j (K row-major m x n rows of the gains, read from HBM), summed in
// j order as the reference's GEMV; the loads of 8 consecutive j are issued before
// their FMAs, so a lane waits for one round trip per 8 entries instead of per entry.
template <class F>
__device__ __forceinline__ double gains_dot(const double* K, int m, int i, int n, F dx) {
  double s = 0.;
  int j = 0;
#pragma unroll 1
  for (; j + 8 <= n; j += 8) {
    double k[8], d[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      k[q] = K[(int64_t)(j + q) * m + i];
      d[q] = dx(j + q);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) s = fma(k[q], d[q], s);
  }
  if (j < n) {  // the tail as one guarded batch
    double k[8], d[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      k[q] = j + q < n ? K[(int64_t)(j + q) * m + i] : 0.;
      d[q] = j + q < n ? dx(j + q) : 0.;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (j + q < n) s = fma(k[q], d[q], s);
  }
  return s;
}

template <int NT, bool MB = false>
__device__ __forceinline__ bool fwd_trial(const Dev& D, int b, const ElemState& s, double alpha, double* xv, double* uv, double* xn,
                          double* red, int* flag, double& cost_try, double& dv, double* pl, int64_t pcap,
                          const double*& cached, double* mbw, double* dxv, int slot = 0, int* nwritten = nullptr) {
  const int n = D.n, nx = D.nx, m = D.m, T = D.T, tid = threadIdx.x;
  const int c = s.cur, o = 1 - c;
  const TrialOut out(D, o, slot);
  const bool feas = s.is_feasible != 0;
  const bool full = feas || alpha == 1.;
  const bool ff = nx != n;  // free-flyer state (dxv: 2 sN doubles of LDS)
  const double* x0 = D.x0 + (int64_t)b * D.sX;
  for (int i = tid; i < nx; i += NT) xn[i] = x0[i];
  cost_try = 0.;
  double* dvp = out.dvp + D.knot(b, 0);
  // (diagnostic phase timer, FDDP_STAMPS=1 on the stamps build: per wave, summed)
  Stamp stamp(D.stamps && tid < kWave ? D.stamps + (int64_t)D.B * 128 + (int64_t)b * 8 : nullptr);  // (wave 0's)
  __syncthreads();
  for (int t = 0; t <= T; ++t) {
    const int64_t kk = D.knot(b, t);
    const double* fs = D.fs + kk * D.sN;
    const double* xs = D.xs[c] + kk * D.sX;
    double* xt = out.xs + kk * D.sX;
    // xs_try[t] = xnext  or  integrate(xnext, fs[t] * (alpha - 1))
    // (the trial's outputs xs_try[t], us_try[t], xnext[t] are stored after the knot's calc,
    // from LDS: a store before the calc made its first spill reloads wait (vmcnt, in
    // order) for the store to reach memory)
    double pd = 0.;
    if (!ff) {
      for (int i = tid; i < nx; i += NT) {
        const double v = full ? xn[i] : xn[i] + fs[i] * (alpha - 1);
        xv[i] = v;
        if (!feas) pd += (v - xs[i]) * D.Vxxfs[kk * D.sN + i];  // -fs^T Vxx diff(xs_try, xs)
      }
      __syncthreads();
    } else {  // on the manifold: dx = diff(xs, xs_try) for the gains, diff(xs_try, xs) for dv
      if (full)
        for (int i = tid; i < nx; i += NT) xv[i] = xn[i];
      else
        state_integrate_wg<NT>(D, xn, fs, alpha - 1, xv);
      __syncthreads();
      state_diff_wg<NT>(D, xs, xv, dxv);
      if (!feas) state_diff_wg<NT>(D, xv, xs, dxv + D.sN, kWave);
      __syncthreads();
      if (!feas)
        for (int i = tid; i < n; i += NT) pd -= dxv[D.sN + i] * D.Vxxfs[kk * D.sN + i];
    }
    const bool running = t < T;
    const fddp_knot_desc kd = D.knots[t];
    stamp.mark(0);
    const double* P = stage_params<NT>(D.pblock(b, t), block_doubles_dev(kd.kind, nx, kd.nu, D.pblock(b, t)), pl, pcap, cached);
    stamp.mark(1);
    if (running) {
      const int nu = kd.nu;
      const double* us = D.us[c] + D.run(b, t) * D.sM;
      const double* K = D.K + D.run(b, t) * D.sNM;
      const double* kv = D.k + D.run(b, t) * D.sM;
      // us_try = us - k * alpha - K * dx ,  dx = diff(xs, xs_try)
      // K (HBM) moves into the knot calc's LDS scratch (free between knots) by LDS-DMA
      // issued by the whole workgroup: one round trip to HBM, no registers. Control i's
      // product is then one FMA chain in j order on lane i, the summation order of the
      // reference's GEMV row (fddp.cpp:199) and of the oracle (gain_row_dot), so us_try
      // rounds as theirs. (Round 5 split the row into 8 partial sums over the workgroup:
      // the reordered sums moved the C5 smoke's xs after 3 iterations 2.4e-8 -> 3.8e-8.)
      if (m <= NT && D.mbw_fwd - (D.dxv_mbw ? 2 * D.sN : 0) >= (int64_t)m * n) {
        if (!ff)
          for (int j = tid; j < n; j += NT) dxv[j] = xv[j] - xs[j];
        dma_vec<NT / kWave>(mbw, K, m * n, tid / kWave, tid & (kWave - 1));
        dma_barrier();
        if (tid < m) {
          double v = 0.;
          if (tid < nu) {
            const double* Kl = lds_ptr(mbw) + tid;
            const double* dl = lds_ptr(dxv);
            double kd2 = 0.;
            int j = 0;
#pragma unroll 1
            for (; j + 8 <= n; j += 8) {  // 8 LDS loads in flight, then their chain
              double kq[8], dq[8];
#pragma unroll
              for (int q = 0; q < 8; ++q) kq[q] = Kl[(j + q) * m], dq[q] = dl[j + q];
#pragma unroll
              for (int q = 0; q < 8; ++q) kd2 = fma(kq[q], dq[q], kd2);
            }
            for (; j < n; ++j) kd2 = fma(Kl[j * m], dl[j], kd2);
            v = fma(-kv[tid], alpha, us[tid]) - kd2;
            // SolverBoxFDDP::forwardPass: cwiseMax(u_lb).cwiseMin(u_ub) (box-fddp.cpp:100-102)
            if (D.box_knot(b, t))
              v = std_min(std_max(v, D.ulb[D.run(b, t) * D.sM + tid]), D.uub[D.run(b, t) * D.sM + tid]);
          }
          uv[tid] = v;
        }
      } else {
        for (int i = tid; i < m; i += NT) {
          double v = 0.;
          if (i < nu) {
            const double kd2 = ff ? gains_dot(K, m, i, n, [&](int j) { return dxv[j]; })
                                  : gains_dot(K, m, i, n, [&](int j) { return xv[j] - xs[j]; });
            v = fma(-kv[i], alpha, us[i]) - kd2;
            if (D.box_knot(b, t)) v = std_min(std_max(v, D.ulb[D.run(b, t) * D.sM + i]), D.uub[D.run(b, t) * D.sM + i]);
          }
          uv[i] = v;
        }
      }
      __syncthreads();
    }
    stamp.mark(2);
    const double ct = knot_calc<NT, MB>(kd, P, nx, xv, uv, running, xn, red, mbw);
    stamp.mark(3);
    bool bad = false;
    for (int i = tid; i < nx; i += NT) gstore(xt + i, xv[i]);
    if (running) {
      double* ut = out.us + D.run(b, t) * D.sM;
      for (int i = tid; i < m; i += NT) gstore(ut + i, uv[i]);
      double* xo = out.xnext + D.run(b, t) * D.sX;
      for (int i = tid; i < nx; i += NT) {
        gstore(xo + i, xn[i]);
        bad |= bad_entry(xn[i]);
      }
    }
    if (!feas) pd = wg_sum<NT>(pd, red);
    if (tid == 0) {
      gstore(out.kcost + kk, ct);
      gstore(dvp + t, pd);
    }
    cost_try += ct;
    bad |= raise_if_nan(cost_try);
    if (wg_any(bad, flag)) {
      if (nwritten) *nwritten = t + 1;  // the knots of the trial buffers this trial wrote
      stamp.flush();
      return false;
    }
    stamp.mark(4);
  }
  stamp.flush();
  if (nwritten) *nwritten = T + 1;
  // dv: terminal first, then t = 0..T-1 (fddp.cpp:110-119). Summed by the
  // thread that stored the terms (program order), broadcast through LDS.
  if (tid == 0) {
    double acc = 0.;
    if (!feas) {
      acc += dvp[T];
      for (int t = 0; t < T; ++t) acc += dvp[t];
    }
    red[0] = acc;
  }
  __syncthreads();
  dv = red[0];
  __syncthreads();
  return true;
}

template <int NT, bool FAST>
__device__ __forceinline__ bool fwd_trial_fast(const Dev& D, int b, const ElemState& s, double alpha, double* xu,
                                               double* dxv, double* xn, double* pa, double* pdyn, double* red,
                                               int* flag, double& cost_try, double& dv, double* pl, int64_t pcap,
                                               const double*& cached);

// Forward-pass LDS beyond the parameter block (doubles): generic trial
// [xv sX | uv sM | xn sX | red 5*NW+8 | flag 2 | dxv 2 sN | multibody scratch D.mbw_fwd], fast trial
// [xu sX+sM | dxv sN | xn sX | pa NT | pdyn NT | red 24 | flag].
template <int NT, bool FAST>
__host__ __device__ inline int64_t fwd_lds_doubles(int64_t sX, int64_t sN, int64_t sM) {
  return FAST ? (sX + sM) + sN + sX + 2 * NT + 24 + 2 : 2 * sX + sM + 5 * (NT / 64) + 8 + 2 + 2 * sN;
}

// The line search's test of one finished trial (fddp.cpp:57-78): fills the
// trial's bookkeeping into s; true if alpha is accepted (then s holds the new state).
__device__ __forceinline__ bool ls_accept(const Prm& prm, ElemState& s, double alpha, double ct, double dv) {
  s.cost_try = ct;
  s.dV = s.cost - ct;
  s.dv = dv;
  s.d0 = s.dg + dv;
  s.d1 = s.dq - 2 * dv;
  s.dVexp = alpha * (s.d0 + 0.5 * alpha * s.d1);
  bool acc;
  if (s.dVexp >= 0)
    acc = s.d0 < prm.th_grad || s.dV > prm.th_acceptstep * s.dVexp;
  else
    acc = s.dV > prm.th_acceptnegstep * s.dVexp;
  if (acc) {
    s.was_feasible = s.is_feasible;
    s.is_feasible = (s.was_feasible || alpha == 1.) ? 1 : 0;
    s.cur = 1 - s.cur;
    s.cost = ct;
  }
  return acc;
}

// After the line search: regularisation schedule (fddp.cpp:83-91) and the loop's
// convergence / abort test (fddp.cpp:92-103).
__device__ __forceinline__ void ls_finish(const Prm& prm, ElemState& s, bool accepted) {
  s.recalc = accepted ? 1 : 0;
  // an accepted trial became xs_ (setCandidate(xs_try_, ...)), so a later
  // expectedImprovement() (e.g. CallbackLogger's) sees diff(xs_try, xs) = 0; d_ keeps
  // the accepted trial's value (fddp.cpp:107-124)
  if (accepted) s.dv = 0.;
  bool abort = false;
  if (s.steplength > prm.th_stepdec) {
    s.xreg /= prm.regfactor;
    if (s.xreg < prm.regmin) s.xreg = prm.regmin;
    s.ureg = s.xreg;
  }
  if (s.steplength <= prm.th_stepinc) {
    s.xreg *= prm.regfactor;
    if (s.xreg > prm.regmax) s.xreg = prm.regmax;
    s.ureg = s.xreg;
    if (s.xreg == prm.regmax) abort = true;
  }
  s.n_iter_run += 1;
  if (abort) {
    s.status = FDDP_STATUS_REGMAX;
    s.active = 0;
  } else if (s.was_feasible && s.stop < prm.th_stop) {  // fddp.cpp:100-102
    s.status = FDDP_STATUS_CONVERGED;
    s.active = 0;
  } else {
    s.iter += 1;
  }
}

// mode 0: the serial line search + update; mode 1 (tryStep): one trial at alpha1;
// mode 2: trial alphas[group * npar + blockIdx.y] of a parallel group into slot
// blockIdx.y, its outcome into ptrial (ls_select_kernel decides).
// MB: every knot is a multibody kind (h->all_mb), only that calc is compiled in.
#ifndef FDDP_FWD_WPE
#define FDDP_FWD_WPE 2
#endif
// the multibody rollout at three workgroups per CU (its LDS, knot_calc_dense_x, allows it on
// the C5 walk): 168 VGPRs
#ifndef FDDP_FWD_WPE_MB
#define FDDP_FWD_WPE_MB 3
#endif
// (the generic variant, for horizons that mix multibody and dense knots, gets the
// whole register file: under the 2-waves cap its spills trip a backend error)
// MBW: waves per EU of the multibody variant (3: three workgroups per CU where the LDS
// allows it, at 168 VGPRs; 2: the 256-VGPR build for batches that fit two per CU anyway)
template <int NT, bool FAST, bool MB = false, int MBW = FDDP_FWD_WPE_MB>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(MB ? MBW : FAST ? FDDP_FWD_WPE : 1))) void forward_kernel(Dev D, Prm prm, int mode, double alpha1, int* active_count,
                                                     int64_t pcap, int group = 0) {
  // (workgroups are dispatched roughly in index order: the elements whose last line
  // search took the most trials start first, so they do not trail the launch)
  const int b = D.ls_order ? D.ls_order[blockIdx.x] : (int)blockIdx.x;
  ElemState* st = D.st + b;
  if (mode != 1 && !st->active) return;
  const int slot = mode == 2 ? (int)blockIdx.y : 0;
  const int a2 = group * D.npar + slot;
  if (mode == 2 && (D.ls_done[b] || a2 >= prm.n_alphas)) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* pl = sm;
  const double* cached = nullptr;
  double *xv, *uv, *xn, *red, *dxv = nullptr, *pa = nullptr, *pdyn = nullptr;
  int* flag;
  if (FAST) {
    xv = pl + pcap;             // xu: x then u
    uv = xv + D.sX;
    dxv = xv + D.sX + D.sM;
    xn = dxv + D.sN;
    pa = xn + D.sX;
    pdyn = pa + NT;
    red = pdyn + NT;
    flag = (int*)(red + 24);
  } else {
    xv = pl + pcap;
    uv = xv + D.sX;
    xn = uv + D.sM;
    red = xn + D.sX;
    flag = (int*)(red + 5 * (NT / kWave) + 8);
  }
  // The element's solver state lives in LDS during the line search: a register copy
  // would be held across every trial's rollout (the knot calc runs at the VGPR cap); the
  // threads take a copy after each trial, and thread 0 writes the changes back.
  __shared__ ElemState ss;
  if (threadIdx.x == 0) ss = *st;
#ifdef FDDP_STAMPS_BUILD
  // (diagnostic: this workgroup's residency, real time and hardware ids; fddp_destroy)
  unsigned long long* rs = D.stamps ? D.stamps + (int64_t)D.B * 136 + (int64_t)b * 4 : nullptr;
  if (rs && threadIdx.x == 0) {
    rs[0] = __builtin_amdgcn_s_memrealtime();
    rs[1] = (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
            ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32);
  }
#endif
  __syncthreads();
  int nwr = D.T + 1;
  // (generic trial) the knot calc's scratch, and dx: its own 2 sN doubles before the scratch,
  // or (D.dxv_mbw) the scratch's last 2 sN doubles: dx is dead once the gains are applied, and
  // the gains' K staging stays below it (fddp_create checks the room)
  double* const mbw = (double*)flag + 2 + (D.dxv_mbw ? 0 : 2 * D.sN);
  double* const dxv_ = D.dxv_mbw ? mbw + D.mbw_fwd - 2 * D.sN : (double*)flag + 2;
  auto trial = [&](double alpha, double& ct, double& dv) {
    if constexpr (FAST)
      return fwd_trial_fast<NT, true>(D, b, ss, alpha, xv, dxv, xn, pa, pdyn, red, flag, ct, dv, pl, pcap, cached);
    else
      return fwd_trial<NT, MB>(D, b, ss, alpha, xv, uv, xn, red, flag, ct, dv, pl, pcap, cached, mbw, dxv_, slot, &nwr);
  };
  // line search (fddp.cpp:53-81). One call site of the trial, so it is inlined (its
  // LDS pointers keep their address space).
  bool accepted = false;
  const int na = mode == 0 ? prm.n_alphas : 1;
  for (int a = 0; a < na; ++a) {
    const double alpha = mode == 1 ? alpha1 : prm.alphas[mode == 2 ? a2 : a];
    double ct, dv;
    bool ok;
    [[clang::always_inline]] ok = trial(alpha, ct, dv);
    if (mode == 1) {
      if (threadIdx.x == 0) {
        st->fwd_fail = ok ? 0 : 1;
        st->cost_try = ct;
        st->dV = ss.cost - ct;
        st->dv = ok ? dv : 0.;
      }
      return;
    }
    if (mode == 2) {
      if (threadIdx.x == 0) {
        double* r = D.ptrial + ((int64_t)b * D.npar + slot) * 4;
        r[0] = ok ? 1. : 0.;
        r[1] = ct;
        r[2] = dv;
        r[3] = (double)nwr;  // knots written (a failed trial stops early)
      }
      return;
    }
    ElemState s = ss;
    s.steplength = alpha;
    const bool acc = ok && ls_accept(prm, s, alpha, ct, dv);
    __syncthreads();  // (every thread has read ss)
    if (threadIdx.x == 0) ss = s;
    __syncthreads();
    if (acc) {
      accepted = true;
      break;
    }
  }
  ElemState s = ss;
  ls_finish(prm, s, accepted);
#ifdef FDDP_STAMPS_BUILD
  if (rs && threadIdx.x == 0) rs[2] = __builtin_amdgcn_s_memrealtime();
#endif
  if (threadIdx.x == 0) {
    *st = s;
    if (s.active && active_count) atomicAdd(active_count, 1);
  }
}

// Decision after parallel group `group`: the first accepted trial in alpha order
// (the serial line search's choice); its slot is copied into the other trajectory
// buffer when it is not slot 0. Undecided elements wait for the next group; the
// last group resets ls_done for the next iteration.
template <int NT>
__global__ __launch_bounds__(NT) void ls_select_kernel(Dev D, Prm prm, int group, int last, int* active_count) {
  const int b = blockIdx.x, tid = threadIdx.x;
  ElemState* st = D.st + b;
  if (!st->active || D.ls_done[b]) {
    if (last && tid == 0) D.ls_done[b] = 0;
    return;
  }
  ElemState s = *st;
  int acc_slot = -1;
  bool exhausted = false;
  for (int p = 0; p < D.npar; ++p) {
    const int a = group * D.npar + p;
    if (a >= prm.n_alphas) {
      exhausted = true;
      break;
    }
    const double alpha = prm.alphas[a];
    s.steplength = alpha;
    const double* r = D.ptrial + ((int64_t)b * D.npar + p) * 4;
    if (r[0] == 0.) continue;
    if (ls_accept(prm, s, alpha, r[1], r[2])) {
      acc_slot = p;
      break;
    }
  }
  if (group * D.npar + D.npar >= prm.n_alphas) exhausted = true;
  // copy the knots slot p's trial wrote (a trial stopped by a forward_error leaves the
  // rest of the buffer as it was, as in the serial search) into trajectory buffer `buf`
  auto copy_slot = [&](int p, int buf) {
    const TrialOut src(D, 0, p), dst(D, buf, 0);
    const int64_t K1 = (int64_t)D.ptrial[((int64_t)b * D.npar + p) * 4 + 3];
    const int64_t K0 = K1 < D.T ? K1 : D.T;
    for (int64_t i = tid; i < K1 * D.sX; i += NT) dst.xs[D.knot(b, 0) * D.sX + i] = src.xs[D.knot(b, 0) * D.sX + i];
    for (int64_t i = tid; i < K0 * D.sM; i += NT) dst.us[D.run(b, 0) * D.sM + i] = src.us[D.run(b, 0) * D.sM + i];
    for (int64_t i = tid; i < K0 * D.sX; i += NT)
      dst.xnext[D.run(b, 0) * D.sX + i] = src.xnext[D.run(b, 0) * D.sX + i];
    for (int64_t i = tid; i < K1; i += NT) dst.kcost[D.knot(b, 0) + i] = src.kcost[D.knot(b, 0) + i];
  };
  if (acc_slot < 0) {
    // no trial of this group accepted: its trials' outputs over the trial buffer in
    // alpha order (slot 0 wrote it directly), so each knot holds the last trial that
    // reached it, as the serial search leaves xs_try_ / us_try_ (fddp.cpp:149-225).
    // A thread copies the same entries for every slot, so the order holds per entry.
    const int np = prm.n_alphas - group * D.npar < D.npar ? prm.n_alphas - group * D.npar : D.npar;
    for (int p = 1; p < np; ++p) copy_slot(p, 1 - s.cur);
    if (!exhausted) {  // next group
      if (tid == 0) *st = s;
      return;
    }
  } else if (acc_slot > 0) {
    // the accepted slot's trajectories into the new current buffer (ls_accept flipped cur)
    copy_slot(acc_slot, s.cur);
  }
  ls_finish(prm, s, acc_slot >= 0);
  if (tid == 0) {
    *st = s;
    D.ls_done[b] = last ? 0 : 1;
    if (s.active && active_count) atomicAdd(active_count, 1);
  }
}

// x0 <- xs[1]; xs[t] <- xs[t+1]; us[t] <- us[t+1] (last kept), into the other buffer.
template <int NT>
__global__ __launch_bounds__(NT) void mpc_shift_kernel(Dev D) {
  const int b = blockIdx.x;
  ElemState* st = D.st + b;
  const int c = st->cur, o = 1 - c, T = D.T;
  const double* xs = D.xs[c] + D.knot(b, 0) * D.sX;
  double* xo = D.xs[o] + D.knot(b, 0) * D.sX;
  const double* us = D.us[c] + D.run(b, 0) * D.sM;
  double* uo = D.us[o] + D.run(b, 0) * D.sM;
  for (int64_t e = threadIdx.x; e < (int64_t)(T + 1) * D.sX; e += NT) {
    const int64_t t = e / D.sX, i = e % D.sX;
    const int64_t ts = t < T ? t + 1 : T;
    xo[e] = xs[ts * D.sX + i];
  }
  for (int64_t e = threadIdx.x; e < (int64_t)T * D.sM; e += NT) {
    const int64_t t = e / D.sM, i = e % D.sM;
    const int64_t ts = t + 1 < T ? t + 1 : T - 1;
    uo[e] = us[ts * D.sM + i];
  }
  for (int i = threadIdx.x; i < D.nx; i += NT) D.x0[(int64_t)b * D.sX + i] = xs[D.sX + i];
  __syncthreads();
  if (threadIdx.x == 0) st->cur = o;
}

// Solve prologue: per-element state (fddp.cpp:21-31, solver-base.cpp:66).
#if defined(FDDP_TU_MAIN)
__global__ void init_state_kernel(Dev D, int is_feasible, double xreg) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= D.B) return;
  ElemState& s = D.st[b];
  s.is_feasible = is_feasible;
  s.xreg = xreg;
  s.ureg = xreg;
  s.was_feasible = 0;
  s.recalc = 1;
  s.iter = 0;
  s.status = FDDP_STATUS_RUNNING;
  s.active = 1;
  s.n_iter_run = 0;
  s.bwd_fail = 0;
  s.fwd_fail = 0;
  // the parallel line search's per-element "decided" flag: a solve never starts with a
  // stale one (a failed launch between groups would otherwise skip a line search)
  if (D.ls_done) D.ls_done[b] = 0;
}
#endif


// Copy xs/us of the current buffer of every element into a dense output.
#if defined(FDDP_TU_MAIN)
__global__ void gather_traj_kernel(Dev D, int which, double* out) {
  const int b = blockIdx.y;
  const int c = D.st[b].cur;
  const int64_t rows = which == 0 ? D.T + 1 : D.T;
  const int w = which == 0 ? D.nx : D.m;
  const int64_t sw = which == 0 ? D.sX : D.sM;
  const double* src = (which == 0 ? D.xs[c] : D.us[c]) + (int64_t)b * rows * sw;
  double* dst = out + (int64_t)b * rows * w;
  for (int64_t e = blockIdx.x * blockDim.x + threadIdx.x; e < rows * w; e += (int64_t)gridDim.x * blockDim.x)
    dst[e] = src[(e / w) * sw + e % w];
}
#endif


#if defined(FDDP_TU_MAIN)
__global__ void scatter_traj_kernel(Dev D, int which, const double* in, int use_zero) {
  const int b = blockIdx.y;
  const int c = D.st[b].cur;
  const int64_t rows = which == 0 ? D.T + 1 : D.T;
  const int w = which == 0 ? D.nx : D.m;
  const int64_t sw = which == 0 ? D.sX : D.sM;
  double* dst = (which == 0 ? D.xs[c] : D.us[c]) + (int64_t)b * rows * sw;
  const double* src = in + (int64_t)b * rows * w;
  // state.zero() of a free-flyer state: the identity quaternion (pinocchio::neutral)
  const int qw = (which == 0 && D.nx != D.n) ? 6 : -1;
  for (int64_t e = blockIdx.x * blockDim.x + threadIdx.x; e < rows * w; e += (int64_t)gridDim.x * blockDim.x)
    dst[(e / w) * sw + e % w] = use_zero ? ((e % w) == qw ? 1. : 0.) : src[e];
}
#endif



// ---------------------------------------------------------------------------
// Standalone batched box QP (fddp_boxqp_solve): BoxQP::solve (box-qp.cpp:
// 51-182), one wave per problem, H and the free-Hessian inverse in LDS.
// ---------------------------------------------------------------------------
#if defined(FDDP_TU_MAIN)
__global__ __launch_bounds__(64) void boxqp_kernel(int nx, const double* H, const double* q, const double* lb,
                                                   const double* ub, const double* xinit, BoxQPCfg c, double* x,
                                                   uint64_t* free_mask, uint64_t* inv_mask, double* Hinv,
                                                   int32_t* status) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int b = blockIdx.x, lane = threadIdx.x;
  const int64_t nn = (int64_t)nx * nx;
  double* Hs = sm;
  double* Qi = sm + nn;
  double* vb = Qi + nn;
  for (int64_t e = lane; e < nn; e += 64) Hs[e] = H[b * nn + e];
  __syncthreads();
  const bool valid = lane < nx;
  const int64_t o = (int64_t)b * nx + lane;
  double xv = valid ? xinit[o] : 0.;
  uint64_t fs = 0, fi = 0;
  int iters = 0;
  auto inv = [&](const InvMap& mp) { return wave_sweep_inverse_lds(Hs, nx, Qi, nx, vb, nx, mp, lane); };
  const bool ok = box_qp_wave(Hs, nx, Qi, nx, vb, nx, lane, valid ? q[o] : 0., valid ? lb[o] : 0.,
                              valid ? ub[o] : 0., xv, c, inv, false, fs, fi, iters);
  __syncthreads();
  if (valid) x[o] = xv;
  for (int64_t e = lane; e < nn; e += 64) Hinv[b * nn + e] = ok ? Qi[e] : 0.;
  if (lane == 0) {
    free_mask[b] = fs;
    inv_mask[b] = fi;
    status[b] = ok ? 0 : 1;
  }
}
#endif


}  // namespace fddp
