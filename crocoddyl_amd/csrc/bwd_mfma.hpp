// Backward Riccati sweep on the fp64 matrix cores (v_mfma_f64_16x16x4_f64).
//
// Same computation as bwd_sweep (SolverDDP::backwardPass + computeGains,
// src/core/solvers/ddp.cpp:180-253, 298-310), reorganised for gfx950:
//
//   Z  = [Fx | Fu]                 (n x (n+m), staged in LDS by LDS-DMA)
//   G  = Vxx' Z                    (MFMA; Vxx' LDS-resident)
//   H  = G^T Z + [Lxx Lxu; . Luu]  = [[Qxx, Qxu], [Qux, Quu]]   (MFMA; the G
//        accumulators are the A operands of H with no data movement:
//        accumulator register r holds rows 4r..4r+3 of a 16-row block, which
//        is exactly the k-slice of one 16x16x4 step; Vxx' is symmetric so
//        G^T = Z^T Vxx' = Fx^T Vxx' as the reference forms it)
//   Qx = Lx + Fx^T Vx', Qu = Lu + Fu^T Vx'  (VALU, folded into the G loop: the
//        lane already holds the Z fragment)
//   C = Lc^-1, the inverse Cholesky factor of Quu (chol_inv_sweep) on wave 0,
//        overlapped with the Qxx/Qxu tiles of waves 1-3; a pivot <= 0 is the
//        reference's LLT failure
//   K  = C^T (C Qxu^T) (two MFMA products), k = C^T (C Qu) (VALU): as accurate as
//        the reference's LLT solves (an explicit Quu^-1 is not, on graded Quu)
//   Vxx = Qxx - K^T Qxu^T (+ xreg I), written symmetric; the owner of x block
//        i keeps its K(:, i) tiles in registers and finds its Qxx(i, :) tiles
//        in the (dead) Vxx' buffer, updating them in place
//   Vx  = Qx + K^T Quu k - 2 K^T Qu (+ Vxx fs)
//
// Pipeline per knot t:
//   P1  the knot's cost blocks (Lxx, Lxu, Luu) are loaded into registers in
//       accumulator layout; G (LDS only) covers their latency; B0; then H,
//       Qx/Qu ; wave 0: Quu^-1
//   B1  -> an LDS-DMA of Fx, Fu, Lx, Lu of knot t-1 is issued; it lands
//       while P2/P3 run (raw s_barrier, no vmcnt wait until B3).
//       fs of knot t-1 follows right after B3 (its buffer is read in P3).
//   P2  K, V update (waves 1-3); k, Quu k (wave 0)
//   B2
//   P3  Vx, Vxx fs, reduction terms
//   B3  vmcnt(0) + barrier: the knot t-1 operands are resident.
// (4 barriers per knot in all.)
//
// One workgroup (4 waves, one per SIMD) per batch element; the element's
// horizon is swept serially. n and m are padded to 16-multiples (NTL, MTL
// tiles); padded rows/cols are kept exactly zero.
// MFMA fragment maps (MI355X guide, f64 16x16x4): A[i=lane&15][k=lane>>4],
// B[k=lane>>4][j=lane&15], C/D col=lane&15, row=(lane>>4)+4*reg.
#pragma once

#include "box_qp.hpp"
#include "fddp_device.hpp"

namespace fddp {

typedef double f64x4 __attribute__((ext_vector_type(4)));

// 1/d from v_rcp_f64 and Newton steps (the IEEE division sequence is ~3x
// longer on the sweep's critical path; dependent f64 FMA latency is 32 cycles)
__device__ __forceinline__ double rcp_f64(double d) {
  double x = __builtin_amdgcn_rcp(d);
#ifndef FDDP_RCP_NO_NEWTON
  x = fma(fma(-d, x, 1.), x, x);
#ifndef FDDP_RCP_ONE_NEWTON
  x = fma(fma(-d, x, 1.), x, x);
#endif
#endif
  return x;
}

__device__ __forceinline__ f64x4 mfma4(double a, double b, f64x4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// dma_cols: ncols columns of nr doubles (global ld nr) into LDS columns of
// stride ld (a multiple of 2); one column per wave instruction (16-B chunks
// when nr is even, else 4-byte pieces). Rows [nr, ld) are left untouched.
template <int NW>
__device__ __forceinline__ void dma_cols(double* lds, int ld, const double* g, int nr, int ncols, int wid, int lane) {
  if ((nr & 1) == 0) {
    const int nch = nr >> 1;
    for (int col = wid; col < ncols; col += NW)
      for (int base = 0; base < nch; base += 64)
        if (base + lane < nch)
          __builtin_amdgcn_global_load_lds(g + (int64_t)col * nr + 2 * (base + lane),
                                           (lds_void_ptr)(lds + col * ld + 2 * base), 16, 0, 0);
  } else {
    const int nw = 2 * nr;
    for (int col = wid; col < ncols; col += NW)
      for (int base = 0; base < nw; base += 64)
        if (base + lane < nw)
          __builtin_amdgcn_global_load_lds((const char*)(g + (int64_t)col * nr) + 4 * (base + lane),
                                           (lds_void_ptr)((char*)(lds + col * ld) + 4 * base), 4, 0, 0);
  }
}

// The columns of an n x ncols column-major global block into LDS columns of
// LDZ doubles (LDZ even, nr even): every wave instruction moves a full 1 KiB
// (64 lanes x 16 B, a per-lane gather), the LDZ - nr padding rows of each
// column are filled from a 16-byte zero source. 39% fewer instructions than
// one per column at n = 76, and a DMA instruction costs ~60-185 cycles of
// issue whatever its size.
template <int NWD, int LDZ>
__device__ __forceinline__ void dma_cols_full(double* lds, const double* g, int nr, int ncols, const double* zero16,
                                              int rank, int lane) {
  constexpr int CPC = LDZ / 2;  // 16-B chunks per LDS column
  const int dpc = nr >> 1;      // of which data
  const int tot = ncols * CPC;
  for (int base = rank * 64; base < tot; base += NWD * 64) {
    const int e = base + lane;
    if (e < tot) {
      const int col = e / CPC, p = e - col * CPC;
      const double* src = p < dpc ? g + (int64_t)col * nr + 2 * p : zero16;
      __builtin_amdgcn_global_load_lds(src, (lds_void_ptr)(lds + 2 * base), 16, 0, 0);
    }
  }
}

template <int NTL, int MTL>
struct MfmaCfg {
  static constexpr int NP = 16 * NTL;
  static constexpr int MP = 16 * MTL;
  static constexpr int JT = NTL + MTL;
  // V / Qxu leading dimension = 2 (mod 4) doubles: 16 lanes stepping along
  // the leading dimension hit 16 distinct bank pairs (stores of tiles in the
  // transposed direction, the transposed P2 tiles), and a fragment read along
  // it (lanes c consecutive, q rows apart) is nearly conflict-free
  static constexpr int LDV = NP + 2;
  static constexpr int LDQ = MP;
  static_assert(MP <= 64, "u block must fit one wave for the factorisation");
  // LDS carve (doubles). Z = [Fx | Fu] is stored with the compile-time
  // column stride NP (zero rows/cols beyond n, m) so that every fragment
  // address is a per-lane base plus an immediate offset.
  static constexpr int oV = 0;
  static constexpr int oQxu = oV + LDV * NP;
  static constexpr int oQuu = oQxu + LDV * MP;
  static constexpr int oQi = oQuu + LDQ * MP;
  static constexpr int oVx = oQi + LDQ * MP;
  static constexpr int oQx = oVx + NP;
  static constexpr int oLx = oQx + NP;
  static constexpr int oFs = oLx + NP;
  static constexpr int oQu = oFs + NP;
  static constexpr int oLu = oQu + MP;
  static constexpr int oKv = oLu + MP;  // kv + quuk: the sweep's 64-double row buffer (wave 0, P1)
  static constexpr int oQuuk = oKv + MP;
  static constexpr int oRed = oKv + (2 * MP > 64 ? 2 * MP : 64);  // 5 sums x up to 8 waves
  static constexpr int oFlag = oRed + 40;  // flag; Quu-ready, G-done, P2-done, H-done counters (5 ints)
  // Z column stride ZLD = NP - 2 (= 2 mod 4): the 16 lanes of a B fragment
  // read 16 columns at a stride of 2*ZLD = 4 (mod 8) banks, conflict-free
  // (a stride of NP was an 8-way conflict). k-steps past ZLD read the next
  // column's first rows (or the 2 zero doubles after the last column); they
  // only ever multiply the zero rows of Vxx' / G, so nothing changes.
  static constexpr int ZLD = NP - 2;
  static constexpr int oZx = (oFlag + 4 + 1) & ~1;
  static constexpr int oZu = oZx + NP * ZLD;
  static constexpr int total0 = oZu + MP * ZLD + 2;
  // C^T, the transposed inverse Cholesky factor (chol_inv_sweep), at the odd leading
  // dimension LDT (its fragment reads step along it: conflict-free): its own area when
  // it fits the 160 KB, else over Zu, which is dead from the H tiles of a knot until
  // the next knot's LDS-DMA (issued after B2 by the 8-wave plan, see bwd_knot)
  static constexpr int LDT = MP + 1;
  static constexpr bool ct_own = sizeof(double) * (total0 + MP * LDT) <= 160 * 1024;
  static constexpr int oCt = ct_own ? total0 : oZu;
  // the prefetch plan's second operand buffers (BwdPlan::prefetch; C^T in its own area):
  // Z, then lx, lu, fs
  static constexpr int oZx2 = (total0 + MP * LDT + 1) & ~1;
  static constexpr int oZu2 = oZx2 + NP * ZLD;
  static constexpr int oLx2 = oZu2 + MP * ZLD + 2;
  static constexpr int oLu2 = oLx2 + NP;
  static constexpr int oFs2 = oLu2 + MP;
  // and the cost blocks Lxx | Lxu | Luu of a knot (n x n, n x m, m x m, column-major as in
  // HBM), twice: the prefetch plan stages them with the knot's other operands
  static constexpr int CB = NP * NP + NP * MP + MP * MP;
  static constexpr int oCb = (oFs2 + NP + 1) & ~1;
  static constexpr bool pre_fits = ct_own && sizeof(double) * (oCb + 2 * CB) <= 160 * 1024;
  static constexpr int total = pre_fits ? oCb + 2 * CB : (ct_own ? total0 + MP * LDT : total0);
  static_assert(ct_own || MP * LDT <= MP * ZLD, "C^T over Zu");
  static constexpr size_t bytes = sizeof(double) * total;
};


// Quu^-1 by the symmetric sweep operator on one wave (Gauss-Jordan without
// pivoting, which SPD matrices do not need). Pivot k is the k-th Schur
// complement = L(k,k)^2 of the Cholesky factor, so `pivot <= 0` is exactly
// Eigen LLT's failure (ddp.cpp:300-304); after sweeping every pivot the
// matrix holds -Quu^-1. Lane l owns column jc = l % MP and rows h*RPL + r
// (h = l / MP). Returns true if a pivot was not positive.
// Fully unrolled so that the pivot register A[k % RPL] is static. Every lane
// publishes one register per step (rb[lane], unconditionally, so the step
// stays one basic block): the lanes of row group k / RPL publish row k, which
// by symmetry doubles as column k. The next step's row is updated and
// published first, so its LDS round trip overlaps the rest of this step's
// updates. No s_waitcnt is needed: one wave's LDS accesses execute in order;
// the empty asm fences only stop the compiler from forwarding a lane's own
// write to its reads. Quu / Qi: column-major, leading dimension LDQ; rb: 64
// doubles of LDS.
template <int MP, int LDQ>
__device__ __forceinline__ bool sym_sweep_inverse(const double* Quu, double* Qi, double* rb, int m, int lane) {
  constexpr int RPL = MP * MP / 64;
  static_assert(MP * MP % 64 == 0 && 64 % MP == 0, "sweep lane layout");
  const int jc = lane % MP, h = lane / MP;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  double A[RPL];
#pragma unroll
  for (int r = 0; r < RPL; ++r) A[r] = Quu[(h * RPL + r) * LDQ + jc];
  bool bad = false;
  rb[lane] = A[0];
#pragma unroll
  for (int k = 0; k < MP; ++k) {
    if (k < m) {
      const int hk = k / RPL, rk = k % RPL;
      const int r1 = (k + 1) % RPL;
      asm volatile("" ::: "memory");
      // step k's broadcast operands: pivot d = A(k, k), A(k, jc), row k at
      // rows h*RPL + r (= column k by symmetry)
      const double d = rb[hk * MP + k];
      const double akj = rb[hk * MP + jc];
      double ak[RPL];
#pragma unroll
      for (int r = 0; r < RPL; ++r) ak[r] = rb[hk * MP + h * RPL + r];
      bad |= !(d > 0.);
      const bool colk = jc == k;
      // next step's row first, with the dependent chain kept short
      // (A - (a_ik a_kj) * (1/d): the product does not wait for 1/d), then
      // published so its LDS round trip overlaps this step's other updates
      const double p1 = ak[r1] * akj;
      const double dinv = rcp_f64(d);
      {
        const double u = colk ? ak[r1] * dinv : fma(-p1, dinv, A[r1]);
        A[r1] = (r1 == rk && h == hk) ? (colk ? -dinv : akj * dinv) : u;
      }
      asm volatile("" ::: "memory");
      rb[lane] = A[r1];
      __builtin_amdgcn_sched_barrier(0);
      // the rest: one FMA per element on every lane, then the lane(s) owning
      // column k (exec-masked) overwrite theirs with A(i, k) / d, and row k's
      // register becomes A(k, jc) / d (-1/d at (k, k))
      const double w = akj * dinv;
#pragma unroll
      for (int r = 0; r < RPL; ++r)
        if (r != r1) A[r] = fma(-ak[r], w, A[r]);
      if (colk) {
#pragma unroll
        for (int r = 0; r < RPL; ++r)
          if (r != r1) A[r] = ak[r] * dinv;
      }
      if (rk != r1 && h == hk) A[rk] = colk ? -dinv : w;
    }
  }
#pragma unroll
  for (int r = 0; r < RPL; ++r) {
    const int i = h * RPL + r;
    Qi[i * LDQ + jc] = (i < m && jc < m) ? -A[r] : 0.;
  }
  return bad;
}

// The inverse Cholesky factor C = Lc^-1 of Quu = Lc Lc^T (the reference's LLT,
// ddp.cpp:298-310) on one wave, in the lane layout of sym_sweep_inverse. Gaussian
// elimination without pivoting (Quu = L D L^T, L unit lower) with the multipliers
// applied to the identity in place: after pivot k, for every row i > k,
//   A(i, j) -= l_ik A(k, j) (j != k),   A(i, k) = -l_ik,   l_ik = A(i, k) / d_k,
// so the strictly lower part accumulates L^-1 (its row k holds L^-1(k, j < k), the
// trailing block stays the symmetric Schur complement, which supplies A(i, k) from
// the published row k) and the diagonal the pivots d_k; then C = D^-1/2 L^-1. The
// gains are formed as K = C^T (C Qxu^T): on the C5 walk's Quu (cond 1e9 .. 5e10,
// graded) the explicit inverse's product Quu^-1 Qxu^T was 200x further from the
// LLT solves than the solves from each other (the round-4 parity trace: K 3e-8 vs
// 1.5e-10), the two triangular products as close as the solves. A pivot <= 0 is the
// LLT failure. C: lower triangular, zero above the diagonal and beyond m.
// Cx (may be null): C's transpose as well, C(i, j) at Cx[i * LDQ + j]; Ct null: no C^T.
template <int MP, int LDQ, int LDT>
__device__ __forceinline__ bool chol_inv_sweep(const double* Quu, double* C, double* Ct, double* rb, int m, int lane,
                                               int* ct_ready, int ct_target, double* Cx = nullptr) {
  constexpr int RPL = MP * MP / 64;
  static_assert(MP * MP % 64 == 0 && 64 % MP == 0, "sweep lane layout");
  const int jc = lane % MP, h = lane / MP;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  double A[RPL];
#pragma unroll
  for (int r = 0; r < RPL; ++r) A[r] = Quu[(h * RPL + r) * LDQ + jc];
  bool bad = false;
  rb[lane] = A[0];
#pragma unroll
  for (int k = 0; k < MP; ++k) {
    if (k < m) {
      const int hk = k / RPL;
      const int r1 = (k + 1) % RPL;
      asm volatile("" ::: "memory");
      // row k (published by its lanes): the pivot, A(k, jc), and A(k, i) = A(i, k)
      // for my rows i > k (the trailing block is symmetric)
      const double d = rb[hk * MP + k];
      const double akj = rb[hk * MP + jc];
      double ak[RPL];
#pragma unroll
      for (int r = 0; r < RPL; ++r) ak[r] = rb[hk * MP + h * RPL + r];
      bad |= !(d > 0.);
      const bool colk = jc == k;
      // next pivot row first (its product does not wait for 1/d), then published
      const double p1 = ak[r1] * akj;
      const double dinv = rcp_f64(d);
      if (h * RPL + r1 > k) A[r1] = colk ? -ak[r1] * dinv : fma(-p1, dinv, A[r1]);
      asm volatile("" ::: "memory");
      rb[lane] = A[r1];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < RPL; ++r)
        if (r != r1 && h * RPL + r > k) A[r] = colk ? -ak[r] * dinv : fma(-ak[r] * akj, dinv, A[r]);
    }
  }
  // 1 / sqrt(d_i) by the diagonal's lanes (one each), published; C(i, j) = L^-1(i, j) / sqrt(d_i)
  // into C (column-major, ld LDQ) and C^T (column-major, ld LDT)
  asm volatile("" ::: "memory");
#pragma unroll
  for (int r = 0; r < RPL; ++r)
    if (h * RPL + r == jc) rb[jc] = (jc < m && A[r] > 0.) ? 1. / sqrt(A[r]) : 0.;
  asm volatile("" ::: "memory");
  // C^T's area may still be read by other waves (ct_target > 0: wait for them)
  if (Ct && ct_target > 0) {
    lds_wait_ge(ct_ready, ct_target);
  }
#pragma unroll
  for (int r = 0; r < RPL; ++r) {
    const int i = h * RPL + r;
    const double s = rb[i];
    double v = 0.;
    if (i < m && jc < m) v = i == jc ? s : (jc < i ? A[r] * s : 0.);
    C[jc * LDQ + i] = v;
    if (Ct) Ct[i * LDT + jc] = v;
    if (Cx) Cx[i * LDQ + jc] = v;
  }
  return bad;
}

// The same factor for a 32-wide Quu (the C5 walk's m = 32) in 16-blocks, so that the
// latency-bound sweeps run 2 x 16 light steps (4 rows per lane) instead of 32 steps of
// 16 rows per lane: Quu = [A11 A21^T; A21 A22] = L L^T, C = L^-1 =
// [C11 0; C21 C22]:
//   C11 = chol_inv(A11);  G = C11 A21^T (= L21^T);  S = A22 - G^T G;
//   C22 = chol_inv(S);    C21 = -C22 (L21 C11)
// (the blocked right-looking Cholesky, the off-diagonal products on MFMA in registers:
// the accumulator register s of G / T is the A and B fragment of k-step s). C as
// chol_inv_sweep's (col-major, ld LDQ, zero above the diagonal and beyond m), then C^T
// (ld LDT) once the other waves are done with its area.
template <int LDQ, int LDT>
__device__ __forceinline__ bool chol_inv_blocked2(const double* Quu, double* C, double* Ct, double* rb, int m, int lane,
                                                  int* ct_ready, int ct_target) {
  const int q = lane >> 4, c = lane & 15;
  const int m1 = m < 16 ? m : 16, m2 = m - 16;
  // C11, and its transpose in the lower-left block (free until C21 lands there)
  bool bad = chol_inv_sweep<16, LDQ, LDT>(Quu, C, nullptr, rb, m1, lane, nullptr, 0, C + 16);
  asm volatile("" ::: "memory");
  if (m2 > 0) {
    f64x4 G = {0., 0., 0., 0.}, T = {0., 0., 0., 0.}, S, X = {0., 0., 0., 0.};
    // G = C11 A12: A(c, 4s+q) = C11(c, 4s+q); B(4s+q, c) = A12(4s+q, c) = Quu(16+c, 4s+q)
#pragma unroll
    for (int s = 0; s < 4; ++s) G = mfma4(C[(4 * s + q) * LDQ + c], Quu[(4 * s + q) * LDQ + 16 + c], G);
    // S = A22 - G^T G, held as S(q+4r, c); staged (by symmetry) at (c, 16+q+4r), the
    // upper-right block (zero in C, rewritten below)
#pragma unroll
    for (int r = 0; r < 4; ++r) S[r] = Quu[(16 + q + 4 * r) * LDQ + 16 + c];
#pragma unroll
    for (int s = 0; s < 4; ++s) S = mfma4(-G[s], G[s], S);
#pragma unroll
    for (int r = 0; r < 4; ++r) C[(16 + q + 4 * r) * LDQ + c] = S[r];
    // T = L21 C11: A(c, 4s+q) = L21(c, 4s+q) = G(4s+q, c); B(4s+q, c) = C11(4s+q, c),
    // stored transposed at (16+c, 4s+q)
#pragma unroll
    for (int s = 0; s < 4; ++s) T = mfma4(G[s], C[(4 * s + q) * LDQ + 16 + c], T);
    asm volatile("" ::: "memory");
    bad = chol_inv_sweep<16, LDQ, LDT>(C + 16 * LDQ, C + 16 * LDQ + 16, nullptr, rb, m2, lane, nullptr, 0) || bad;
    asm volatile("" ::: "memory");
    // C21 = -C22 T: A(c, 4s+q) = C22(c, 4s+q) at (16+c, 16+4s+q); B = T's register s
#pragma unroll
    for (int s = 0; s < 4; ++s) X = mfma4(-C[(16 + 4 * s + q) * LDQ + 16 + c], T[s], X);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      C[c * LDQ + 16 + q + 4 * r] = X[r];
      C[(16 + q + 4 * r) * LDQ + c] = 0.;  // the staging of S
    }
  } else {
#pragma unroll
    for (int r = 0; r < 8; ++r) {  // rows 16..31 (C11^T's block too), then the upper-right block
      const int e = lane + 64 * r, i = 16 + (e & 15), j = e >> 4;
      C[j * LDQ + i] = 0.;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) C[(16 + q + 4 * r) * LDQ + c] = 0.;
  }
  asm volatile("" ::: "memory");
  if (ct_target > 0) {
    lds_wait_ge(ct_ready, ct_target);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int e = lane + 64 * r, i = e & 31, j = e >> 5;
    Ct[i * LDT + j] = C[j * LDQ + i];
  }
  return bad;
}

// Same sweep with each lane owning a BS x BS block of the matrix (BS = MP/8,
// an 8 x 8 grid of blocks over the 64 lanes): per step one FMA per element
// as before, but the column-k / row-k fix-ups touch BS elements of 8 lanes
// instead of MP elements of 2 lanes, and the broadcast reads are 2 x BS
// contiguous doubles. VALU-issue bound (f64 ops issue at 8 cycles), so this
// is ~1.8x fewer cycles per pivot than the column-per-lane layout.
template <int MP, int LDQ>
__device__ __forceinline__ bool sym_sweep_inverse_blk(const double* Quu, double* Qi, double* rb, int m, int lane) {
  constexpr int BS = MP / 8;
  static_assert(MP % 8 == 0 && BS >= 1, "8 x 8 lane grid");
  const int bi = lane >> 3, bj = lane & 7;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  double A[BS][BS];
#pragma unroll
  for (int a = 0; a < BS; ++a)
#pragma unroll
    for (int b = 0; b < BS; ++b) A[a][b] = Quu[(BS * bj + b) * LDQ + BS * bi + a];
  bool bad = false;
  if (bi == 0) {
#pragma unroll
    for (int b = 0; b < BS; ++b) rb[BS * bj + b] = A[0][b];
  }
#pragma unroll
  for (int k = 0; k < MP; ++k) {
    if (k < m) {
      const int kb = k / BS, kr = k % BS;
      const int k1 = k + 1, kb1 = k1 / BS, kr1 = k1 % BS;
      (void)k1;
      asm volatile("" ::: "memory");
      const double d = rb[k];
      double rowv[BS], colv[BS];
#pragma unroll
      for (int b = 0; b < BS; ++b) rowv[b] = rb[BS * bj + b];  // A(k, my columns)
#pragma unroll
      for (int a = 0; a < BS; ++a) colv[a] = rb[BS * bi + a];  // A(my rows, k) by symmetry
      bad |= !(d > 0.);
      const double dinv = rcp_f64(d);
      double w[BS];
#pragma unroll
      for (int b = 0; b < BS; ++b) w[b] = rowv[b] * dinv;
      const bool colk = bj == kb, rowk = bi == kb;
      auto fix = [&](int a, int b, double v) {  // column-k / row-k / (k, k) fix-ups
        if (colk && b == kr) v = colv[a] * dinv;
        if (rowk && a == kr) v = (colk && b == kr) ? -dinv : w[b];
        return v;
      };
      // next step's row first (register row kr1 holds it in lanes bi == kb1;
      // after the last pivot the publish is dead and harmless)
#pragma unroll
      for (int b = 0; b < BS; ++b) A[kr1][b] = fix(kr1, b, fma(-colv[kr1], w[b], A[kr1][b]));
      asm volatile("" ::: "memory");
      if (bi == kb1) {
#pragma unroll
        for (int b = 0; b < BS; ++b) rb[BS * bj + b] = A[kr1][b];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int a = 0; a < BS; ++a) {
        if (a == kr1) continue;
#pragma unroll
        for (int b = 0; b < BS; ++b) A[a][b] = fix(a, b, fma(-colv[a], w[b], A[a][b]));
      }
    }
  }
#pragma unroll
  for (int a = 0; a < BS; ++a)
#pragma unroll
    for (int b = 0; b < BS; ++b) {
      const int i = BS * bi + a, j = BS * bj + b;
      Qi[j * LDQ + i] = (i < m && j < m) ? -A[a][b] : 0.;
    }
  return bad;
}

// The masked / relabelled inverse an InvMap describes (the box QP's free
// Hessian, box_qp.hpp) with the register sweep: the masked matrix is staged
// into Qi, swept in place (the sweep reads all of it before writing), and
// the result is cut to the `out` set.
template <int MP, int LDQ>
__device__ __forceinline__ bool sym_sweep_inverse_masked(const double* H, double* Qi, double* rb, int m, int lane,
                                                         const InvMap& mp) {
  // staged four entries per lane at a time, loads before stores (one LDS round trip per four)
  int e = lane;
  for (; e + 3 * 64 < m * m; e += 4 * 64) {
    double v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = mp.load(H, LDQ, (e + 64 * q) % m, (e + 64 * q) / m);
#pragma unroll
    for (int q = 0; q < 4; ++q) Qi[((e + 64 * q) / m) * LDQ + (e + 64 * q) % m] = v[q];
  }
  for (; e < m * m; e += 64) {
    const int i = e % m, j = e / m;
    Qi[j * LDQ + i] = mp.load(H, LDQ, i, j);
  }
  const bool bad = sym_sweep_inverse<MP, LDQ>(Qi, Qi, rb, m, lane);
  asm volatile("" ::: "memory");
  for (int e = lane; e < m * m; e += 64) {
    const int i = e % m, j = e / m;
    if (!(mp.out(i) && mp.out(j))) Qi[j * LDQ + i] = 0.;
  }
  asm volatile("" ::: "memory");
  return bad;
}

// Compile-time work plan of the sweep: which wave owns which column blocks
// of Z (G = Vxx' Z_i and the H tiles (i, j >= jstart(i))), and which wave
// updates which Vxx tile in P2. With the plan static, every wave's code path
// has only its own tiles, statically indexed registers and no per-tile
// predicates.
//  NW = 4: wave 0 takes the u blocks (Quu and its inverse), waves 1-3 share
//          the x blocks by longest-processing-time on their MFMA count.
//  NW = 8: two waves per SIMD (wave w on SIMD w % 4). Wave 0 only inverts Quu
//          (VALU), sharing its SIMD with the smallest block; the other blocks
//          are paired largest-with-smallest so that the SIMDs get equal MFMA
//          loads, and the u-block owners signal wave 0 through an LDS counter
//          as soon as their Quu rows are stored.
// V tile (i, j), i <= j, is updated by the owner of i or of j (whoever has
// fewer), using the K(:, i) or K(:, j) tiles that owner holds in registers.
template <int NTL, int MTL>
__host__ __device__ constexpr int bwd_block_cost(int i) {
  return 4 * NTL * NTL + (i < NTL ? (NTL - i + MTL) : MTL) * 4 * NTL;
}

template <int NTL, int MTL, int NW>
struct BwdPlan {
  static constexpr int JT = NTL + MTL;
  static_assert(NW == 1 || NW == 4 || NW == 8, "1, 4 or 8 waves");
  static_assert(NW != 1 || JT <= 8, "1-wave plan: at most 8 column blocks");
  static_assert(NW == 4 || JT <= 7, "8-wave plan: at most 7 column blocks");
  int nown[8];
  int blk[8][8];
  int ntile[8];
  int tile[8][24][2];
  int uwaves;  // waves other than 0 that own u blocks
  int gwaves;  // waves owning any block (they read Vxx' in G)
  int ndma;    // waves issuing the LDS-DMA of the next knot's operands
  int dmarank[8];
  int xwaves;  // waves owning x blocks (the P3 consumers)
  bool prefetch;  // double-buffered operands, DMA at the knot's start (see below)
  constexpr BwdPlan()
      : nown{}, blk{}, ntile{}, tile{}, uwaves(0), gwaves(0), ndma(0), dmarank{}, xwaves(0), prefetch(false) {
    int owner[16] = {};
    if (NW == 1) {  // small knots: one wave owns every block (no partial barrier ever waits)
      for (int u = 0; u < MTL; ++u) blk[0][nown[0]++] = NTL + u;
      for (int i = 0; i < NTL; ++i) blk[0][nown[0]++] = i;
    } else if (NW == 4) {
      for (int u = 0; u < MTL; ++u) {
        blk[0][nown[0]++] = NTL + u;
        owner[NTL + u] = 0;
      }
      int load[4] = {0, 0, 0, 0};
      for (int i = 0; i < NTL; ++i) {  // the cost decreases with i: LPT order
        int best = 1;
        for (int w = 2; w < 4; ++w)
          if (load[w] < load[best]) best = w;
        blk[best][nown[best]++] = i;
        owner[i] = best;
        load[best] += bwd_block_cost<NTL, MTL>(i);
      }
    } else {
      // eight items: the blocks, the inversion (-1) and empty slots (-2)
      int item[8] = {}, cost[8] = {};
      for (int k = 0; k < 8; ++k) {
        item[k] = k < JT ? k : (k == JT ? -1 : -2);
        // the inversion counts as the largest item, so it shares its SIMD with
        // the smallest block (a u block, done before the inversion starts):
        // it is VALU-issue bound, and an MFMA partner steals its issue slots
        cost[k] = k < JT ? bwd_block_cost<NTL, MTL>(k) : (k == JT ? 1 << 20 : 0);
      }
      for (int a = 0; a < 8; ++a)  // sort by cost, descending
        for (int b2 = a + 1; b2 < 8; ++b2)
          if (cost[b2] > cost[a]) {
            const int ti = item[a], tc = cost[a];
            item[a] = item[b2];
            cost[a] = cost[b2];
            item[b2] = ti;
            cost[b2] = tc;
          }
      int gp = 0;  // the pair holding the inversion goes to SIMD 0
      for (int p = 0; p < 4; ++p)
        if (item[p] == -1 || item[7 - p] == -1) gp = p;
      int simd = 1;
      for (int p = 0; p < 4; ++p) {
        const int s2 = p == gp ? 0 : simd++;
        const int a2 = item[p], b3 = item[7 - p];
        int wa = s2, wb = s2 + 4;
        if (b3 == -1) {  // the inversion item always takes wave 0
          wa = s2 + 4;
          wb = s2;
        }
        if (a2 >= 0) {
          blk[wa][nown[wa]++] = a2;
          owner[a2] = wa;
        }
        if (b3 >= 0) {
          blk[wb][nown[wb]++] = b3;
          owner[b3] = wb;
        }
      }
    }
    for (int w = 1; w < NW; ++w)
      for (int o = 0; o < nown[w]; ++o)
        if (blk[w][o] >= NTL) {
          ++uwaves;
          break;
        }
    for (int w = 0; w < NW; ++w) gwaves += nown[w] > 0 ? 1 : 0;
    // the next knot's LDS-DMA: each instruction blocks its wave for a few
    // hundred cycles, so in the 8-wave plan it goes to the waves that have no
    // x blocks (no P2 / P3 MFMA work); they skip B2 (see bwd_knot)
    for (int w = 0; w < NW; ++w) dmarank[w] = -1;
    // Prefetch plan (C^T in its own area, some wave other than 0 owns no block): the
    // operands are double-buffered and those idle waves issue knot t-1's DMA at the start
    // of knot t, a whole knot before B3 waits for it (and B1 waits for LDS only)
    int idle = 0;
    for (int w = 1; w < NW; ++w) idle += nown[w] == 0 ? 1 : 0;
    prefetch = MfmaCfg<NTL, MTL>::pre_fits && idle >= 1;
    if (prefetch) {
      for (int w = 1; w < NW; ++w)
        if (nown[w] == 0) dmarank[w] = ndma++;
    } else if (NW <= 4) {
      for (int w = 0; w < NW; ++w) dmarank[w] = ndma++;
    } else {  // the waves without x blocks: no MFMA work in P2 / P3
      for (int w = 0; w < NW; ++w)
        if (!owns_x(w)) dmarank[w] = ndma++;
    }
    for (int w = 0; w < NW; ++w) xwaves += owns_x(w) ? 1 : 0;
    // V tiles: the diagonal with its owner, the rest greedily
    int vload[8] = {};
    for (int i = 0; i < NTL; ++i) {
      const int w = owner[i];
      tile[w][ntile[w]][0] = i;
      tile[w][ntile[w]][1] = i;
      ++ntile[w];
      vload[w] += 3;  // K(:, i) + the diagonal tile
    }
    for (int i = 0; i < NTL; ++i)
      for (int j = i + 1; j < NTL; ++j) {
        const int w = vload[owner[j]] < vload[owner[i]] ? owner[j] : owner[i];
        tile[w][ntile[w]][0] = i;
        tile[w][ntile[w]][1] = j;
        ++ntile[w];
        vload[w] += 1;
      }
  }
  constexpr bool owns_x(int w) const {
    for (int o = 0; o < nown[w]; ++o)
      if (blk[w][o] < NTL) return true;
    return false;
  }
  constexpr bool owns_u(int w) const {
    for (int o = 0; o < nown[w]; ++o)
      if (blk[w][o] >= NTL) return true;
    return false;
  }
  constexpr int slot(int w, int blockid) const {  // index o of blockid in blk[w], or -1
    for (int o = 0; o < nown[w]; ++o)
      if (blk[w][o] == blockid) return o;
    return -1;
  }
};
template <int NTL>
__host__ __device__ constexpr int bwd_jstart(int i) {
  return i < NTL ? i : NTL;
}

// A knot descriptor's nu by a scalar (constant address space) load: the descriptors do
// not change during a kernel.
__device__ __forceinline__ int knot_nu_const(const Dev& D, int t) {
  typedef const __attribute__((address_space(4))) fddp_knot_desc* const_knot_ptr;
  return ((const_knot_ptr)(uintptr_t)D.knots)[t].nu;
}

// LDS carve of one workgroup (see MfmaCfg).
struct BwdLds {
  double *V, *Qxu, *Quu, *Qi, *vx, *qx, *lxv, *fsb, *qu, *luv, *kv, *quuk, *rowbuf, *red, *Zx, *Zu, *Ct;
  double *Zx2, *Zu2, *lxv2, *luv2, *fsb2;  // the prefetch plan's second buffers (else = the first)
  double *cb0, *cb1;                       // the prefetch plan's cost-block buffers
  int* flag;
};

// SolverBoxFDDP::computeGains on wave 0 (box-fddp.cpp:48-79): the box QP
// (box_qp.hpp) on Quu, Qu with bounds u_lb - us, u_ub - us, warm-started at
// the previous k; leaves Quu_inv in Qi, k = -x in kv (and in D.k), and Qu
// zeroed on the clamped set. Returns false where the reference raises
// backward_error (including its qp_ size check: the QP has
// runningModels[0]->nu variables, box-fddp.cpp:16, box-qp.cpp:53-72).
template <int MP, int LDQ>
__device__ __forceinline__ bool box_gains_wave(const Dev& D, const BwdLds& L, int b, int t, int cur, int lane) {
  const int nu = D.knots[t].nu;
  if (nu != D.knots[0].nu) return false;
  const int64_t rr = D.run(b, t);
  const bool valid = lane < nu;
  double q = 0., lb = 0., ub = 0., x = 0.;
  if (valid) {
    const double u = D.us[cur][rr * D.sM + lane];
    q = L.qu[lane];
    lb = D.ulb[rr * D.sM + lane] - u;
    ub = D.uub[rr * D.sM + lane] - u;
    x = D.k[rr * D.sM + lane];
  }
  uint64_t fsol, finv;
  int iters;
  int ninv = 0;
  auto inv = [&](const InvMap& mp) {
    ++ninv;
    return sym_sweep_inverse_masked<MP, LDQ>(L.Quu, L.Qi, L.rowbuf, nu, lane, mp);
  };
  const bool qp_ok = box_qp_wave(L.Quu, LDQ, L.Qi, LDQ, L.rowbuf, nu, lane, q, lb, ub, x, D.boxcfg, inv, true, fsol,
                                 finv, iters);
  if (D.box_stats && lane == 0) {
    atomicAdd(D.box_stats, 1ull);
    atomicAdd(D.box_stats + 1, (unsigned long long)iters);
    atomicAdd(D.box_stats + 2, (unsigned long long)ninv);
  }
  if (!qp_ok) return false;
  asm volatile("" ::: "memory");
  if (lane < MP) L.kv[lane] = valid ? -x : 0.;
  if (valid) {
    D.k[rr * D.sM + lane] = -x;
    if (!((fsol >> lane) & 1)) L.qu[lane] = 0.;
  }
  if (D.dQuuInv)
    for (int e = lane; e < nu * nu; e += 64) D.dQuuInv[rr * D.sMM + (e / nu) * D.m + e % nu] = L.Qi[(e / nu) * LDQ + e % nu];
  return true;
}

// One knot of the sweep, as executed by wave W (all four waves call this
// with their own W; the barriers inside line up one to one).
template <int NTL, int MTL, int NW, int W>
__device__ __forceinline__ bool bwd_knot(const Dev& D, const BwdLds& L, int b, int t, bool feas, double xreg,
                                         double ureg, int cur, Stamp& stamp, double (&red5)[5]) {
  using Cfg = MfmaCfg<NTL, MTL>;
  constexpr int NP = Cfg::NP, MP = Cfg::MP, JT = Cfg::JT, LDV = Cfg::LDV, LDQ = Cfg::LDQ, ZLD = Cfg::ZLD;
  constexpr BwdPlan<NTL, MTL, NW> P{};
  constexpr int NO = P.nown[W];
  constexpr int NA = NO > 0 ? NO : 1;
  static_assert(NO <= 8, "column blocks per wave");
  // The lane id and the dimensions are laundered through empty asm on every
  // knot: otherwise LICM hoists every per-lane address of the unrolled code
  // out of the knot loop and keeps them all live (hundreds of registers).
  // m: the padded control dimension of the blocks (nu_max); mu: this knot's nu (an
  // impulse knot has none: Quu_inv, K and k vanish, Vx = Qx, Vxx = Qxx as the reference's
  // backwardPass does for nu = 0, ddp.cpp:229-253); the blocks' columns beyond mu are
  // not read
  // (the knot's nu by a scalar load through the constant address space: a vector load
  // would wait, in-order, behind the previous knot's stores still in flight)
  int lane = threadIdx.x & 63, n = D.n, m = D.m, mu = knot_nu_const(D, t);
  asm volatile("" : "+v"(lane));
  asm volatile("" : "+s"(n), "+s"(m));
  mu = __builtin_amdgcn_readfirstlane(mu);
  const int q = lane >> 4, c = lane & 15;
  const bool xr = !isnan(xreg), ur = !isnan(ureg);
  const int64_t kk = D.knot(b, t), rr = D.run(b, t);
  const bool boxk = feas && mu > 0 && D.box_knot(b, t);  // SolverBoxFDDP gains on this knot (box-fddp.cpp:47)
  if constexpr (W != 0 && P.owns_u(W)) __builtin_amdgcn_s_setprio(2);  // Quu first: the inversion waits on it
  // the next knot's operands (LDS-DMA; lands during P2 / P3)
  // this knot's operand buffers (prefetch plan: by the knot's parity) and knot t-1's
  constexpr bool pre = P.prefetch;
  const bool odd = pre && (t & 1);
  double* const Zx = odd ? L.Zx2 : L.Zx;
  double* const Zu = odd ? L.Zu2 : L.Zu;
  const double* const lxv = odd ? L.lxv2 : L.lxv;
  const double* const luv = odd ? L.luv2 : L.luv;
  const double* const fsb = odd ? L.fsb2 : L.fsb;
  // part 1: Fx (the Zx buffer: no reader after P1) by the DMA waves other than 0, so it can
  // go right after B1 even where C^T lives over Zu; part 2: the rest (Fu into Zu, Lx, Lu and
  // the prefetch plan's blocks); 3: everything
  constexpr int NDX = P.ndma - (P.dmarank[0] >= 0 ? 1 : 0);
  constexpr int CTC = (MP * Cfg::LDT + ZLD - 1) / ZLD;  // Zu columns C^T covers (when it lies over Zu)
  constexpr int RKX = P.dmarank[W] - (P.dmarank[0] >= 0 && P.dmarank[W] > P.dmarank[0] ? 1 : 0);
  auto issue_dma = [&](int part) {
  if constexpr (P.dmarank[W] >= 0) {
    if (t > 0) {  // operands of knot t-1 (prefetch plan: into the other buffers, with fs)
      constexpr int ND = P.ndma, RK = P.dmarank[W];
      const int64_t k1 = kk - 1;
      const bool nb = pre && !odd;
      double* const nZx = nb ? L.Zx2 : L.Zx;
      double* const nZu = nb ? L.Zu2 : L.Zu;
      const bool full = (n & 1) == 0 && ZLD - n <= 2 * 64;
      if (part == 3) {
        if (full) {
          dma_cols_full<ND, ZLD>(nZx, D.Fx + k1 * D.sNN, n, n, D.zero16, RK, lane);
        } else {
          dma_cols<ND>(nZx, ZLD, D.Fx + k1 * D.sNN, n, n, RK, lane);
        }
      } else if (part == 1) {
        // (and the columns of Fu past the ones C^T lies over: CTC Zu columns hold C^T)
        if constexpr (W != 0 && NDX > 0) {
          const int c0 = CTC < m ? CTC : m;
          if (full) {
            dma_cols_full<NDX, ZLD>(nZx, D.Fx + k1 * D.sNN, n, n, D.zero16, RKX, lane);
            if (c0 < m)
              dma_cols_full<NDX, ZLD>(nZu + c0 * ZLD, D.Fu + k1 * D.sNM + (int64_t)c0 * n, n, m - c0, D.zero16, RKX,
                                      lane);
          } else {
            dma_cols<NDX>(nZx, ZLD, D.Fx + k1 * D.sNN, n, n, RKX, lane);
            if (c0 < m) dma_cols<NDX>(nZu + c0 * ZLD, ZLD, D.Fu + k1 * D.sNM + (int64_t)c0 * n, n, m - c0, RKX, lane);
          }
        }
        return;
      }
      // part 2 of a split: only the Fu columns under C^T
      const int mu2 = part == 2 ? (CTC < m ? CTC : m) : m;
      if (full) {
        dma_cols_full<ND, ZLD>(nZu, D.Fu + k1 * D.sNM, n, mu2, D.zero16, RK, lane);
      } else {
        dma_cols<ND>(nZu, ZLD, D.Fu + k1 * D.sNM, n, mu2, RK, lane);
      }
      dma_vec<ND>(nb ? L.lxv2 : L.lxv, D.Lx + k1 * D.sN, n, RK, lane);
      dma_vec<ND>(nb ? L.luv2 : L.luv, D.Lu + k1 * D.sM, m, RK, lane);
      if constexpr (pre) {
        dma_vec<ND>(nb ? L.fsb2 : L.fsb, D.fs + k1 * D.sN, n, RK, lane);
        double* const cb = nb ? L.cb1 : L.cb0;
        dma_vec<ND>(cb, D.Lxx + k1 * D.sNN, n * n, RK, lane);
        dma_vec<ND>(cb + n * n + (n * n & 1), D.Lxu + k1 * D.sNM, n * m, RK, lane);
        dma_vec<ND>(cb + n * n + (n * n & 1) + n * m + (n * m & 1), D.Luu + k1 * D.sMM, m * m, RK, lane);
      }
    }
  }
  };
  if constexpr (pre) issue_dma(3);
  double* V = L.V;
  double* Qxu = L.Qxu;
  double* Quu = L.Quu;
  double* Qi = L.Qi;

  // ---- P1: cost blocks in accumulator layout (both triangles of Lxx: Qxx
  // uses its symmetric part, which the reference reaches through its Vxx
  // symmetrisation); their latency is covered by the G loop
  // Lv: both triangles of Lxx at this wave's P2 V tiles (Qxx uses the
  // symmetric part of Lxx, which the reference reaches through its Vxx
  // symmetrisation; it is added to the G^T Z part in P2). Lq: the Lxu / Luu
  // inits of this wave's Qxu / Quu tiles.
  constexpr int NVT = P.ntile[W] > 0 ? P.ntile[W] : 1;
  double Lv[NVT][4][2];
  double Lq[NA][MTL][4];
  {
    // (the prefetch plan: from their LDS copies, staged a knot ahead)
    const double* const cbk = odd ? L.cb1 : L.cb0;
    const int o1 = n * n + (n * n & 1), o2 = o1 + n * m + (n * m & 1);
    const double* Lxx = pre ? cbk : D.Lxx + kk * D.sNN;
    const double* Lxu = pre ? cbk + o1 : D.Lxu + kk * D.sNM;
    const double* Luu = pre ? cbk + o2 : D.Luu + kk * D.sMM;
#pragma unroll
    for (int k3 = 0; k3 < P.ntile[W]; ++k3) {
      const int i = P.tile[W][k3][0], j = P.tile[W][k3][1];
      const bool rowf = P.slot(W, i) >= 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // the Qxx(i, j) element that acc[r] of this tile holds in P2
        const int R = rowf ? 16 * i + q + 4 * r : 16 * i + c, C = rowf ? 16 * j + c : 16 * j + q + 4 * r;
        const bool ok = R < n && C < n;
        Lv[k3][r][0] = ok ? Lxx[(int64_t)C * n + R] : 0.;
        Lv[k3][r][1] = ok ? Lxx[(int64_t)R * n + C] : 0.;
      }
    }
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      const int i = P.blk[W][o];
#pragma unroll
      for (int ju = 0; ju < MTL; ++ju)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int Cu = 16 * ju + c;
          double v = 0.;
          if (i < NTL) {
            const int R = 16 * i + q + 4 * r;
            if (R < n && Cu < mu) v = Lxu[(int64_t)Cu * n + R];
          } else {
            const int Ru = 16 * (i - NTL) + q + 4 * r;
            if (Ru < mu && Cu < mu) v = Luu[(int64_t)Cu * m + Ru];
          }
          Lq[o][ju][r] = v;
        }
    }
  }
  // G_o = V' Z_i (i = owned block o) and the q-partials of Z_i^T Vx'
  f64x4 G[NA][NTL];
  double qp[NA];
#pragma unroll
  for (int o = 0; o < NA; ++o) {
    qp[o] = 0.;
#pragma unroll
    for (int a = 0; a < NTL; ++a) G[o][a] = f64x4{0., 0., 0., 0.};
  }
  // software-pipelined two k-steps ahead; sched_barriers stop the scheduler
  // from hoisting every fragment read of the unrolled loop (register blowup)
  double vf[3][NTL], zf[3][NA], vxf[3];
  auto gload = [&](int s, int buf) {
    const int row = 4 * s + q;
#pragma unroll
    for (int a = 0; a < NTL; ++a) vf[buf][a] = V[row * LDV + 16 * a + c];
    vxf[buf] = L.vx[row];
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      const int i = P.blk[W][o];
      zf[buf][o] = i < NTL ? Zx[(16 * i + c) * ZLD + row] : Zu[(16 * (i - NTL) + c) * ZLD + row];
    }
  };
  // (rows >= n of V' are exactly zero, so the padded k-steps add nothing;
  // running them keeps the unrolled loop branch-free)
  if (NO > 0) {
    gload(0, 0);
    gload(1, 1);
  }
#pragma unroll
  for (int s = 0; s < 4 * NTL; ++s) {
    if (NO > 0) {
      if (s + 2 < 4 * NTL) gload(s + 2, (s + 2) % 3);
      const int cb = s % 3;
#pragma unroll
      for (int o = 0; o < NO; ++o) {
        qp[o] += zf[cb][o] * vxf[cb];
#pragma unroll
        for (int a = 0; a < NTL; ++a) G[o][a] = mfma4(vf[cb][a], zf[cb][o], G[o][a]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int o = 0; o < NO; ++o) {
    double v = qp[o];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    const int i = P.blk[W][o];
    if (q == 0) {
      if (i < NTL) {
        const int R = 16 * i + c;
        L.qx[R] = R < n ? lxv[R] + v : 0.;
      } else {
        const int Ru = 16 * (i - NTL) + c;
        L.qu[Ru] = Ru < mu ? luv[Ru] + v : 0.;
      }
    }
  }
  stamp.mark(0);
  // B0 (partial, LDS counter): the x-block owners write Qxx into the V'
  // buffer, so they wait until every block owner is done reading V' in G.
  // The u-block owners only write Quu and go on (their Quu rows are what the
  // inversion waits for); the inversion wave does not read V' at all.
  if constexpr (NO > 0) {
    if (lane == 0) lds_signal(L.flag + 2);
  }
  if constexpr (P.owns_x(W)) {
    const int target = P.gwaves * (D.T - t);
    lds_wait_ge(L.flag + 2, target);
  }
  // H(i, j) = G_i^T Z_j (+ Lxu / Luu + ureg I), j >= jstart(i). Qxx(i, j) goes to the
  // dead V' buffer at the mirrored position (R, C) -> V[R * LDV + C]
  // (conflict-free, and a lower tile that no other wave touches before this
  // wave updates it in place in P2); Qxu / Quu tiles go to their buffers.
  // Column j's Z fragments are read into registers while column j-1's MFMAs
  // run (any(j) is monotone in j, so the next column always exists). With two
  // waves per SIMD the partner wave covers that latency instead, and the
  // second buffer's registers are better spent elsewhere.
  constexpr bool ZDB = NW <= 4;
  double zc[4 * NTL], zn[ZDB ? 4 * NTL : 1];
  bool first = true;
  auto zload = [&](double(&zz)[4 * NTL], int j) {
#pragma unroll
    for (int s = 0; s < 4 * NTL; ++s)
      zz[s] = j < NTL ? Zx[(16 * j + c) * ZLD + 4 * s + q] : Zu[(16 * (j - NTL) + c) * ZLD + 4 * s + q];
  };
#pragma unroll
  for (int j = 0; j < JT; ++j) {
    bool any = false;
#pragma unroll
    for (int o = 0; o < NO; ++o) any = any || j >= bwd_jstart<NTL>(P.blk[W][o]);
    if (!any) continue;
    if constexpr (ZDB) {
      if (first) zload(zc, j);
      first = false;
      if (j + 1 < JT) zload(zn, j + 1);
    } else {
      zload(zc, j);
    }
    __builtin_amdgcn_sched_barrier(0);
    const bool isx = j < NTL;
    const int ju = j - NTL;
    f64x4 acc[NA];
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      const int i = P.blk[W][o];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double v;
        if (isx) {
          v = 0.;  // + sym(Lxx) in P2
        } else {
          v = Lq[o][isx ? 0 : ju][r];
          if (ur && i >= NTL && 16 * (i - NTL) + q + 4 * r == 16 * ju + c && 16 * ju + c < mu) v += ureg;
        }
        acc[o][r] = v;
      }
    }
#pragma unroll
    for (int s = 0; s < 4 * NTL; ++s) {
#pragma unroll
      for (int o = 0; o < NO; ++o)
        if (j >= bwd_jstart<NTL>(P.blk[W][o])) acc[o] = mfma4(G[o][s >> 2][s & 3], zc[s], acc[o]);
    }
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      const int i = P.blk[W][o];
      if (j >= bwd_jstart<NTL>(i)) {
        if (isx) {
#pragma unroll
          for (int r = 0; r < 4; ++r) V[(16 * i + q + 4 * r) * LDV + 16 * j + c] = acc[o][r];
        } else if (i < NTL) {
#pragma unroll
          for (int r = 0; r < 4; ++r) Qxu[(16 * ju + c) * LDV + 16 * i + q + 4 * r] = acc[o][r];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) Quu[(16 * ju + c) * LDQ + 16 * (i - NTL) + q + 4 * r] = acc[o][r];
        }
      }
    }
    if constexpr (ZDB) {
#pragma unroll
      for (int s = 0; s < 4 * NTL; ++s) zc[s] = zn[s < (ZDB ? 4 * NTL : 1) ? s : 0];
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (W != 0 && P.owns_u(W)) {  // this wave's Quu rows are stored: tell wave 0
    if (lane == 0) lds_signal(L.flag + 1);
    __builtin_amdgcn_s_setprio(0);
  }
  if constexpr (!Cfg::ct_own && NO > 0) {  // H done: its reads of Zu are over (C^T lands there)
    if (lane == 0) lds_signal(L.flag + 4);
  }
  stamp.mark(1);
  // ---- wave 0: Quu^-1 by the symmetric sweep (overlaps waves 1-3) ----------
  if constexpr (W == 0) {
    if constexpr (P.uwaves > 0) {  // wait for the other u-block owners' Quu rows
      const int target = P.uwaves * (D.T - t);
      lds_wait_ge(L.flag + 1, target);
    }
    if (boxk) {
      if (!box_gains_wave<MP, LDQ>(D, L, b, t, cur, lane) && lane == 0) *L.flag = 1;
    } else {
      // C = Lc^-1 into Qi (the gains as K = C^T (C Qxu^T), k = C^T (C Qu))
      // (C^T over Zu: written once every wave's H tiles have read Zu)
      const int htarget = Cfg::ct_own ? 0 : P.gwaves * (D.T - t);
      __builtin_amdgcn_s_setprio(3);  // the sweeps' latency chain is the knot's critical path
      bool bad;
      if constexpr (MP == 32)
        bad = chol_inv_blocked2<LDQ, Cfg::LDT>(Quu, Qi, L.Ct, L.rowbuf, mu, lane, L.flag + 4, htarget);
      else
        bad = chol_inv_sweep<MP, LDQ, Cfg::LDT>(Quu, Qi, L.Ct, L.rowbuf, mu, lane, L.flag + 4, htarget);
      __builtin_amdgcn_s_setprio(0);
      if (bad && lane == 0) *L.flag = 1;
    }
  }
  stamp.mark(2);
  // B1 (without the prefetch plan it also retires the fs DMA issued at the end of the
  // last knot; with it, the knot's DMA in flight stays in flight)
  if constexpr (pre)
    lds_barrier();
  else
    dma_barrier();
  stamp.mark(3);
  if (*L.flag) return false;
  // the next knot's operands: right after B1, except in the 8-wave plan with C^T over Zu
  // (after B2, once every C^T read is done)
  constexpr bool early_dma = NW <= 4 || Cfg::ct_own;
  // (with C^T over Zu: the Fx part now, the rest after B2)
  constexpr bool split_dma = !early_dma && !pre && NDX > 0;
  if constexpr (early_dma && !pre) issue_dma(3);
  if constexpr (split_dma) issue_dma(1);
  // ---- P2: K(:, i) = Quu^-1 Qxu(i, :)^T ; Vxx(i, j) = Qxx(i, j) - K(:, i)^T Qxu(j, :)^T
  f64x4 Kt[NA][MTL];
  double kst = 0.;   // wave 0: k(row) (lanes part == 0)
  double vfs[NA];    // Vxx fs (lanes q == 0 of the x blocks)
  // This knot's K, k and Vxx fs to HBM. With C^T in its own area (the small shapes) after
  // B3: their stores would otherwise hold B3's vmcnt wait, and they drain while the next
  // knot's G runs. The C5 shape stores them where they are formed (measured: deferring
  // costs its spilling kernel 3 %).
  constexpr bool defer = Cfg::ct_own;
  auto store_K = [&]() {
    double* Kg = D.K + rr * D.sNM;
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      const int i = P.blk[W][o];
      if (i < NTL) {
        const int C = 16 * i + c;
#pragma unroll
        for (int it = 0; it < MTL; ++it)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int R = 16 * it + q + 4 * r;
            if (R < m && C < n) Kg[(int64_t)C * m + R] = Kt[o][it][r];
          }
      }
    }
  };
  auto store_fs = [&]() {
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      const int C = 16 * P.blk[W][o] + c;
      if (P.blk[W][o] < NTL && !feas && q == 0 && C < n) D.Vxxfs[kk * D.sN + C] = vfs[o];
    }
  };
  auto store_k = [&]() {
    if constexpr (W == 0) {
      const int row = lane % MP, part = lane / MP;
      if (!boxk && part == 0 && row < m) D.k[rr * D.sM + row] = kst;
    }
  };
  {
    bool bad = false;
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      const int i = P.blk[W][o];
      if (i < NTL) {
#pragma unroll
        for (int it = 0; it < MTL; ++it) Kt[o][it] = f64x4{0., 0., 0., 0.};
#pragma unroll
        for (int s = 0; s < 4 * MTL; ++s) {
          const double bq = Qxu[(4 * s + q) * LDV + 16 * i + c];
#pragma unroll
          for (int it = 0; it < MTL; ++it) Kt[o][it] = mfma4(Qi[(4 * s + q) * LDQ + 16 * it + c], bq, Kt[o][it]);
        }
        if (!boxk) {
          // Kt holds W = C Qxu^T; K = C^T W: W's accumulator register s' holds rows
          // q + 4 s' of its 16-row tile, which is the B fragment of k-step s'. C is
          // lower triangular, so C^T's tile (it, kt) vanishes for kt < it: tile it of
          // K reads W's tiles kt >= it only, so it replaces W's tile it in place
          // (one extra tile of registers, not MTL)
#pragma unroll
          for (int it = 0; it < MTL; ++it) {
            f64x4 kn = f64x4{0., 0., 0., 0.};
#pragma unroll
            for (int kt = it; kt < MTL; ++kt)
#pragma unroll
              for (int s = 0; s < 4; ++s)
                kn = mfma4(L.Ct[(16 * kt + 4 * s + q) * Cfg::LDT + 16 * it + c], Kt[o][kt][s], kn);
            Kt[o][it] = kn;
          }
        }
      }
    }
    if constexpr (!defer) store_K();
    stamp.mark(4);
    // this wave's V tiles (i, j), i <= j: with K(:, i) when it owns block i
    // ("row" form, V(i, j) = Qxx(i, j) - K(:, i)^T Qxu(j, :)^T), else with
    // K(:, j) on the transposed tile V(j, i) = Qxx(i, j)^T - K(:, j)^T Qxu(i, :)^T
#pragma unroll
    for (int k3 = 0; k3 < P.ntile[W]; ++k3) {
      const int i = P.tile[W][k3][0], j = P.tile[W][k3][1];
      const int oi = P.slot(W, i);
      const bool rowf = oi >= 0;
      const int oa = rowf ? oi : P.slot(W, j);
      const int ra = rowf ? i : j, ca = rowf ? j : i;  // tile rows / cols of the result
      f64x4 acc;
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // Qxx(i, j) lives at V[R * LDV + C] (R in i, C in j)
        const double fvf = rowf ? V[(16 * i + q + 4 * r) * LDV + 16 * j + c] : V[(16 * i + c) * LDV + 16 * j + q + 4 * r];
        acc[r] = 0.5 * (Lv[k3][r][0] + Lv[k3][r][1]) + fvf;
      }
      const f64x4 qxx = acc;
#pragma unroll
      for (int s = 0; s < 4 * MTL; ++s)
        acc = mfma4(-Kt[oa < 0 ? 0 : oa][s >> 2][s & 3], Qxu[(4 * s + q) * LDV + 16 * ca + c], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int R = 16 * ra + q + 4 * r, C2 = 16 * ca + c;
        double v = acc[r];
        if (xr && R == C2 && R < n) v += xreg;
        if (ra != ca || R <= C2) {
          V[C2 * LDV + R] = v;
          V[R * LDV + C2] = v;
          if (R < n && C2 < n) bad |= bad_entry(v);
        }
      }
      if (D.dQxx) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int R = 16 * ra + q + 4 * r, C2 = 16 * ca + c;
          if (R < n && C2 < n) {
            D.dQxx[rr * D.sNN + (int64_t)C2 * n + R] = qxx[r];
            if (ra != ca) D.dQxx[rr * D.sNN + (int64_t)R * n + C2] = qxx[r];
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (W == 0) {  // k = Quu^-1 Qu (box knots: k = -x, set) ; Quuk = Quu k (64 / MP lanes per row)
      constexpr int LPR = 64 / MP;
      const int row = lane % MP, part = lane / MP;
      double a0 = 0., a1 = 0.;
      if (!boxk) {
        // y = C Qu (into kv), then k = C^T y
        for (int k2 = part; k2 < mu; k2 += 2 * LPR) {
          a0 = fma(Qi[k2 * LDQ + row], L.qu[k2], a0);
          if (k2 + LPR < mu) a1 = fma(Qi[(k2 + LPR) * LDQ + row], L.qu[k2 + LPR], a1);
        }
        double a = a0 + a1;
#pragma unroll
        for (int o2 = MP; o2 < 64; o2 <<= 1) a += __shfl_xor(a, o2, 64);
        if (part == 0) L.kv[row] = row < mu ? a : 0.;
        asm volatile("" ::: "memory");
        a0 = 0.;
        a1 = 0.;
        for (int k2 = part; k2 < mu; k2 += 2 * LPR) {
          a0 = fma(L.Ct[k2 * Cfg::LDT + row], L.kv[k2], a0);
          if (k2 + LPR < mu) a1 = fma(L.Ct[(k2 + LPR) * Cfg::LDT + row], L.kv[k2 + LPR], a1);
        }
        a = a0 + a1;
#pragma unroll
        for (int o2 = MP; o2 < 64; o2 <<= 1) a += __shfl_xor(a, o2, 64);
        asm volatile("" ::: "memory");
        if (part == 0) {
          if (row >= mu) a = 0.;
          L.kv[row] = a;
          kst = a;
        }
        if constexpr (!defer) store_k();
      }
      asm volatile("" ::: "memory");
      double a;
      a0 = 0.;
      a1 = 0.;
      for (int k2 = part; k2 < mu; k2 += 2 * LPR) {
        a0 = fma(Quu[k2 * LDQ + row], L.kv[k2], a0);
        if (k2 + LPR < mu) a1 = fma(Quu[(k2 + LPR) * LDQ + row], L.kv[k2 + LPR], a1);
      }
      a = a0 + a1;
#pragma unroll
      for (int o2 = MP; o2 < 64; o2 <<= 1) a += __shfl_xor(a, o2, 64);
      if (part == 0) L.quuk[row] = row < mu ? a : 0.;
    }
    if (bad) *L.flag = 1;
  }
  stamp.mark(5);
  // B2 (partial, LDS counter): P3 (the x-block owners) needs every V tile
  // and wave 0's Quu k; the other waves only signal (when they produced
  // something) and go on issuing the DMA.
  if constexpr (W == 0 || P.owns_x(W)) {
    if (lane == 0) lds_signal(L.flag + 3);
  }
  // With C^T over Zu (!ct_own) the next knot's LDS-DMA into Zu must also wait for every
  // C^T read (the K products of the x-block owners, wave 0's k): the waves that only
  // signal would otherwise issue it while those still run (a race seen as 1 in 256 solves
  // differing between trial-group sizes)
  if constexpr (P.owns_x(W) || (!Cfg::ct_own && NW == 8)) {
    const int target = (P.xwaves + (P.owns_x(0) ? 0 : 1)) * (D.T - t);
    lds_wait_ge(L.flag + 3, target);
  }
  if constexpr (!early_dma) issue_dma(split_dma ? 2 : 3);
  // ---- P3: Vx = Qx + K^T Quuk - 2 K^T Qu (+ Vxx fs), reduction terms -------
  {
    const double* fsv = fsb;
    bool bad = false;
    double pv[5] = {0., 0., 0., 0., 0.};
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      if constexpr (defer) vfs[o] = 0.;
      const int i = P.blk[W][o];
      if (i < NTL) {
        const int R = 16 * i + c;
        double a = 0., c2 = 0., f = 0.;
#pragma unroll
        for (int it = 0; it < MTL; ++it)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int k2 = 16 * it + 4 * r + q;
            a += Kt[o][it][r] * L.quuk[k2];
            c2 += Kt[o][it][r] * L.qu[k2];
          }
        if (!feas) {
          double f0 = 0., f1 = 0., f2 = 0., f3 = 0.;
          int j = q;
          for (; j + 12 < n; j += 16) {
            f0 = fma(V[j * LDV + R], fsv[j], f0);
            f1 = fma(V[(j + 4) * LDV + R], fsv[j + 4], f1);
            f2 = fma(V[(j + 8) * LDV + R], fsv[j + 8], f2);
            f3 = fma(V[(j + 12) * LDV + R], fsv[j + 12], f3);
          }
          for (; j < n; j += 4) f0 = fma(V[j * LDV + R], fsv[j], f0);
          f = (f0 + f1) + (f2 + f3);
        }
        a += __shfl_xor(a, 16, 64);
        a += __shfl_xor(a, 32, 64);
        c2 += __shfl_xor(c2, 16, 64);
        c2 += __shfl_xor(c2, 32, 64);
        f += __shfl_xor(f, 16, 64);
        f += __shfl_xor(f, 32, 64);
        if (q == 0) {
          double v = 0.;
          if (R < n) {
            v = ur ? (L.qx[R] + a) - 2 * c2 : L.qx[R] - c2;
            if (!feas) {
              if constexpr (defer)
                vfs[o] = f;
              else
                D.Vxxfs[kk * D.sN + R] = f;
              v += f;
              pv[2] += v * fsv[R];
              pv[3] += fsv[R] * f;
            }
            bad |= bad_entry(v);
          }
          L.vx[R] = v;
        }
      }
    }
    if constexpr (W == 0) {
      if (lane < m) {
        pv[0] = L.qu[lane] * L.kv[lane];
        pv[1] = L.kv[lane] * L.quuk[lane];
        pv[4] = L.qu[lane] * L.qu[lane];
      }
    }
    // the expected-improvement / stopping terms. Small shapes: per-lane running sums over
    // the knots, reduced over the workgroup once at the end of the sweep; the C5 shape
    // (its kernel at the register cap): per-knot wave sums into D.part
    if constexpr (defer) {
#pragma unroll
      for (int j = 0; j < 5; ++j) red5[j] += pv[j];
    } else {
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        const double s = wave_sum(pv[j]);
        if (lane == 0) L.red[j * NW + W] = s;
      }
    }
    if (bad) *L.flag = 1;
  }
  stamp.mark(6);
  dma_barrier();  // B3: knot t-1 operands resident
  // fs of knot t-1 (read in its P3; landed by the vmcnt(0) of its B1)
  if constexpr (P.dmarank[W] >= 0 && !pre) {
    if (t > 0) dma_vec<P.ndma>(L.fsb, D.fs + (kk - 1) * D.sN, n, P.dmarank[W], lane);
  }
  if constexpr (defer) {
    store_K();
    store_fs();
    store_k();
  }
  return true;
}

template <int NTL, int MTL, int NW>
__device__ __forceinline__ bool bwd_sweep_mfma(const Dev& D, int b, bool feas, double xreg, double ureg, int cur,
                                               double* sm, double (&ei)[3]) {
  double red5[5] = {0., 0., 0., 0., 0.};  // running sums (C^T in its own area: the small shapes)
  using Cfg = MfmaCfg<NTL, MTL>;
  constexpr int NP = Cfg::NP, MP = Cfg::MP, LDV = Cfg::LDV, LDQ = Cfg::LDQ;
  constexpr int NT = NW * 64;
  const int n = D.n, m = D.m, T = D.T, tid = threadIdx.x;
  const int wid = tid >> 6, lane = tid & 63;
  BwdLds L;
  L.V = sm + Cfg::oV;
  L.Qxu = sm + Cfg::oQxu;
  L.Quu = sm + Cfg::oQuu;
  L.Qi = sm + Cfg::oQi;
  L.vx = sm + Cfg::oVx;
  L.qx = sm + Cfg::oQx;
  L.lxv = sm + Cfg::oLx;
  L.fsb = sm + Cfg::oFs;
  L.qu = sm + Cfg::oQu;
  L.luv = sm + Cfg::oLu;
  L.kv = sm + Cfg::oKv;
  L.quuk = sm + Cfg::oQuuk;
  L.rowbuf = sm + Cfg::oKv;
  L.red = sm + Cfg::oRed;
  L.flag = (int*)(sm + Cfg::oFlag);
  L.Zx = sm + Cfg::oZx;
  L.Zu = sm + Cfg::oZu;
  L.Ct = sm + Cfg::oCt;
  constexpr bool pre = BwdPlan<NTL, MTL, NW>{}.prefetch;
  L.Zx2 = pre ? sm + Cfg::oZx2 : L.Zx;
  L.Zu2 = pre ? sm + Cfg::oZu2 : L.Zu;
  L.lxv2 = pre ? sm + Cfg::oLx2 : L.lxv;
  L.luv2 = pre ? sm + Cfg::oLu2 : L.luv;
  L.fsb2 = pre ? sm + Cfg::oFs2 : L.fsb;
  L.cb0 = sm + Cfg::oCb;
  L.cb1 = sm + Cfg::oCb + Cfg::CB;
  static_assert(Cfg::ct_own || NW == 8, "C^T over Zu needs the 8-wave plan's late LDS-DMA");
  double* V = L.V;
  const bool xr = !isnan(xreg);
  Stamp stamp(D.stamps ? D.stamps + ((int64_t)b * 8 + wid) * 8 : nullptr);

  if (tid == 0) {
    L.flag[0] = 0;
    L.flag[1] = 0;  // Quu-ready counter (8-wave plan)
    L.flag[2] = 0;  // G-done counter (partial B0)
    L.flag[3] = 0;  // P2-done counter (partial B2)
    L.flag[4] = 0;  // H-done counter (C^T over Zu)
  }
  // ---- terminal: Vxx = Lxx_T (+ xreg I), Vx = Lx_T (+ Vxx fs_T) ------------
  {
    const int64_t kk = D.knot(b, T);
    const double* Lxx = D.Lxx + kk * D.sNN;
    const double* Lx = D.Lx + kk * D.sN;
    const double* fs = D.fs + kk * D.sN;
    double* fsv = L.fsb;
    // stored transposed so that G = V Z uses Lxx_T itself (it may be asymmetric)
    for (int e = tid; e < NP * NP; e += NT) {
      const int i = e % NP, j = e / NP;
      double v = (i < n && j < n) ? Lxx[(int64_t)i * n + j] : 0.;
      if (xr && i == j && i < n) v += xreg;
      V[j * LDV + i] = v;
    }
    for (int i = tid; i < NP; i += NT) fsv[i] = i < n ? fs[i] : 0.;
    // zero the padding of the per-knot vector buffers once (DMA fills [0, n))
    // (and of Z: rows >= n, columns >= n / m are never written by the DMA)
    for (int i = tid; i < NP; i += NT) L.lxv[i] = 0.;
    for (int i = tid; i < MP; i += NT) L.luv[i] = 0.;
    for (int e = tid; e < (NP + MP) * Cfg::ZLD + 2; e += NT) L.Zx[e] = 0.;
    if constexpr (pre) {  // the second buffers: Z, lx, lu, fs (contiguous)
      for (int e = tid; e < (NP + MP) * Cfg::ZLD + 2 + 2 * NP + MP; e += NT) L.Zx2[e] = 0.;
    }
    __syncthreads();
    double pv[2] = {0., 0.};
    for (int i = tid; i < NP; i += NT) {
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
      L.vx[i] = v;
    }
    if constexpr (Cfg::ct_own) {
      red5[2] += pv[0];
      red5[3] += pv[1];
    } else {
      wg_sums<NT, 2>(pv, L.red);
      if (tid == 0) {
        double* p = D.part + kk * 8;
        p[0] = 0.; p[1] = 0.; p[2] = pv[0]; p[3] = pv[1]; p[4] = 0.;
      }
    }
    if (D.dVxx) {
      for (int e = tid; e < n * n; e += NT) {
        const int i = e % n, j = e / n;
        D.dVxx[kk * D.sNN + e] = Lxx[e] + ((xr && i == j) ? xreg : 0.);
      }
      for (int i = tid; i < n; i += NT) D.dVx[kk * D.sN + i] = L.vx[i];
    }
    __syncthreads();
    if (T > 0) {  // operands of knot T-1 (prefetch plan: into the buffers of its parity)
      const int64_t k1 = kk - 1;
      const bool o1 = pre && ((T - 1) & 1);
      dma_cols<NW>(o1 ? L.Zx2 : L.Zx, Cfg::ZLD, D.Fx + k1 * D.sNN, n, n, wid, lane);
      dma_cols<NW>(o1 ? L.Zu2 : L.Zu, Cfg::ZLD, D.Fu + k1 * D.sNM, n, m, wid, lane);
      dma_vec<NW>(o1 ? L.lxv2 : L.lxv, D.Lx + k1 * D.sN, n, wid, lane);
      dma_vec<NW>(o1 ? L.luv2 : L.luv, D.Lu + k1 * D.sM, m, wid, lane);
      dma_vec<NW>(o1 ? L.fsb2 : L.fsb, D.fs + k1 * D.sN, n, wid, lane);
      if constexpr (pre) {
        double* const cb = o1 ? L.cb1 : L.cb0;
        dma_vec<NW>(cb, D.Lxx + k1 * D.sNN, n * n, wid, lane);
        dma_vec<NW>(cb + n * n + (n * n & 1), D.Lxu + k1 * D.sNM, n * m, wid, lane);
        dma_vec<NW>(cb + n * n + (n * n & 1) + n * m + (n * m & 1), D.Luu + k1 * D.sMM, m * m, wid, lane);
      }
    }
    dma_barrier();
  }

  for (int t = T - 1; t >= 0; --t) {
    const int64_t kk = D.knot(b, t);
    const int64_t rr = D.run(b, t);
    stamp.mark(7);
    bool ok = false;
    switch (wid) {
      case 0: ok = bwd_knot<NTL, MTL, NW, 0>(D, L, b, t, feas, xreg, ureg, cur, stamp, red5); break;
      case 1: ok = bwd_knot<NTL, MTL, NW, 1>(D, L, b, t, feas, xreg, ureg, cur, stamp, red5); break;
      case 2: ok = bwd_knot<NTL, MTL, NW, 2>(D, L, b, t, feas, xreg, ureg, cur, stamp, red5); break;
      case 3: ok = bwd_knot<NTL, MTL, NW, 3>(D, L, b, t, feas, xreg, ureg, cur, stamp, red5); break;
      case 4: if constexpr (NW > 4) ok = bwd_knot<NTL, MTL, NW, 4>(D, L, b, t, feas, xreg, ureg, cur, stamp, red5); break;
      case 5: if constexpr (NW > 4) ok = bwd_knot<NTL, MTL, NW, 5>(D, L, b, t, feas, xreg, ureg, cur, stamp, red5); break;
      case 6: if constexpr (NW > 4) ok = bwd_knot<NTL, MTL, NW, 6>(D, L, b, t, feas, xreg, ureg, cur, stamp, red5); break;
      default: if constexpr (NW > 4) ok = bwd_knot<NTL, MTL, NW, 7>(D, L, b, t, feas, xreg, ureg, cur, stamp, red5); break;
    }
    if (!ok) {  // the factorisation failed (every wave saw the flag)
      stamp.flush();
      return false;
    }
    if constexpr (!Cfg::ct_own) {
      if (tid == 0) {
        double* p = D.part + kk * 8;
        const double* red = L.red;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          double a = 0.;
          for (int w = 0; w < NW; ++w) a += red[j * NW + w];
          p[j] = a;
        }
      }
    }
    if (D.dQxx) {
      for (int e = tid; e < n * n; e += NT) D.dVxx[kk * D.sNN + e] = V[(e / n) * LDV + e % n];
      for (int e = tid; e < n * m; e += NT) D.dQxu[rr * D.sNM + e] = L.Qxu[(e / n) * LDV + e % n];
      for (int e = tid; e < m * m; e += NT) D.dQuu[rr * D.sMM + e] = L.Quu[(e / m) * LDQ + e % m];
      for (int i = tid; i < n; i += NT) {
        D.dQx[rr * D.sN + i] = L.qx[i];
        D.dVx[kk * D.sN + i] = L.vx[i];
      }
      for (int i = tid; i < m; i += NT) D.dQu[rr * D.sM + i] = L.qu[i];
      __syncthreads();
    }
    if (*L.flag) {
      stamp.flush();
      return false;
    }
  }
  stamp.flush();
  // updateExpectedImprovement / stoppingCriteria (fddp.cpp:126-146, ddp.cpp:132-142):
  // ei = {dg, dq, stop}, in thread 0
  if constexpr (Cfg::ct_own) {  // the running sums over the workgroup
    wg_sums<NT, 5>(red5, L.red);
    ei[0] = feas ? red5[0] : red5[0] - red5[2];
    ei[1] = feas ? -red5[1] : red5[3] - red5[1];
    ei[2] = red5[4];
  }  // (else: the per-knot sums in D.part, summed by the kernel's epilogue)
  return true;
}

// LDS bytes of a plan: the prefetch plan's second buffers only where the plan uses them
// (a four-wave plan with every wave owning blocks keeps the smaller carve, so two of its
// workgroups fit a CU)
template <int NTL, int MTL, int NW>
constexpr size_t bwd_lds_bytes() {
  using Cfg = MfmaCfg<NTL, MTL>;
  return BwdPlan<NTL, MTL, NW>{}.prefetch ? Cfg::bytes
                                          : sizeof(double) * (Cfg::ct_own ? Cfg::total0 + Cfg::MP * Cfg::LDT : Cfg::total0);
}

// (the four-wave plans at two waves per SIMD: two workgroups per CU, which is what the
// residency-based plan choice counts on)
template <int NTL, int MTL, int NW>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(NW == 4 ? 2 : 1))) void backward_mfma_kernel(
    Dev D, Prm prm, int mode) {
  const int b = blockIdx.x;
  ElemState* st = D.st + b;
  if (mode == 0 && !st->active) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const bool feas = st->is_feasible != 0;
  double xreg = st->xreg, ureg = st->ureg;
  bool ok;
  int tries = 0;
  const int max_tries = reg_retry_bound(prm, xreg);
  double ei[3];  // dg, dq, stop (thread 0)
  for (;;) {
    ok = bwd_sweep_mfma<NTL, MTL, NW>(D, b, feas, xreg, ureg, st->cur, sm, ei);
    __syncthreads();
    if (ok || mode == 1) break;
    xreg *= prm.regfactor;  // increaseRegularization (ddp.cpp:312-318)
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
    if (!ok && mode == 0) {
      st->status = FDDP_STATUS_REGMAX;
      st->active = 0;
      st->n_iter_run += 1;
    }
    if (ok) {
      if constexpr (!MfmaCfg<NTL, MTL>::ct_own) {  // the per-knot sums, in knot order
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
        ei[0] = dg;
        ei[1] = dq;
        ei[2] = stop;
      }
      st->dg = ei[0];
      st->dq = ei[1];
      st->stop = ei[2];
    }
  }
}

}  // namespace fddp
