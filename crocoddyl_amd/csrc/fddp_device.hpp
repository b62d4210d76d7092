// Device-side data layout, per-element solver state and workgroup helpers
// shared by the libfddp_hip kernels (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fddp_hip.h"

namespace fddp {

// Multibody knots (variable-size blocks, multibody.hpp): free and contact dynamics.
__host__ __device__ inline bool is_mb_kind(int kind) {
  return kind == FDDP_KNOT_EULER_FREEFWD || kind == FDDP_KNOT_EULER_CONTACTFWD || kind == FDDP_KNOT_IMPULSEFWD;
}

constexpr int kWave = 64;

// Per-element FDDP state machine (SolverAbstract/SolverDDP/SolverFDDP members,
// solver-base.hpp:230-276, ddp.hpp:270-306, fddp.hpp:95-101).
struct ElemState {
  double cost;        // cost_
  double cost_try;    // cost_try_
  double stop;        // stop_
  double xreg, ureg;  // xreg_, ureg_
  double steplength;  // steplength_
  double dV, dVexp;   // dV_, dVexp_
  double dg, dq, dv;  // dg_, dq_, dv_
  double d0, d1;      // d_
  int32_t is_feasible, was_feasible;
  int32_t recalc;      // recalcDiff
  int32_t iter;        // iter_
  int32_t status;      // FDDP_STATUS_*
  int32_t active;      // still iterating inside fddp_solve
  int32_t cur;         // which of the two trajectory buffers holds xs_/us_
  int32_t n_iter_run;  // loop bodies executed
  int32_t bwd_fail;    // last backward pass raised backward_error
  int32_t fwd_fail;    // last trial raised forward_error
};

static_assert(sizeof(ElemState) % 8 == 0, "ElemState alignment");


__host__ __device__ inline int64_t pad2(int64_t v) { return (v + 1) & ~int64_t(1); }

// A pointer known to address LDS: the assumption lets the address-space inference
// compile accesses through it to ds_* instructions even where the compiler cannot
// trace it back to the kernel's __shared__ array (a pointer that is LDS on one path
// and global on another is otherwise accessed with flat instructions).
template <class T>
__device__ __forceinline__ T* lds_ptr(T* p) {
  __builtin_assume(__builtin_amdgcn_is_shared((const __attribute__((address_space(0))) void*)(p)));
  return p;
}

// ---- LDS progress counters between the waves of a workgroup ------------------------
// For data exchanged through LDS only: the fences order LDS accesses alone (an LDS-only
// s_waitcnt lgkmcnt(0)). A generic workgroup release would also wait for every vector
// memory operation in flight (vmcnt(0)): the backward sweep's LDS-DMA of the next knot's
// operands, which the counters are meant to overlap. Data in global memory needs the
// generic fences instead (multibody.hpp tree_side_barrier).
__device__ __forceinline__ void lds_signal(int* ctr) {  // after this wave's LDS writes / reads
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_publish(int* ctr, int v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __hip_atomic_store(ctr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_wait_ge(int* ctr, int target) {  // before the LDS accesses it guards
#ifdef FDDP_SPIN_POLL  // diagnostic build (make spin): busy polls, no s_sleep between them
  while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
  }
#else
  while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
#endif
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

typedef __attribute__((address_space(3))) void* lds_void_ptr;

// Barrier that waits only for this wave's LDS traffic: an LDS-DMA in flight
// stays in flight across it (a __syncthreads() would add vmcnt(0)).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// Barrier after which every LDS-DMA issued by the workgroup has landed.
__device__ __forceinline__ void dma_barrier() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Asynchronous copy global -> LDS by LDS-DMA (global_load_lds: the LDS
// destination of one wave instruction is a wave-uniform base + lane * size).
// dma_vec: nd contiguous doubles (16-B aligned both sides) over the 4 waves;
// an odd tail double moves as two 4-byte DMAs.
template <int NW>  // NW participating waves, wid = this wave's rank among them
__device__ __forceinline__ void dma_vec(double* lds, const double* g, int nd, int wid, int lane) {
  const int nch = nd >> 1;
  for (int base = wid * 64; base < nch; base += NW * 64) {
    const int ch = base + lane;
    if (ch < nch) __builtin_amdgcn_global_load_lds(g + 2 * ch, (lds_void_ptr)(lds + 2 * base), 16, 0, 0);
  }
  if ((nd & 1) && wid == NW - 1 && lane < 2)
    __builtin_amdgcn_global_load_lds((const char*)(g + nd - 1) + 4 * lane, (lds_void_ptr)(lds + nd - 1), 4, 0, 0);
}
// Diagnostic phase timer (built with -DFDDP_STAMPS_BUILD, enabled by
// FDDP_STAMPS=1): per wave, core cycles spent per phase, accumulated in
// registers (a global read-modify-write per mark would drain the LDS-DMA in
// flight) and flushed at the end of the sweep. Compiled out otherwise.
struct Stamp {
#ifdef FDDP_STAMPS_BUILD
  unsigned long long* out;
  unsigned long long t0;
  unsigned long long acc[8];
  __device__ Stamp(unsigned long long* o) : out(o), t0(__builtin_amdgcn_s_memtime()), acc{} {}
  __device__ __forceinline__ void mark(int ph) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    acc[ph] += t - t0;
    t0 = t;
  }
  __device__ __forceinline__ void flush() {
    if (out && (threadIdx.x & 63) == 0)
      for (int i = 0; i < 8; ++i) out[i] += acc[i];
  }
#else
  __device__ Stamp(unsigned long long*) {}
  __device__ __forceinline__ void mark(int) {}
  __device__ __forceinline__ void flush() {}
#endif
};

// ---- register broadcasts within a wave (64 lanes = 4 rows of 16) -------------------
// lane n of every row of 16 lanes, to the whole row (DPP row_newbcast: a VALU move, no
// LDS-crossbar round trip as __shfl's ds_bpermute); n a compile-time constant
template <int N>
__device__ __forceinline__ double row_bcast_d(double v) {
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)bits, 0x150 + N, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(bits >> 32), 0x150 + N, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int I = 0>
__device__ __forceinline__ double row_bcast_d(double v, int n) {  // n in [I, 16), unrolled
  if constexpr (I < 15) {
    if (n != I) return row_bcast_d<I + 1>(v, n);
  }
  return row_bcast_d<I>(v);
}
// row r (lanes 16 r .. 16 r + 15) of a wave to all four rows, lane for lane (= __shfl(v,
// (lane & 15) + 16 r)) by two permlane swaps per half (gfx950 v_permlane16/32_swap: odd
// rows of the first operand with even rows of the second; upper 32 lanes of the first
// with lower 32 of the second)
template <int R>
__device__ __forceinline__ int row_to_all_i(int h) {
  const auto a = __builtin_amdgcn_permlane16_swap(h, h, false, false);  // rows [0,0,2,2] | [1,1,3,3]
  const int t = (R & 1) ? a[1] : a[0];
  const auto c = __builtin_amdgcn_permlane32_swap(t, t, false, false);  // [t0,t1,t0,t1] | [t2,t3,t2,t3]
  return (R & 2) ? c[1] : c[0];
}
template <int R>
__device__ __forceinline__ double row_to_all_d(double v) {
  const long long bits = __double_as_longlong(v);
  const int lo = row_to_all_i<R>((int)bits), hi = row_to_all_i<R>((int)(bits >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int I = 0>
__device__ __forceinline__ double row_to_all_d(double v, int r) {  // r in [I, 4), unrolled
  if constexpr (I < 3) {
    if (r != I) return row_to_all_d<I + 1>(v, r);
  }
  return row_to_all_d<I>(v);
}
// lane l's value to every lane (v_readlane, a scalar)
__device__ __forceinline__ double lane_read_d(double v, int l) {
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)bits, l);
  const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// fddp_boxqp_params on the device (BoxQP, box-qp.hpp:92-93)
struct BoxQPCfg {
  int maxiter, n_alphas;
  double th_acceptstep, th_grad, reg;
  double alphas[16];
};

// All device buffers of one handle. Every per-knot array is [b][t][...] with
// the per-knot stride padded to an even number of doubles (16-B aligned rows).
struct Dev {
  int nx, n, m, T, B;  // n = ndx, m = nu_max
  int64_t sX, sN, sM, sNN, sNM, sMM;
  const fddp_knot_desc* knots;  // T+1
  const double* params;
  double* x0;                // [B][sX]
  double* xs[2];             // [B][T+1][sX]
  double* us[2];             // [B][T][sM]
  double* xnext[2];          // [B][T][sX]   data[t].xnext of that trajectory
  double* kcost[2];          // [B][T+1]     data[t].cost of that trajectory
  double *Fx, *Fu, *Lxx, *Lxu, *Luu, *Lx, *Lu;  // [B][T+1][...]
  double* fs;                // [B][T+1][sN]
  double* K;                 // [B][T][sNM]  (nu x ndx, ld = m)
  double* k;                 // [B][T][sM]
  double* Vxxfs;             // [B][T+1][sN] Vxx[t] * fs[t]
  double* part;              // [B][T+1][8]  per-knot reduction terms
  double* dvp;               // [B][T+1]     per-knot expectedImprovement terms
  // debug per-knot stores (null unless fddp_set_debug)
  double *dVxx, *dVx, *dQxx, *dQxu, *dQuu, *dQx, *dQu;
  ElemState* st;             // [B]
  double* bwork;             // generic sweep's global workspace when LDS is too small (else null)
  double* zero16;            // 16 zero bytes: source of the LDS-DMA gap fill
  const int* segend;         // [T+1] end of the run of knots from t sharing desc + parameter block
  unsigned long long* stamps;  // diagnostic: [B][4 waves][8 phases] cycles (null = off)
  // SolverBoxFDDP (box-fddp.cpp:15-160): box QP gains on limited knots once
  // feasible, clamped controls in the forward pass
  int box;                         // solver kind == FDDP_SOLVER_BOXFDDP
  const double *ulb, *uub;         // [B][T][sM] control limits (null = none set)
  const unsigned char* haslim;     // [B][T] has_control_limits (null = none)
  double* dQuuInv;                 // debug [B][T][sMM] Quu_inv_ (null unless debug + box)
  unsigned long long* box_stats;   // diagnostics (FDDP_BOX_STATS=1): box QPs, Newton iterations, inverses
  BoxQPCfg boxcfg;                 // qp_(nu, 100, 0.1, 1e-5, 0.) (box-fddp.cpp:16)
  int64_t mbw;                     // LDS doubles of the multibody calc scratch (0: no multibody knots)
  int64_t mbw_fwd;                 // ... of the forward kernels' calc (mb::calc_dense_doubles)
  int dxv_mbw;                     // forward kernels: dx (2 sN) in the tail of that scratch (dead during the calc)
  int64_t mbd;                     // LDS doubles of the multibody calcDiff work area (its parameter block follows)
  int mbspill;                     // its plan's spill flags (multibody.hpp diff_spill)
  // parallel line search (generic trials): npar trials of one element run in
  // npar workgroups; trial slot 0 writes the other trajectory buffer, slots
  // 1..npar-1 their own copies (same [b][t] layout), accepted ones are copied back
  int npar;                        // trials per element evaluated together (1: serial line search)
  const int* ls_order;             // [B] rollout workgroup -> element (longest line search first), or null
  double *pxs, *pus, *pxnext, *pkcost, *pdvp;  // slots 1..npar-1: [slot][B][T+1|T][...]
  double* ptrial;                  // [B][npar][4]: ok, cost_try, dv, -
  int* ls_done;                    // [B] line search decided in an earlier group of this iteration
  __device__ bool box_knot(int b, int t) const { return box && haslim && haslim[(int64_t)b * T + t]; }

  __device__ __host__ int64_t knot(int b, int t) const { return (int64_t)b * (T + 1) + t; }
  __device__ __host__ int64_t run(int b, int t) const { return (int64_t)b * T + t; }
  __device__ __host__ const double* pblock(int b, int t) const {
    return params + knots[t].param_offset + (int64_t)b * knots[t].param_stride;
  }
};

// Solver thresholds (fddp_params) passed by value.
struct Prm {
  double th_acceptstep, th_stop, th_grad, th_stepdec, th_stepinc, th_acceptnegstep;
  double regfactor, regmin, regmax;
  int n_alphas;
  double alphas[16];
};

// Bound on the backward kernels' regularisation retries within one sweep. The reference
// retries until xreg reaches regmax (fddp.cpp:35-47): from a positive xreg that is
// ceil(log(regmax / xreg) / log(regfactor)) increases (set_regfactor rejects <= 1); two
// more absorb the rounding of the products. A zero / NaN xreg never reaches regmax (the
// reference would not stop): one try, then the element stops at regmax.
__host__ __device__ inline int reg_retry_bound(const Prm& prm, double xreg) {
  if (!(xreg > 0.) || !(prm.regfactor > 1.) || !(xreg < prm.regmax)) return 1;
  const double k = ceil(log(prm.regmax / xreg) / log(prm.regfactor));
  return k < 1e6 ? (int)k + 2 : 1000000;
}

// Which batch elements a launch works on (host-side selectors).
enum Sel { SEL_ACTIVE = 0, SEL_ALL = 1, SEL_ITER0 = 2, SEL_RECALC = 3 };

__device__ inline bool selected(const ElemState& s, int sel) {
  switch (sel) {
    case SEL_ACTIVE: return s.active != 0;
    case SEL_ALL: return true;
    case SEL_ITER0: return s.iter == 0;
    default: return s.active != 0 && s.recalc != 0;
  }
}

// Knot descriptors and segment ends through the constant address space:
// scalar loads (lgkmcnt), which do not queue behind the global stores in
// flight the way vector loads do (loads and stores share vmcnt, in order).
__device__ __forceinline__ fddp_knot_desc knot_desc_s(const Dev& D, int t) {
  typedef __attribute__((address_space(4))) const fddp_knot_desc* cptr;
  const cptr p = (cptr)D.knots + t;
  fddp_knot_desc k;
  k.kind = p->kind;
  k.nu = p->nu;
  k.param_offset = p->param_offset;
  k.param_stride = p->param_stride;
  return k;
}
// A parameter-pool double through the constant address space (the pool does not change
// during a kernel): a scalar load
__device__ __forceinline__ double param_s(const double* p) {
  typedef __attribute__((address_space(4))) const double* cptr;
  return *(cptr)p;
}

// raiseIfNaN — src/core/solver-base.cpp:175-181
__device__ inline bool raise_if_nan(double v) { return isnan(v) || isinf(v) || v >= 1e30; }
// |x| value that trips raiseIfNaN(lpNorm<Infinity>) for an element of a vector
__device__ inline bool bad_entry(double v) {
  const double a = fabs(v);
  return isnan(a) || isinf(a) || a >= 1e30;
}

// ---------------------------------------------------------------------------
// Workgroup reductions (wave64 shuffles + LDS).
// ---------------------------------------------------------------------------
__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Sum of v over the workgroup; `red` is LDS scratch of >= 2*nwaves doubles.
// Ends with every thread holding the total; contains two barriers.
template <int NT>
__device__ inline double wg_sum(double v, double* red) {
  constexpr int NW = NT / kWave;
  v = wave_sum(v);
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.;
#pragma unroll
  for (int i = 0; i < NW; ++i) s += red[i];
  __syncthreads();
  return s;
}

// Several sums at once (same structure; red >= NV*NW doubles).
template <int NT, int NV>
__device__ inline void wg_sums(double (&v)[NV], double* red) {
  constexpr int NW = NT / kWave;
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    double x = wave_sum(v[j]);
    if (lane == 0) red[j * NW + w] = x;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    double s = 0.;
#pragma unroll
    for (int i = 0; i < NW; ++i) s += red[j * NW + i];
    v[j] = s;
  }
  __syncthreads();
}

// OR of a predicate over the workgroup.
__device__ inline bool wg_any(bool p, int* flag) {
  if (threadIdx.x == 0) *flag = 0;
  __syncthreads();
  if (p) *flag = 1;
  __syncthreads();
  const bool r = *flag != 0;
  __syncthreads();
  return r;
}

}  // namespace fddp
