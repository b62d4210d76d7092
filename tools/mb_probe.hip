// Diagnostic (not product): per-phase cycle breakdown of the multibody knot
// calcDiff / calc (crocoddyl_amd/csrc/multibody.hpp) on one packed block.
// Usage: mb_probe <input.bin> <nwg>  (input from tools/mb_probe.py).
// Every executor phase (run / run_w0 / sync) is stamped with s_memtime by
// thread 0 of workgroup 0; nwg workgroups run concurrently (load as in the
// knot-parallel kernel).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
// stamps inside the blocked Gauss-Jordan (multibody.hpp gj_mfma), thread 0 of workgroup 0
__device__ unsigned long long g_gjst[32];
// phase labels (first stamped launch only): the source location of each phase's lambda,
// cut from the executor method's __PRETTY_FUNCTION__ ("... (lambda at FILE:LINE:COL) ...")
constexpr int kLabelLen = 48;
__device__ char g_labels[256][kLabelLen];
__device__ int g_label_on;
#define MB_GJ_MARK(id)                                                            \
  do {                                                                            \
    if (threadIdx.x == 0 && blockIdx.x == 0) g_gjst[id] = __builtin_amdgcn_s_memtime(); \
  } while (0)
// LDS matrices of the calcDiff of workgroup 0 (multibody.hpp MB_DUMP), column-major
// rows x cols per slot; the first launch fills them
constexpr int kDumpSlots = 12, kDumpCap = 4096;
__device__ double g_dump[kDumpSlots][kDumpCap];
__device__ int g_dump_shape[kDumpSlots][2];
#define MB_DUMP(slot, ptr, rows, cols, ld)                                                  \
  do {                                                                                      \
    __syncthreads();                                                                        \
    if (blockIdx.x == 0) {                                                                  \
      const double* p_ = (const double*)(ptr);                                              \
      const int r_ = (rows), c_ = (cols), l_ = (ld);                                        \
      for (int e_ = threadIdx.x; e_ < r_ * c_ && e_ < kDumpCap; e_ += blockDim.x)            \
        g_dump[slot][e_] = p_[(e_ / r_) * l_ + e_ % r_];                                    \
      if (threadIdx.x == 0) {                                                               \
        g_dump_shape[slot][0] = r_;                                                         \
        g_dump_shape[slot][1] = c_;                                                         \
      }                                                                                     \
    }                                                                                       \
    __syncthreads();                                                                        \
  } while (0)
#include "../crocoddyl_amd/csrc/multibody.hpp"

using namespace fddp::mb;
using fddp::pad2;

struct StampExec {
  int nt;
  unsigned long long* st;  // LDS: [0] = count, then stamps
  template <class F>
  __device__ __forceinline__ void run(F f) const {
    [[clang::always_inline]] f((int)threadIdx.x);
    __syncthreads();
    mark(__PRETTY_FUNCTION__);
  }
  template <class F>
  __device__ __forceinline__ void run_w0(F f) const {
    if (threadIdx.x < 64) {
      [[clang::always_inline]] f((int)threadIdx.x);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (threadIdx.x == 0) {
      unsigned long long i = st[0]++;
      if (i < 254) st[2 + i] = __builtin_amdgcn_s_memtime() | (1ull << 63);
      label(i, __PRETTY_FUNCTION__);
    }
  }
  __device__ __forceinline__ void sync() const {
    __syncthreads();
    mark();
  }
  template <class T>
  __device__ __forceinline__ T* lds(T* p) const {
    return fddp::lds_ptr(p);
  }
  __device__ __forceinline__ void mark(const char* who = "sync / solver") const {
    if (threadIdx.x == 0) {
      unsigned long long i = st[0]++;
      if (i < 254) st[2 + i] = __builtin_amdgcn_s_memtime();
      label(i, who);
    }
  }
  // (after the stamp: the copy is not timed in the phase it names)
  __device__ __forceinline__ void label(unsigned long long i, const char* who) const {
    if (!g_label_on || blockIdx.x != 0 || i >= 254) return;
    const char* s = who;
    for (const char* q = who; *q; ++q)
      if (q[0] == 'a' && q[1] == 't' && q[2] == ' ' && q > who && q[-1] == ' ') s = q + 3;
    int k = 0;
    for (const char* q = s; *q && k < kLabelLen - 1; ++q)  // keep "file:line" past the last '/'
      if (*q == '/') k = 0; else if (*q == ')') break; else g_labels[i][k++] = *q;
    g_labels[i][k] = 0;
  }
};

// found by argument-dependent lookup (StampExec is in the global namespace)
template <int SPW>
__device__ inline bool gauss_jordan(const StampExec& ex, double* A, int nr, int ld, int nc, int* flag, double* pb,
                                    int id0 = 1 << 30) {
  const bool ok = gauss_jordan_regs<SPW>(A, nr, ld, nc, flag, pb, id0);
  ex.mark();
  return ok;
}
__device__ constexpr bool mb_inv_inplace(const StampExec& ex) { return mb_inv_inplace(DevExec{ex.nt}); }
__device__ inline bool mb_solve(const StampExec& ex, double* A, int nr, int ld, int nc, int* flag, double* pb) {
  const bool ok = mb_solve(DevExec{ex.nt}, A, nr, ld, nc, flag, pb);
  ex.mark();
  return ok;
}
template <class Side>
__device__ inline bool mb_invert(const StampExec& ex, double* A, int nr, int ld, int* flag, double* pb,
                                 double** Minv, Side side, int* nslots) {
  const bool ok = mb_invert(DevExec{ex.nt}, A, nr, ld, flag, pb, Minv, side, nslots);
  ex.mark();
  return ok;
}

// (2 waves / EU as the library's mb_knot_kernel / _s2: two 256-thread workgroups per CU
// when the LDS plan allows it)
template <int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2))) void probe_diff(const double* Pg, int nx, int m, const double* xg,
                                                        const double* ug, int use_u, double* out, int64_t so,
                                                        unsigned long long* stamps, int mode, int spill) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int psz = (int)Pg[3];
  const Blk bk = parse(Pg);
  bool vc;
  const int njac = count_jac_costs(bk, &vc);
  const DiffLayout l = diff_layout(bk.nj, njac, bk.nc, vc, bk.nj - bk.nun, count_cost_rows(bk, bk.nj - bk.nun), spill);
  double* P = sm + pad2(l.total);
  unsigned long long* st = (unsigned long long*)(P + pad2(psz));
  for (int e = threadIdx.x; e < psz; e += NT) P[e] = Pg[e];
  if (threadIdx.x == 0) {
    st[0] = 0;
    st[1] = __builtin_amdgcn_s_memtime();
  }
  __syncthreads();
  StampExec ex{NT, st};
  double* o = out + so * blockIdx.x;
  const int n = 2 * (int)Pg[1];
  double xn[1];
  (void)xn;
  if (mode == 0)
    knot_calc_diff_x(ex, P, nx, m, xg, ug, use_u != 0, sm, o, o + n * n, o + n * n + n * m, o + 2 * n * n + n * m,
                     o + 2 * n * n + 2 * n * m, o + 2 * n * n + 2 * n * m + m * m, o + 2 * n * n + 2 * n * m + m * m + n,
                     o + 2 * n * n + 2 * n * m + m * m + n + m, o + 2 * n * n + 2 * n * m + m * m + n + m + nx,
                     nullptr, spill);
  else  // without the fused calc's outputs (next state, cost)
    knot_calc_diff_x(ex, P, nx, m, xg, ug, use_u != 0, sm, o, o + n * n, o + n * n + n * m, o + 2 * n * n + n * m,
                     o + 2 * n * n + 2 * n * m, o + 2 * n * n + 2 * n * m + m * m, o + 2 * n * n + 2 * n * m + m * m + n,
                     nullptr, nullptr);
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const unsigned long long c = st[0] < 254 ? st[0] : 254;
    stamps[0] = c;
    stamps[1] = st[1];
    for (unsigned long long i = 0; i < c; ++i) stamps[2 + i] = st[2 + i];
  }
}

__global__ __launch_bounds__(256) void probe_calc(const double* Pg, int nx, const double* xg, const double* ug,
                                                  int use_u, double* out, unsigned long long* stamps) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int psz = (int)Pg[3];
#ifdef MB_CALC_DENSE
  const int64_t w = pad2(calc_dense_doubles((int)Pg[1], parse(Pg).nc));
#else
  const int64_t w = pad2(calc_work_doubles((int)Pg[1], parse(Pg).nc));
#endif
  double* P = sm + w;
  unsigned long long* st = (unsigned long long*)(P + pad2(psz));
  for (int e = threadIdx.x; e < psz; e += 256) P[e] = Pg[e];
  if (threadIdx.x == 0) {
    st[0] = 0;
    st[1] = __builtin_amdgcn_s_memtime();
  }
  __syncthreads();
  StampExec ex{256, st};
#ifdef MB_CALC_DENSE
  const double c = knot_calc_dense_x(ex, P, nx, xg, ug, use_u != 0, out + (int64_t)blockIdx.x * (nx + 1), sm);
#else
  const double c = knot_calc_x(ex, P, nx, xg, ug, use_u != 0, out + (int64_t)blockIdx.x * (nx + 1), sm);
#endif
  if (threadIdx.x == 0) out[(int64_t)blockIdx.x * (nx + 1) + nx] = c;
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const unsigned long long cc = st[0] < 254 ? st[0] : 254;
    stamps[0] = cc;
    stamps[1] = st[1];
    for (unsigned long long i = 0; i < cc; ++i) stamps[2 + i] = st[2 + i];
  }
}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  int hdr[4];  // nx, nu, m, psz
  if (fread(hdr, 4, 4, f) != 4) return 2;
  const int nx = hdr[0], nu = hdr[1], m = hdr[2], psz = hdr[3];
  std::vector<double> P(psz), x(nx), u(m > 0 ? m : 1);
  if (fread(P.data(), 8, psz, f) != (size_t)psz || fread(x.data(), 8, nx, f) != (size_t)nx ||
      fread(u.data(), 8, u.size(), f) != u.size())
    return 2;
  fclose(f);
  const int nwg = atoi(argv[2]);
  const int nj = (int)P[1], n = 2 * nj;
  const Blk bk = parse(P.data());
  bool vc;
  const int njac = count_jac_costs(bk, &vc);
  // the library's plan (spilled on the large trees; PROBE_SPILL=0 forces the all-LDS plan)
  const int spill = getenv("PROBE_SPILL") && getenv("PROBE_SPILL")[0] == '0'
                        ? 0
                        : diff_spill(nj, njac, bk.nc, vc, bk.nj - bk.nun, count_cost_rows(bk, bk.nj - bk.nun), psz, m);
  const DiffLayout l = diff_layout(nj, njac, bk.nc, vc, bk.nj - bk.nun, count_cost_rows(bk, bk.nj - bk.nun), spill);
  const size_t smd = 8 * (pad2(l.total) + pad2(psz) + 256);
#ifdef MB_CALC_DENSE
  const size_t smc = 8 * (pad2(calc_dense_doubles(nj, bk.nc)) + pad2(psz) + 256);
#else
  const size_t smc = 8 * (pad2(calc_work_doubles(nj, bk.nc)) + pad2(psz) + 256);
#endif
  printf("nj %d nx %d nu %d m %d psz %d lds diff %zu calc %zu\n", nj, nx, nu, m, psz, smd, smc);
  printf("  layout (spill %d): wv %ld A %ld half %ld dtau %ld da %ld qp %ld vec %ld J %ld red %ld Jc %ld Y %ld da0 %ld R %ld total %ld (njac %d vcols %d nc %d nrows %d)\n",
         spill, (long)l.wv, (long)l.A, (long)l.half, (long)l.dtau, (long)l.da, (long)l.qp, (long)l.vec, (long)l.J,
         (long)l.red, (long)l.Jc, (long)l.Y, (long)l.da0, (long)l.R, (long)l.total, njac, (int)vc, bk.nc,
         count_cost_rows(bk, bk.nj - bk.nun));
  fflush(stdout);
  if (argc > 3 && std::string(argv[3]) != "dump") return 0;  // layout only
  const bool dump = argc > 3;
  double *dP, *dx, *du, *dout;
  unsigned long long* dst;
  CK(hipMalloc(&dP, 8 * psz));
  CK(hipMalloc(&dx, 8 * nx));
  CK(hipMalloc(&du, 8 * u.size()));
  const int64_t so = 2 * n * n + 2 * n * m + m * m + n + m + nx + 2;
  CK(hipMalloc(&dout, 8 * so * nwg + 8 * (nx + 1) * nwg));
  CK(hipMalloc(&dst, 8 * 256));
  CK(hipMemcpy(dP, P.data(), 8 * psz, hipMemcpyHostToDevice));
  CK(hipMemcpy(dx, x.data(), 8 * nx, hipMemcpyHostToDevice));
  CK(hipMemcpy(du, u.data(), 8 * u.size(), hipMemcpyHostToDevice));
  const int pnt = getenv("PROBE_NT") ? atoi(getenv("PROBE_NT")) : kMbDiffNT;  // calcDiff workgroup size
  printf("calcDiff workgroup: %d threads\n", pnt == 512 || pnt == 128 ? pnt : 256);
  CK(hipFuncSetAttribute((const void*)probe_diff<128>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smd));
  CK(hipFuncSetAttribute((const void*)probe_diff<256>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smd));
  CK(hipFuncSetAttribute((const void*)probe_diff<512>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smd));
  CK(hipFuncSetAttribute((const void*)probe_calc, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smc));
  std::vector<unsigned long long> st(256);
  std::vector<char> labels(256 * kLabelLen, 0);
  for (int which = 0; which < 2; ++which) {
    for (int rep = 0; rep < 4; ++rep) {
      {  // the last launch records the phase labels (its times are not reported)
        const int on = rep == 3;
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_label_on), &on, sizeof(int)));
      }
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0));
      if (which == 0) {
        if (pnt == 128)
          hipLaunchKernelGGL(probe_diff<128>, dim3(nwg), dim3(128), smd, 0, dP, nx, m, dx, du, nu > 0 ? 1 : 0, dout, so,
                             dst, getenv("PROBE_DIFF_NOCOST") ? 1 : 0, spill);
        else if (pnt == 512)
          hipLaunchKernelGGL(probe_diff<512>, dim3(nwg), dim3(512), smd, 0, dP, nx, m, dx, du, nu > 0 ? 1 : 0, dout, so,
                             dst, getenv("PROBE_DIFF_NOCOST") ? 1 : 0, spill);
        else
          hipLaunchKernelGGL(probe_diff<256>, dim3(nwg), dim3(256), smd, 0, dP, nx, m, dx, du, nu > 0 ? 1 : 0, dout, so,
                             dst, getenv("PROBE_DIFF_NOCOST") ? 1 : 0, spill);
      } else {
        hipLaunchKernelGGL(probe_calc, dim3(nwg), dim3(256), smc, 0, dP, nx, dx, du, nu > 0 ? 1 : 0, dout, dst);
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      CK(hipMemcpy(st.data(), dst, 8 * 256, hipMemcpyDeviceToHost));
      if (rep < 3) printf("%s nwg %d: %.3f ms (%.2f us per WG-knot at 256 CUs)\n", which == 0 ? "calcDiff" : "calc", nwg, ms,
             1e3 * ms / (nwg / 256.0 > 1 ? nwg / 256.0 : 1));
      if (dump && which == 0 && rep == 0) {  // the LDS matrices and the output blocks
        std::vector<double> dm((size_t)kDumpSlots * kDumpCap);
        std::vector<int> sh(2 * kDumpSlots);
        CK(hipMemcpyFromSymbol(dm.data(), HIP_SYMBOL(g_dump), 8 * dm.size()));
        CK(hipMemcpyFromSymbol(sh.data(), HIP_SYMBOL(g_dump_shape), 4 * sh.size()));
        std::vector<double> ob(so);
        CK(hipMemcpy(ob.data(), dout, 8 * so, hipMemcpyDeviceToHost));
        std::string path = std::string(argv[1]) + ".dump";
        FILE* g = fopen(path.c_str(), "wb");
        fwrite(sh.data(), 4, sh.size(), g);
        fwrite(dm.data(), 8, dm.size(), g);
        fwrite(&so, 8, 1, g);
        fwrite(ob.data(), 8, ob.size(), g);
        fclose(g);
        printf("dumped %s\n", path.c_str());
      }
      if (rep == 3) {
        CK(hipMemcpyFromSymbol(labels.data(), HIP_SYMBOL(g_labels), labels.size()));
        printf("  phase labels:");
        for (unsigned long long i = 0; i < st[0] && i < 254; ++i) printf(" [%llu %s]", i, &labels[i * kLabelLen]);
        printf("\n");
      }
      if (rep == 2) {
        unsigned long long prev = st[1];
        printf("  phases (s_memtime ticks; * = wave-0 phase):");
        for (unsigned long long i = 0; i < st[0]; ++i) {
          const bool w0 = st[2 + i] >> 63;
          const unsigned long long t = st[2 + i] & ~(1ull << 63);
          printf(" %llu%s", t - prev, w0 ? "*" : "");
          prev = t;
        }
        printf("\n  total %llu\n", prev - st[1]);
        unsigned long long gj[32];
        CK(hipMemcpyFromSymbol(gj, HIP_SYMBOL(g_gjst), sizeof(gj)));
        printf("  gauss-jordan marks (ticks from its start; per block: sweep, update, barrier):");
        for (int i = 1; i < 32; ++i)
          if (gj[i] >= gj[0] && gj[i] - gj[0] < 10000000ull) printf(" %d:%llu", i, gj[i] - gj[0]);
        printf("\n");
        std::vector<unsigned long long> z(32, 0ull);
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_gjst), z.data(), sizeof(gj)));
      }
    }
  }
  return 0;
}
