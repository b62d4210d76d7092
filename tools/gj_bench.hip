// Diagnostic (not product): the multibody Gauss-Jordan variants in isolation, one
// workgroup, on a random SPD matrix: the blocked MFMA sweep (gj_mfma, inverse and
// [M | B] solve) and the unblocked register sweep (gauss_jordan_rows), with phase
// stamps; plus dependent-chain latencies of the sweep's instructions.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/gj_bench tools/gj_bench.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
__device__ unsigned long long g_gjst[32];
#define MB_GJ_MARK(id)                                                                    \
  do {                                                                                    \
    if (threadIdx.x == 0 && blockIdx.x == 0) g_gjst[id] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#include "../crocoddyl_amd/csrc/multibody.hpp"

using namespace fddp::mb;

// mode 0: gj_mfma inverse (nc = nr); 1: gj_mfma solve (nc columns); 2: gauss_jordan_rows on [M | I];
// 3: gauss_jordan_rows on [M | B]
template <int NT>
__global__ __launch_bounds__(NT) void gj_kernel(const double* Ag, int nr, int ld, int nc, int mode, double* out,
                                                unsigned long long* cyc, int* okp) {
  __shared__ double A[64 * 130];
  __shared__ double pb[128];
  __shared__ int flag;
  for (int e = threadIdx.x; e < ld * nc; e += NT) A[e] = Ag[e];
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  bool ok = false;
#if defined(__HIP_DEVICE_COMPILE__)
  if (mode == 0)
    ok = gj_mfma(A, nr, ld, nr, true, &flag);
  else if (mode == 1)
    ok = gj_mfma(A, nr, ld, nc, false, &flag);
  else
    ok = gauss_jordan_rows<8, 3>(A, nr, ld, nc, pb, &flag, mode == 2 ? nr : 1 << 30);
#endif
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  for (int e = threadIdx.x; e < ld * nc; e += NT) out[e] = A[e];
  if (threadIdx.x == 0) {
    cyc[0] = t1 - t0;
    *okp = ok ? 1 : 0;
  }
}

__global__ void lat_kernel(double* out, unsigned long long* cyc, int iters) {
  const int lane = threadIdx.x;
  double x = 1.0 + lane * 1e-9, y = 1.0 + lane * 1e-12;
  unsigned long long t[8];
  t[0] = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) x = __builtin_fma(x, y, 1e-30);
  t[1] = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) x = __builtin_amdgcn_rcp(x);
  t[2] = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) x = __shfl(x, (lane + 5) & 63) + 1e-30;
  t[3] = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) x = readlane_d(x, 7) * y;
  t[4] = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) x = 1. / x;
  t[5] = __builtin_amdgcn_s_memtime();
  out[lane] = x;
  if (lane == 0)
    for (int k = 0; k < 5; ++k) cyc[k] = (t[k + 1] - t[k]) / iters;
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
  const int nr = argc > 1 ? atoi(argv[1]) : 38, nb = argc > 2 ? atoi(argv[2]) : 13;
  const int ld = nr | 1;
  srand(1);
  std::vector<double> X(nr * nr), M(nr * nr);
  for (auto& v : X) v = (rand() / (double)RAND_MAX) - 0.5;
  for (int i = 0; i < nr; ++i)
    for (int j = 0; j < nr; ++j) {
      double s = i == j ? nr : 0.;
      for (int k = 0; k < nr; ++k) s += X[i * nr + k] * X[j * nr + k];
      M[i + nr * j] = s;
    }
  double *dA, *dO, *dl;
  unsigned long long *dc, cyc[8];
  int* dok;
  CK(hipMalloc(&dA, 8 * ld * 130));
  CK(hipMalloc(&dO, 8 * ld * 130));
  CK(hipMalloc(&dl, 8 * 64));
  CK(hipMalloc(&dc, 8 * 8));
  CK(hipMalloc(&dok, 4));
  hipLaunchKernelGGL(lat_kernel, dim3(1), dim3(64), 0, 0, dl, dc, 256);
  CK(hipMemcpy(cyc, dc, 8 * 5, hipMemcpyDeviceToHost));
  printf("dependent latency (cycles): fma_f64 %llu rcp_f64 %llu shfl_f64 %llu readlane_f64+mul %llu div_f64 %llu\n",
         cyc[0], cyc[1], cyc[2], cyc[3], cyc[4]);
  for (int mode = 0; mode < 4; ++mode) {
    const int nc = mode == 0 ? nr : (mode == 2 ? 2 * nr : nr + nb);
    std::vector<double> A(ld * nc, 0.);
    for (int c = 0; c < nc; ++c)
      for (int r = 0; r < nr; ++r)
        A[r + ld * c] = c < nr ? M[r + nr * c] : (mode == 2 ? (c - nr == r ? 1. : 0.) : std::sin(1. + r + 3. * c));
    CK(hipMemcpy(dA, A.data(), 8 * A.size(), hipMemcpyHostToDevice));
    for (int nt : {256, 512}) {
      for (int rep = 0; rep < 3; ++rep) {
        if (nt == 256)
          hipLaunchKernelGGL(gj_kernel<256>, dim3(1), dim3(256), 0, 0, dA, nr, ld, nc, mode, dO, dc, dok);
        else
          hipLaunchKernelGGL(gj_kernel<512>, dim3(1), dim3(512), 0, 0, dA, nr, ld, nc, mode, dO, dc, dok);
        CK(hipDeviceSynchronize());
      }
      std::vector<double> O(ld * nc);
      int ok;
      unsigned long long gj[32];
      CK(hipMemcpy(O.data(), dO, 8 * O.size(), hipMemcpyDeviceToHost));
      CK(hipMemcpy(cyc, dc, 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(&ok, dok, 4, hipMemcpyDeviceToHost));
      CK(hipMemcpyFromSymbol(gj, HIP_SYMBOL(g_gjst), sizeof(gj)));
      // residual: M * X - (I or B) over the result columns
      double err = 0.;
      const int c0 = (mode == 0) ? 0 : nr, c1 = (mode == 0) ? nr : nc;
      for (int c = c0; c < c1; ++c)
        for (int r = 0; r < nr; ++r) {
          double s = 0.;
          for (int k = 0; k < nr; ++k) s += M[r + nr * k] * O[k + ld * c];
          const double rhs = mode == 0 ? (r == c ? 1. : 0.) : A[r + ld * c];
          err = fmax(err, fabs(s - rhs));
        }
      printf("mode %d (%s) nr %d nc %d threads %d: %llu cycles ok %d residual %.2e", mode,
             mode == 0 ? "mfma inverse" : mode == 1 ? "mfma solve" : mode == 2 ? "rows [M|I]" : "rows [M|B]", nr, nc,
             nt, cyc[0], ok, err);
      if (mode < 2) {
        printf("  marks:");
        for (int i = 1; i < 32; ++i)
          if (gj[i] >= gj[0] && gj[i] - gj[0] < 10000000ull) printf(" %d:%llu", i, gj[i] - gj[0]);
        std::vector<unsigned long long> z(32, 0ull);
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_gjst), z.data(), sizeof(gj)));
      }
      printf("\n");
    }
  }
  return 0;
}
