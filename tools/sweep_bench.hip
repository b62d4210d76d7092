// Micro-benchmark (diagnostic): cycles of the backward sweep's Quu factorisations on
// wave 0 in isolation, one wave per workgroup: variant 0 sym_sweep_inverse<32> (the
// explicit inverse, round 3), 1 chol_inv_sweep<32>, 2 chol_inv_blocked2 (round 4),
// 3 chol_inv_sweep<16> on the leading 16 x 16 block.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/sweep_bench tools/sweep_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include "../crocoddyl_amd/csrc/bwd_mfma.hpp"

__global__ void k_sweep(const double* Q, double* Qi_out, unsigned long long* cyc, int reps, int m, int variant) {
  __shared__ double Quu[32 * 32], Qi[32 * 32], Ct[32 * 33], rb[64];
  const int lane = threadIdx.x;
  for (int e = lane; e < 1024; e += 64) Quu[e] = Q[e];
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  bool bad = false;
  for (int r = 0; r < reps; ++r) {
    if (variant == 0)
      bad |= fddp::sym_sweep_inverse<32, 32>(Quu, Qi, rb, m, lane);
    else if (variant == 1)
      bad |= fddp::chol_inv_sweep<32, 32, 33>(Quu, Qi, Ct, rb, m, lane, nullptr, 0);
    else if (variant == 2)
      bad |= fddp::chol_inv_blocked2<32, 33>(Quu, Qi, Ct, rb, m, lane, nullptr, 0);
    else
      bad |= fddp::chol_inv_sweep<16, 32, 33>(Quu, Qi, Ct, rb, m < 16 ? m : 16, lane, nullptr, 0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  for (int e = lane; e < 1024; e += 64) Qi_out[blockIdx.x * 1024 + e] = Qi[e];
  if (lane == 0) cyc[blockIdx.x] = (t1 - t0) / reps + (bad ? 1000000000ull : 0);
}

// relative accuracy of rcp_f64 over a wide range of pivots
__global__ void k_rcp(const double* d, double* err, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) err[i] = fabs(fddp::rcp_f64(d[i]) * d[i] - 1.0);
}

int main() {
  {
    const int N = 1 << 16;
    double* h = (double*)malloc(N * 8);
    for (int i = 0; i < N; ++i) h[i] = exp(-30.0 + 60.0 * (rand() / (double)RAND_MAX)) * (1 + 1e-3 * i);
    double *dd, *de;
    hipMalloc(&dd, N * 8);
    hipMalloc(&de, N * 8);
    hipMemcpy(dd, h, N * 8, hipMemcpyHostToDevice);
    k_rcp<<<N / 256, 256>>>(dd, de, N);
    hipMemcpy(h, de, N * 8, hipMemcpyDeviceToHost);
    double mx = 0;
    for (int i = 0; i < N; ++i) mx = fmax(mx, h[i]);
    printf("rcp_f64: max |rcp(d) d - 1| = %.3e\n", mx);
  }
  const int m = 32;
  double Q[1024], X[1024];
  srand(1);
  for (int i = 0; i < 1024; ++i) X[i] = (rand() / (double)RAND_MAX) - 0.5;
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < m; ++j) {
      double s = 0;
      for (int k = 0; k < m; ++k) s += X[i * 32 + k] * X[j * 32 + k];
      Q[j * 32 + i] = s + (i == j ? 1.0 : 0.0);
    }
  double *dQ, *dQi;
  unsigned long long* dc;
  hipMalloc(&dQ, sizeof(Q));
  hipMalloc(&dQi, sizeof(double) * 1024 * 256);
  hipMalloc(&dc, 8 * 256);
  hipMemcpy(dQ, Q, sizeof(Q), hipMemcpyHostToDevice);
  for (int variant = 0; variant < 4; ++variant)
    for (int blocks : {1, 256}) {
      k_sweep<<<blocks, 64>>>(dQ, dQi, dc, 20, m, variant);
      hipDeviceSynchronize();
      unsigned long long c[256];
      hipMemcpy(c, dc, 8 * blocks, hipMemcpyDeviceToHost);
      double Qi[1024];
      hipMemcpy(Qi, dQi, sizeof(Qi), hipMemcpyDeviceToHost);
      // variant 0: |Q Qi - I|; 1, 2: |C Q C^T - I| (C = L^-1); 3: on the leading 16 block
      const int mm = variant == 3 ? 16 : m;
      double err = 0;
      for (int i = 0; i < mm; ++i)
        for (int j = 0; j < mm; ++j) {
          double s = 0;
          if (variant == 0) {
            for (int k = 0; k < mm; ++k) s += Q[k * 32 + i] * Qi[j * 32 + k];
          } else {
            for (int k = 0; k < mm; ++k)
              for (int l = 0; l < mm; ++l) s += Qi[k * 32 + i] * Q[l * 32 + k] * Qi[l * 32 + j];
          }
          err = fmax(err, fabs(s - (i == j)));
        }
      printf("variant %d blocks=%d: %llu cycles (%.0f per pivot), residual %.2e\n", variant, blocks, c[0],
             c[0] / (double)mm, err);
    }
  return 0;
}
