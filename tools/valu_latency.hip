// Micro-benchmark (diagnostic): dependent-chain latency of f64 VALU ops and
// LDS round trips on gfx950, one wave.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(double* out, unsigned long long* cyc, int iters, double seed) {
  __shared__ double buf[128];
  const int lane = threadIdx.x;
  double x = seed + lane * 1e-9, y = 1.0 + lane * 1e-12;
  buf[lane] = x;
  __syncthreads();
  unsigned long long t[8];
  t[0] = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) x = fma(x, y, 1e-30);  // dependent fma chain
  t[1] = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) x = __builtin_amdgcn_rcp(x);  // dependent rcp chain
  t[2] = __builtin_amdgcn_s_memtime();
  double a0 = x, a1 = x + 1, a2 = x + 2, a3 = x + 3, a4 = x + 4, a5 = x + 5, a6 = x + 6, a7 = x + 7;
  for (int i = 0; i < iters; ++i) {  // 8 independent fma (throughput)
    a0 = fma(a0, y, 1e-30); a1 = fma(a1, y, 1e-30); a2 = fma(a2, y, 1e-30); a3 = fma(a3, y, 1e-30);
    a4 = fma(a4, y, 1e-30); a5 = fma(a5, y, 1e-30); a6 = fma(a6, y, 1e-30); a7 = fma(a7, y, 1e-30);
  }
  t[3] = __builtin_amdgcn_s_memtime();
  x += a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  for (int i = 0; i < iters; ++i) {  // LDS: write own, read a broadcast value, dependent
    asm volatile("" ::: "memory");
    buf[lane] = x;
    asm volatile("" ::: "memory");
    x = buf[(i & 31)] * 0.5 + 1e-30;
  }
  t[4] = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {  // LDS read only, dependent address chain
    asm volatile("" ::: "memory");
    x = buf[((int)x & 63)] + 1e-30;
  }
  t[5] = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {  // select on f64 (2x v_cndmask) chain
    x = (lane & 1) ? x * y : x;
  }
  t[6] = __builtin_amdgcn_s_memtime();
  out[lane] = x;
  if (lane == 0)
    for (int j = 0; j < 6; ++j) cyc[j] = t[j + 1] - t[j];
}
int main() {
  double* d; unsigned long long* c;
  hipMalloc(&d, 64 * 8); hipMalloc(&c, 8 * 8);
  const int iters = 1000;
  k<<<1, 64>>>(d, c, iters, 1.0);
  hipDeviceSynchronize();
  k<<<1, 64>>>(d, c, iters, 1.0);
  hipDeviceSynchronize();
  unsigned long long h[8];
  hipMemcpy(h, c, 6 * 8, hipMemcpyDeviceToHost);
  const char* names[6] = {"dependent v_fma_f64", "dependent v_rcp_f64", "8 independent v_fma_f64 (per fma)",
                          "LDS write+broadcast read+fma chain", "LDS dependent read chain", "f64 select*mul chain"};
  for (int j = 0; j < 6; ++j) printf("%-40s %.1f cycles\n", names[j], h[j] / (double)iters / (j == 2 ? 8 : 1));
  return 0;
}
