// Micro-benchmark (diagnostic, not part of the library): cycles per
// v_mfma_f64_16x16x4_f64 on one wave for 1, 2, 4, 8 independent accumulator
// chains, plus an LDS write->read broadcast round trip.
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/mfma_lat mfma_f64_latency.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int NC>
__global__ void chain(double* out, unsigned long long* cyc, int iters) {
  f64x4 acc[NC];
  for (int i = 0; i < NC; ++i) acc[i] = f64x4{0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
#pragma unroll
      for (int i = 0; i < NC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int i = 0; i < NC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void lds_rt(double* out, unsigned long long* cyc, int iters) {
  __shared__ double buf[64];
  const int lane = threadIdx.x;
  double v = lane;
  buf[lane] = v;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    asm volatile("" ::: "memory");
    const double d = buf[it & 31];
    v = v * 0.5 + d;
    asm volatile("" ::: "memory");
    buf[lane] = v;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[lane] = v;
  if (lane == 0) cyc[0] = t1 - t0;
}

template <int NC>
double run_chain(double* d_out, unsigned long long* d_cyc, int blocks) {
  const int iters = 200;
  chain<NC><<<blocks, 64>>>(d_out, d_cyc, iters);
  hipDeviceSynchronize();
  chain<NC><<<blocks, 64>>>(d_out, d_cyc, iters);
  hipDeviceSynchronize();
  unsigned long long c[1024];
  hipMemcpy(c, d_cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
  double mean = 0;
  for (int i = 0; i < blocks; ++i) mean += (double)c[i];
  mean /= blocks;
  return mean / (iters * 16.0 * NC);
}

int main() {
  double* d_out;
  unsigned long long* d_cyc;
  hipMalloc(&d_out, sizeof(double) * 1024 * 64);
  hipMalloc(&d_cyc, sizeof(unsigned long long) * 1024);
  for (int blocks : {1, 1024}) {
    printf("blocks=%d  cycles per MFMA: 1 chain %.1f | 2 chains %.1f | 4 chains %.1f | 8 chains %.1f\n", blocks,
           run_chain<1>(d_out, d_cyc, blocks), run_chain<2>(d_out, d_cyc, blocks), run_chain<4>(d_out, d_cyc, blocks),
           run_chain<8>(d_out, d_cyc, blocks));
  }
  const int iters = 1000;
  lds_rt<<<1, 64>>>(d_out, d_cyc, iters);
  hipDeviceSynchronize();
  unsigned long long c;
  hipMemcpy(&c, d_cyc, sizeof(c), hipMemcpyDeviceToHost);
  printf("LDS write->read->fma->write loop: %.1f cycles/iter\n", (double)c / iters);
  return 0;
}
