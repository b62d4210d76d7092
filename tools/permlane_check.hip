// Diagnostic (not product): checks multibody.hpp's register broadcasts against __shfl
// on the device: row_bcast_d<n> (DPP row_newbcast) and row_to_all_d<r> (permlane swaps).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../crocoddyl_amd/csrc -o permlane_check permlane_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "multibody.hpp"
using namespace fddp;
__global__ void k(int* bad) {
  const int lane = threadIdx.x;
  const double v = 1000.0 * lane + 0.25;
  int nb = 0;
#pragma unroll
  for (int n = 0; n < 16; ++n) nb += row_bcast_d(v, n) != __shfl(v, n + 16 * (lane >> 4)) ? 1 : 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) nb += row_to_all_d(v, r) != __shfl(v, (lane & 15) + 16 * r) ? 1 : 0;
  bad[lane] = nb;  // (per-lane, summed on the host)
}
int main() {
  int* d;
  hipMalloc(&d, 64 * 4);
  k<<<1, 64>>>(d);
  int hv[64], h = 0;
  hipMemcpy(hv, d, 64 * 4, hipMemcpyDeviceToHost);
  for (int i = 0; i < 64; ++i) h += hv[i];
  printf("permlane_check: %d mismatches\n", h);
  return h != 0;
}
