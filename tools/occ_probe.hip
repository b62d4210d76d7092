// Diagnostic (not product): how many 256-thread workgroups one CU holds at once for a given
// dynamic LDS size and per-lane scratch, measured (real-time start / end and the CU of every
// workgroup) rather than taken from the occupancy API.
// Usage: occ_probe <lds_bytes> <scratch: 0|1> <nwg>
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

template <bool SCRATCH>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void spin(unsigned long long* rec, int iters,
                                                                                      int sel) {
  extern __shared__ double sm[];
  unsigned long long* r = rec + 4 * blockIdx.x;
  if (threadIdx.x == 0) {
    r[0] = __builtin_amdgcn_s_memrealtime();
    r[1] = (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
           ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32);
  }
  double acc = threadIdx.x;
  if (SCRATCH) {
    // a private array indexed by a runtime value lives in scratch (160 doubles = 1280 B)
    double a[160];
    for (int i = 0; i < 160; ++i) a[i] = i * acc;
    for (int it = 0; it < iters; ++it) acc += a[(it * 7 + sel + threadIdx.x) % 160];
  } else {
    for (int it = 0; it < iters; ++it) acc = fma(acc, 1.0000001, 0.5);
  }
  sm[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    r[2] = __builtin_amdgcn_s_memrealtime();
    r[3] = (unsigned long long)sm[1];
  }
}

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  const int lds = atoi(argv[1]), scr = atoi(argv[2]), nwg = atoi(argv[3]);
  unsigned long long* d;
  if (hipMalloc(&d, 32 * (size_t)nwg) != hipSuccess) return 1;
  hipMemset(d, 0, 32 * (size_t)nwg);
  const void* k = scr ? (const void*)spin<true> : (const void*)spin<false>;
  hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  int per_cu = 0;
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256, lds);
  hipFuncAttributes fa;
  hipFuncGetAttributes(&fa, k);
  for (int rep = 0; rep < 2; ++rep) {
    if (scr)
      hipLaunchKernelGGL(spin<true>, dim3(nwg), dim3(256), lds, 0, d, 20000, 1);
    else
      hipLaunchKernelGGL(spin<false>, dim3(nwg), dim3(256), lds, 0, d, 20000, 1);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
  }
  std::vector<unsigned long long> h(4 * (size_t)nwg);
  hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
  struct Ev {
    unsigned long long t;
    int dlt;
  };
  std::vector<std::pair<unsigned long long, std::vector<Ev>>> cus;
  for (int b = 0; b < nwg; ++b) {
    const unsigned long long key = ((h[4 * b + 1] >> 32) << 16) | ((h[4 * b + 1] >> 8) & 0xff);
    size_t i = 0;
    while (i < cus.size() && cus[i].first != key) ++i;
    if (i == cus.size()) cus.push_back({key, {}});
    cus[i].second.push_back({h[4 * b], 1});
    cus[i].second.push_back({h[4 * b + 2], -1});
  }
  int most = 0;
  for (auto& c : cus) {
    std::sort(c.second.begin(), c.second.end(),
              [](const Ev& a, const Ev& b) { return a.t < b.t || (a.t == b.t && a.dlt < b.dlt); });
    int cur = 0;
    for (auto& e : c.second) most = std::max(most, cur += e.dlt);
  }
  printf("lds %d scratch %d (private %zu B/lane, vgpr %d): occupancy API %d per CU; measured at most %d on one CU (%zu CUs)\n",
         lds, scr, (size_t)fa.localSizeBytes, fa.numRegs, per_cu, most, cus.size());
  return 0;
}
