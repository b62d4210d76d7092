// Dense / generic knot kernels: calc_kernel, calc_diff_kernel (fddp_kernels.hpp) and the
// fused dense-knot calc/calcDiff calc_tiled_kernel (fast_path.hpp).
#include "fast_path.hpp"
#include "fddp_kernels.hpp"
#include "ktab.hpp"

namespace fddp {
namespace ktab {

const void* calc_fn() { return (const void*)calc_kernel<kNT>; }
const void* calc_diff_fn() { return (const void*)calc_diff_kernel<kNT>; }
const void* calc_tiled_fn() { return (const void*)calc_tiled_kernel<kNTF>; }
hipError_t calc(dim3 grid, size_t smem, hipStream_t s, const Dev& D, int sel, int64_t pcap, int skip_mb) {
  hipLaunchKernelGGL(calc_kernel<kNT>, grid, dim3(kNT), smem, s, D, sel, pcap, skip_mb);
  return hipGetLastError();
}
hipError_t calc_diff(dim3 grid, size_t smem, hipStream_t s, const Dev& D, int sel, int gaps, int64_t pcap) {
  hipLaunchKernelGGL(calc_diff_kernel<kNT>, grid, dim3(kNT), smem, s, D, sel, gaps, pcap);
  return hipGetLastError();
}
hipError_t calc_tiled(dim3 grid, size_t smem, hipStream_t s, const Dev& D, int sel_calc, int sel_diff, int gaps,
                      int64_t pcap) {
  hipLaunchKernelGGL(calc_tiled_kernel<kNTF>, grid, dim3(kNTF), smem, s, D, sel_calc, sel_diff, gaps, pcap);
  return hipGetLastError();
}

}  // namespace ktab
}  // namespace fddp
