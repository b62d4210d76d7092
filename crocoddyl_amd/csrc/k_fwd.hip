// Line-search rollout kernels (fddp_kernels.hpp forward_kernel, ls_select_kernel).
// FDDP_TU_FWD = 0: the generic and dense fast-path variants + ls_select; 1 / 2: the
// multibody-only variants at three / two waves per EU (the large ones), so they compile in
// parallel.
// The rollout's knot calc solves [M | Jc^T | tau - nle] by the dense blocked Gauss-Jordan
// (multibody.hpp MB_CALC_DENSE): measured on the C5 walk, the tree-sparse LTDL with the
// cost records on its idle waves has to be called out of line here (the backend's register
// alignment check trips on it inlined at the 256-VGPR cap), and the calls cost the rollout
// 6 % (29.9 -> 31.8 ms per step), more than the solve gains.
#define MB_CALC_DENSE 1
#include "fast_path.hpp"
#include "fddp_kernels.hpp"
#include "ktab.hpp"

#ifndef FDDP_TU_FWD
#error "k_fwd.hip is compiled with -DFDDP_TU_FWD=0|1|2"
#endif

namespace fddp {
namespace ktab {

#if FDDP_TU_FWD == 0
const void* forward_fn_0(int v) {
  return v == FWD_FAST ? (const void*)forward_kernel<kNT, true> : (const void*)forward_kernel<kNT, false>;
}
hipError_t forward_0(int v, dim3 grid, size_t smem, hipStream_t s, const Dev& D, const Prm& prm, int mode,
                     double alpha, int* count, int64_t pcap, int group) {
  if (v == FWD_FAST)
    hipLaunchKernelGGL((forward_kernel<kNT, true>), grid, dim3(kNT), smem, s, D, prm, mode, alpha, count, pcap, group);
  else
    hipLaunchKernelGGL((forward_kernel<kNT, false>), grid, dim3(kNT), smem, s, D, prm, mode, alpha, count, pcap, group);
  return hipGetLastError();
}
hipError_t ls_select(dim3 grid, hipStream_t s, const Dev& D, const Prm& prm, int group, int last, int* count) {
  hipLaunchKernelGGL((ls_select_kernel<kNT>), grid, dim3(kNT), 0, s, D, prm, group, last, count);
  return hipGetLastError();
}
#elif FDDP_TU_FWD == 2
const void* forward_fn_2() { return (const void*)forward_kernel<kNT, false, true, 2>; }
hipError_t forward_2(dim3 grid, size_t smem, hipStream_t s, const Dev& D, const Prm& prm, int mode, double alpha,
                     int* count, int64_t pcap, int group) {
  hipLaunchKernelGGL((forward_kernel<kNT, false, true, 2>), grid, dim3(kNT), smem, s, D, prm, mode, alpha, count, pcap,
                     group);
  return hipGetLastError();
}
#else
const void* forward_fn_1() { return (const void*)forward_kernel<kNT, false, true>; }
hipError_t forward_1(dim3 grid, size_t smem, hipStream_t s, const Dev& D, const Prm& prm, int mode, double alpha,
                     int* count, int64_t pcap, int group) {
  hipLaunchKernelGGL((forward_kernel<kNT, false, true>), grid, dim3(kNT), smem, s, D, prm, mode, alpha, count, pcap,
                     group);
  return hipGetLastError();
}
#endif

}  // namespace ktab
}  // namespace fddp
