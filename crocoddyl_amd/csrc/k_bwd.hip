// Riccati sweep kernels (bwd_mfma.hpp backward_mfma_kernel, fddp_kernels.hpp
// backward_kernel). FDDP_TU_BWD = 0: the C5-sized MFMA variant (5 x 2 tiles); 1: the
// other MFMA variants and the generic VALU sweep.
#include "bwd_mfma.hpp"
#include "fddp_kernels.hpp"
#include "ktab.hpp"

#ifndef FDDP_TU_BWD
#error "k_bwd.hip is compiled with -DFDDP_TU_BWD=0|1"
#endif

namespace fddp {
namespace ktab {

namespace {
template <int NTL, int MTL, int NW>
int setup_one(int n, int* per_cu) {
  using Cfg = MfmaCfg<NTL, MTL>;
  const size_t lds = bwd_lds_bytes<NTL, MTL, NW>();
  if (lds > 160 * 1024 || n > Cfg::ZLD) return -1;
  const void* f = (const void*)backward_mfma_kernel<NTL, MTL, NW>;
  if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return -1;
  // resident workgroups per CU (registers and LDS): the plan choice weighs it
  if (per_cu && hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, f, NW * 64, lds) != hipSuccess) *per_cu = 1;
  // column-block ownership per wave is static (BwdPlan in bwd_mfma.hpp)
  return (NTL * 10 + MTL) * 10 + NW;
}
template <int NTL, int MTL, int NW>
void launch_one(dim3 grid, hipStream_t s, const Dev& D, const Prm& prm, int mode) {
  backward_mfma_kernel<NTL, MTL, NW><<<grid, dim3(NW * 64), bwd_lds_bytes<NTL, MTL, NW>(), s>>>(D, prm, mode);
}
}  // namespace

#if FDDP_TU_BWD == 0
int backward_mfma_setup_0(int ntl, int mtl, int nw, int n, int* per_cu) {
  return (ntl == 5 && mtl == 2 && nw == 8) ? setup_one<5, 2, 8>(n, per_cu) : -2;
}
hipError_t backward_mfma_0(int code, dim3 grid, hipStream_t s, const Dev& D, const Prm& prm, int mode) {
  if (code != 528) return hipErrorInvalidDeviceFunction;
  launch_one<5, 2, 8>(grid, s, D, prm, mode);
  return hipGetLastError();
}
#else
int backward_mfma_setup_1(int ntl, int mtl, int nw, int n, int* per_cu) {  // -1: no such variant or it does not fit
#define FDDP_BWD_CASE(A, B, W) \
  if (ntl == A && mtl == B && nw == W) return setup_one<A, B, W>(n, per_cu);
  FDDP_BWD_CASE(3, 1, 8) FDDP_BWD_CASE(3, 1, 4) FDDP_BWD_CASE(3, 1, 1)
  FDDP_BWD_CASE(2, 1, 8) FDDP_BWD_CASE(2, 1, 4) FDDP_BWD_CASE(2, 1, 1)
  FDDP_BWD_CASE(1, 1, 8) FDDP_BWD_CASE(1, 1, 4) FDDP_BWD_CASE(1, 1, 1)
#undef FDDP_BWD_CASE
  return -1;
}
hipError_t backward_mfma_1(int code, dim3 grid, hipStream_t s, const Dev& D, const Prm& prm, int mode) {
  switch (code) {
    case 318: launch_one<3, 1, 8>(grid, s, D, prm, mode); break;
    case 314: launch_one<3, 1, 4>(grid, s, D, prm, mode); break;
    case 311: launch_one<3, 1, 1>(grid, s, D, prm, mode); break;
    case 218: launch_one<2, 1, 8>(grid, s, D, prm, mode); break;
    case 214: launch_one<2, 1, 4>(grid, s, D, prm, mode); break;
    case 211: launch_one<2, 1, 1>(grid, s, D, prm, mode); break;
    case 118: launch_one<1, 1, 8>(grid, s, D, prm, mode); break;
    case 114: launch_one<1, 1, 4>(grid, s, D, prm, mode); break;
    case 111: launch_one<1, 1, 1>(grid, s, D, prm, mode); break;
    default: return hipErrorInvalidDeviceFunction;
  }
  return hipGetLastError();
}
const void* backward_generic_fn() { return (const void*)backward_kernel<kNT>; }
hipError_t backward_generic(dim3 grid, size_t smem, hipStream_t s, const Dev& D, const Prm& prm, int mode) {
  hipLaunchKernelGGL(backward_kernel<kNT>, grid, dim3(kNT), smem, s, D, prm, mode);
  return hipGetLastError();
}
#endif

}  // namespace ktab
}  // namespace fddp
