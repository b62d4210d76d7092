// Multibody knot kernels (fddp_kernels.hpp mb_knot_kernel*), one variant per object:
// the Makefile compiles this file once per FDDP_TU_MB = ktab::MB_W2 .. MB_S2.
#include "fddp_kernels.hpp"
#include "ktab.hpp"

#ifndef FDDP_TU_MB
#error "k_mb.hip is compiled with -DFDDP_TU_MB=<variant>"
#endif

namespace fddp {
namespace ktab {

namespace {
#if FDDP_TU_MB == 0
constexpr int kThreads = mb::kMbDiffNT;
const void* const kFn = (const void*)mb_knot_kernel;
#define MB_KERNEL mb_knot_kernel
#elif FDDP_TU_MB == 1
constexpr int kThreads = mb::kMbDiffNT;
const void* const kFn = (const void*)mb_knot_kernel_w1;
#define MB_KERNEL mb_knot_kernel_w1
#elif FDDP_TU_MB == 2
constexpr int kThreads = mb::kMbDiffNT / 2;
const void* const kFn = (const void*)mb_knot_kernel_x2;
#define MB_KERNEL mb_knot_kernel_x2
#elif FDDP_TU_MB == 3
constexpr int kThreads = 2 * mb::kMbDiffNT;
const void* const kFn = (const void*)mb_knot_kernel_x8;
#define MB_KERNEL mb_knot_kernel_x8
#else
constexpr int kThreads = mb::kMbDiffNT;
const void* const kFn = (const void*)mb_knot_kernel_s2;
#define MB_KERNEL mb_knot_kernel_s2
#endif
}  // namespace

#define MB_CAT2(a, b) a##b
#define MB_CAT(a, b) MB_CAT2(a, b)
// per-variant entry points, dispatched by ktab::mb_knot* in fddp_hip.hip
int MB_CAT(mb_knot_threads_, FDDP_TU_MB)() { return kThreads; }
const void* MB_CAT(mb_knot_fn_, FDDP_TU_MB)() { return kFn; }
hipError_t MB_CAT(mb_knot_, FDDP_TU_MB)(dim3 grid, size_t smem, hipStream_t s, const Dev& D, int sel_calc,
                                        int sel_diff) {
  hipLaunchKernelGGL(MB_KERNEL, grid, dim3(kThreads), smem, s, D, sel_calc, sel_diff);
  return hipGetLastError();
}

}  // namespace ktab
}  // namespace fddp
