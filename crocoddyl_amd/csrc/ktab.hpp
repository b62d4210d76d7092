// Kernel table of libfddp_hip: the large kernels are compiled in their own translation
// units (k_mb.hip, k_fwd.hip, k_bwd.hip, k_calc.hip; the Makefile builds them in
// parallel) and fddp_hip.hip reaches them only through these typed launchers and
// function handles (for hipFuncSetAttribute / occupancy queries). Each launcher returns
// the launch's hipError_t.
#ifndef CROCODDYL_AMD_KTAB_HPP_
#define CROCODDYL_AMD_KTAB_HPP_

#include <hip/hip_runtime.h>

#include "fddp_device.hpp"

namespace fddp {
namespace ktab {

constexpr int kNT = 256;   // threads of the per-element kernels
constexpr int kNTF = 512;  // fused calc/calcDiff: 8 waves per CU keep the derivative stores streaming

// Multibody knot calc/calcDiff, one workgroup per (knot, element) (k_mb.hip):
//   MB_W2 256 threads at 2 waves/EU, MB_W1 256 threads at 1 wave/EU,
//   MB_X2 128 threads (small trees), MB_X8 512 threads (the one-per-CU plans),
//   MB_S2 256 threads at 2 waves/EU on the spilled plan (multibody.hpp diff_spill)
enum { MB_W2 = 0, MB_W1 = 1, MB_X2 = 2, MB_X8 = 3, MB_S2 = 4, MB_NVAR = 5 };
int mb_knot_threads(int v);
const void* mb_knot_fn(int v);
hipError_t mb_knot(int v, dim3 grid, size_t smem, hipStream_t s, const Dev& D, int sel_calc, int sel_diff);

// Line-search rollout (k_fwd.hip): FWD_GENERIC any knot mix, FWD_FAST the dense-knot
// fast path, FWD_MB multibody-only horizons at three workgroups per CU (168 VGPRs),
// FWD_MB2 the same at two (256 VGPRs)
enum { FWD_GENERIC = 0, FWD_FAST = 1, FWD_MB = 2, FWD_MB2 = 3 };
const void* forward_fn(int v);
hipError_t forward(int v, dim3 grid, size_t smem, hipStream_t s, const Dev& D, const Prm& prm, int mode, double alpha,
                   int* count, int64_t pcap, int group);
hipError_t ls_select(dim3 grid, hipStream_t s, const Dev& D, const Prm& prm, int group, int last, int* count);

// Riccati sweep (k_bwd.hip). MFMA variants are named (NTL*10+MTL)*10+NW (n, m in
// 16-tiles, waves per element). backward_mfma_setup: the variant for (NTL, MTL, NW)
// with its dynamic LDS set, or -1 if the shape does not fit (n > its padded width, LDS).
int backward_mfma_setup(int ntl, int mtl, int nw, int n, int* per_cu = nullptr);
hipError_t backward_mfma(int code, dim3 grid, hipStream_t s, const Dev& D, const Prm& prm, int mode);
const void* backward_generic_fn();
hipError_t backward_generic(dim3 grid, size_t smem, hipStream_t s, const Dev& D, const Prm& prm, int mode);

// Dense / generic knot kernels (k_calc.hip)
const void* calc_fn();
const void* calc_diff_fn();
const void* calc_tiled_fn();
hipError_t calc(dim3 grid, size_t smem, hipStream_t s, const Dev& D, int sel, int64_t pcap, int skip_mb);
hipError_t calc_diff(dim3 grid, size_t smem, hipStream_t s, const Dev& D, int sel, int gaps, int64_t pcap);
hipError_t calc_tiled(dim3 grid, size_t smem, hipStream_t s, const Dev& D, int sel_calc, int sel_diff, int gaps,
                      int64_t pcap);

}  // namespace ktab
}  // namespace fddp


// Per-object entry points behind the dispatchers above (defined in the k_*.hip objects;
// the dispatchers live in fddp_hip.hip).
namespace fddp {
namespace ktab {
int mb_knot_threads_0();
int mb_knot_threads_1();
int mb_knot_threads_2();
int mb_knot_threads_3();
int mb_knot_threads_4();
const void* mb_knot_fn_0();
const void* mb_knot_fn_1();
const void* mb_knot_fn_2();
const void* mb_knot_fn_3();
const void* mb_knot_fn_4();
hipError_t mb_knot_0(dim3 grid, size_t smem, hipStream_t s, const Dev& D, int sel_calc, int sel_diff);
hipError_t mb_knot_1(dim3 grid, size_t smem, hipStream_t s, const Dev& D, int sel_calc, int sel_diff);
hipError_t mb_knot_2(dim3 grid, size_t smem, hipStream_t s, const Dev& D, int sel_calc, int sel_diff);
hipError_t mb_knot_3(dim3 grid, size_t smem, hipStream_t s, const Dev& D, int sel_calc, int sel_diff);
hipError_t mb_knot_4(dim3 grid, size_t smem, hipStream_t s, const Dev& D, int sel_calc, int sel_diff);
const void* forward_fn_0(int v);
hipError_t forward_0(int v, dim3 grid, size_t smem, hipStream_t s, const Dev& D, const Prm& prm, int mode,
                     double alpha, int* count, int64_t pcap, int group);
const void* forward_fn_1();
hipError_t forward_1(dim3 grid, size_t smem, hipStream_t s, const Dev& D, const Prm& prm, int mode, double alpha,
                     int* count, int64_t pcap, int group);
const void* forward_fn_2();
hipError_t forward_2(dim3 grid, size_t smem, hipStream_t s, const Dev& D, const Prm& prm, int mode, double alpha,
                     int* count, int64_t pcap, int group);
int backward_mfma_setup_0(int ntl, int mtl, int nw, int n, int* per_cu);  // -2: not in this object
int backward_mfma_setup_1(int ntl, int mtl, int nw, int n, int* per_cu);
hipError_t backward_mfma_0(int code, dim3 grid, hipStream_t s, const Dev& D, const Prm& prm, int mode);
hipError_t backward_mfma_1(int code, dim3 grid, hipStream_t s, const Dev& D, const Prm& prm, int mode);
}  // namespace ktab
}  // namespace fddp

#endif  // CROCODDYL_AMD_KTAB_HPP_
