// libfddp_hip — C ABI implementation (see include/fddp_hip.h).
//
// One handle = one ShootingProblem replicated over B batch elements (each
// element with its own x0, warm start and optionally its own model
// parameters) + one SolverFDDP state machine per element, all resident on one
// gfx950 device. fddp_solve enqueues, per FDDP iteration:
//   [iter 0] calc_kernel + cost_sum      ShootingProblem::calc (ddp.cpp:158)
//   calc_diff_kernel (+gaps)             SolverDDP::calcDiff (ddp.cpp:157-178)
//   backward_kernel (reg retries)        computeDirection loop (fddp.cpp:35-48)
//   forward_kernel (line search, update) fddp.cpp:49-103
// Elements that converge or abort drop out (masked); the host only reads one
// counter per iteration to stop early.
// (the large kernels are compiled in the k_*.hip objects and reached through ktab.hpp)
#define FDDP_TU_MAIN 1
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/fddp_hip.h"
#include "fddp_device.hpp"
#include "fddp_kernels.hpp"
#include "fast_path.hpp"
#include "bwd_mfma.hpp"
#include "ktab.hpp"

using namespace fddp;

// ---- kernel-table dispatchers (ktab.hpp): variant -> the object that compiled it ----
namespace fddp {
namespace ktab {
int mb_knot_threads(int v) {
  return v == MB_W1   ? mb_knot_threads_1()
         : v == MB_X2 ? mb_knot_threads_2()
         : v == MB_X8 ? mb_knot_threads_3()
         : v == MB_S2 ? mb_knot_threads_4()
                      : mb_knot_threads_0();
}
const void* mb_knot_fn(int v) {
  return v == MB_W1   ? mb_knot_fn_1()
         : v == MB_X2 ? mb_knot_fn_2()
         : v == MB_X8 ? mb_knot_fn_3()
         : v == MB_S2 ? mb_knot_fn_4()
                      : mb_knot_fn_0();
}
hipError_t mb_knot(int v, dim3 grid, size_t smem, hipStream_t s, const Dev& D, int sel_calc, int sel_diff) {
  switch (v) {
    case MB_W1: return mb_knot_1(grid, smem, s, D, sel_calc, sel_diff);
    case MB_X2: return mb_knot_2(grid, smem, s, D, sel_calc, sel_diff);
    case MB_X8: return mb_knot_3(grid, smem, s, D, sel_calc, sel_diff);
    case MB_S2: return mb_knot_4(grid, smem, s, D, sel_calc, sel_diff);
    default: return mb_knot_0(grid, smem, s, D, sel_calc, sel_diff);
  }
}
const void* forward_fn(int v) {
  return v == FWD_MB ? forward_fn_1() : v == FWD_MB2 ? forward_fn_2() : forward_fn_0(v);
}
hipError_t forward(int v, dim3 grid, size_t smem, hipStream_t s, const Dev& D, const Prm& prm, int mode, double alpha,
                   int* count, int64_t pcap, int group) {
  if (v == FWD_MB) return forward_1(grid, smem, s, D, prm, mode, alpha, count, pcap, group);
  if (v == FWD_MB2) return forward_2(grid, smem, s, D, prm, mode, alpha, count, pcap, group);
  return forward_0(v, grid, smem, s, D, prm, mode, alpha, count, pcap, group);
}
int backward_mfma_setup(int ntl, int mtl, int nw, int n, int* per_cu) {
  const int v = backward_mfma_setup_0(ntl, mtl, nw, n, per_cu);
  return v != -2 ? v : backward_mfma_setup_1(ntl, mtl, nw, n, per_cu);
}
hipError_t backward_mfma(int code, dim3 grid, hipStream_t s, const Dev& D, const Prm& prm, int mode) {
  return code == 528 ? backward_mfma_0(code, grid, s, D, prm, mode) : backward_mfma_1(code, grid, s, D, prm, mode);
}
}  // namespace ktab
}  // namespace fddp

namespace {

thread_local std::string g_err;

using ktab::kNT;
using ktab::kNTF;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                           \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess)                                                                       \
      return fail(FDDP_ERR_RUNTIME, std::string(#expr) + ": " + hipGetErrorString(e_));         \
  } while (0)

#define LAUNCH_CHECK()                                                                          \
  do {                                                                                          \
    hipError_t e_ = hipGetLastError();                                                          \
    if (e_ != hipSuccess) return fail(FDDP_ERR_RUNTIME, std::string("launch: ") + hipGetErrorString(e_)); \
  } while (0)

// a launch through the kernel table (ktab.hpp), which returns the launch's error
#define KLAUNCH(expr)                                                                           \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess) return fail(FDDP_ERR_RUNTIME, std::string("launch: ") + hipGetErrorString(e_)); \
  } while (0)

int64_t block_doubles(int kind, int nx, int nu) {
  switch (kind) {
    case FDDP_KNOT_LQR:
      return FDDP_PARAM_HEADER + 2LL * nx * nx + 2LL * nx * nu + (int64_t)nu * nu + 2LL * nx + nu;
    case FDDP_KNOT_UNICYCLE:
      return FDDP_PARAM_HEADER;
    case FDDP_KNOT_EULER_DIFFLQR: {
      const int64_t nq = nx / 2;
      return FDDP_PARAM_HEADER + 2 * nq * nq + nq * nu + nq + (int64_t)nx * nx + (int64_t)nx * nu +
             (int64_t)nu * nu + nx + nu;
    }
  }
  return -1;
}


// Checks one FDDP_KNOT_EULER_FREEFWD / _CONTACTFWD / FDDP_KNOT_IMPULSEFWD block
// (layouts in include/fddp_hip.h) against nx / nu and the space left in the
// pool. Returns its size in doubles, or -1 with `why` set. nj / njac / nc:
// dofs, jac costs and contact rows (LDS sizing).
int64_t mb_block_check(const double* P, int64_t avail, int kind, int nx, int nu, std::string& why, int* nj_out,
                       int* njac_out, int* nc_out, bool* vcols_out = nullptr, int* nu_out = nullptr,
                       int* nrows_out = nullptr) {
  using namespace fddp::mb;
  if (avail < FDDP_PARAM_HEADER) return why = "block out of range", -1;
  const double dt = P[0];
  const int nj = (int)P[1], ncost = (int)P[2];
  const int64_t size = (int64_t)P[3];
  if (!(dt >= 0.) || !std::isfinite(dt)) return why = "dt has positive value", -1;
  if ((double)nj != P[1] || nj < 1 || nj > kMaxJ) return why = "number of dofs out of [1, 64]", -1;
  if (size > avail || (double)size != P[3]) return why = "block out of range", -1;
  int64_t o = FDDP_PARAM_HEADER + 3 + nj;
  if (o + kJRec > size) return why = "block too small for its joints", -1;
  const bool ff = (int)P[o] == J_FREEFLYER;
  if (ff && nj < 6) return why = "a free-flyer root needs nv >= 6", -1;
  const int nb = ff ? nj - 5 : nj, nq = ff ? nj + 1 : nj;
  if (nx != nq + nj) return why = "multibody knots need nx = nq + nv", -1;
  const bool contact = kind == FDDP_KNOT_EULER_CONTACTFWD, impulse = kind == FDDP_KNOT_IMPULSEFWD;
  if (!contact && !impulse && (nu != nj || ff)) return why = "ActuationModelFull needs nu = nv and no free-flyer", -1;
  if (impulse && nu != 0) return why = "impulse knots have nu = 0", -1;
  if (impulse && dt != 0.) return why = "impulse blocks carry dt = 0 (no integrator)", -1;
  if ((double)ncost != P[2] || ncost < 0 || ncost > kMaxCosts) return why = "number of costs out of [0, 64]", -1;
  int force_rows = 0;  // rows the contact-force costs read
  if (o + (int64_t)kJRec * nb > size) return why = "block too small for its joints", -1;
  for (int i = 0; i < nb; ++i) {
    const double* J = P + o + (int64_t)kJRec * i;
    const int type = (int)J[0], par = (int)J[1];
    if ((double)type != J[0] || (type != J_REVOLUTE && type != J_FREEFLYER)) return why = "unknown joint type", -1;
    if (type == J_FREEFLYER && (i != 0 || par != -1)) return why = "a free-flyer may only be the root joint", -1;
    if ((double)par != J[1] || par < -1 || par >= i) return why = "joint parents must precede their children", -1;
    if (type == J_REVOLUTE) {
      const double an = std::sqrt(J[2] * J[2] + J[3] * J[3] + J[4] * J[4]);
      if (!(std::fabs(an - 1.) < 1e-9)) return why = "joint axes must be unit vectors", -1;
    }
    if (!(J[17] >= 0.)) return why = "negative body mass", -1;
  }
  o += (int64_t)kJRec * nb;
  int njac = 0;
  bool vcols = false;
  for (int k = 0; k < ncost; ++k) {
    if (o + kCHdr > size) return why = "cost records out of range", -1;
    const double* C = P + o;
    const int type = (int)C[0];
    const int64_t rs = (int64_t)C[3];
    const int act = (int)C[2];
    if ((double)act != C[2] || act < A_QUAD || act > A_WEIGHTED_QUAD_BARRIER)
      return why = "unknown activation kind", -1;
    const int ap = act <= A_WEIGHTED_QUAD ? 1 : (act == A_QUAD_BARRIER ? 2 : 3);  // parameter rows per residual
    int64_t want = -1;
    if (type == C_STATE) want = kCHdr + nx + ap * 2 * nj;
    if (type == C_CONTROL) want = kCHdr + nu + ap * (int64_t)nu;
    if (type == C_FRAME_PLACEMENT) want = kCHdr + 25 + ap * 6;
    if (type == C_FRAME_TRANSLATION) want = kCHdr + 16 + ap * 3;
    if (type == C_FRAME_VELOCITY) {
      if (impulse) return why = "frame-velocity costs are covered on Euler knots only", -1;
      want = kCHdr + 19 + ap * 6;
    }
    if (type == C_COM_POSITION) want = kCHdr + 3 + ap * 3;
    if (type == C_CONTACT_FORCE || type == C_FRICTION_CONE) {
      // [row0, nr, fref(6)] | [row0, nc, nr, A(3 nr)]; rows checked against the contacts below
      if (kind != FDDP_KNOT_EULER_CONTACTFWD) return why = "force costs need contact knots", -1;
      if (o + kCHdr + 3 > size) return why = "cost records out of range", -1;
      const int row0 = (int)C[kCHdr];
      if ((double)row0 != C[kCHdr] || (row0 < 0 && row0 != kInactiveForceRow))
        return why = "contact-force cost row out of range", -1;
      if (type == C_CONTACT_FORCE) {
        const int nrf = (int)C[kCHdr + 1];
        if (nrf != 3 && nrf != 6) return why = "contact-force costs need a 3- or 6-row force", -1;
        want = kCHdr + 8 + ap * nrf;
        if (row0 >= 0) force_rows = std::max(force_rows, row0 + nrf);
      } else {
        const int ncc = (int)C[kCHdr + 1], nrc = (int)C[kCHdr + 2];
        if ((double)nrc != C[kCHdr + 2] || nrc < 1 || nrc > 6) return why = "friction cone rows out of [1, 6]", -1;
        if (row0 >= 0 && ncc != 3 && ncc != 6) return why = "friction cone on a contact of 3 or 6 rows", -1;
        want = kCHdr + 3 + 3 * nrc + ap * nrc;
        if (row0 >= 0) force_rows = std::max(force_rows, row0 + ncc);
      }
    }
    if (want < 0) return why = "unknown cost type " + std::to_string(type), -1;
    if (rs != want || o + rs > size) return why = "cost record of the wrong size", -1;
    if (type == C_FRAME_PLACEMENT || type == C_FRAME_TRANSLATION || type == C_FRAME_VELOCITY) {
      const int fj = (int)C[kCHdr];
      if ((double)fj != C[kCHdr] || fj < 0 || fj >= nb) return why = "frame attached to an unknown joint", -1;
    }
    if (type == C_STATE && ff)  // the reference state's free-flyer pose must be finite
      for (int e = 0; e < 7; ++e)
        if (!std::isfinite(C[kCHdr + e])) return why = "non-finite reference state", -1;
    if (type == C_FRAME_PLACEMENT || type == C_FRAME_TRANSLATION || type == C_COM_POSITION ||
        type == C_FRAME_VELOCITY || (type == C_STATE && ff))
      ++njac;
    if (type == C_FRAME_VELOCITY) vcols = true;
    o += rs;
  }
  int nc = 0;
  std::vector<std::pair<int, int>> crow;  // (row0, rows) of every contact record
  if (contact || impulse) {  // [nun | r_coeff, damping, ncontact, 0 | 1 | 2] + contact / impulse records
    if (o + 4 > size) return why = "contact section out of range", -1;
    const int nun = (int)P[o], ncon = (int)P[o + 2];
    const double damping = P[o + 1];
    if (impulse ? P[o + 3] != 1. : (P[o + 3] != 0. && P[o + 3] != 2.))
      return why = "contact / impulse section flag does not match the kind", -1;
    if (impulse) {
      if (!(P[o] >= 0.) || !std::isfinite(P[o])) return why = "The restitution coefficient has to be positive", -1;
    } else {
      if ((double)nun != P[o] || nun < 0 || nun >= nj) return why = "unactuated dofs out of [0, nv)", -1;
      if (ff && nun != 6) return why = "ActuationModelFloatingBase on a free-flyer leaves 6 dofs unactuated", -1;
      if (nu != nj - nun) return why = "ActuationModelFloatingBase needs nu = nv - nun", -1;
    }
    if (!(damping >= 0.) || !std::isfinite(damping)) return why = "The damping factor has to be positive", -1;
    if ((double)ncon != P[o + 2] || ncon < 0) return why = "negative number of contacts", -1;
    o += 4;
    for (int k = 0; k < ncon; ++k) {
      if (o + kCHdr + 1 > size) return why = "contact records out of range", -1;
      const double* C = P + o;
      const int type = (int)C[0];
      const int64_t rs = (int64_t)C[3];
      int64_t want = -1;
      if (type == C_CONTACT_3D) want = kCHdr + (impulse ? 13 : 16);
      if (type == C_CONTACT_6D) want = kCHdr + (impulse ? 13 : 25);
      if (want < 0) return why = "unknown contact type " + std::to_string(type), -1;
      if (rs != want || o + rs > size) return why = "contact record of the wrong size", -1;
      const int fj = (int)C[kCHdr];
      if ((double)fj != C[kCHdr] || fj < 0 || fj >= nb) return why = "contact frame attached to an unknown joint", -1;
      if (!std::isfinite(C[1]) || !std::isfinite(C[2])) return why = "non-finite contact gains", -1;
      const int rows = type == C_CONTACT_3D ? 3 : 6;
      crow.emplace_back(nc, rows);
      nc += rows;
      o += rs;
    }
    if (nc > kMaxNc) return why = "more than 24 contact rows in one knot", -1;
  }
  if (force_rows > nc) return why = "contact-force cost reads rows beyond the contacts", -1;
  if (force_rows > 0) {  // each contact-force cost reads exactly one contact of its size
    int64_t oc = FDDP_PARAM_HEADER + 3 + nj + (int64_t)kJRec * nb;
    for (int k = 0; k < ncost; ++k) {
      const double* C = P + oc;
      if (((int)C[0] == C_CONTACT_FORCE || (int)C[0] == C_FRICTION_CONE) && (int)C[kCHdr] >= 0) {
        bool hit = false;
        for (const auto& r : crow) hit = hit || (r.first == (int)C[kCHdr] && r.second == (int)C[kCHdr + 1]);
        if (!hit) return why = "a force cost must read one whole contact of its size", -1;
      }
      oc += (int64_t)C[3];
    }
  }
  if (o != size) return why = "block size does not match its records", -1;
  if (njac > kMaxJacCosts) return why = "more than 8 frame / CoM / frame-velocity / free-flyer state costs in one knot", -1;
  const int nrows = count_cost_rows(parse(P), nu);
  if (nrows > kMaxCostRows) return why = "more than 64 cost residual rows with dense Jacobians in one knot", -1;
  if ((pad2(diff_layout(nj, njac, nc, vcols, nu, nrows).total) + pad2(size)) * 8 > 160 * 1024)
    return why = "too many dofs for the calcDiff LDS plan", -1;
  if (nj_out) *nj_out = std::max(*nj_out, nj);
  if (njac_out) *njac_out = std::max(*njac_out, njac);
  if (nc_out) *nc_out = std::max(*nc_out, nc);
  if (vcols_out) *vcols_out = *vcols_out || vcols;
  if (nu_out) *nu_out = std::max(*nu_out, nu);
  if (nrows_out) *nrows_out = std::max(*nrows_out, nrows);
  return size;
}

// Validation of a knot sequence against the handle's dims (fddp_create,
// fddp_set_knots, fddp_set_model_params). exact_nu_max: the running knots' max
// nu must equal nu_max (creation); otherwise it may be smaller (the
// reference's circularAppend / updateNode checks, shooting.hxx:249-252).
// Multibody blocks are checked for every batch element they cover.
int check_knots(const fddp_dims& d, const fddp_knot_desc* knots, const double* params, int64_t n_params,
                const char* who, bool exact_nu_max) {
  const std::string w(who);
  int nu_max = 0;
  for (int t = 0; t <= d.T; ++t) {
    const fddp_knot_desc& k = knots[t];
    if (k.nu < 0) return fail(FDDP_ERR_INVALID_ARG, w + ": negative nu");
    if (t < d.T && k.nu > nu_max) nu_max = k.nu;
    if (d.nx != d.ndx && !is_mb_kind(k.kind))
      return fail(FDDP_ERR_INVALID_ARG, w + ": a free-flyer state needs multibody knots");
    if (k.kind == FDDP_KNOT_UNICYCLE && (d.nx != 3 || k.nu != 2))
      return fail(FDDP_ERR_INVALID_ARG, w + ": unicycle knots need nx=3, nu=2");
    if (k.kind == FDDP_KNOT_EULER_DIFFLQR && (d.nx % 2))
      return fail(FDDP_ERR_INVALID_ARG, w + ": Euler(DiffLQR) knots need an even nx");
    if (k.param_offset < 0 || k.param_stride < 0 || k.param_offset + (int64_t)(d.B - 1) * k.param_stride >= n_params)
      return fail(FDDP_ERR_INVALID_ARG, w + ": knot " + std::to_string(t) + " parameter block out of range");
    int64_t sz;
    if (is_mb_kind(k.kind)) {
      if (!params) return fail(FDDP_ERR_INVALID_ARG, w + ": null parameter pool");
      sz = 0;
      const int nb = k.param_stride > 0 ? d.B : 1;
      for (int b = 0; b < nb; ++b) {
        const int64_t off = k.param_offset + (int64_t)b * k.param_stride;
        std::string why;
        const int64_t s1 = mb_block_check(params + off, n_params - off, k.kind, d.nx, k.nu, why, nullptr, nullptr, nullptr);
        if (s1 < 0) return fail(FDDP_ERR_INVALID_ARG, w + ": knot " + std::to_string(t) + ": " + why);
        if (k.param_stride > 0 && s1 > k.param_stride)
          return fail(FDDP_ERR_INVALID_ARG, w + ": knot " + std::to_string(t) + " blocks overlap (stride too small)");
        sz = std::max(sz, s1);
      }
    } else {
      sz = block_doubles(k.kind, d.nx, k.nu);
    }
    if (sz < 0) return fail(FDDP_ERR_UNSUPPORTED, w + ": unknown knot kind " + std::to_string(k.kind));
    if (k.param_offset + (int64_t)(d.B - 1) * k.param_stride + sz > n_params)
      return fail(FDDP_ERR_INVALID_ARG, w + ": knot " + std::to_string(t) + " parameter block out of range");
  }
  if (exact_nu_max ? nu_max != d.nu_max : nu_max > d.nu_max)
    return fail(FDDP_ERR_INVALID_ARG, exact_nu_max ? w + ": nu_max must equal the max nu over the running knots"
                                                   : w + ": nu node is bigger than the maximum nu");
  if (knots[d.T].nu > d.nu_max) return fail(FDDP_ERR_INVALID_ARG, w + ": terminal nu exceeds nu_max");
  return FDDP_OK;
}

}  // namespace

struct fddp_handle_s {
  fddp_dims dims;
  int device = 0;
  int npar_env = 0;    // CROCODDYL_AMD_LS_PAR (0: chosen per problem)
  int npar_alloc = 1;  // trial slots allocated for the parallel line search
  bool npar_adapt = false;  // trial-group size re-chosen after every solve (choose_npar)
  bool npar_chosen = false;  // choose_npar has set D.npar
  double ls_slots = 0.;     // rollout workgroups resident on the device at once
  int fwd_mb_variant = -1;  // rollout_variant's choice (-1: not yet made; reset by apply_knots)
  hipStream_t stream = nullptr;
  std::vector<fddp_knot_desc> knots;
  int64_t n_params = 0;
  int64_t params_cap = 0;  // doubles allocated for the parameter pool
  fddp_params prm;
  Dev D;
  std::vector<void*> allocs;
  double* staging = nullptr;
  int64_t staging_len = 0;
  double* d_out = nullptr;  // B doubles
  int* d_count = nullptr;
  int* h_count = nullptr;   // pinned
  bool debug = false;
  double* dbg[7] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  double* dqi = nullptr;  // SolverBoxFDDP::Quu_inv_ debug store (allocated with debug on)
  int solver_kind = FDDP_SOLVER_FDDP;
  double* d_ulb = nullptr;  // control limits, allocated on first fddp_set_control_limits
  double* d_uub = nullptr;
  unsigned char* d_haslim = nullptr;
  int64_t bytes = 0;
  size_t bwd_smem = 0, fwd_smem = 0, calc_smem = 0, cdiff_smem = 0;
  bool fast = false;  // dense-knot fast path (fast_path.hpp) for calc / calcDiff / forward
  size_t fused_smem = 0, fwd_fast_smem = 0;
  int64_t pcap = 0;  // doubles of LDS reserved for a resident parameter block
  bool has_mb = false;     // multibody knots present (mb_knot_kernel)
  bool all_mb = false;     // every knot is a multibody knot
  size_t mb_diff_smem = 0; // its dynamic LDS
  int mb_nj = 0;            // largest multibody tree (dofs)
  int bwd_variant = 0;  // 0 generic, else (NTL*10+MTL)*10+waves of the MFMA sweep
  int ls_npar_last = 0;      // trial-group size of the last line search (1: serial)
  std::vector<int> h_order;  // host copy of D.ls_order (kept alive for the async upload)
  int ls_launches_last = 0;  // rollout (forward_kernel) dispatches of the last line search
  fddp_iteration_callback cb = nullptr;  // per-iteration callback (fddp_set_callback)
  void* cb_user = nullptr;
  bool in_solve = false;
  // timing
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev_rec;
  double t_ms[4] = {0, 0, 0, 0};
  int64_t t_cnt[4] = {0, 0, 0, 0};
};

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

int dalloc(fddp_handle* h, double** p, int64_t n) {
  void* q = nullptr;
  const size_t bytes = sizeof(double) * (size_t)(n > 0 ? n : 1);
  HIP_TRY(hipMalloc(&q, bytes));
  HIP_TRY(hipMemsetAsync(q, 0, bytes, h->stream));
  h->allocs.push_back(q);
  h->bytes += (int64_t)bytes;
  *p = (double*)q;
  return FDDP_OK;
}

hipEvent_t take_event(fddp_handle* h) {
  if (!h->ev_pool.empty()) {
    hipEvent_t e = h->ev_pool.back();
    h->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

struct Timed {
  fddp_handle* h;
  int cls;
  hipEvent_t a = nullptr, b = nullptr;
  Timed(fddp_handle* hh, int c) : h(hh), cls(c) {
    if (h->timing) {
      a = take_event(h);
      b = take_event(h);
      if (a) (void)hipEventRecord(a, h->stream);
    }
  }
  ~Timed() {
    if (h->timing && a && b) {
      (void)hipEventRecord(b, h->stream);
      h->ev_rec.push_back({cls, {a, b}});
    }
  }
};

Prm to_prm(const fddp_params& p) {
  Prm q;
  q.th_acceptstep = p.th_acceptstep;
  q.th_stop = p.th_stop;
  q.th_grad = p.th_grad;
  q.th_stepdec = p.th_stepdec;
  q.th_stepinc = p.th_stepinc;
  q.th_acceptnegstep = p.th_acceptnegstep;
  q.regfactor = p.regfactor;
  q.regmin = p.regmin;
  q.regmax = p.regmax;
  q.n_alphas = p.n_alphas;
  for (int i = 0; i < 16; ++i) q.alphas[i] = p.alphas[i];
  return q;
}

BoxQPCfg to_boxcfg(const fddp_boxqp_params& p) {
  BoxQPCfg c;
  c.maxiter = p.maxiter;
  c.n_alphas = p.n_alphas;
  c.th_acceptstep = p.th_acceptstep;
  c.th_grad = p.th_grad;
  c.reg = p.reg;
  for (int i = 0; i < 16; ++i) c.alphas[i] = p.alphas[i];
  return c;
}

// ---- kernel launchers ------------------------------------------------------
int launch_fused(fddp_handle* h, int sel_calc, int sel_diff, int gaps) {
  Timed tm(h, sel_diff >= 0 ? 1 : 0);
  const Dev& D = h->D;
  KLAUNCH(ktab::calc_tiled(dim3(D.B), h->fused_smem, h->stream, D, sel_calc, sel_diff, gaps, h->pcap));
  return FDDP_OK;
}
// The knot-parallel kernel's LDS plan leaves room for one workgroup per CU: take the
// 1-wave/EU build (no spills; FDDP_MB_W1=0 forces the 2-wave one, for A/B runs).
static bool mb_one_per_cu(const fddp_handle* h) {
  static const int env = [] {
    const char* e = std::getenv("FDDP_MB_W1");
    return e ? (e[0] == '0' ? 0 : 1) : -1;
  }();
  return env >= 0 ? env == 1 : h->mb_diff_smem > 80 * 1024;
}
// 512-thread (8-wave) workgroups for the one-per-CU plans: two waves per SIMD where the
// 256-thread plan has one (C5 calcDiff 66 -> 59 ms); FDDP_MB_NT=256 / 512 forces
static bool mb_x8(const fddp_handle* h) {
  static const int env = [] {
    const char* e = std::getenv("FDDP_MB_NT");
    return e ? std::atoi(e) : 0;
  }();
  return env ? env == 512 : mb_one_per_cu(h);
}
// 128-thread (2-wave) workgroups for the small trees whose LDS plan fits four per CU
static bool mb_x2(const fddp_handle* h) {
  static const int env = [] {
    const char* e = std::getenv("FDDP_MB_NT");
    return e ? std::atoi(e) : 0;
  }();
  return env ? env == 128 : (h->mb_nj <= 16 && h->mb_diff_smem <= 40 * 1024);
}
// Multibody knots (knot-parallel): calc for sel_calc, calcDiff for sel_diff (-1: none).
int launch_mb(fddp_handle* h, int sel_calc, int sel_diff) {
  const Dev& D = h->D;
  const int v = D.mbspill ? ktab::MB_S2
                           : mb_x2(h) ? ktab::MB_X2 : (mb_x8(h) ? ktab::MB_X8 : (mb_one_per_cu(h) ? ktab::MB_W1 : ktab::MB_W2));
  KLAUNCH(ktab::mb_knot(v, dim3(D.T + 1, D.B), h->mb_diff_smem, h->stream, D, sel_calc, sel_diff));
  return FDDP_OK;
}
int launch_calc(fddp_handle* h, int sel) {
  if (h->fast) return launch_fused(h, sel, -1, 0);
  Timed tm(h, 0);
  const Dev& D = h->D;
  if (h->has_mb) {
    int rc;
    if ((rc = launch_mb(h, sel, -1))) return rc;
    if (!h->all_mb) KLAUNCH(ktab::calc(dim3(D.B), h->calc_smem, h->stream, D, sel, h->pcap, 1));
  } else {
    KLAUNCH(ktab::calc(dim3(D.B), h->calc_smem, h->stream, D, sel, h->pcap, 0));
  }
  return FDDP_OK;
}
int launch_cost_sum(fddp_handle* h, int sel, double* out) {
  const Dev& D = h->D;
  hipLaunchKernelGGL(cost_sum_kernel, dim3((D.B + 255) / 256), dim3(256), 0, h->stream, D, sel, out);
  LAUNCH_CHECK();
  return FDDP_OK;
}
int launch_calc_diff(fddp_handle* h, int sel, int gaps) {
  if (h->fast) return launch_fused(h, -1, sel, gaps);
  Timed tm(h, 1);
  const Dev& D = h->D;
  if (h->has_mb) {  // multibody knots: one workgroup per knot, before the gaps pass
    int rc;
    if ((rc = launch_mb(h, -1, sel))) return rc;
  }
  KLAUNCH(ktab::calc_diff(dim3(D.B), h->cdiff_smem, h->stream, D, sel, gaps, h->pcap));
  return FDDP_OK;
}
// problem.calc (sel_calc) + cost_ = sum of knot costs, then problem.calcDiff
// (sel_diff, + gaps): one fused pass on the fast path.
int launch_calc_then_diff(fddp_handle* h, int sel_calc, int sel_calc_sum, int sel_diff, int gaps) {
  int rc;
  if (h->fast) {
    if ((rc = launch_fused(h, sel_calc, sel_diff, gaps))) return rc;
    return launch_cost_sum(h, sel_calc_sum, nullptr);
  }
  if (h->has_mb) {  // multibody knots: their calc fused into the knot-parallel calcDiff
    // one timer record per calcDiff call (class 1): the knot-parallel kernel, the
    // dense knots' calc (mixed horizons only), the cost sum and the gaps pass
    Timed tm(h, 1);
    const Dev& D = h->D;
    if ((rc = launch_mb(h, sel_calc, sel_diff))) return rc;
    if (!h->all_mb) KLAUNCH(ktab::calc(dim3(D.B), h->calc_smem, h->stream, D, sel_calc, h->pcap, 1));
    if ((rc = launch_cost_sum(h, sel_calc_sum, nullptr))) return rc;
    KLAUNCH(ktab::calc_diff(dim3(D.B), h->cdiff_smem, h->stream, D, sel_diff, gaps, h->pcap));
    return FDDP_OK;
  }
  if ((rc = launch_calc(h, sel_calc))) return rc;
  if ((rc = launch_cost_sum(h, sel_calc_sum, nullptr))) return rc;
  return launch_calc_diff(h, sel_diff, gaps);
}
int launch_backward(fddp_handle* h, int mode) {
  Timed tm(h, 2);
  const Dev& D = h->D;
  if (h->bwd_variant)
    KLAUNCH(ktab::backward_mfma(h->bwd_variant, dim3(D.B), h->stream, D, to_prm(h->prm), mode));
  else
    KLAUNCH(ktab::backward_generic(dim3(D.B), h->bwd_smem, h->stream, D, to_prm(h->prm), mode));
  return FDDP_OK;
}

// slot buffers of the parallel line search (generic trials), allocated on first use
static int ensure_par_slots(fddp_handle* h) {
  Dev& D = h->D;
  if (D.npar <= h->npar_alloc) return FDDP_OK;  // (buffers of a smaller npar stay until fddp_destroy)
  const int64_t B = D.B, K1 = D.T + 1, K0 = D.T, q = D.npar - 1;
  int rc;
  double* done = nullptr;
  if ((rc = dalloc(h, &D.pxs, q * B * K1 * D.sX)) || (rc = dalloc(h, &D.pus, q * B * K0 * D.sM)) ||
      (rc = dalloc(h, &D.pxnext, q * B * K0 * D.sX)) || (rc = dalloc(h, &D.pkcost, q * B * K1)) ||
      (rc = dalloc(h, &D.pdvp, q * B * K1)) || (rc = dalloc(h, &D.ptrial, B * D.npar * 4)) ||
      (rc = dalloc(h, &done, (B + 1) / 2)))
    return rc;
  D.ls_done = (int*)done;
  h->npar_alloc = D.npar;
  return FDDP_OK;
}

// every knot multibody: the rollout variant with only the multibody calc compiled in
// (FDDP_FWD_MB=0 selects the generic one, for A/B runs)
static bool mb_rollout(const fddp_handle* h) {
  static const bool off = [] {
    const char* e = std::getenv("FDDP_FWD_MB");
    return e && e[0] == '0';
  }();
  return h->all_mb && !off;
}

// Workgroups of `fn` one CU holds at once with `smem` bytes of dynamic LDS: the occupancy
// API's answer, capped by the LDS allocated in 2 KB granules (measured on gfx950,
// tools/occ_probe.hip: 53,248 B per workgroup fit three per CU, 53,776 B two, where the API
// still says three).
static int resident_per_cu(const void* fn, size_t smem) {
  int per_cu = 0;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kNT, smem);
  hipFuncAttributes fa{};
  (void)hipFuncGetAttributes(&fa, fn);
  const size_t g = 2048, lds = ((smem + fa.sharedSizeBytes + g - 1) / g) * g;
  const int by_lds = lds > 0 ? (int)((160 * 1024) / lds) : per_cu;
  return std::max(1, std::min(per_cu, by_lds));
}
// The rollout variant: the generic one for mixed horizons; for multibody-only horizons the
// three-workgroups-per-CU build (168 VGPRs, spills) when its LDS allows three per CU and the
// batch needs more than two per CU, else the 256-VGPR build (FDDP_FWD_MBW=2|3 forces one).
static int rollout_variant(fddp_handle* h) {
  if (!mb_rollout(h)) return ktab::FWD_GENERIC;
  if (h->fwd_mb_variant >= 0) return h->fwd_mb_variant;
  static const int env = [] {
    const char* e = std::getenv("FDDP_FWD_MBW");
    return e ? std::atoi(e) : 0;
  }();
  int dev_cus = 0;
  (void)hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, h->device);
  const bool three = resident_per_cu(ktab::forward_fn(ktab::FWD_MB), h->fwd_smem) >= 3;
  const bool take3 = env ? env == 3 : (three && h->D.B > 2 * std::max(1, dev_cus));
  h->fwd_mb_variant = take3 ? ktab::FWD_MB : ktab::FWD_MB2;
  return h->fwd_mb_variant;
}

// Trial-group size of the next line searches from the trial counts of the last one
// (the results are bit-identical for every size; only the work and the number of
// sequential launches change). With S rollout workgroups resident at once and t_b the
// trials element b needed: serial (1) takes ~max(sum t_b / S, max t_b) trial-times, one
// group launch per g trials ~sum_k max(U_k / S, 1) with U_k the trial slots of group k.
static void choose_npar(fddp_handle* h, const std::vector<ElemState>& st) {
  if (!h->npar_adapt || h->fast) return;
  const int na = h->prm.n_alphas;
  if (h->ls_slots <= 0.) {
    int dev_cus = 0;
    (void)hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, h->device);
    const int per_cu = resident_per_cu(ktab::forward_fn(rollout_variant(h)), h->fwd_smem);
    h->ls_slots = (double)std::max(1, dev_cus) * std::max(1, per_cu);
    if (std::getenv("FDDP_STAMPS"))  // (diagnostic runs: the rollout's residency)
      std::fprintf(stderr, "[fddp] rollout: %d workgroups per CU x %d CUs (LDS %zu B per workgroup)\n", per_cu, dev_cus,
                   h->fwd_smem);
  }
  std::vector<int> t;
  t.reserve(st.size());
  for (const ElemState& s : st) {
    if (s.n_iter_run <= 0) continue;
    int k = na;  // exhausted: every alpha tried
    for (int a = 0; a < na; ++a)
      if (s.steplength == h->prm.alphas[a]) {
        k = a + 1;
        break;
      }
    t.push_back(k);
  }
  if (t.empty()) return;
  // (in whole rounds of resident workgroups: a launch with one workgroup more than the
  // slots takes two trial-times)
  const double S = h->ls_slots;
  double best = 0.;
  int best_g = 1;
  for (int g : {1, 2, 4}) {
    double time = 0.;
    if (g == 1) {
      double w = 0.;
      int tmax = 0;
      for (int v : t) w += v, tmax = std::max(tmax, v);
      time = std::max(std::ceil(w / S), (double)tmax);
    } else {
      for (int k0 = 0; k0 < na; k0 += g) {
        const int slots = std::min(g, na - k0);
        double u = 0.;
        for (int v : t) u += v > k0 ? slots : 0;
        if (u > 0.) time += std::ceil(u / S);
      }
    }
    if (g == 1 || time < best) best = time, best_g = g;
  }
  h->D.npar = best_g;
  h->npar_chosen = true;
}

// Longest-processing-time-first dispatch of the next line search: the rollout's
// workgroups map to the elements in descending order of their last line search's trial
// count (the fixed MPC protocol repeats it exactly; a heuristic otherwise). Each element's
// work is unchanged, so are its results. A simulation of the C5 walk's trial histogram on
// 512 resident workgroups: 8 trial-lengths in element order, 6 longest-first (ideal 5.1).
static int update_ls_order(fddp_handle* h, const std::vector<ElemState>& st) {
  Dev& D = h->D;
  const int B = D.B, na = h->prm.n_alphas;
  if (B < 2 || h->fast) return FDDP_OK;
  if (!D.ls_order) {
    double* p = nullptr;
    int rc;
    if ((rc = dalloc(h, &p, (B + 1) / 2))) return rc;
    D.ls_order = (const int*)p;
  }
  std::vector<int> key(B);
  for (int b = 0; b < B; ++b) {
    const ElemState& s = st[b];
    int k = 0;
    if (s.n_iter_run > 0) {
      k = na;
      for (int a = 0; a < na; ++a)
        if (s.steplength == h->prm.alphas[a]) {
          k = a + 1;
          break;
        }
    }
    key[b] = k;
  }
  h->h_order.resize(B);
  for (int b = 0; b < B; ++b) h->h_order[b] = b;
  std::stable_sort(h->h_order.begin(), h->h_order.end(), [&](int x, int y) { return key[x] > key[y]; });
  HIP_TRY(hipMemcpyAsync((void*)D.ls_order, h->h_order.data(), sizeof(int) * B, hipMemcpyHostToDevice, h->stream));
  return FDDP_OK;
}

int launch_forward(fddp_handle* h, int mode, double alpha, int* count) {
  Timed tm(h, 3);
  const Dev& D = h->D;
  if (!h->fast && mode == 0 && D.npar > 1) {
    // the line search in groups of npar trials evaluated together; every group
    // is launched (decided elements exit at once), so there is no host round trip
    int rc;
    if ((rc = ensure_par_slots(h))) return rc;
    const int na = h->prm.n_alphas, G = (na + D.npar - 1) / D.npar;
    h->ls_npar_last = D.npar;
    h->ls_launches_last = G;
    const int v = rollout_variant(h);
    for (int g = 0; g < G; ++g) {
      KLAUNCH(ktab::forward(v, dim3(D.B, D.npar), h->fwd_smem, h->stream, D, to_prm(h->prm), 2, 1., nullptr, h->pcap,
                            g));
      KLAUNCH(ktab::ls_select(dim3(D.B), h->stream, D, to_prm(h->prm), g, g == G - 1 ? 1 : 0, count));
    }
    return FDDP_OK;
  }
  if (mode == 0) {
    h->ls_npar_last = 1;
    h->ls_launches_last = 1;
  }
  if (h->fast)
    KLAUNCH(ktab::forward(ktab::FWD_FAST, dim3(D.B), h->fwd_fast_smem, h->stream, D, to_prm(h->prm), mode, alpha,
                          count, h->pcap, 0));
  else
    KLAUNCH(ktab::forward(rollout_variant(h), dim3(D.B), h->fwd_smem, h->stream, D,
                          to_prm(h->prm), mode, alpha, count, h->pcap, 0));
  return FDDP_OK;
}

__global__ void set_feasible_kernel(Dev D, int is_feasible) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < D.B) D.st[b].is_feasible = is_feasible;
}
__global__ void ei_kernel(Dev D, double* out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= D.B) return;
  ElemState& s = D.st[b];
  s.d0 = s.dg + s.dv;
  s.d1 = s.dq - 2 * s.dv;
  out[2 * b] = s.d0;
  out[2 * b + 1] = s.d1;
}
__global__ void step_state_kernel(Dev D, int iter, double xreg, double ureg, int was_feasible) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= D.B) return;
  ElemState& s = D.st[b];
  s.iter = iter;
  s.xreg = xreg;
  s.ureg = ureg;
  s.was_feasible = was_feasible;
}

int download_states(fddp_handle* h, std::vector<ElemState>& v) {
  v.resize(h->dims.B);
  HIP_TRY(hipMemcpyAsync(v.data(), h->D.st, sizeof(ElemState) * h->dims.B, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return FDDP_OK;
}

void fill_result(const ElemState& s, fddp_result* r) {
  r->status = s.status;
  r->iter = s.iter;
  r->is_feasible = s.is_feasible;
  r->n_iter_run = s.n_iter_run;
  r->cost = s.cost;
  r->stop = s.stop;
  r->xreg = s.xreg;
  r->ureg = s.ureg;
  r->steplength = s.steplength;
  r->dV = s.dV;
  r->dVexp = s.dVexp;
  r->d0 = s.d0;
  r->d1 = s.d1;
}

int gather_traj(fddp_handle* h, int which, int other_buf, double* out, int on_device) {
  const Dev& D0 = h->D;
  Dev D = D0;
  if (other_buf) {  // view the trial buffer as current: swap the pointers
    std::swap(D.xs[0], D.xs[1]);
    std::swap(D.us[0], D.us[1]);
  }
  const int64_t len = which == 0 ? (int64_t)D.B * (D.T + 1) * D.nx : (int64_t)D.B * D.T * D.m;
  double* dst = on_device ? out : h->staging;
  hipLaunchKernelGGL(gather_traj_kernel, dim3(8, D.B), dim3(256), 0, h->stream, D, which, dst);
  LAUNCH_CHECK();
  if (!on_device) {
    HIP_TRY(hipMemcpyAsync(out, h->staging, sizeof(double) * len, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
  }
  return FDDP_OK;
}

}  // namespace

extern "C" {

const char* fddp_last_error(void) { return g_err.c_str(); }

void fddp_default_params(fddp_params* p) {
  // ddp.cpp:15-37 ; fddp.cpp:14-15 ; solver-base.cpp:24-25
  p->th_acceptstep = 0.1;
  p->th_stop = 1e-9;
  p->th_grad = 1e-12;
  p->th_stepdec = 0.5;
  p->th_stepinc = 0.01;
  p->th_acceptnegstep = 2.;
  p->regfactor = 10.;
  p->regmin = 1e-9;
  p->regmax = 1e9;
  p->n_alphas = 10;
  p->pad_ = 0;
  for (int i = 0; i < 16; ++i) p->alphas[i] = i < 10 ? 1. / std::pow(2., (double)i) : 0.;
}

namespace {

// Knot-dependent device state of a handle: LDS plans and the fast-path
// choice, the parameter pool, the knot descriptors, the knot segments of the
// tiled calc, and the Riccati sweep variant (fddp_create, fddp_set_knots).
int apply_knots(fddp_handle* h, const fddp_knot_desc* knots, const double* params, int64_t n_params) {
  Dev& D = h->D;
  const fddp_dims& d = h->dims;
  const int64_t K1 = (int64_t)d.T + 1;
  int rc;
  h->knots.assign(knots, knots + K1);
  {
    int64_t pmax = 0;
    int mb_nj = 0, mb_njac = 0, mb_nc = 0;
    bool mb_vcols = false;
    int mb_nu = 0, mb_nrows = 0;
    // each multibody block's own shape: the device lays out a knot's calcDiff LDS from its
    // own block, so the plan to allocate is the largest knot's, not the plan of the largest
    // value of every parameter (on the Solo12 trot those come from different knots: 82.2 KB,
    // one workgroup per CU, against the largest knot's 79.6 KB)
    struct MbShape {
      int nj, njac, nc, nu, nrows;
      bool vcols;
    };
    std::vector<MbShape> shapes;
    h->has_mb = false;
    for (int t = 0; t <= d.T; ++t) {
      int64_t sz;
      if (is_mb_kind(knots[t].kind)) {
        h->has_mb = true;
        sz = 0;
        const int nb = knots[t].param_stride > 0 ? d.B : 1;
        for (int b = 0; b < nb; ++b) {  // validated by check_knots
          const int64_t off = knots[t].param_offset + (int64_t)b * knots[t].param_stride;
          std::string why;
          MbShape k{0, 0, 0, 0, 0, false};
          sz = std::max(sz, mb_block_check(params + off, n_params - off, knots[t].kind, d.nx, knots[t].nu, why, &k.nj,
                                           &k.njac, &k.nc, &k.vcols, &k.nu, &k.nrows));
          mb_nj = std::max(mb_nj, k.nj);
          mb_njac = std::max(mb_njac, k.njac);
          mb_nc = std::max(mb_nc, k.nc);
          mb_vcols = mb_vcols || k.vcols;
          mb_nu = std::max(mb_nu, k.nu);
          mb_nrows = std::max(mb_nrows, k.nrows);
          bool seen = false;
          for (const MbShape& q : shapes)
            seen = seen || (q.nj == k.nj && q.njac == k.njac && q.nc == k.nc && q.nu == k.nu && q.nrows == k.nrows &&
                            q.vcols == k.vcols);
          if (!seen) shapes.push_back(k);
        }
      } else {
        sz = block_doubles(knots[t].kind, d.nx, knots[t].nu);
      }
      pmax = std::max<int64_t>(pmax, sz);
    }
    h->all_mb = true;
    for (int t = 0; t <= d.T; ++t) h->all_mb = h->all_mb && is_mb_kind(knots[t].kind);
    D.mbw = h->has_mb ? pad2(fddp::mb::calc_work_doubles(mb_nj, mb_nc)) : 0;
    D.mbw_fwd = h->has_mb ? pad2(fddp::mb::calc_dense_doubles(mb_nj, mb_nc)) : 0;
    h->mb_nj = mb_nj;
    // parallel line-search trials: they pay on the large trees (C5 Talos, nv = 38:
    // forward -12 %), where one rollout keeps a CU busy longest; on small ones (C4
    // Solo12, nv = 18) the extra trials cost more than the shorter chains save
    // (a re-application of the knots — fddp_set_knots, the MPC loop's circularAppend —
    // keeps the size chosen from the last line search's trial counts: resetting it every
    // step cost the C5 shift protocol's rollout 52.3 -> 65.8 ms)
    if (!(h->npar_chosen && h->has_mb && !h->npar_env))
      D.npar = h->npar_env ? h->npar_env : (h->has_mb && mb_nj >= 24 ? 4 : 1);
    h->npar_adapt = !h->npar_env && h->has_mb;
    int64_t mb_pmax = 0;  // largest multibody parameter block (staged in LDS by mb_knot_kernel)
    for (int t = 0; t <= d.T; ++t)
      if (is_mb_kind(knots[t].kind)) {
        const int nb = knots[t].param_stride > 0 ? d.B : 1;
        for (int b = 0; b < nb; ++b)
          mb_pmax = std::max<int64_t>(mb_pmax, (int64_t)params[knots[t].param_offset + (int64_t)b * knots[t].param_stride + 3]);
      }
    // the calcDiff's LDS plan: spilled to the output blocks where the all-LDS plan would
    // leave room for one workgroup per CU only (multibody.hpp diff_spill; FDDP_MB_SPILL=0
    // forces the all-LDS plan, for A/B runs)
    static const int spill_env = [] {
      const char* e = std::getenv("FDDP_MB_SPILL");
      return e ? std::atoi(e) : -1;
    }();
    auto plan_doubles = [&](int spill) {  // the largest knot's plan under spill flags `spill`
      int64_t mx = 0;
      for (const MbShape& q : shapes)
        mx = std::max<int64_t>(mx, pad2(fddp::mb::diff_layout(q.nj, q.njac, q.nc, q.vcols, q.nu, q.nrows, spill).total));
      return mx;
    };
    // (the spill flags themselves from the largest value of every parameter: the spilled
    // arrays must fit their output blocks on every knot)
    D.mbspill = h->has_mb && spill_env != 0 && (plan_doubles(0) + pad2(mb_pmax)) * 8 > 80 * 1024
                    ? fddp::mb::diff_spill(mb_nj, mb_njac, mb_nc, mb_vcols, mb_nu, mb_nrows, mb_pmax, D.m)
                    : 0;
    D.mbd = h->has_mb ? plan_doubles(D.mbspill) : 0;
    h->mb_diff_smem = h->has_mb ? sizeof(double) * (D.mbd + pad2(mb_pmax)) : 0;
    const int64_t budget = (150 * 1024) / 8 - (2 * D.sX + D.sM + 2 * D.sN + 5 * (kNT / kWave) + 16) - D.mbw;
    // LDS-staged parameter blocks up to pcap doubles; larger (dense) blocks are read from
    // global memory. The multibody calc reads its block from LDS only (knots.hpp), so
    // pcap covers at least the largest multibody block.
    h->pcap = pmax <= budget ? pad2(pmax) : (pad2(mb_pmax) <= budget ? pad2(mb_pmax) : 0);
    if (h->has_mb && h->pcap < pad2(mb_pmax))
      return fail(FDDP_ERR_INVALID_ARG, "multibody parameter blocks exceed the LDS budget of the calc / rollout kernels");
  }
  // (dx in the tail of the calc's scratch when the gains' K staging leaves room: on the C5 walk
  // that takes the rollout's LDS to 52.6 KB, three workgroups per CU; the LDS is allocated in
  // 2 KB granules (measured: tools/occ_probe.hip), which the occupancy API does not model)
  D.dxv_mbw = D.mbw_fwd >= (int64_t)D.m * D.n + 2 * D.sN ? 1 : 0;
  h->fwd_smem = sizeof(double) * (h->pcap + fwd_lds_doubles<kNT, false>(D.sX, D.sN, D.sM) - (D.dxv_mbw ? 2 * D.sN : 0) +
                                  D.mbw_fwd);
  h->fwd_mb_variant = -1;  // (re-chosen with the new LDS size)
  h->ls_slots = 0.;
  h->calc_smem = sizeof(double) * (h->pcap + 2 * D.sX + D.sM + 5 * (kNT / kWave) + 16 + D.mbw);
  h->cdiff_smem = sizeof(double) * (h->pcap + D.sX + D.sM);
  {  // dense-knot fast path: every knot LQR / Euler∘DiffLQR, block LDS-resident
    bool dense = h->pcap > 0 && d.nx == d.ndx && d.nx <= kNT && d.nu_max <= kNT;
    for (int t = 0; t <= d.T; ++t)
      dense = dense && (knots[t].kind == FDDP_KNOT_LQR || knots[t].kind == FDDP_KNOT_EULER_DIFFLQR);
    h->fused_smem = sizeof(double) * (h->pcap + calc_tiled_lds(D.sX, D.sM));
    h->fwd_fast_smem = sizeof(double) * (h->pcap + fwd_lds_doubles<kNT, true>(D.sX, D.sN, D.sM));
    const char* env = std::getenv("FDDP_FAST");
    const bool off = env && env[0] == '0';
    h->fast = dense && !off && h->fused_smem <= 160 * 1024 && h->fwd_fast_smem <= 160 * 1024;
  }
  if (n_params > h->params_cap) {  // the old pool stays owned by the handle until fddp_destroy
    double* p = nullptr;
    if ((rc = dalloc(h, &p, n_params))) return rc;
    D.params = p;
    h->params_cap = n_params;
  }
  h->n_params = n_params;
  HIP_TRY(hipMemcpyAsync((void*)D.params, params, sizeof(double) * n_params, hipMemcpyHostToDevice, h->stream));
  if (!D.knots) {
    fddp_knot_desc* kd = nullptr;
    if ((rc = dalloc(h, (double**)&kd, (sizeof(fddp_knot_desc) * K1 + 7) / 8))) return rc;
    D.knots = kd;
  }
  HIP_TRY(hipMemcpyAsync((void*)D.knots, knots, sizeof(fddp_knot_desc) * K1, hipMemcpyHostToDevice, h->stream));
  {  // knot segments: runs of knots with the same desc and parameter block
     // (running runs stop before the terminal knot), for the tiled calc
    std::vector<int> se(d.T + 1);
    for (int t = d.T; t >= 0; --t) {
      const bool same = t + 1 < d.T && knots[t + 1].kind == knots[t].kind && knots[t + 1].nu == knots[t].nu &&
                        knots[t + 1].param_offset == knots[t].param_offset &&
                        knots[t + 1].param_stride == knots[t].param_stride;
      se[t] = same ? se[t + 1] : t + 1;
    }
    if (!D.segend) {
      double* sp = nullptr;
      if ((rc = dalloc(h, &sp, (d.T + 2) / 2 + 1))) return rc;
      D.segend = (const int*)sp;
    }
    HIP_TRY(hipMemcpyAsync((void*)D.segend, se.data(), sizeof(int) * se.size(), hipMemcpyHostToDevice, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));  // the host staging vectors go out of scope
  }
  {  // dynamic LDS of every kernel the handle may launch (a refusal names the kernel and size)
    struct Req {
      const void* f;
      size_t bytes;
      bool use;
      const char* name;
    } reqs[] = {
        {ktab::backward_generic_fn(), h->bwd_smem, true, "backward_kernel"},
        {ktab::forward_fn(ktab::FWD_GENERIC), h->fwd_smem, true, "forward_kernel"},
        {ktab::forward_fn(ktab::FWD_FAST), h->fwd_fast_smem, true, "forward_kernel<fast>"},
        {ktab::forward_fn(ktab::FWD_MB), h->fwd_smem, h->has_mb, "forward_kernel<multibody>"},
        {ktab::forward_fn(ktab::FWD_MB2), h->fwd_smem, h->has_mb, "forward_kernel<multibody, 2 waves/EU>"},
        {ktab::calc_tiled_fn(), h->fused_smem, true, "calc_tiled_kernel"},
        {ktab::calc_fn(), h->calc_smem, true, "calc_kernel"},
        {ktab::calc_diff_fn(), h->cdiff_smem, true, "calc_diff_kernel"},
        {ktab::mb_knot_fn(ktab::MB_W2), h->mb_diff_smem, h->has_mb, "mb_knot_kernel"},
        {ktab::mb_knot_fn(ktab::MB_W1), h->mb_diff_smem, h->has_mb, "mb_knot_kernel_w1"},
        {ktab::mb_knot_fn(ktab::MB_X8), h->mb_diff_smem, h->has_mb, "mb_knot_kernel_x8"},
        {ktab::mb_knot_fn(ktab::MB_X2), h->mb_diff_smem, h->has_mb, "mb_knot_kernel_x2"},
        {ktab::mb_knot_fn(ktab::MB_S2), h->mb_diff_smem, h->has_mb, "mb_knot_kernel_s2"},
    };
    for (const Req& r : reqs) {
      if (!r.use) continue;
      const hipError_t e = hipFuncSetAttribute(r.f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)r.bytes);
      if (e != hipSuccess)
        return fail(FDDP_ERR_RUNTIME, std::string("hipFuncSetAttribute(dynamic LDS) of ") + r.name + ": " +
                                          std::to_string(r.bytes) + " bytes: " + hipGetErrorString(e));
    }
  }
  {  // backward sweep variant: MFMA tiles when every running knot has nu == nu_max, or on
    // multibody horizons (their calcDiff zero-fills the Fu columns beyond a knot's nu, so
    // the sweep runs a knot on its own nu: the impulse knots of the gaits)
    bool uniform_nu = d.nu_max > 0;
    for (int t = 0; t < d.T; ++t) uniform_nu = uniform_nu && knots[t].nu == d.nu_max;
    uniform_nu = uniform_nu || (h->all_mb && d.nu_max > 0);
    const char* env = std::getenv("FDDP_BACKWARD");
    const bool force_generic = env && std::strcmp(env, "generic") == 0;
    const int ntl = (d.ndx + 15) / 16, mtl = (d.nu_max + 15) / 16;
    int v = -1;
    if (uniform_nu && !force_generic) {
      // eight waves per element, the fastest knot (measured round 4: one wave (C3) or four
      // (C2) per element are slower, 12.1 / 1.06 ms against 3.6 / 0.89 ms), unless the
      // four-wave plan keeps more elements resident: the sweep is a serial chain per
      // element, so its time goes with the rounds of resident workgroups, ceil(B / slots),
      // and a four-wave knot takes ~1.15x an eight-wave one (C3, B = 512 on 256 CUs: two
      // four-wave workgroups per CU, one round, 3.20 -> 2.16 ms; C4 and C2 keep eight).
      // FDDP_BWD_WAVES=1|4|8 overrides.
      const char* ew = std::getenv("FDDP_BWD_WAVES");
      int nw = 8;
      if (ew) nw = ew[0] == '1' ? 1 : (ew[0] == '4' ? 4 : 8);
      // one-wave plans exist for the small shapes (NTL + MTL <= 4, MTL = 1); four-wave
      // plans where C^T has its own LDS area (else C^T over Zu needs the 8-wave plan's
      // late LDS-DMA); everything else runs eight waves (ktab::backward_mfma_setup)
      const bool known = (ntl == 5 && mtl == 2) || (mtl == 1 && ntl >= 1 && ntl <= 3);
      if (known) {
        if (nw == 1 && !(ntl + mtl <= 4 && mtl == 1)) nw = 8;
        int occ = 0;
        v = ktab::backward_mfma_setup(ntl, mtl, nw, d.ndx, &occ);
        if (v < 0 && nw == 4) v = ktab::backward_mfma_setup(ntl, mtl, 8, d.ndx, &occ);
        if (!ew && v > 0 && mtl == 1) {
          int cus = 0, occ4 = 0;
          (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device);
          const int v4 = ktab::backward_mfma_setup(ntl, mtl, 4, d.ndx, &occ4);
          if (v4 > 0 && cus > 0 && occ > 0 && occ4 > 0) {
            const int64_t r8 = (d.B + (int64_t)cus * occ - 1) / ((int64_t)cus * occ);
            const int64_t r4 = (d.B + (int64_t)cus * occ4 - 1) / ((int64_t)cus * occ4);
            if (1.2 * (double)r4 < (double)r8) v = v4;
          }
        }
      }
    }
    h->bwd_variant = v > 0 ? v : 0;
  }
  return FDDP_OK;
}

}  // namespace

int fddp_create(const fddp_dims* dims, const fddp_knot_desc* knots, const double* params, int64_t n_params,
                int device, fddp_handle** out) {
  g_err.clear();
  if (!dims || !knots || !params || !out) return fail(FDDP_ERR_INVALID_ARG, "fddp_create: null argument");
  *out = nullptr;
  const fddp_dims d = *dims;
  if (d.T < 1 || d.B < 1 || d.nx < 1 || d.nu_max < 0)
    return fail(FDDP_ERR_INVALID_ARG, "fddp_create: T, B, nx must be positive");
  if (d.nx != d.ndx) {  // StateMultibody with a free-flyer root: nq = nv + 1, ndx = 2 nv (multibody.hxx:16-17)
    if (d.nx != d.ndx + 1 || d.ndx % 2 || d.ndx < 12)
      return fail(FDDP_ERR_UNSUPPORTED, "fddp_create: nx != ndx is supported for free-flyer states (nx = ndx + 1)");
    for (int t = 0; t <= d.T; ++t)
      if (!is_mb_kind(knots[t].kind))
        return fail(FDDP_ERR_INVALID_ARG, "fddp_create: a free-flyer state needs multibody knots");
  }
  if (d.B > 65535) return fail(FDDP_ERR_INVALID_ARG, "fddp_create: B > 65535 per handle");
  {
    const int rc0 = check_knots(d, knots, params, n_params, "fddp_create", true);
    if (rc0) return rc0;
  }

  int ndev = 0;
  const hipError_t ce = hipGetDeviceCount(&ndev);
  if (ce != hipSuccess || ndev == 0) {
    int rtv = 0;
    (void)hipRuntimeGetVersion(&rtv);
    return fail(FDDP_ERR_NO_DEVICE, std::string("fddp_create: no HIP device visible (") + hipGetErrorString(ce) +
                                        ", runtime " + std::to_string(rtv) + ")");
  }
  if (device < 0 || device >= ndev) return fail(FDDP_ERR_INVALID_ARG, "fddp_create: bad device index");
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(FDDP_ERR_UNSUPPORTED, std::string("fddp_create: device is ") + prop.gcnArchName +
                                          ", libfddp_hip is built for gfx950 (MI355X) only");

  DeviceGuard g(device);
  auto* h = new fddp_handle_s();
  h->dims = d;
  h->device = device;
  fddp_default_params(&h->prm);
  int rc;
  auto bail = [&](int code) {
    fddp_destroy(h);
    return code;
  };
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess)
    return bail(fail(FDDP_ERR_RUNTIME, "hipStreamCreate failed"));

  Dev& D = h->D;
  std::memset(&D, 0, sizeof(D));
  D.nx = d.nx;
  D.n = d.ndx;
  D.m = d.nu_max;
  D.T = d.T;
  D.B = d.B;
  D.sX = pad2(d.nx);
  D.sN = pad2(d.ndx);
  D.sM = pad2(d.nu_max > 0 ? d.nu_max : 1);
  D.sNN = pad2((int64_t)d.ndx * d.ndx);
  D.sNM = pad2((int64_t)d.ndx * (d.nu_max > 0 ? d.nu_max : 1));
  D.sMM = pad2((int64_t)d.nu_max * d.nu_max > 0 ? (int64_t)d.nu_max * d.nu_max : 1);
  // line-search trials evaluated together per element on the generic (multibody)
  // path: the same trials and the same choice as the serial search, fewer serial
  // rollouts for the elements that backtrack (CROCODDYL_AMD_LS_PAR = 1 is serial)
  D.npar = 1;
  D.ls_order = nullptr;
  if (const char* e = std::getenv("CROCODDYL_AMD_LS_PAR")) D.npar = h->npar_env = std::max(1, std::min(16, std::atoi(e)));
  const int64_t B = d.B, K1 = (int64_t)d.T + 1, K0 = d.T;
  {  // SolverBoxFDDP's qp_(nu, 100, 0.1, 1e-5, 0.) (box-fddp.cpp:16); unused until BOXFDDP
    fddp_boxqp_params bp;
    fddp_boxqp_default_params(&bp);
    bp.th_grad = 1e-5;
    bp.reg = 0.;
    D.boxcfg = to_boxcfg(bp);
  }

  h->bwd_smem = BwdSmem::bytes(D.n, D.m, false);
  if (h->bwd_smem > 160 * 1024) {
    h->bwd_smem = BwdSmem::bytes(D.n, D.m, true);
    if (h->bwd_smem > 160 * 1024)
      return bail(fail(FDDP_ERR_UNSUPPORTED, "fddp_create: (ndx, nu_max) too large for the Riccati sweep"));
    if ((rc = dalloc(h, &D.bwork, (int64_t)d.B * BwdSmem::work_doubles(D.n, D.m)))) return bail(rc);
  }
  struct A {
    double** p;
    int64_t n;
  } plan[] = {
      {&D.x0, B * D.sX},          {&D.xs[0], B * K1 * D.sX}, {&D.xs[1], B * K1 * D.sX}, {&D.us[0], B * K0 * D.sM},
      {&D.us[1], B * K0 * D.sM},  {&D.xnext[0], B * K0 * D.sX}, {&D.xnext[1], B * K0 * D.sX},
      {&D.kcost[0], B * K1},      {&D.kcost[1], B * K1},     {&D.Fx, B * K1 * D.sNN},   {&D.Fu, B * K1 * D.sNM},
      {&D.Lxx, B * K1 * D.sNN},   {&D.Lxu, B * K1 * D.sNM},  {&D.Luu, B * K1 * D.sMM},  {&D.Lx, B * K1 * D.sN},
      {&D.Lu, B * K1 * D.sM},     {&D.fs, B * K1 * D.sN},    {&D.K, B * K0 * D.sNM},    {&D.k, B * K0 * D.sM},
      {&D.Vxxfs, B * K1 * D.sN},  {&D.part, B * K1 * 8},     {&D.dvp, B * K1},
      {&D.zero16, 2},
  };
  for (auto& a : plan)
    if ((rc = dalloc(h, a.p, a.n))) return bail(rc);
  double* stp = nullptr;
  if ((rc = dalloc(h, &stp, (int64_t)(sizeof(ElemState) / 8) * B))) return bail(rc);
  D.st = (ElemState*)stp;
  h->staging_len = std::max<int64_t>(std::max<int64_t>(B * K1 * d.nx, B * K0 * D.sM), B * K1);
  if ((rc = dalloc(h, &h->staging, h->staging_len))) return bail(rc);
  if ((rc = dalloc(h, &h->d_out, 2 * B))) return bail(rc);
  double* cnt = nullptr;
  if ((rc = dalloc(h, &cnt, 1))) return bail(rc);
  h->d_count = (int*)cnt;
  if (hipHostMalloc((void**)&h->h_count, sizeof(int)) != hipSuccess)
    return bail(fail(FDDP_ERR_RUNTIME, "hipHostMalloc"));

  // SolverAbstract constructor state (solver-base.cpp:14-26): xreg = ureg = NaN
  std::vector<ElemState> st0(B);
  for (auto& s : st0) {
    std::memset(&s, 0, sizeof(s));
    s.xreg = NAN;
    s.ureg = NAN;
    s.steplength = 1.;
  }
  if (hipMemcpyAsync(D.st, st0.data(), sizeof(ElemState) * B, hipMemcpyHostToDevice, h->stream) != hipSuccess)
    return bail(fail(FDDP_ERR_RUNTIME, "upload state"));
  if ((rc = apply_knots(h, knots, params, n_params))) return bail(rc);
  if (const char* e = std::getenv("FDDP_STAMPS")) {
    if (e[0] == '1') {
      double* p2 = nullptr;
      if ((rc = dalloc(h, &p2, (int64_t)d.B * 140))) return bail(rc);
      D.stamps = (unsigned long long*)p2;
    }
  }
  if (hipStreamSynchronize(h->stream) != hipSuccess) return bail(fail(FDDP_ERR_RUNTIME, "sync after create"));
  *out = h;
  return FDDP_OK;
}

void fddp_destroy(fddp_handle* h) {
  if (!h) return;
  DeviceGuard g(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  if (h->D.stamps) {  // diagnostic summary: mean cycles per element per wave and phase
    std::vector<unsigned long long> v((size_t)h->dims.B * 140);
    if (hipMemcpy(v.data(), h->D.stamps, v.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
      const char* names[8] = {"p1_G", "p1_H", "p1_inv", "b1_dma", "p2_K", "p2_Vupd", "b2_p3", "b3_wait"};
      std::fprintf(stderr, "[fddp stamps] mean cycles per element (variant %d):\n", h->bwd_variant);
      for (int w = 0; w < h->bwd_variant % 10; ++w) {
        std::fprintf(stderr, "  wave %d:", w);
        for (int ph = 0; ph < 8; ++ph) {
          double s2 = 0;
          for (int b = 0; b < h->dims.B; ++b) s2 += (double)v[((size_t)b * 8 + w) * 8 + ph];
          std::fprintf(stderr, " %s=%.0f", names[ph], s2 / h->dims.B);
        }
        std::fprintf(stderr, "\n");
      }
      if (h->has_mb || h->fast) {
        const char* mn[5] = {"state", "params", "gains", "calc", "stores_checks"};
        std::fprintf(stderr, "[fddp stamps] %s rollout, wave 0's mean cycles per element (all trials):",
                     h->fast ? "dense fast-path" : "multibody");
        for (int ph = 0; ph < 5; ++ph) {
          double s2 = 0;
          for (int b = 0; b < h->dims.B; ++b) s2 += (double)v[(size_t)h->dims.B * 128 + (size_t)b * 8 + ph];
          std::fprintf(stderr, " %s=%.0f", mn[ph], s2 / h->dims.B);
        }
        std::fprintf(stderr, "\n");
      }
      {  // the rollout's residency: per workgroup (element) of its last launch, the real-time
         // start / end (100 MHz) and the CU it ran on (HW_ID, XCC_ID); the most workgroups one
         // CU held at once, and the mean over the launch
        struct Ev {
          unsigned long long t;
          int d;
        };
        std::vector<std::pair<unsigned long long, std::vector<Ev>>> cus;
        std::vector<std::pair<unsigned long long, std::vector<Ev>>>* pc = &cus;
        unsigned long long t0 = ~0ull, t1 = 0;
        int n = 0;
        for (int b = 0; b < h->dims.B; ++b) {
          const unsigned long long* r = &v[(size_t)h->dims.B * 136 + (size_t)b * 4];
          if (r[0] == 0 || r[2] == 0) continue;
          const unsigned long long hw = r[1];
          // cu: HW_ID cu_id [11:8], sh_id [12], se_id [15:13]; XCC_ID in the high word
          const unsigned long long key = ((hw >> 32) << 16) | ((hw >> 8) & 0xff);
          size_t i = 0;
          while (i < pc->size() && (*pc)[i].first != key) ++i;
          if (i == pc->size()) pc->push_back({key, {}});
          (*pc)[i].second.push_back({r[0], 1});
          (*pc)[i].second.push_back({r[2], -1});
          t0 = std::min(t0, r[0]);
          t1 = std::max(t1, r[2]);
          ++n;
        }
        int most = 0;
        double area = 0.;
        for (auto& c : cus) {
          std::sort(c.second.begin(), c.second.end(), [](const Ev& a, const Ev& b) { return a.t < b.t || (a.t == b.t && a.d < b.d); });
          int cur = 0;
          for (size_t k = 0; k < c.second.size(); ++k) {
            cur += c.second[k].d;
            most = std::max(most, cur);
            if (k + 1 < c.second.size()) area += (double)cur * (double)(c.second[k + 1].t - c.second[k].t);
          }
        }
        if (n > 0)
          std::fprintf(stderr,
                       "[fddp stamps] rollout residency: %d workgroups on %zu CUs, at most %d on one CU, mean %.2f per used "
                       "CU over the launch (%.3f ms)\n",
                       n, cus.size(), most, area / ((double)(t1 - t0) * (double)cus.size()), (t1 - t0) * 1e-5);
      }
      if (h->fast) {
        const char* fn[8] = {"stage", "compute", "-", "-", "-", "blocks", "-", "-"};
        std::fprintf(stderr, "[fddp stamps] fused calc/calcDiff, mean cycles per element:\n");
        for (int w = 0; w < 8; ++w) {
          std::fprintf(stderr, "  wave %d:", w);
          for (int ph = 0; ph < 8; ++ph) {
            double s2 = 0;
            for (int b = 0; b < h->dims.B; ++b) s2 += (double)v[(size_t)h->dims.B * 64 + ((size_t)b * 8 + w) * 8 + ph];
            std::fprintf(stderr, " %s=%.0f", fn[ph], s2 / h->dims.B);
          }
          std::fprintf(stderr, "\n");
        }
      }
    }
  }
  for (void* p : h->allocs) (void)hipFree(p);
  for (auto& r : h->ev_rec) {
    (void)hipEventDestroy(r.second.first);
    (void)hipEventDestroy(r.second.second);
  }
  for (auto e : h->ev_pool) (void)hipEventDestroy(e);
  if (h->h_count) (void)hipHostFree(h->h_count);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

int fddp_set_model_params(fddp_handle* h, const double* params, int64_t n_params) {
  if (!h || !params || n_params != h->n_params) return fail(FDDP_ERR_INVALID_ARG, "fddp_set_model_params: size");
  DeviceGuard g(h->device);
  if (h->has_mb) {  // variable-size multibody blocks: re-validate and re-plan the LDS
    int rc;
    if ((rc = check_knots(h->dims, h->knots.data(), params, n_params, "fddp_set_model_params", false))) return rc;
    HIP_TRY(hipStreamSynchronize(h->stream));
    const std::vector<fddp_knot_desc> kn = h->knots;
    return apply_knots(h, kn.data(), params, n_params);
  }
  HIP_TRY(hipMemcpyAsync((void*)h->D.params, params, sizeof(double) * n_params, hipMemcpyHostToDevice, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return FDDP_OK;
}

int fddp_set_x0(fddp_handle* h, const double* x0) {
  if (!h || !x0) return fail(FDDP_ERR_INVALID_ARG, "fddp_set_x0: null");
  DeviceGuard g(h->device);
  const Dev& D = h->D;
  HIP_TRY(hipMemcpy2DAsync(D.x0, sizeof(double) * D.sX, x0, sizeof(double) * D.nx, sizeof(double) * D.nx, D.B,
                           hipMemcpyHostToDevice, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return FDDP_OK;
}

int fddp_get_x0(fddp_handle* h, double* x0) {
  if (!h || !x0) return fail(FDDP_ERR_INVALID_ARG, "fddp_get_x0: null");
  DeviceGuard g(h->device);
  const Dev& D = h->D;
  HIP_TRY(hipMemcpy2DAsync(x0, sizeof(double) * D.nx, D.x0, sizeof(double) * D.sX, sizeof(double) * D.nx, D.B,
                           hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return FDDP_OK;
}

int fddp_set_params(fddp_handle* h, const fddp_params* p) {
  if (!h || !p) return fail(FDDP_ERR_INVALID_ARG, "fddp_set_params: null");
  // validation as the reference setters
  if (0. >= p->th_acceptstep || p->th_acceptstep > 1)
    return fail(FDDP_ERR_INVALID_ARG, "th_acceptstep value should between 0 and 1.");  // solver-base.cpp:159-165
  if (p->th_stop <= 0.) return fail(FDDP_ERR_INVALID_ARG, "th_stop value has to higher than 0.");  // :167-173
  if (0. > p->th_grad) return fail(FDDP_ERR_INVALID_ARG, "th_grad value has to be positive.");    // ddp.cpp:480-486
  if (0. >= p->th_stepdec || p->th_stepdec > 1.)
    return fail(FDDP_ERR_INVALID_ARG, "th_stepdec value should between 0 and 1.");  // ddp.cpp:464-470
  if (0. >= p->th_stepinc || p->th_stepinc > 1.)
    return fail(FDDP_ERR_INVALID_ARG, "th_stepinc value should between 0 and 1.");  // ddp.cpp:472-478
  if (0. > p->th_acceptnegstep)
    return fail(FDDP_ERR_INVALID_ARG, "th_acceptnegstep value has to be positive.");  // fddp.cpp:229-235
  if (p->regfactor <= 1.) return fail(FDDP_ERR_INVALID_ARG, "regfactor value is higher than 1.");  // ddp.cpp:420-426
  if (0. > p->regmin) return fail(FDDP_ERR_INVALID_ARG, "regmin value has to be positive.");
  if (0. > p->regmax) return fail(FDDP_ERR_INVALID_ARG, "regmax value has to be positive.");
  if (p->n_alphas < 1 || p->n_alphas > 16) return fail(FDDP_ERR_INVALID_ARG, "n_alphas must be in [1, 16]");
  for (int i = 1; i < p->n_alphas; ++i) {  // ddp.cpp:444-462
    if (0. >= p->alphas[i]) return fail(FDDP_ERR_INVALID_ARG, "alpha values has to be positive.");
    if (p->alphas[i] >= p->alphas[i - 1])
      return fail(FDDP_ERR_INVALID_ARG, "alpha values are monotonously decreasing.");
  }
  h->prm = *p;
  return FDDP_OK;
}

int fddp_get_params(fddp_handle* h, fddp_params* p) {
  if (!h || !p) return fail(FDDP_ERR_INVALID_ARG, "fddp_get_params: null");
  *p = h->prm;
  return FDDP_OK;
}

int fddp_set_candidate(fddp_handle* h, const double* xs, const double* us, int is_feasible) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "fddp_set_candidate: null handle");
  DeviceGuard g(h->device);
  const Dev& D = h->D;
  const int64_t lx = (int64_t)D.B * (D.T + 1) * D.nx, lu = (int64_t)D.B * D.T * D.m;
  if (xs) HIP_TRY(hipMemcpyAsync(h->staging, xs, sizeof(double) * lx, hipMemcpyHostToDevice, h->stream));
  hipLaunchKernelGGL(scatter_traj_kernel, dim3(8, D.B), dim3(256), 0, h->stream, D, 0, h->staging, xs ? 0 : 1);
  LAUNCH_CHECK();
  if (D.m > 0) {
    if (us) HIP_TRY(hipMemcpyAsync(h->staging, us, sizeof(double) * lu, hipMemcpyHostToDevice, h->stream));
    hipLaunchKernelGGL(scatter_traj_kernel, dim3(8, D.B), dim3(256), 0, h->stream, D, 1, h->staging, us ? 0 : 1);
    LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(set_feasible_kernel, dim3((D.B + 255) / 256), dim3(256), 0, h->stream, D, is_feasible ? 1 : 0);
  LAUNCH_CHECK();
  HIP_TRY(hipStreamSynchronize(h->stream));
  return FDDP_OK;
}

int fddp_set_candidate_device(fddp_handle* h, const double* xs, const double* us, int is_feasible) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "fddp_set_candidate_device: null handle");
  DeviceGuard g(h->device);
  const Dev& D = h->D;
  hipLaunchKernelGGL(scatter_traj_kernel, dim3(8, D.B), dim3(256), 0, h->stream, D, 0, xs, xs ? 0 : 1);
  LAUNCH_CHECK();
  if (D.m > 0) {
    hipLaunchKernelGGL(scatter_traj_kernel, dim3(8, D.B), dim3(256), 0, h->stream, D, 1, us, us ? 0 : 1);
    LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(set_feasible_kernel, dim3((D.B + 255) / 256), dim3(256), 0, h->stream, D, is_feasible ? 1 : 0);
  LAUNCH_CHECK();
  return FDDP_OK;
}

int fddp_solve(fddp_handle* h, int maxiter, int is_feasible, double reg_init, fddp_result* out) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "fddp_solve: null handle");
  if (h->in_solve) return fail(FDDP_ERR_INVALID_ARG, "fddp_solve: called from its own iteration callback");
  if (maxiter < 0) return fail(FDDP_ERR_INVALID_ARG, "fddp_solve: maxiter < 0");
  DeviceGuard g(h->device);
  static const bool box_stats = getenv("FDDP_BOX_STATS") && atoi(getenv("FDDP_BOX_STATS")) == 1;
  if (box_stats && h->D.box && !h->D.box_stats) {
    int rc0;
    if ((rc0 = dalloc(h, (double**)&h->D.box_stats, 4))) return rc0;
  }
  if (h->D.box_stats) HIP_TRY(hipMemsetAsync(h->D.box_stats, 0, 4 * sizeof(unsigned long long), h->stream));
  const Dev& D = h->D;
  const double xreg0 = std::isnan(reg_init) ? h->prm.regmin : reg_init;
  hipLaunchKernelGGL(init_state_kernel, dim3((D.B + 255) / 256), dim3(256), 0, h->stream, D, is_feasible ? 1 : 0,
                     xreg0);
  LAUNCH_CHECK();
  int rc;
  // per-iteration callbacks (fddp.cpp:92-98): the states read back after every body
  std::vector<ElemState> cbst;
  std::vector<fddp_result> cbres;
  std::vector<int32_t> cbrep, cbrun(h->cb ? D.B : 0, 0);
  struct InSolve {
    bool& f;
    explicit InSolve(bool& f_) : f(f_) { f = true; }
    ~InSolve() { f = false; }
  } in_solve(h->in_solve);
  for (int it = 0; it < maxiter; ++it) {
    if (it == 0) {
      if ((rc = launch_calc_then_diff(h, SEL_ACTIVE, SEL_ACTIVE, SEL_RECALC, 1))) return rc;
    } else {
      if ((rc = launch_calc_diff(h, SEL_RECALC, 1))) return rc;
    }
    if ((rc = launch_backward(h, 0))) return rc;
    HIP_TRY(hipMemsetAsync(h->d_count, 0, sizeof(int), h->stream));
    if ((rc = launch_forward(h, 0, 1., h->d_count))) return rc;
    if (h->cb) {
      // reported: ran this body (n_iter_run advanced) and did not abort at regmax in it
      if ((rc = download_states(h, cbst))) return rc;
      cbres.resize(D.B);
      cbrep.assign(D.B, 0);
      int any = 0;
      for (int b = 0; b < D.B; ++b) {
        fill_result(cbst[b], &cbres[b]);
        cbrep[b] = (cbst[b].n_iter_run > cbrun[b] && cbst[b].status != FDDP_STATUS_REGMAX) ? 1 : 0;
        if (cbrep[b]) cbres[b].iter = it;  // the loop counter of this body; finished elements keep theirs
        cbrun[b] = cbst[b].n_iter_run;
        any |= cbrep[b];
      }
      const int stop = any ? h->cb(h->cb_user, it, cbres.data(), cbrep.data(), D.B) : 0;
      (void)hipSetDevice(h->device);  // (the callback may have switched devices)
      if (stop) {  // the reference's exception out of the loop body: the state stays at this iteration
        if (out) std::copy(cbres.begin(), cbres.end(), out);
        return fail(FDDP_ERR_CALLBACK_ABORT, "fddp_solve: stopped by the iteration callback at iteration " +
                                                 std::to_string(it));
      }
    }
    if (it + 1 < maxiter) {
      HIP_TRY(hipMemcpyAsync(h->h_count, h->d_count, sizeof(int), hipMemcpyDeviceToHost, h->stream));
      HIP_TRY(hipStreamSynchronize(h->stream));
      if (*h->h_count == 0) break;
    }
  }
  if (out) {
    std::vector<ElemState> st;
    if ((rc = download_states(h, st))) return rc;
    for (int b = 0; b < D.B; ++b) fill_result(st[b], &out[b]);
    choose_npar(h, st);
    if ((rc = update_ls_order(h, st))) return rc;
  } else {
    HIP_TRY(hipStreamSynchronize(h->stream));
  }
  if (D.box_stats) {  // diagnostics: mean Newton iterations / inverses per box QP of this solve
    unsigned long long bs[4];
    HIP_TRY(hipMemcpy(bs, D.box_stats, sizeof(bs), hipMemcpyDeviceToHost));
    fprintf(stderr, "fddp box stats: %llu QPs, %.3f Newton iterations and %.3f inverses per QP\n", bs[0],
            bs[0] ? (double)bs[1] / bs[0] : 0., bs[0] ? (double)bs[2] / bs[0] : 0.);
  }
  return FDDP_OK;
}

int fddp_get_line_search_info(fddp_handle* h, int* group_size, int* launches) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "fddp_get_line_search_info: null handle");
  if (group_size) *group_size = h->ls_npar_last;
  if (launches) *launches = h->ls_launches_last;
  return FDDP_OK;
}

int fddp_set_callback(fddp_handle* h, fddp_iteration_callback cb, void* user) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "fddp_set_callback: null handle");
  if (h->in_solve) return fail(FDDP_ERR_INVALID_ARG, "fddp_set_callback: not from inside a callback");
  h->cb = cb;
  h->cb_user = cb ? user : nullptr;
  return FDDP_OK;
}

int fddp_get_results(fddp_handle* h, fddp_result* out) {
  if (!h || !out) return fail(FDDP_ERR_INVALID_ARG, "fddp_get_results: null");
  DeviceGuard g(h->device);
  std::vector<ElemState> st;
  int rc;
  if ((rc = download_states(h, st))) return rc;
  for (int b = 0; b < h->dims.B; ++b) fill_result(st[b], &out[b]);
  return FDDP_OK;
}

int fddp_get_xs(fddp_handle* h, double* out, int on_device) {
  if (!h || !out) return fail(FDDP_ERR_INVALID_ARG, "fddp_get_xs: null");
  DeviceGuard g(h->device);
  return gather_traj(h, 0, 0, out, on_device);
}
int fddp_get_us(fddp_handle* h, double* out, int on_device) {
  if (!h || !out) return fail(FDDP_ERR_INVALID_ARG, "fddp_get_us: null");
  DeviceGuard g(h->device);
  if (h->D.m == 0) return FDDP_OK;
  return gather_traj(h, 1, 0, out, on_device);
}
int fddp_get_xs_try(fddp_handle* h, double* out) {
  if (!h || !out) return fail(FDDP_ERR_INVALID_ARG, "fddp_get_xs_try: null");
  DeviceGuard g(h->device);
  return gather_traj(h, 0, 1, out, 0);
}
int fddp_get_us_try(fddp_handle* h, double* out) {
  if (!h || !out) return fail(FDDP_ERR_INVALID_ARG, "fddp_get_us_try: null");
  DeviceGuard g(h->device);
  if (h->D.m == 0) return FDDP_OK;
  return gather_traj(h, 1, 1, out, 0);
}

// ---- step API ---------------------------------------------------------------
int fddp_problem_calc(fddp_handle* h, double* cost) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "null handle");
  DeviceGuard g(h->device);
  int rc;
  if ((rc = launch_calc(h, SEL_ALL))) return rc;
  if ((rc = launch_cost_sum(h, SEL_ALL, h->d_out))) return rc;
  if (cost) HIP_TRY(hipMemcpyAsync(cost, h->d_out, sizeof(double) * h->dims.B, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return FDDP_OK;
}

int fddp_problem_calc_diff(fddp_handle* h, double* cost) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "null handle");
  DeviceGuard g(h->device);
  int rc;
  if ((rc = launch_calc_diff(h, SEL_ALL, 0))) return rc;
  if ((rc = launch_cost_sum(h, SEL_ALL, h->d_out))) return rc;
  if (cost) HIP_TRY(hipMemcpyAsync(cost, h->d_out, sizeof(double) * h->dims.B, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return FDDP_OK;
}

int fddp_compute_direction(fddp_handle* h, int recalc, int32_t* status) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "null handle");
  DeviceGuard g(h->device);
  int rc;
  if (recalc) {
    if ((rc = launch_calc_then_diff(h, SEL_ITER0, SEL_ITER0, SEL_ALL, 1))) return rc;
    if ((rc = launch_cost_sum(h, SEL_ALL, nullptr))) return rc;
  }
  if ((rc = launch_backward(h, 1))) return rc;
  if (status) {
    std::vector<ElemState> st;
    if ((rc = download_states(h, st))) return rc;
    for (int b = 0; b < h->dims.B; ++b) status[b] = st[b].bwd_fail;
  } else {
    HIP_TRY(hipStreamSynchronize(h->stream));
  }
  return FDDP_OK;
}

// SolverDDP::calcDiff (ddp.cpp:157-178): the first half of computeDirection(true)
int fddp_calc_diff(fddp_handle* h, double* cost) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "fddp_calc_diff: null handle");
  DeviceGuard g(h->device);
  int rc;
  if ((rc = launch_calc_then_diff(h, SEL_ITER0, SEL_ITER0, SEL_ALL, 1))) return rc;
  if ((rc = launch_cost_sum(h, SEL_ALL, h->d_out))) return rc;
  if (cost) HIP_TRY(hipMemcpyAsync(cost, h->d_out, sizeof(double) * h->dims.B, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return FDDP_OK;
}

// SolverDDP::backwardPass (ddp.cpp:180-253): the second half of computeDirection
int fddp_backward_pass(fddp_handle* h, int32_t* status) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "fddp_backward_pass: null handle");
  return fddp_compute_direction(h, 0, status);
}

// SolverFDDP::forwardPass (fddp.cpp:149-225): tryStep without the cost difference
int fddp_forward_pass(fddp_handle* h, double step_length, double* cost_try, int32_t* status) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "fddp_forward_pass: null handle");
  if (step_length > 1. || step_length < 0.)
    return fail(FDDP_ERR_INVALID_ARG, "invalid step length, value is between 0. to 1.");  // fddp.cpp:150-153
  DeviceGuard g(h->device);
  int rc;
  if ((rc = launch_forward(h, 1, step_length, nullptr))) return rc;
  std::vector<ElemState> st;
  if ((rc = download_states(h, st))) return rc;
  for (int b = 0; b < h->dims.B; ++b) {
    if (cost_try) cost_try[b] = st[b].cost_try;
    if (status) status[b] = st[b].fwd_fail;
  }
  return FDDP_OK;
}

int fddp_abi_version(void) { return FDDP_ABI_VERSION; }

int fddp_update_expected_improvement(fddp_handle* h) {
  // dg/dq are reduced inside the backward kernel (same terms, same order).
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "null handle");
  return FDDP_OK;
}

int fddp_try_step(fddp_handle* h, double alpha, double* dV, int32_t* status) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "null handle");
  if (alpha > 1. || alpha < 0.)
    return fail(FDDP_ERR_INVALID_ARG, "invalid step length, value is between 0. to 1.");  // fddp.cpp:150-153
  DeviceGuard g(h->device);
  int rc;
  if ((rc = launch_forward(h, 1, alpha, nullptr))) return rc;
  std::vector<ElemState> st;
  if ((rc = download_states(h, st))) return rc;
  for (int b = 0; b < h->dims.B; ++b) {
    if (dV) dV[b] = st[b].dV;
    if (status) status[b] = st[b].fwd_fail;
  }
  return FDDP_OK;
}

int fddp_expected_improvement(fddp_handle* h, double* d) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "null handle");
  DeviceGuard g(h->device);
  const Dev& D = h->D;
  hipLaunchKernelGGL(ei_kernel, dim3((D.B + 255) / 256), dim3(256), 0, h->stream, D, h->d_out);
  LAUNCH_CHECK();
  if (d) HIP_TRY(hipMemcpyAsync(d, h->d_out, sizeof(double) * 2 * D.B, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return FDDP_OK;
}

int fddp_stopping_criteria(fddp_handle* h, double* stop) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "null handle");
  DeviceGuard g(h->device);
  std::vector<ElemState> st;
  int rc;
  if ((rc = download_states(h, st))) return rc;
  if (stop)
    for (int b = 0; b < h->dims.B; ++b) stop[b] = st[b].stop;
  return FDDP_OK;
}

// Solver state for the step API (reference: a fresh solver has iter_ = 0 and
// xreg_ = ureg_ = NaN; tests also set them explicitly).
int fddp_set_solver_state(fddp_handle* h, int iter, double xreg, double ureg, int was_feasible) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "null handle");
  DeviceGuard g(h->device);
  const Dev& D = h->D;
  hipLaunchKernelGGL(step_state_kernel, dim3((D.B + 255) / 256), dim3(256), 0, h->stream, D, iter, xreg, ureg,
                     was_feasible);
  LAUNCH_CHECK();
  HIP_TRY(hipStreamSynchronize(h->stream));
  return FDDP_OK;
}

int fddp_set_debug(fddp_handle* h, int on) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "null handle");
  DeviceGuard g(h->device);
  Dev& D = h->D;
  if (on && !h->dbg[0]) {
    const int64_t B = D.B, K1 = D.T + 1, K0 = D.T;
    const int64_t sizes[7] = {B * K1 * D.sNN, B * K1 * D.sN, B * K0 * D.sNN, B * K0 * D.sNM,
                              B * K0 * D.sMM, B * K0 * D.sN, B * K0 * D.sM};
    int rc;
    for (int i = 0; i < 7; ++i)
      if ((rc = dalloc(h, &h->dbg[i], sizes[i]))) return rc;
  }
  double* const* p = h->dbg;
  const bool a = on != 0;
  D.dVxx = a ? p[0] : nullptr;
  D.dVx = a ? p[1] : nullptr;
  D.dQxx = a ? p[2] : nullptr;
  D.dQxu = a ? p[3] : nullptr;
  D.dQuu = a ? p[4] : nullptr;
  D.dQx = a ? p[5] : nullptr;
  D.dQu = a ? p[6] : nullptr;
  if (on && !h->dqi) {
    int rc;
    if ((rc = dalloc(h, &h->dqi, (int64_t)D.B * D.T * D.sMM))) return rc;
  }
  D.dQuuInv = a ? h->dqi : nullptr;
  h->debug = a;
  HIP_TRY(hipStreamSynchronize(h->stream));
  return FDDP_OK;
}

int fddp_get_quantity(fddp_handle* h, int which, double* out) {
  if (!h || !out) return fail(FDDP_ERR_INVALID_ARG, "fddp_get_quantity: null");
  DeviceGuard g(h->device);
  const Dev& D = h->D;
  const int64_t n = D.n, m = D.m;
  const double* src = nullptr;
  int64_t per = 0, stride = 0, nk = 0;
  int cur = -1;
  switch (which) {
    case FDDP_Q_FX: src = D.Fx; per = n * n; stride = D.sNN; nk = D.T + 1; break;
    case FDDP_Q_FU: src = D.Fu; per = n * m; stride = D.sNM; nk = D.T + 1; break;
    case FDDP_Q_LXX: src = D.Lxx; per = n * n; stride = D.sNN; nk = D.T + 1; break;
    case FDDP_Q_LXU: src = D.Lxu; per = n * m; stride = D.sNM; nk = D.T + 1; break;
    case FDDP_Q_LUU: src = D.Luu; per = m * m; stride = D.sMM; nk = D.T + 1; break;
    case FDDP_Q_LX: src = D.Lx; per = n; stride = D.sN; nk = D.T + 1; break;
    case FDDP_Q_LU: src = D.Lu; per = m; stride = D.sM; nk = D.T + 1; break;
    case FDDP_Q_XNEXT: cur = 1; per = D.nx; stride = D.sX; nk = D.T; break;
    case FDDP_Q_COST: cur = 2; per = 1; stride = 1; nk = D.T + 1; break;
    case FDDP_Q_FS: src = D.fs; per = n; stride = D.sN; nk = D.T + 1; break;
    case FDDP_Q_K: src = D.K; per = m * n; stride = D.sNM; nk = D.T; break;
    case FDDP_Q_KV: src = D.k; per = m; stride = D.sM; nk = D.T; break;
    case FDDP_Q_VXX: src = D.dVxx; per = n * n; stride = D.sNN; nk = D.T + 1; break;
    case FDDP_Q_VX: src = D.dVx; per = n; stride = D.sN; nk = D.T + 1; break;
    case FDDP_Q_QXX: src = D.dQxx; per = n * n; stride = D.sNN; nk = D.T; break;
    case FDDP_Q_QXU: src = D.dQxu; per = n * m; stride = D.sNM; nk = D.T; break;
    case FDDP_Q_QUU: src = D.dQuu; per = m * m; stride = D.sMM; nk = D.T; break;
    case FDDP_Q_QX: src = D.dQx; per = n; stride = D.sN; nk = D.T; break;
    case FDDP_Q_QU: src = D.dQu; per = m; stride = D.sM; nk = D.T; break;
    case FDDP_Q_QUU_INV: src = D.dQuuInv; per = m * m; stride = D.sMM; nk = D.T; break;
    default: return fail(FDDP_ERR_INVALID_ARG, "fddp_get_quantity: unknown quantity");
  }
  if (per == 0) return FDDP_OK;
  if (cur >= 0) {
    // xnext / knot costs live in the current trajectory buffer of each element
    std::vector<ElemState> st;
    int rc;
    if ((rc = download_states(h, st))) return rc;
    for (int b = 0; b < D.B; ++b) {
      const double* s = (cur == 2 ? D.kcost[st[b].cur] : D.xnext[st[b].cur]) + (int64_t)b * nk * stride;
      HIP_TRY(hipMemcpy2DAsync(out + (int64_t)b * nk * per, sizeof(double) * per, s, sizeof(double) * stride,
                               sizeof(double) * per, nk, hipMemcpyDeviceToHost, h->stream));
    }
  } else {
    if (!src) return fail(FDDP_ERR_INVALID_ARG, "fddp_get_quantity: enable fddp_set_debug first");
    HIP_TRY(hipMemcpy2DAsync(out, sizeof(double) * per, src, sizeof(double) * stride, sizeof(double) * per,
                             (size_t)D.B * nk, hipMemcpyDeviceToHost, h->stream));
  }
  HIP_TRY(hipStreamSynchronize(h->stream));
  return FDDP_OK;
}

int fddp_set_knots(fddp_handle* h, const fddp_knot_desc* knots, const double* params, int64_t n_params) {
  if (!h || !knots || !params) return fail(FDDP_ERR_INVALID_ARG, "fddp_set_knots: null argument");
  int rc;
  if ((rc = check_knots(h->dims, knots, params, n_params, "fddp_set_knots", false))) return rc;
  DeviceGuard g(h->device);
  HIP_TRY(hipStreamSynchronize(h->stream));  // no launch may still read the old knots
  return apply_knots(h, knots, params, n_params);
}

int fddp_set_solver_kind(fddp_handle* h, int kind) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "fddp_set_solver_kind: null handle");
  if (kind != FDDP_SOLVER_FDDP && kind != FDDP_SOLVER_BOXFDDP)
    return fail(FDDP_ERR_INVALID_ARG, "fddp_set_solver_kind: unknown solver kind");
  if (kind == FDDP_SOLVER_BOXFDDP && h->dims.nu_max > 64)
    return fail(FDDP_ERR_UNSUPPORTED, "fddp_set_solver_kind: the box QP holds at most 64 controls (one wave)");
  h->solver_kind = kind;
  h->D.box = kind == FDDP_SOLVER_BOXFDDP ? 1 : 0;
  return FDDP_OK;
}

int fddp_get_solver_kind(fddp_handle* h, int* kind) {
  if (!h || !kind) return fail(FDDP_ERR_INVALID_ARG, "fddp_get_solver_kind: null");
  *kind = h->solver_kind;
  return FDDP_OK;
}

int fddp_set_control_limits(fddp_handle* h, const double* u_lb, const double* u_ub) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "fddp_set_control_limits: null handle");
  if ((u_lb == nullptr) != (u_ub == nullptr))
    return fail(FDDP_ERR_INVALID_ARG, "fddp_set_control_limits: give both u_lb and u_ub, or neither");
  DeviceGuard g(h->device);
  Dev& D = h->D;
  if (!u_lb) {
    D.ulb = D.uub = nullptr;
    D.haslim = nullptr;
    return FDDP_OK;
  }
  const int64_t B = D.B, T = D.T, m = D.m;
  int rc;
  if (!h->d_ulb) {
    if ((rc = dalloc(h, &h->d_ulb, B * T * D.sM))) return rc;
    if ((rc = dalloc(h, &h->d_uub, B * T * D.sM))) return rc;
    double* hl = nullptr;
    if ((rc = dalloc(h, &hl, (B * T + 7) / 8))) return rc;
    h->d_haslim = (unsigned char*)hl;
  }
  // update_has_control_limits (action-base.hxx:142-144) per knot and element
  std::vector<unsigned char> lim((size_t)(B * T));
  std::vector<double> lb((size_t)(B * T * D.sM), -INFINITY), ub((size_t)(B * T * D.sM), INFINITY);
  for (int64_t b = 0; b < B; ++b)
    for (int64_t t = 0; t < T; ++t) {
      const int nu = h->knots[t].nu;
      bool al = false, au = false;
      for (int64_t i = 0; i < m; ++i) {
        const double l = u_lb[(b * T + t) * m + i], u = u_ub[(b * T + t) * m + i];
        lb[(b * T + t) * D.sM + i] = l;
        ub[(b * T + t) * D.sM + i] = u;
        if (i < nu) {
          al = al || std::isfinite(l);
          au = au || std::isfinite(u);
        }
      }
      lim[b * T + t] = (al && au) ? 1 : 0;
    }
  HIP_TRY(hipMemcpyAsync(h->d_ulb, lb.data(), sizeof(double) * lb.size(), hipMemcpyHostToDevice, h->stream));
  HIP_TRY(hipMemcpyAsync(h->d_uub, ub.data(), sizeof(double) * ub.size(), hipMemcpyHostToDevice, h->stream));
  HIP_TRY(hipMemcpyAsync(h->d_haslim, lim.data(), lim.size(), hipMemcpyHostToDevice, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  D.ulb = h->d_ulb;
  D.uub = h->d_uub;
  D.haslim = h->d_haslim;
  return FDDP_OK;
}

void fddp_boxqp_default_params(fddp_boxqp_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->maxiter = 100;
  p->n_alphas = 10;
  p->th_acceptstep = 0.1;
  p->th_grad = 1e-9;
  p->reg = 1e-9;
  for (int i = 0; i < 10; ++i) p->alphas[i] = 1. / std::pow(2., (double)i);
}

int fddp_boxqp_solve(int device, int B, int nx, const double* H, const double* q, const double* lb,
                     const double* ub, const double* xinit, const fddp_boxqp_params* p, double* x,
                     uint64_t* free_mask, uint64_t* inv_mask, double* Hff_inv, int32_t* status) {
  g_err.clear();
  if (B < 0 || nx < 1 || !H || !q || !lb || !ub || !xinit || !p)
    return fail(FDDP_ERR_INVALID_ARG, "fddp_boxqp_solve: invalid argument");
  if (nx > 64) return fail(FDDP_ERR_UNSUPPORTED, "fddp_boxqp_solve: nx > 64 (one wave per QP)");
  // BoxQP setters' validation (box-qp.cpp:203-249)
  if (p->th_grad < 0.) return fail(FDDP_ERR_INVALID_ARG, "th_grad value has to be positive.");
  if (p->reg < 0.) return fail(FDDP_ERR_INVALID_ARG, "reg value has to be positive.");
  if (p->n_alphas < 1 || p->n_alphas > 16) return fail(FDDP_ERR_INVALID_ARG, "n_alphas must be in [1, 16]");
  for (int i = 1; i < p->n_alphas; ++i) {
    if (0. >= p->alphas[i]) return fail(FDDP_ERR_INVALID_ARG, "alpha values has to be positive.");
    if (p->alphas[i] >= p->alphas[i - 1]) return fail(FDDP_ERR_INVALID_ARG, "alpha values are monotonously decreasing.");
  }
  if (B == 0) return FDDP_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(FDDP_ERR_NO_DEVICE, "fddp_boxqp_solve: no HIP device");
  if (device < 0 || device >= ndev) return fail(FDDP_ERR_INVALID_ARG, "fddp_boxqp_solve: bad device index");
  DeviceGuard g(device);
  const size_t nn = (size_t)B * nx * nx, nv = (size_t)B * nx;
  // one allocation: H | q lb ub xinit | x | Hinv | masks (2B) | status (B)
  const size_t nd = 2 * nn + 5 * nv + 2 * (size_t)B + ((size_t)B + 1) / 2;
  double* buf = nullptr;
  HIP_TRY(hipMalloc(&buf, sizeof(double) * nd));
  double *dH = buf, *dq = dH + nn, *dl = dq + nv, *du = dl + nv, *dx0 = du + nv, *dx = dx0 + nv, *dHi = dx + nv;
  uint64_t* dm = (uint64_t*)(dHi + nn);
  int32_t* ds = (int32_t*)(dm + 2 * (size_t)B);
  int rc = FDDP_OK;
  auto run = [&]() -> int {
    HIP_TRY(hipMemcpy(dH, H, sizeof(double) * nn, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dq, q, sizeof(double) * nv, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dl, lb, sizeof(double) * nv, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(du, ub, sizeof(double) * nv, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dx0, xinit, sizeof(double) * nv, hipMemcpyHostToDevice));
    const size_t smem = sizeof(double) * (2 * (size_t)nx * nx + 64);
    HIP_TRY(hipFuncSetAttribute((const void*)boxqp_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
    hipLaunchKernelGGL(boxqp_kernel, dim3(B), dim3(64), smem, 0, nx, dH, dq, dl, du, dx0, to_boxcfg(*p), dx, dm,
                       dm + B, dHi, ds);
    LAUNCH_CHECK();
    HIP_TRY(hipDeviceSynchronize());
    if (x) HIP_TRY(hipMemcpy(x, dx, sizeof(double) * nv, hipMemcpyDeviceToHost));
    if (free_mask) HIP_TRY(hipMemcpy(free_mask, dm, sizeof(uint64_t) * B, hipMemcpyDeviceToHost));
    if (inv_mask) HIP_TRY(hipMemcpy(inv_mask, dm + B, sizeof(uint64_t) * B, hipMemcpyDeviceToHost));
    if (Hff_inv) HIP_TRY(hipMemcpy(Hff_inv, dHi, sizeof(double) * nn, hipMemcpyDeviceToHost));
    if (status) HIP_TRY(hipMemcpy(status, ds, sizeof(int32_t) * B, hipMemcpyDeviceToHost));
    return FDDP_OK;
  };
  rc = run();
  (void)hipFree(buf);
  return rc;
}

int fddp_mpc_shift(fddp_handle* h) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "null handle");
  DeviceGuard g(h->device);
  const Dev& D = h->D;
  hipLaunchKernelGGL(mpc_shift_kernel<kNT>, dim3(D.B), dim3(kNT), 0, h->stream, D);
  LAUNCH_CHECK();
  return FDDP_OK;
}

int fddp_synchronize(fddp_handle* h) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "null handle");
  DeviceGuard g(h->device);
  HIP_TRY(hipStreamSynchronize(h->stream));
  return FDDP_OK;
}

int fddp_get_stream(fddp_handle* h, void** stream) {
  if (!h || !stream) return fail(FDDP_ERR_INVALID_ARG, "null");
  *stream = (void*)h->stream;
  return FDDP_OK;
}

int fddp_set_timing(fddp_handle* h, int on) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "null handle");
  h->timing = on != 0;
  return FDDP_OK;
}

int fddp_get_timing(fddp_handle* h, double* ms_out, int64_t* counts_out) {
  if (!h) return fail(FDDP_ERR_INVALID_ARG, "null handle");
  DeviceGuard g(h->device);
  HIP_TRY(hipStreamSynchronize(h->stream));
  for (auto& r : h->ev_rec) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, r.second.first, r.second.second) == hipSuccess) {
      h->t_ms[r.first] += ms;
      h->t_cnt[r.first] += 1;
    }
    h->ev_pool.push_back(r.second.first);
    h->ev_pool.push_back(r.second.second);
  }
  h->ev_rec.clear();
  for (int i = 0; i < 4; ++i) {
    if (ms_out) ms_out[i] = h->t_ms[i];
    if (counts_out) counts_out[i] = h->t_cnt[i];
    h->t_ms[i] = 0.;
    h->t_cnt[i] = 0;
  }
  return FDDP_OK;
}

int64_t fddp_device_bytes(fddp_handle* h) { return h ? h->bytes : 0; }

}  // extern "C"
