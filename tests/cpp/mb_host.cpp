// Test harness (CPU): the device multibody knot code of
// crocoddyl_amd/csrc/multibody.hpp compiled for the host and run with the
// sequential-lane executor, so tests/test_multibody_host.py can check the
// exact device arithmetic against the numpy oracle without a GPU.
#include <cstdio>
#include <cstdlib>
#include <vector>

// the calcDiff's LDS matrices (multibody.hpp MB_DUMP), column-major per slot, for the
// parity diagnosis (tools/mb_dump_check.py --host)
static double g_dump[12][4096];
static int g_dump_shape[12][2];
#define MB_DUMP(slot, ptr, rows, cols, ld)                                   \
  do {                                                                       \
    const double* p_ = (const double*)(ptr);                                 \
    const int r_ = (rows), c_ = (cols), l_ = (ld);                           \
    for (int e_ = 0; e_ < r_ * c_ && e_ < 4096; ++e_) g_dump[slot][e_] = p_[(e_ / r_) * l_ + e_ % r_]; \
    g_dump_shape[slot][0] = r_;                                              \
    g_dump_shape[slot][1] = c_;                                              \
  } while (0)
#include "../../crocoddyl_amd/csrc/multibody.hpp"

using namespace fddp::mb;

extern "C" {

double mb_host_calc(const double* P, int nx, const double* x, const double* u, int use_u, double* xnext) {
  const Blk b = parse(P);
  std::vector<double> w(calc_work_doubles(b.nj, b.nc), 0.);
  return knot_calc_x(HostExec{256}, P, nx, x, u, use_u != 0, xnext, w.data());
}

void mb_host_calc_diff(const double* P, int nx, int m, const double* x, const double* u, int use_u, double* Fx,
                       double* Fu, double* Lxx, double* Lxu, double* Luu, double* Lx, double* Lu, double* xnext,
                       double* cost) {
  const Blk b = parse(P);
  bool vc = false;
  const int njac = count_jac_costs(b, &vc);
  const int nu = b.nj - b.nun, nrows = count_cost_rows(b, nu);
  // the device's plan for this block (spilled to the output blocks on the large trees);
  // MB_HOST_SPILL=0 forces the all-LDS plan
  const char* sp = std::getenv("MB_HOST_SPILL");
  const int spill = sp && sp[0] == '0' ? 0 : diff_spill(b.nj, njac, b.nc, vc, nu, nrows, (int64_t)P[3], m);
  std::vector<double> w(diff_layout(b.nj, njac, b.nc, vc, nu, nrows, spill).htotal, 0.);
  // MB_HOST_NT: the workgroup size the lanes emulate (128 / 256 / 512: the device's
  // small-tree, default and 8-wave calcDiff kernels)
  const char* e = std::getenv("MB_HOST_NT");
  knot_calc_diff_x(HostExec{e ? std::atoi(e) : kMbDiffNT}, P, nx, m, x, u, use_u != 0, w.data(), Fx, Fu, Lxx, Lxu, Luu,
                   Lx, Lu, xnext, cost, nullptr, spill);
}
}

extern "C" {
// The calcDiff LDS plan of a knot block (doubles): the DiffLayout offsets in field
// order, then total, nj, njac, nc, nrows, vcols, spill flags, half, block size.
// (m: nu_max of the plan, diff_spill)
int mb_host_layout(const double* P, int m, double* out) {
  const Blk b = parse(P);
  bool vc = false;
  const int njac = count_jac_costs(b, &vc);
  const int nu = b.nj - b.nun;
  const int nrows = count_cost_rows(b, nu);
  const int spill = diff_spill(b.nj, njac, b.nc, vc, nu, nrows, (int64_t)P[3], m);
  const DiffLayout l = diff_layout(b.nj, njac, b.nc, vc, nu, nrows, spill);
  const int64_t f[] = {l.wv, l.A, l.dtau, l.da, l.qp, l.vec, l.J, l.red, l.R, l.Jc, l.a0, l.lam, l.Y, l.H,
                       l.Sx, l.da0, l.fx, l.zv, l.dfx, l.dfu, l.total, b.nj, njac, b.nc, nrows, vc ? 1 : 0,
                       spill, l.half, (int64_t)P[3]};
  for (int i = 0; i < (int)(sizeof(f) / sizeof(f[0])); ++i) out[i] = (double)f[i];
  return (int)(sizeof(f) / sizeof(f[0]));
}
}

extern "C" {
// The device's calcDiff plan for a block at nu_max m: the spill flags (diff_spill) and
// the LDS bytes of the plan with the parameter block.
int mb_host_plan(const double* P, int m, int64_t* lds_bytes) {
  const Blk b = parse(P);
  bool vc = false;
  const int njac = count_jac_costs(b, &vc);
  const int nu = b.nj - b.nun, nrows = count_cost_rows(b, nu);
  const int spill = diff_spill(b.nj, njac, b.nc, vc, nu, nrows, (int64_t)P[3], m);
  *lds_bytes = 8 * (fddp::pad2(diff_layout(b.nj, njac, b.nc, vc, nu, nrows, spill).total) + fddp::pad2((int64_t)P[3]));
  return spill;
}
}

extern "C" {
// The multibody rollout's dynamic LDS per workgroup for a block (fddp_hip.hip apply_knots):
// the staged parameter block, the trial's vectors (x, u, next x, the sums, the flag; dx in
// the knot calc's scratch) and the dense knot calc's scratch (calc_dense_doubles, also in
// *dense); in *work the tree calc's scratch (calc_work_doubles), for comparison.
int64_t mb_host_rollout_lds(const double* P, int nx, int nu_max, int64_t* dense, int64_t* work) {
  const Blk b = parse(P);
  const int64_t sX = fddp::pad2(nx), sM = fddp::pad2(nu_max);
  *dense = fddp::pad2(calc_dense_doubles(b.nj, b.nc));
  *work = fddp::pad2(calc_work_doubles(b.nj, b.nc));
  return 8 * (fddp::pad2((int64_t)P[3]) + 2 * sX + sM + 5 * 4 + 8 + 2 + *dense);
}
}

extern "C" {
// The static check of a calcDiff plan (multibody.hpp diff_layout_check): 0, or 1 with the
// conflicting pair's names in msg.
int mb_host_layout_check(int nj, int njac, int nc, int vcols, int nu, int nrows, int spill, char* msg, int cap) {
  const DiffLayout l = diff_layout(nj, njac, nc, vcols != 0, nu, nrows, spill);
  int a = 0, b = 0;
  if (!diff_layout_check(l, nj, njac, nc, vcols != 0, nu, nrows, &a, &b)) return 0;
  DiffRegion r[40];
  diff_layout_regions(l, nj, njac, nc, vcols != 0, nu, nrows, r);
  std::snprintf(msg, cap, "%s [%lld, +%lld) phases %d-%d / %s [%lld, +%lld) phases %d-%d (total %lld)", r[a].name,
                (long long)r[a].off, (long long)r[a].size, r[a].first, r[a].last, r[b].name, (long long)r[b].off,
                (long long)r[b].size, r[b].first, r[b].last, (long long)l.total);
  return 1;
}
}

extern "C" {
// the MB_DUMP slots of the last mb_host_calc_diff: shapes (12 x 2 ints), values (12 x 4096)
void mb_host_dump(int* shape, double* vals) {
  for (int s = 0; s < 12; ++s) {
    shape[2 * s] = g_dump_shape[s][0];
    shape[2 * s + 1] = g_dump_shape[s][1];
    for (int e = 0; e < 4096; ++e) vals[s * 4096 + e] = g_dump[s][e];
  }
}
}
