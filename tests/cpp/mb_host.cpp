// Test harness (CPU): the device multibody knot code of
// crocoddyl_amd/csrc/multibody.hpp compiled for the host and run with the
// sequential-lane executor, so tests/test_multibody_host.py can check the
// exact device arithmetic against the numpy oracle without a GPU.
#include <cstdlib>
#include <vector>

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
  std::vector<double> w(diff_layout(b.nj, kMaxJacCosts, b.nc, true, b.nj - b.nun, count_cost_rows(b, b.nj - b.nun)).total, 0.);
  // MB_HOST_NT: the workgroup size the lanes emulate (128 / 256 / 512: the device's
  // small-tree, default and 8-wave calcDiff kernels)
  const char* e = std::getenv("MB_HOST_NT");
  knot_calc_diff_x(HostExec{e ? std::atoi(e) : kMbDiffNT}, P, nx, m, x, u, use_u != 0, w.data(), Fx, Fu, Lxx, Lxu, Luu, Lx, Lu, xnext, cost);
}
}

extern "C" {
// The calcDiff LDS plan of a knot block (doubles): the DiffLayout offsets in field
// order, then total, nj, njac, nc, nrows, vcols.
int mb_host_layout(const double* P, double* out) {
  const Blk b = parse(P);
  bool vc = false;
  const int njac = count_jac_costs(b, &vc);
  const int nu = b.nj - b.nun;
  const int nrows = count_cost_rows(b, nu);
  const DiffLayout l = diff_layout(b.nj, njac, b.nc, vc, nu, nrows);
  const int64_t f[] = {l.wv, l.A, l.dtau, l.da, l.qp, l.vec, l.J, l.red, l.R, l.Jc, l.a0, l.lam, l.Y, l.H,
                       l.Sx, l.da0, l.fx, l.zv, l.dfx, l.dfu, l.total, b.nj, njac, b.nc, nrows, vc ? 1 : 0};
  for (int i = 0; i < (int)(sizeof(f) / sizeof(f[0])); ++i) out[i] = (double)f[i];
  return (int)(sizeof(f) / sizeof(f[0]));
}
}
