// The reference's benchmark/lqr-optctrl.cpp usage pattern written against the
// crocoddyl_amd C++ facade: only the namespace changes.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <memory>
#include <vector>

#include "crocoddyl_amd/solver_fddp_hip.hpp"

namespace croc = crocoddyl_amd;

// a CallbackLogger-style recorder (bindings/python/crocoddyl/__init__.py:356-381)
struct Logger : croc::CallbackAbstract {
  struct Row {
    std::size_t iter;
    double cost, stop, step, xreg, grad;
  };
  std::vector<Row> rows;
  void operator()(croc::SolverFDDP& s) override {
    rows.push_back({s.get_iter(), s.get_cost(), s.get_stop(), s.get_steplength(), s.get_xreg(), -s.get_d()[1]});
  }
};

int main(int argc, char** argv) {
  try {
    const int T = 100;
    // lqr-optctrl.cpp:28-31: one model object shared by all knots
    auto model = std::make_shared<croc::ActionModelLQR>(24, 12, false);
    std::vector<std::shared_ptr<croc::ActionModelBase> > running(T, model);
    croc::VectorXd x0(24, 0.);
    auto problem = std::make_shared<croc::ShootingProblem>(x0, running, model);
    croc::SolverFDDP solver(problem);
    const bool ok = solver.solve();
    std::printf("lqr converged=%d iter=%zu cost=%.12e stop=%.3e\n", ok, solver.get_iter(), solver.get_cost(),
                solver.get_stop());
    // unicycle towards the origin (examples/notebooks/unicycle_towards_origin.py)
    auto uni = std::make_shared<croc::ActionModelUnicycle>();
    std::vector<std::shared_ptr<croc::ActionModelBase> > urun(30, uni);
    croc::VectorXd ux0 = {-1., -1., 1.};
    auto uprob = std::make_shared<croc::ShootingProblem>(ux0, urun, uni);
    croc::SolverFDDP usolver(uprob);
    const bool uok = usolver.solve();
    const auto xs = usolver.get_xs();
    std::printf("unicycle converged=%d iter=%zu cost=%.12e xT=(%.3e %.3e %.3e)\n", uok, usolver.get_iter(),
                usolver.get_cost(), xs.back()[0], xs.back()[1], xs.back()[2]);
    // per-iteration callbacks (fddp.cpp:92-98): a logger and CallbackVerbose (to stderr)
    auto logger = std::make_shared<Logger>();
    croc::SolverFDDP lsolver(uprob);
    lsolver.setCallbacks({logger, std::make_shared<croc::CallbackVerbose>(2, stderr)});
    lsolver.solve();
    for (const auto& r : logger->rows)
      std::printf("trace%zu cost=%.17e stop=%.17e step=%.17e xreg=%.17e grad=%.17e\n", r.iter, r.cost, r.stop, r.step,
                  r.xreg, r.grad);
    // control-limited LQR with SolverBoxFDDP (box-fddp.cpp)
    auto bmodel = std::make_shared<croc::ActionModelLQR>(24, 12, false);
    bmodel->set_u_lb(croc::VectorXd(12, -0.05));
    bmodel->set_u_ub(croc::VectorXd(12, 0.05));
    std::vector<std::shared_ptr<croc::ActionModelBase> > brun(T, bmodel);
    auto bprob = std::make_shared<croc::ShootingProblem>(x0, brun, bmodel);
    croc::SolverBoxFDDP bsolver(bprob);
    const bool bok = bsolver.solve();
    double umax = 0.;
    for (const auto& u : bsolver.get_us())
      for (double v : u) umax = std::max(umax, std::fabs(v));
    std::printf("box converged=%d iter=%zu cost=%.12e umax=%.6f th_stop=%.1e\n", bok, bsolver.get_iter(),
                bsolver.get_cost(), umax, bsolver.get_th_stop());
    try {
      usolver.set_th_stepdec(2.0);  // ddp.cpp:464-470 rejects this
      std::printf("setter validation MISSING\n");
      return 3;
    } catch (const croc::Exception&) {
      std::printf("setter validation ok\n");
    }
    return (ok && uok && bok && umax <= 0.05) ? 0 : 2;
  } catch (const croc::Exception& e) {
    std::printf("exception: %s\n", e.what());
    return 1;
  }
}
