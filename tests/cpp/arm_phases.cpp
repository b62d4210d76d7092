// The reference's DDP-phase timing loop (benchmark/arm-kinova-codegen.cpp:258-285:
// calcDiff once, then backwardPass and forwardPass(0.005) timed call by call) on the
// crocoddyl_amd C++ facade: a 6-DoF Jaco-class arm (kinova.urdf is absent offline; the
// chain is built in code) with the kinova factory's knots (benchmark/factory/arm-kinova.hpp:
// Euler(dt = 1e-3) over FreeFwdDynamics, ActuationModelFull, gripperPose FramePlacement at
// (I, (0, 0, 0.4)) weight 1, xReg 1e-4, uReg 1e-4; terminal Euler(dt = 0) over the same
// differential model), N = 100 nodes, x0 random in [-1, 1] (Eigen::VectorXd::Random).
//
// usage: arm_phases pack FILE           the knot descriptors + parameter pool (for the oracle)
//        arm_phases phases FILE [TRIALS] calcDiff, TRIALS x backwardPass, TRIALS x forwardPass(0.005);
//                                        writes [cost, K, k, cost_try, xs_try, us_try, x0] to FILE
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "crocoddyl_amd/multibody.hpp"

namespace croc = crocoddyl_amd;
using croc::Vec3;
using croc::VectorXd;

static const int N = 100;  // number of nodes (arm-kinova-codegen.cpp:25)

static std::shared_ptr<croc::Model> sample_jaco6() {
  auto m = std::make_shared<croc::Model>();
  struct Link {
    Vec3 axis, p;
    double mass;
    Vec3 c, d;
  };
  const Link links[6] = {
      {Vec3(0., 0., 1.), Vec3(0., 0., 0.1564), 0.75, Vec3(0., -0.002, -0.06), Vec3(0.0021, 0.0022, 0.0010)},
      {Vec3(0., 1., 0.), Vec3(0., 0.0054, 0.1284), 0.99, Vec3(0., -0.21, 0.), Vec3(0.0110, 0.0009, 0.0111)},
      {Vec3(0., 1., 0.), Vec3(0., -0.41, 0.), 0.68, Vec3(0., 0.08, -0.01), Vec3(0.0038, 0.0004, 0.0038)},
      {Vec3(0., 0., 1.), Vec3(0., 0.2073, -0.0114), 0.43, Vec3(0., 0.03, -0.05), Vec3(0.0010, 0.0010, 0.0003)},
      {Vec3(0., 1., 0.), Vec3(0., 0., -0.1038), 0.43, Vec3(0., 0.03, -0.05), Vec3(0.0010, 0.0010, 0.0003)},
      {Vec3(0., 0., 1.), Vec3(0., 0.1038, 0.), 0.73, Vec3(0., 0., -0.06), Vec3(0.0010, 0.0010, 0.0006)},
  };
  int parent = 0;
  for (int j = 0; j < 6; ++j) {
    const Link& L = links[j];
    parent = m->addJoint(parent, croc::JointModelRevoluteUnaligned(L.axis[0], L.axis[1], L.axis[2]),
                         croc::SE3(croc::Mat3::Identity(), L.p), "j2s6s200_joint_" + std::to_string(j + 1));
    m->appendBodyToJoint(parent, croc::Inertia(L.mass, L.c, croc::Mat3::Diag(L.d[0], L.d[1], L.d[2])));
  }
  m->addFrame("j2s6s200_end_effector", parent, croc::SE3(croc::Mat3::Identity(), Vec3(0., 0., -0.16)));
  return m;
}

static bool write_all(const char* path, const std::vector<std::pair<const void*, size_t> >& parts) {
  FILE* f = std::fopen(path, "wb");
  if (!f) return false;
  for (const auto& p : parts) std::fwrite(p.first, 1, p.second, f);
  std::fclose(f);
  return true;
}

// Timer (core/utils/timer.hpp): microseconds
struct Timer {
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  double get_us_duration() const {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  }
};

static void report(const char* name, const std::vector<double>& d) {
  double avg = 0., var = 0., mx = 0., mn = 1e300;
  for (double v : d) avg += v, mx = std::max(mx, v), mn = std::min(mn, v);
  avg /= d.size();
  for (double v : d) var += (v - avg) * (v - avg);
  const double sd = std::sqrt(var / d.size());
  std::printf("%s [us]:\t%g +- %g (max: %g, min: %g, per nodes: %g +- %g)\n", name, avg, sd, mx, mn, avg / N, sd / N);
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s pack|phases FILE [TRIALS]\n", argv[0]);
    return 2;
  }
  try {
    auto rmodel = sample_jaco6();
    auto state = std::make_shared<croc::StateMultibody>(rmodel);
    const int nu = state->get_nv();
    const int ee = rmodel->getFrameId("j2s6s200_end_effector");
    auto goal = std::make_shared<croc::CostModelFramePlacement>(
        state, croc::FramePlacement(ee, croc::SE3(croc::Mat3::Identity(), Vec3(0., 0., 0.4))), nu);
    auto xreg = std::make_shared<croc::CostModelState>(state, state->zero(), nu);
    auto ureg = std::make_shared<croc::CostModelControl>(state, nu);
    auto costs = std::make_shared<croc::CostModelSum>(state, nu);
    costs->addCost("gripperPose", goal, 1.);
    costs->addCost("xReg", xreg, 1e-4);
    costs->addCost("uReg", ureg, 1e-4);
    auto actuation = std::make_shared<croc::ActuationModelFull>(state);
    auto dam = std::make_shared<croc::DifferentialActionModelFreeFwdDynamics>(state, actuation, costs);
    auto running = std::make_shared<croc::IntegratedActionModelEuler>(dam, 1e-3);
    auto terminal = std::make_shared<croc::IntegratedActionModelEuler>(dam, 0.);

    // x0 = (q0, v0) uniform in [-1, 1] (a fixed LCG: the test replays it exactly)
    uint64_t s = 0x5EEDull;
    auto rnd = [&]() {
      s = s * 6364136223846793005ull + 1442695040888963407ull;
      return 2. * ((s >> 11) * (1. / 9007199254740992.)) - 1.;
    };
    VectorXd x0(state->get_nx());
    for (double& v : x0) v = rnd();
    std::vector<std::shared_ptr<croc::ActionModelBase> > models(N, running);
    auto problem = std::make_shared<croc::ShootingProblem>(x0, models, terminal);
    if (!std::strcmp(argv[1], "pack")) {
      std::vector<fddp_knot_desc> knots;
      VectorXd pool;
      problem->pack(knots, pool);
      const int64_t nk = (int64_t)knots.size(), np = (int64_t)pool.size();
      const int32_t dims[4] = {problem->get_nx(), problem->get_ndx(), problem->get_nu_max(), problem->get_T()};
      if (!write_all(argv[2], {{dims, sizeof(dims)}, {&nk, 8}, {knots.data(), sizeof(fddp_knot_desc) * nk}, {&np, 8},
                               {pool.data(), 8 * np}}))
        return 3;
      std::printf("packed T=%d nx=%d ndx=%d nu_max=%d\n", problem->get_T(), problem->get_nx(), problem->get_ndx(),
                  problem->get_nu_max());
      return 0;
    }
    const int trials = argc > 3 ? std::atoi(argv[3]) : 100;
    croc::SolverFDDP ddp(problem);
    // the harness's warm start (arm-kinova-codegen.cpp:60-70): xs = x0 everywhere; us = 0
    // here (its quasiStatic controls need the RNEA of the URDF model)
    std::vector<VectorXd> xs(N + 1, x0), us(N, VectorXd(nu, 0.));
    ddp.setCandidate(xs, us, false);
    ddp.set_solver_state(0, NAN, NAN, false);  // a fresh solver (iter 0, no regularisation)

    const double cost = ddp.calcDiff();
    std::vector<double> dur(trials);
    for (int i = 0; i < trials; ++i) {
      Timer timer;
      ddp.backwardPass();
      dur[i] = timer.get_us_duration();
    }
    report("backwardPass", dur);
    for (int i = 0; i < trials; ++i) {
      Timer timer;
      ddp.forwardPass(0.005);
      dur[i] = timer.get_us_duration();
    }
    report("forwardPass", dur);

    VectorXd out{cost};
    for (const auto& K : ddp.get_K()) out.insert(out.end(), K.begin(), K.end());
    for (const auto& k : ddp.get_k()) out.insert(out.end(), k.begin(), k.end());
    out.push_back(ddp.get_cost_try());
    for (const auto& x : ddp.get_xs_try()) out.insert(out.end(), x.begin(), x.end());
    for (const auto& u : ddp.get_us_try()) out.insert(out.end(), u.begin(), u.end());
    out.insert(out.end(), x0.begin(), x0.end());
    if (!write_all(argv[2], {{out.data(), 8 * out.size()}})) return 3;
    // the argument check of forwardPass (fddp.cpp:150-153)
    bool threw = false;
    try {
      ddp.forwardPass(1.5);
    } catch (const croc::Exception&) {
      threw = true;
    }
    std::printf("phases cost=%.12e cost_try=%.12e invalid_step_throws=%d\n", cost, ddp.get_cost_try(), threw ? 1 : 0);
    return 0;
  } catch (const croc::Exception& e) {
    std::printf("exception: %s\n", e.what());
    return 1;
  }
}
