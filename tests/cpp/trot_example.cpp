// The Solo12 trotting problem (C4) built in C++ against the crocoddyl_amd facade,
// the way a C++ user of the reference writes it (benchmark/quadrupedal-gaits-optctrl.cpp:
// 40-64 with SimpleQuadrupedGaitProblem, utils/quadruped.py:162-208 / 357-553 for the
// phase and cost structure): robot model, contact-dynamics knots with 3D contacts,
// friction cones, CoM / foot tracking, state bounds, impulse foot switches; then
// SolverFDDP on the GPU through the C ABI.
//
// usage: trot_example pack FILE          write the knot descriptors + parameter pool
//        trot_example solve FILE MAXITER solve from the default state, write results
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "crocoddyl_amd/multibody.hpp"

namespace croc = crocoddyl_amd;
using croc::Vec3;
using croc::VectorXd;

// robots.sample_solo12(): free-flyer + 4 legs (HAA x, HFE y, KFE y), feet 0.16 m below the knees
static std::shared_ptr<croc::Model> sample_solo12() {
  auto m = std::make_shared<croc::Model>(croc::JointModelFreeFlyer());
  auto body = [&](int j, double mass, Vec3 c, Vec3 d) {
    m->appendBodyToJoint(j, croc::Inertia(mass, c, croc::Mat3::Diag(d[0], d[1], d[2])));
  };
  body(1, 1.43, Vec3(0., 0., 0.), Vec3(0.0025, 0.0108, 0.0126));
  m->addFrame("root_joint", 1);
  const char* legs[4] = {"FL", "FR", "HL", "HR"};
  const double sxs[4] = {1., 1., -1., -1.}, sys[4] = {1., -1., 1., -1.};
  for (int l = 0; l < 4; ++l) {
    const double sx = sxs[l], sy = sys[l];
    const std::string L = legs[l];
    struct Spec {
      const char* suffix;
      Vec3 ax, p;
      double mass;
      Vec3 c, d;
    } specs[3] = {
        {"_HAA", Vec3(1, 0, 0), Vec3(0.1946 * sx, 0.0875 * sy, 0.0), 0.148, Vec3(-0.078 * sx, 0.015 * sy, 0.0),
         Vec3(0.00002, 0.0001, 0.0001)},
        {"_HFE", Vec3(0, 1, 0), Vec3(0.0, 0.014 * sy, 0.0), 0.148, Vec3(0.0, 0.016 * sy, -0.078),
         Vec3(0.0004, 0.0004, 0.00002)},
        {"_KFE", Vec3(0, 1, 0), Vec3(0.0, 0.03745 * sy, -0.16), 0.033, Vec3(0.0, 0.007 * sy, -0.078),
         Vec3(0.0001, 0.0001, 0.000003)},
    };
    int j = 1;
    int ids[3];
    for (int k = 0; k < 3; ++k) {
      j = m->addJoint(j, croc::JointModelRevoluteUnaligned(specs[k].ax), croc::SE3(croc::Mat3::Identity(), specs[k].p),
                      L + specs[k].suffix);
      body(j, specs[k].mass, specs[k].c, specs[k].d);
      m->addFrame(L + specs[k].suffix, j);  // pinocchio adds a JOINT frame per joint
      ids[k] = j;
    }
    m->addFrame(L + "_FOOT", ids[2], croc::SE3(croc::Mat3::Identity(), Vec3(0.0, 0.008 * sy, -0.16)));
    const double lim[3][2] = {{-0.9, 0.9}, {-1.9, 1.9}, {-3.0, 3.0}};
    for (int k = 0; k < 3; ++k) m->setJointLimits(ids[k], lim[k][0], lim[k][1], 20.0);
  }
  VectorXd q = {0.0, 0.0, 0.235, 0.0, 0.0, 0.0, 1.0};
  for (int l = 0; l < 4; ++l) {
    const bool front = l < 2;
    for (double v : front ? VectorXd{0.0, 0.8, -1.6} : VectorXd{0.0, -0.8, 1.6}) q.push_back(v);
  }
  m->referenceConfigurations["standing"] = q;
  return m;
}

// SimpleQuadrupedGaitProblem, the trotting gait (utils/quadruped.py; the C++ class of
// the reference's benchmark has the same builders)
class SimpleQuadrupedGaitProblem {
 public:
  typedef std::shared_ptr<croc::ActionModelBase> Action;
  SimpleQuadrupedGaitProblem(std::shared_ptr<croc::Model> rmodel, const std::string& lf, const std::string& rf,
                             const std::string& lh, const std::string& rh)
      : rmodel_(rmodel), state_(std::make_shared<croc::StateMultibody>(rmodel)),
        actuation_(std::make_shared<croc::ActuationModelFloatingBase>(state_)) {
    lfId = rmodel->getFrameId(lf);
    rfId = rmodel->getFrameId(rf);
    lhId = rmodel->getFrameId(lh);
    rhId = rmodel->getFrameId(rh);
    VectorXd x0 = rmodel->referenceConfigurations.at("standing");
    x0.resize(rmodel->nq() + rmodel->nv(), 0.);
    rmodel->defaultState = x0;
  }

  std::vector<Action> createTrottingModels(const VectorXd& x0, double stepLength, double stepHeight, double timeStep,
                                           int stepKnots, int supportKnots) {
    const VectorXd q0(x0.begin(), x0.begin() + state_->get_nq());
    Vec3 rfPos0 = rmodel_->framePlacement(q0, rfId).translation, rhPos0 = rmodel_->framePlacement(q0, rhId).translation;
    Vec3 lfPos0 = rmodel_->framePlacement(q0, lfId).translation, lhPos0 = rmodel_->framePlacement(q0, lhId).translation;
    Vec3 comRef = (((rfPos0 + rhPos0) + lfPos0) + lhPos0) / 4.;
    comRef[2] = rmodel_->centerOfMass(q0)[2];
    std::vector<Action> doubleSupport;
    for (int k = 0; k < supportKnots; ++k) doubleSupport.push_back(createSwingFootModel(timeStep, all()));
    const double sl = firstStep ? 0.5 * stepLength : stepLength;
    std::vector<Vec3*> f1 = {&rfPos0, &lhPos0};
    auto rflh = createFootstepModels(comRef, f1, sl, stepHeight, timeStep, stepKnots, {lfId, rhId}, {rfId, lhId});
    firstStep = false;
    std::vector<Vec3*> f2 = {&lfPos0, &rhPos0};
    auto lfrh = createFootstepModels(comRef, f2, stepLength, stepHeight, timeStep, stepKnots, {rfId, lhId}, {lfId, rhId});
    std::vector<Action> out = doubleSupport;
    out.insert(out.end(), rflh.begin(), rflh.end());
    out.insert(out.end(), doubleSupport.begin(), doubleSupport.end());
    out.insert(out.end(), lfrh.begin(), lfrh.end());
    return out;
  }

  int lfId, rfId, lhId, rhId;
  bool firstStep = true;
  double mu = 0.7;
  Vec3 nsurf{0., 0., 1.};

 private:
  std::vector<int> all() const { return {lfId, rfId, lhId, rhId}; }

  // quadruped.py:357-405: comPos0 / feetPos0 advance in place
  std::vector<Action> createFootstepModels(Vec3& comPos0, std::vector<Vec3*>& feetPos0, double stepLength,
                                           double stepHeight, double timeStep, int numKnots,
                                           const std::vector<int>& support, const std::vector<int>& swing) {
    const double comPercentage = (double)swing.size() / (double)(support.size() + swing.size());
    std::vector<Action> out;
    std::vector<croc::FramePlacement> swingFootTask;
    for (int k = 0; k < numKnots; ++k) {
      swingFootTask.clear();
      for (size_t s = 0; s < swing.size(); ++s) {
        const double phKnots = numKnots / 2.;
        Vec3 dp;
        if (k < phKnots)
          dp = Vec3(stepLength * (k + 1) / numKnots, 0., stepHeight * k / phKnots);
        else if (k == phKnots)
          dp = Vec3(stepLength * (k + 1) / numKnots, 0., stepHeight);
        else
          dp = Vec3(stepLength * (k + 1) / numKnots, 0., stepHeight * (1 - double(k - phKnots) / phKnots));
        swingFootTask.push_back(croc::FramePlacement(swing[s], croc::SE3(croc::Mat3::Identity(), *feetPos0[s] + dp)));
      }
      const Vec3 comTask = Vec3(stepLength * (k + 1) / numKnots, 0., 0.) * comPercentage + comPos0;
      out.push_back(createSwingFootModel(timeStep, support, &comTask, &swingFootTask));
    }
    out.push_back(createImpulseModel(support, swingFootTask));
    comPos0 = comPos0 + Vec3(stepLength * comPercentage, 0., 0.);
    for (Vec3* p : feetPos0) *p = *p + Vec3(stepLength, 0., 0.);
    return out;
  }

  std::shared_ptr<croc::CostModelState> stateReg(const VectorXd& w, int nu) const {
    VectorXd w2(w.size());
    for (size_t i = 0; i < w.size(); ++i) w2[i] = w[i] * w[i];
    return std::make_shared<croc::CostModelState>(state_, std::make_shared<croc::ActivationModelWeightedQuad>(w2),
                                                  rmodel_->defaultState, nu);
  }

  // quadruped.py:407-461
  Action createSwingFootModel(double timeStep, const std::vector<int>& support, const Vec3* comTask = nullptr,
                              const std::vector<croc::FramePlacement>* swingFootTask = nullptr) {
    const int nu = actuation_->nu, nv = rmodel_->nv();
    auto contactModel = std::make_shared<croc::ContactModelMultiple>(state_, nu);
    const double gains[2] = {0., 50.};
    for (int i : support)
      contactModel->addContact(rmodel_->frames[i].name + "_contact",
                               std::make_shared<croc::ContactModel3D>(
                                   state_, croc::FrameTranslation(i, Vec3(0., 0., 0.)), nu, gains));
    auto costModel = std::make_shared<croc::CostModelSum>(state_, nu);
    if (comTask) costModel->addCost("comTrack", std::make_shared<croc::CostModelCoMPosition>(state_, *comTask, nu), 1e6);
    for (int i : support) {
      croc::FrictionCone cone(nsurf, mu, 4, false);
      auto fc = std::make_shared<croc::CostModelContactFrictionCone>(
          state_, std::make_shared<croc::ActivationModelQuadraticBarrier>(croc::ActivationBounds(cone.lb, cone.ub)),
          croc::FrameFrictionCone(i, cone), nu);
      costModel->addCost(rmodel_->frames[i].name + "_frictionCone", fc, 1e1);
    }
    if (swingFootTask)
      for (const croc::FramePlacement& t : *swingFootTask)
        costModel->addCost(rmodel_->frames[t.id].name + "_footTrack",
                           std::make_shared<croc::CostModelFrameTranslation>(
                               state_, croc::FrameTranslation(t.id, t.placement.translation), nu),
                           1e6);
    VectorXd w;
    for (int i = 0; i < 3; ++i) w.push_back(0.);
    for (int i = 0; i < 3; ++i) w.push_back(500.);
    for (int i = 0; i < nv - 6; ++i) w.push_back(0.01);
    for (int i = 0; i < 6; ++i) w.push_back(10.);
    for (int i = 0; i < nv - 6; ++i) w.push_back(1.);
    costModel->addCost("stateReg", stateReg(w, nu), 1e1);
    costModel->addCost("ctrlReg", std::make_shared<croc::CostModelControl>(state_, nu), 1e-1);
    // state bounds (quadruped.py:449-454; the free-flyer rows at +-DBL_MAX, see crocoddyl_amd/gaits.py)
    const VectorXd& slb = state_->get_lb();
    const VectorXd& sub = state_->get_ub();
    bool finite = true;
    for (int i = 7; i < state_->get_nq(); ++i) finite = finite && std::isfinite(slb[i]);
    if (finite) {
      VectorXd lb, ub;
      auto clip = [](double v) { return std::isinf(v) ? (v > 0 ? DBL_MAX : -DBL_MAX) : v; };
      for (int i = 1; i < nv + 1; ++i) lb.push_back(clip(slb[i])), ub.push_back(clip(sub[i]));
      for (size_t i = slb.size() - nv; i < slb.size(); ++i) lb.push_back(clip(slb[i])), ub.push_back(clip(sub[i]));
      VectorXd zero(rmodel_->defaultState.size(), 0.);
      costModel->addCost("stateBounds",
                         std::make_shared<croc::CostModelState>(
                             state_,
                             std::make_shared<croc::ActivationModelQuadraticBarrier>(croc::ActivationBounds(lb, ub)),
                             zero, nu),
                         1e3);
    }
    auto dmodel = std::make_shared<croc::DifferentialActionModelContactFwdDynamics>(state_, actuation_, contactModel,
                                                                                    costModel, 0., true);
    return std::make_shared<croc::IntegratedActionModelEuler>(dmodel, timeStep);
  }

  // quadruped.py:522-553: ImpulseModel3D on the support feet
  Action createImpulseModel(const std::vector<int>& support, const std::vector<croc::FramePlacement>& swingFootTask) {
    const int nv = rmodel_->nv();
    auto impulseModel = std::make_shared<croc::ImpulseModelMultiple>(state_);
    for (int i : support)
      impulseModel->addImpulse(rmodel_->frames[i].name + "_impulse", std::make_shared<croc::ImpulseModel3D>(state_, i));
    auto costModel = std::make_shared<croc::CostModelSum>(state_, 0);
    for (const croc::FramePlacement& t : swingFootTask)
      costModel->addCost(rmodel_->frames[t.id].name + "_footTrack",
                         std::make_shared<croc::CostModelFrameTranslation>(
                             state_, croc::FrameTranslation(t.id, t.placement.translation), 0),
                         1e7);
    VectorXd w;
    for (int i = 0; i < 6; ++i) w.push_back(1.);
    for (int i = 0; i < nv - 6; ++i) w.push_back(10.);
    for (int i = 0; i < nv; ++i) w.push_back(10.);
    costModel->addCost("stateReg", stateReg(w, 0), 1e1);
    auto model = std::make_shared<croc::ActionModelImpulseFwdDynamics>(state_, impulseModel, costModel);
    model->set_JMinvJt_damping(1e-12);
    model->set_r_coeff(0.0);
    return model;
  }

  std::shared_ptr<croc::Model> rmodel_;
  std::shared_ptr<croc::StateMultibody> state_;
  std::shared_ptr<croc::ActuationModelFloatingBase> actuation_;
};

static bool write_all(const char* path, const std::vector<std::pair<const void*, size_t> >& parts) {
  FILE* f = std::fopen(path, "wb");
  if (!f) return false;
  for (const auto& p : parts) std::fwrite(p.first, 1, p.second, f);
  std::fclose(f);
  return true;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s pack|solve FILE [MAXITER]\n", argv[0]);
    return 2;
  }
  try {
    const int T = 60;  // C4: 27 step knots + 2 support knots, stretched to T = 60 (crocoddyl_amd/synthetic.py)
    auto solo = sample_solo12();
    SimpleQuadrupedGaitProblem gait(solo, "FL_FOOT", "FR_FOOT", "HL_FOOT", "HR_FOOT");
    const VectorXd x0 = solo->defaultState;
    std::vector<SimpleQuadrupedGaitProblem::Action> models =
        gait.createTrottingModels(x0, 0.15, 0.1, 1e-2, std::max(1, T / 2 - 3), 2);
    models.resize(T);
    auto problem = std::make_shared<croc::ShootingProblem>(x0, models, models.back());
    if (!std::strcmp(argv[1], "pack")) {
      std::vector<fddp_knot_desc> knots;
      VectorXd pool;
      problem->pack(knots, pool);
      const int64_t nk = (int64_t)knots.size(), np = (int64_t)pool.size();
      const int32_t dims[4] = {problem->get_nx(), problem->get_ndx(), problem->get_nu_max(), problem->get_T()};
      if (!write_all(argv[2], {{dims, sizeof(dims)}, {&nk, 8}, {knots.data(), sizeof(fddp_knot_desc) * nk}, {&np, 8},
                               {pool.data(), 8 * np}}))
        return 3;
      std::printf("packed T=%d nx=%d ndx=%d nu_max=%d knots=%lld pool=%lld\n", problem->get_T(), problem->get_nx(),
                  problem->get_ndx(), problem->get_nu_max(), (long long)nk, (long long)np);
      return 0;
    }
    const int maxiter = argc > 3 ? std::atoi(argv[3]) : 3;
    croc::SolverFDDP solver(problem);
    std::vector<VectorXd> xs(T + 1, x0), us;  // the benchmark's warm start: the default state, zero controls
    const bool ok = solver.solve(xs, us, maxiter, false, 1e-9);
    const auto xo = solver.get_xs();
    const auto uo = solver.get_us();
    VectorXd flat;
    for (const auto& x : xo) flat.insert(flat.end(), x.begin(), x.end());
    for (const auto& u : uo) flat.insert(flat.end(), u.begin(), u.end());
    const fddp_result r = solver.get_results()[0];
    if (!write_all(argv[2], {{&r, sizeof(r)}, {flat.data(), 8 * flat.size()}})) return 3;
    std::printf("trot solved=%d iter=%zu cost=%.12e steplength=%g\n", ok, solver.get_iter(), solver.get_cost(),
                solver.get_steplength());
    return 0;
  } catch (const croc::Exception& e) {
    std::printf("exception: %s\n", e.what());
    return 1;
  }
}
