// crocoddyl_amd C++ facade over libfddp_hip (include/fddp_hip.h), header-only.
//
// Mirrors the reference's C++ API for the hot path so a C++ caller switches by
// swapping the namespace:
//   crocoddyl::ShootingProblem(x0, running_models, terminal_model)
//       include/crocoddyl/core/optctrl/shooting.hpp:48-63
//   crocoddyl::SolverFDDP(problem).solve(init_xs, init_us, maxiter, is_feasible, reginit)
//       include/crocoddyl/core/solvers/fddp.hpp:50-101, src/core/solvers/fddp.cpp:19-105
//   crocoddyl::SolverBoxFDDP(problem)  include/crocoddyl/core/solvers/box-fddp.hpp, src/core/solvers/box-fddp.cpp
//   ActionModelAbstract::set_u_lb / set_u_ub / get_has_control_limits  core/action-base.hxx:107-144
//   crocoddyl::ActionModelLQR(nx, nu, drift_free)          core/actions/lqr.hpp:21-60
//   crocoddyl::ActionModelUnicycle()                        core/actions/unicycle.hpp
//   crocoddyl::DifferentialActionModelLQR(nq, nu, drift_free), IntegratedActionModelEuler(model, dt)
// Errors raise crocoddyl_amd::Exception (the reference's throw_pretty /
// crocoddyl::Exception, core/utils/exception.hpp:23-50). Vectors are any type
// with data()/size() (std::vector<double>, Eigen::VectorXd); matrices are
// column-major (Eigen's default order).
// Link: -lfddp_hip (crocoddyl_amd/lib). All numerical work runs on the GPU.
#ifndef CROCODDYL_AMD_SOLVER_FDDP_HIP_HPP_
#define CROCODDYL_AMD_SOLVER_FDDP_HIP_HPP_

#include <cmath>
#include <cstdio>
#include <exception>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../fddp_hip.h"

namespace crocoddyl_amd {

struct Exception : std::runtime_error {
  explicit Exception(const std::string& m) : std::runtime_error(m) {}
};

inline void check(int rc, const char* what) {
  if (rc != FDDP_OK) throw Exception(std::string(what) + ": " + fddp_last_error());
}

typedef std::vector<double> VectorXd;  // column vectors / column-major matrices

template <class V>
inline VectorXd to_vec(const V& v) {
  return VectorXd(v.data(), v.data() + v.size());
}

// Parameter carriers with the reference defaults. pack() appends this
// model's block (layout: include/fddp_hip.h) to `pool`.
// Control limits (action-base.hxx:20-22, 107-144): -inf / +inf by default.
struct ControlLimits {
  template <class V>
  void set_u_lb(const V& v) {
    if ((int)v.size() != limits_nu()) throw Exception("Invalid argument: lower bound has wrong dimension");
    u_lb_ = to_vec(v);
  }
  template <class V>
  void set_u_ub(const V& v) {
    if ((int)v.size() != limits_nu()) throw Exception("Invalid argument: upper bound has wrong dimension");
    u_ub_ = to_vec(v);
  }
  VectorXd get_u_lb() const { return u_lb_.empty() ? VectorXd(limits_nu(), -INFINITY) : u_lb_; }
  VectorXd get_u_ub() const { return u_ub_.empty() ? VectorXd(limits_nu(), INFINITY) : u_ub_; }
  bool get_has_control_limits() const {  // update_has_control_limits (action-base.hxx:142-144)
    bool l = false, u = false;
    for (double v : get_u_lb()) l = l || std::isfinite(v);
    for (double v : get_u_ub()) u = u || std::isfinite(v);
    return l && u;
  }
  virtual ~ControlLimits() {}
  virtual int limits_nu() const = 0;

 protected:
  VectorXd u_lb_, u_ub_;
};

struct ActionModelBase : ControlLimits {
  virtual ~ActionModelBase() {}
  virtual int kind() const = 0;
  virtual int nx() const = 0;
  virtual int ndx() const { return nx(); }  // StateAbstract::get_ndx (nx - 1 on a free-flyer state)
  virtual int nu() const = 0;
  virtual void pack(VectorXd& pool) const = 0;
  int limits_nu() const { return nu(); }
};

// A differential (continuous-time) action model the device integrates with
// IntegratedActionModelEuler (core/diff-action-base.hpp:41-72): its knot kind
// under Euler and the block packer for a step dt.
struct DifferentialActionModelBase : ControlLimits {
  virtual ~DifferentialActionModelBase() {}
  virtual int euler_kind() const = 0;
  virtual int nx() const = 0;
  virtual int ndx() const { return nx(); }
  virtual int nu() const = 0;
  virtual void pack_euler(double dt, VectorXd& pool) const = 0;
  int limits_nu() const { return nu(); }
};

inline VectorXd eye(int r, int c) {
  VectorXd m((size_t)r * c, 0.);
  for (int i = 0; i < r && i < c; ++i) m[(size_t)i * r + i] = 1.;
  return m;
}

struct ActionModelLQR : ActionModelBase {  // lqr.hxx:13-25
  int nx_, nu_;
  bool drift_free;
  VectorXd Fx, Fu, f0, Lxx, Lxu, Luu, lx, lu;
  ActionModelLQR(int nx, int nu, bool drift_free_ = true)
      : nx_(nx), nu_(nu), drift_free(drift_free_), Fx(eye(nx, nx)), Fu(eye(nx, nu)), f0(nx, 1.), Lxx(eye(nx, nx)),
        Lxu(eye(nx, nu)), Luu(eye(nu, nu)), lx(nx, 1.), lu(nu, 1.) {}
  int kind() const { return FDDP_KNOT_LQR; }
  int nx() const { return nx_; }
  int nu() const { return nu_; }
  void pack(VectorXd& p) const {
    const double hdr[FDDP_PARAM_HEADER] = {drift_free ? 1. : 0., 0., 0., 0.};
    p.insert(p.end(), hdr, hdr + FDDP_PARAM_HEADER);
    for (const VectorXd* v : {&Fx, &Fu, &f0, &Lxx, &Lxu, &Luu, &lx, &lu}) p.insert(p.end(), v->begin(), v->end());
  }
};

struct ActionModelUnicycle : ActionModelBase {  // unicycle.hxx:13-16
  double dt = 0.1, wx = 10., wu = 1.;
  int kind() const { return FDDP_KNOT_UNICYCLE; }
  int nx() const { return 3; }
  int nu() const { return 2; }
  void pack(VectorXd& p) const {
    const double hdr[FDDP_PARAM_HEADER] = {dt, wx, wu, 0.};
    p.insert(p.end(), hdr, hdr + FDDP_PARAM_HEADER);
  }
};

struct DifferentialActionModelLQR : DifferentialActionModelBase {  // diff-lqr.hxx:14-28
  int nq, nu_;
  bool drift_free;
  VectorXd Fq, Fv, Fu, f0, Lxx, Lxu, Luu, lx, lu;
  DifferentialActionModelLQR(int nq_, int nu__, bool drift_free_ = true)
      : nq(nq_), nu_(nu__), drift_free(drift_free_), Fq(eye(nq_, nq_)), Fv(eye(nq_, nq_)), Fu(eye(nq_, nu__)),
        f0(nq_, 1.), Lxx(eye(2 * nq_, 2 * nq_)), Lxu(eye(2 * nq_, nu__)), Luu(eye(nu__, nu__)), lx(2 * nq_, 1.),
        lu(nu__, 1.) {}
  int euler_kind() const { return FDDP_KNOT_EULER_DIFFLQR; }
  int nx() const { return 2 * nq; }
  int nu() const { return nu_; }
  void pack_euler(double dt, VectorXd& p) const {
    const double hdr[FDDP_PARAM_HEADER] = {dt, drift_free ? 1. : 0., 0., 0.};
    p.insert(p.end(), hdr, hdr + FDDP_PARAM_HEADER);
    for (const VectorXd* v : {&Fq, &Fv, &Fu, &f0, &Lxx, &Lxu, &Luu, &lx, &lu}) p.insert(p.end(), v->begin(), v->end());
  }
};

struct IntegratedActionModelEuler : ActionModelBase {  // euler.hxx:16-35
  std::shared_ptr<DifferentialActionModelBase> differential;
  double dt;
  IntegratedActionModelEuler(std::shared_ptr<DifferentialActionModelBase> d, double time_step = 1e-3)
      : differential(d), dt(time_step < 0. ? 1e-3 : time_step) {
    set_u_lb(d->get_u_lb());  // euler.hxx:25-26
    set_u_ub(d->get_u_ub());
  }
  int kind() const { return differential->euler_kind(); }
  int nx() const { return differential->nx(); }
  int ndx() const { return differential->ndx(); }
  int nu() const { return differential->nu(); }
  void pack(VectorXd& p) const { differential->pack_euler(dt, p); }
};

// ShootingProblem over one problem (B = 1) or B problems sharing the models
// (x0s of size B*nx).
class ShootingProblem {
 public:
  template <class V>
  ShootingProblem(const V& x0, const std::vector<std::shared_ptr<ActionModelBase> >& running,
                  std::shared_ptr<ActionModelBase> terminal, int batch = 1)
      : x0_(to_vec(x0)), running_(running), terminal_(terminal), B_(batch) {
    if (running.empty()) throw Exception("Invalid argument: no running models");
    nx_ = running[0]->nx();
    ndx_ = running[0]->ndx();
    nu_max_ = 0;
    for (size_t i = 0; i < running.size(); ++i) {  // shooting.hxx:28-49
      if (running[i]->nx() != nx_) throw Exception("Invalid argument: nx in " + std::to_string(i) + " node is not consistent");
      if (running[i]->ndx() != ndx_)
        throw Exception("Invalid argument: ndx in " + std::to_string(i) + " node is not consistent");
      if (running[i]->nu() > nu_max_) nu_max_ = running[i]->nu();
    }
    if (terminal->nx() != nx_) throw Exception("Invalid argument: nx in terminal node is not consistent");
    if ((int)x0_.size() != nx_ * B_) throw Exception("Invalid argument: x0 has wrong dimension");
  }
  int get_T() const { return (int)running_.size(); }
  int get_nx() const { return nx_; }
  int get_ndx() const { return ndx_; }
  int get_nu_max() const { return nu_max_; }
  int get_B() const { return B_; }
  const VectorXd& get_x0() const { return x0_; }
  template <class V>
  void set_x0(const V& x0) {  // shooting.hxx:391-397
    VectorXd v = to_vec(x0);
    if ((int)v.size() != nx_ * B_) throw Exception("Invalid argument: x0 has wrong dimension");
    x0_ = v;
  }
  // knot descriptors + pool (shared models packed once)
  void pack(std::vector<fddp_knot_desc>& knots, VectorXd& pool) const {
    std::vector<const ActionModelBase*> seen;
    std::vector<int64_t> offs;
    knots.clear();
    pool.clear();
    for (int t = 0; t <= get_T(); ++t) {
      const ActionModelBase* m = t < get_T() ? running_[t].get() : terminal_.get();
      int64_t off = -1;
      for (size_t i = 0; i < seen.size(); ++i)
        if (seen[i] == m) off = offs[i];
      if (off < 0) {
        off = (int64_t)pool.size();
        m->pack(pool);
        seen.push_back(m);
        offs.push_back(off);
      }
      fddp_knot_desc d;
      d.kind = m->kind();
      d.nu = m->nu();
      d.param_offset = off;
      d.param_stride = 0;
      knots.push_back(d);
    }
  }
  // control limits of the running knots, B*T*nu_max each (fddp_set_control_limits);
  // false when no model has any limit
  bool pack_limits(VectorXd& lb, VectorXd& ub) const {
    const int T = get_T(), m = nu_max_;
    lb.assign((size_t)B_ * T * m, -INFINITY);
    ub.assign((size_t)B_ * T * m, INFINITY);
    bool any = false;
    for (int t = 0; t < T; ++t) {
      const VectorXd l = running_[t]->get_u_lb(), u = running_[t]->get_u_ub();
      for (int i = 0; i < running_[t]->nu(); ++i) {
        any = any || std::isfinite(l[i]) || std::isfinite(u[i]);
        for (int b = 0; b < B_; ++b) {
          lb[((size_t)b * T + t) * m + i] = l[i];
          ub[((size_t)b * T + t) * m + i] = u[i];
        }
      }
    }
    return any;
  }

 private:
  VectorXd x0_;
  std::vector<std::shared_ptr<ActionModelBase> > running_;
  std::shared_ptr<ActionModelBase> terminal_;
  int nx_, ndx_, nu_max_, B_;
};

class SolverFDDP;

// CallbackAbstract (solver-base.hpp:284-298): called once per iteration of solve(),
// after the regularisation update and stoppingCriteria (fddp.cpp:92-98), with the
// solver's getters reading that iteration's state (element 0 when batched;
// get_results() / reported() give every element).
class CallbackAbstract {
 public:
  virtual ~CallbackAbstract() {}
  virtual void operator()(SolverFDDP& solver) = 0;
};

// SolverFDDP (fddp.hpp:50-101) on the GPU.
class SolverFDDP {
 public:
  explicit SolverFDDP(std::shared_ptr<ShootingProblem> problem, int device = 0) : problem_(problem) {
    std::vector<fddp_knot_desc> knots;
    VectorXd pool;
    problem->pack(knots, pool);
    fddp_dims d;
    d.nx = problem->get_nx();
    d.ndx = problem->get_ndx();
    d.nu_max = problem->get_nu_max();
    d.T = problem->get_T();
    d.B = problem->get_B();
    dims_ = d;
    fddp_handle* h = nullptr;
    if (fddp_abi_version() != FDDP_ABI_VERSION)
      throw Exception("libfddp_hip C ABI version " + std::to_string(fddp_abi_version()) + ", this header is " +
                      std::to_string(FDDP_ABI_VERSION));
    check(fddp_create(&d, knots.data(), pool.data(), (int64_t)pool.size(), device, &h), "fddp_create");
    h_.reset(h, fddp_destroy);
    fddp_default_params(&params_);
    check(fddp_set_x0(h, problem->get_x0().data()), "fddp_set_x0");
    res_.resize(d.B);
  }

  // fddp.cpp:19-105 ; init vectors empty => state.zero() / zeros (solver-base.cpp:46-65)
  template <class V = VectorXd>
  bool solve(const std::vector<V>& init_xs = std::vector<V>(), const std::vector<V>& init_us = std::vector<V>(),
             std::size_t maxiter = 100, bool is_feasible = false, double reginit = 1e-9) {
    setCandidate(init_xs, init_us, is_feasible);
    check(fddp_set_x0(h_.get(), problem_->get_x0().data()), "fddp_set_x0");
    VectorXd lb, ub;  // the models' current limits (SolverFDDP ignores them)
    const bool lim = problem_->pack_limits(lb, ub);
    check(fddp_set_control_limits(h_.get(), lim ? lb.data() : nullptr, lim ? ub.data() : nullptr),
          "fddp_set_control_limits");
    check(fddp_set_params(h_.get(), &params_), "fddp_set_params");
    check(fddp_set_callback(h_.get(), callbacks_.empty() ? nullptr : &SolverFDDP::on_iteration, this),
          "fddp_set_callback");
    cb_error_ = nullptr;
    const int rc = fddp_solve(h_.get(), (int)maxiter, is_feasible ? 1 : 0, reginit, res_.data());
    fddp_set_callback(h_.get(), nullptr, nullptr);
    reported_.clear();
    // a callback that threw stopped the solve after its iteration (fddp.cpp:92-98):
    // res_ holds that iteration's results, and the callback's exception is rethrown as is
    if (rc == FDDP_ERR_CALLBACK_ABORT && cb_error_) {
      std::exception_ptr e = cb_error_;
      cb_error_ = nullptr;
      std::rethrow_exception(e);
    }
    check(rc, "fddp_solve");
    return res_[0].status == FDDP_STATUS_CONVERGED;
  }

  // ---- the solver's phases one at a time (SolverDDP / SolverFDDP methods) --------------
  // SolverDDP::calcDiff (ddp.cpp:157-178): problem.calc at iter 0, problem.calcDiff, the
  // gaps; returns cost_ (element 0; get_costs() every element)
  double calcDiff() {
    costs_.assign(dims_.B, 0.);
    check(fddp_calc_diff(h_.get(), costs_.data()), "fddp_calc_diff");
    return costs_[0];
  }
  // SolverDDP::backwardPass (ddp.cpp:180-253); throws "backward_error" as the reference
  // (batched: when any element fails; get_step_status() says which)
  void backwardPass() {
    check(fddp_set_params(h_.get(), &params_), "fddp_set_params");
    step_status_.assign(dims_.B, 0);
    check(fddp_backward_pass(h_.get(), step_status_.data()), "fddp_backward_pass");
    for (int32_t v : step_status_)
      if (v) throw Exception("backward_error");
  }
  // SolverDDP::computeDirection (ddp.cpp:120-125)
  void computeDirection(bool recalc = true) {
    if (recalc) calcDiff();
    backwardPass();
  }
  // SolverFDDP::forwardPass (fddp.cpp:149-225): xs_try / us_try / cost_try; throws
  // "forward_error" as the reference; stepLength outside [0, 1] is an invalid argument
  void forwardPass(double steplength) {
    costs_try_.assign(dims_.B, 0.);
    step_status_.assign(dims_.B, 0);
    check(fddp_forward_pass(h_.get(), steplength, costs_try_.data(), step_status_.data()), "fddp_forward_pass");
    for (int32_t v : step_status_)
      if (v) throw Exception("forward_error");
  }
  // SolverDDP::tryStep (ddp.cpp:127-130): cost_ - cost_try_
  double tryStep(double steplength = 1.) {
    std::vector<double> dv(dims_.B, 0.);
    step_status_.assign(dims_.B, 0);
    check(fddp_try_step(h_.get(), steplength, dv.data(), step_status_.data()), "fddp_try_step");
    for (int32_t v : step_status_)
      if (v) throw Exception("forward_error");
    return dv[0];
  }
  // SolverDDP::stoppingCriteria (ddp.cpp:132-142)
  double stoppingCriteria() {
    std::vector<double> s(dims_.B, 0.);
    check(fddp_stopping_criteria(h_.get(), s.data()), "fddp_stopping_criteria");
    return s[0];
  }
  // SolverFDDP::updateExpectedImprovement / expectedImprovement (fddp.cpp:107-147)
  void updateExpectedImprovement() { check(fddp_update_expected_improvement(h_.get()), "fddp_update_expected_improvement"); }
  std::vector<double> expectedImprovement() {
    std::vector<double> d(2 * (size_t)dims_.B, 0.);
    check(fddp_expected_improvement(h_.get(), d.data()), "fddp_expected_improvement");
    return {d[0], d[1]};
  }
  double get_cost_try() const { return costs_try_.empty() ? 0. : costs_try_[0]; }
  const std::vector<double>& get_costs() const { return costs_; }
  const std::vector<double>& get_costs_try() const { return costs_try_; }
  const std::vector<int32_t>& get_step_status() const { return step_status_; }
  // SolverDDP getters (ddp.hpp:60-271), element 0: K_[t] (nu x ndx, column-major), k_[t],
  // fs_[t]; Vxx / Vx / Q* need set_debug(true) before the backward pass (device stores)
  std::vector<VectorXd> get_K() const { return quantity(FDDP_Q_K, dims_.T, (size_t)dims_.nu_max * dims_.ndx); }
  std::vector<VectorXd> get_k() const { return quantity(FDDP_Q_KV, dims_.T, dims_.nu_max); }
  std::vector<VectorXd> get_fs() const { return quantity(FDDP_Q_FS, dims_.T + 1, dims_.ndx); }
  std::vector<VectorXd> get_Vxx() const { return quantity(FDDP_Q_VXX, dims_.T + 1, (size_t)dims_.ndx * dims_.ndx); }
  std::vector<VectorXd> get_Vx() const { return quantity(FDDP_Q_VX, dims_.T + 1, dims_.ndx); }
  std::vector<VectorXd> get_Quu() const { return quantity(FDDP_Q_QUU, dims_.T, (size_t)dims_.nu_max * dims_.nu_max); }
  std::vector<VectorXd> get_Qu() const { return quantity(FDDP_Q_QU, dims_.T, dims_.nu_max); }
  void set_debug(bool on) { check(fddp_set_debug(h_.get(), on ? 1 : 0), "fddp_set_debug"); }
  std::vector<VectorXd> get_xs_try() const {
    VectorXd a((size_t)dims_.B * (dims_.T + 1) * dims_.nx);
    check(fddp_get_xs_try(h_.get(), a.data()), "fddp_get_xs_try");
    std::vector<VectorXd> out;
    for (int t = 0; t <= dims_.T; ++t) out.push_back(VectorXd(a.begin() + t * dims_.nx, a.begin() + (t + 1) * dims_.nx));
    return out;
  }
  std::vector<VectorXd> get_us_try() const {
    VectorXd a((size_t)dims_.B * dims_.T * dims_.nu_max);
    check(fddp_get_us_try(h_.get(), a.data()), "fddp_get_us_try");
    std::vector<VectorXd> out;
    for (int t = 0; t < dims_.T; ++t)
      out.push_back(VectorXd(a.begin() + t * dims_.nu_max, a.begin() + (t + 1) * dims_.nu_max));
    return out;
  }
  // the solver members the phases read (a fresh solver: iter 0, xreg = ureg = NaN)
  void set_solver_state(int iter, double xreg, double ureg, bool was_feasible) {
    check(fddp_set_solver_state(h_.get(), iter, xreg, ureg, was_feasible ? 1 : 0), "fddp_set_solver_state");
  }

  // SolverAbstract::setCallbacks / getCallbacks (solver-base.cpp:69-77)
  void setCallbacks(const std::vector<std::shared_ptr<CallbackAbstract> >& callbacks) { callbacks_ = callbacks; }
  const std::vector<std::shared_ptr<CallbackAbstract> >& getCallbacks() const { return callbacks_; }
  // inside a callback: which elements ran the current iteration
  const std::vector<int32_t>& reported() const { return reported_; }

  template <class V>
  void setCandidate(const std::vector<V>& xs_warm, const std::vector<V>& us_warm, bool is_feasible) {
    const int T = dims_.T, nx = dims_.nx, nu = dims_.nu_max, B = dims_.B;
    VectorXd xs, us;
    if (!xs_warm.empty()) {
      if ((int)xs_warm.size() != T + 1) throw Exception("Warm start state has wrong dimension");
      for (int b = 0; b < B; ++b)
        for (const V& x : xs_warm) xs.insert(xs.end(), x.data(), x.data() + nx);
    }
    if (!us_warm.empty()) {
      if ((int)us_warm.size() != T) throw Exception("Warm start control has wrong dimension");
      for (int b = 0; b < B; ++b)
        for (const V& u : us_warm) {
          VectorXd row(nu, 0.);
          for (int i = 0; i < (int)u.size() && i < nu; ++i) row[i] = u.data()[i];
          us.insert(us.end(), row.begin(), row.end());
        }
    }
    check(fddp_set_candidate(h_.get(), xs.empty() ? nullptr : xs.data(), us.empty() ? nullptr : us.data(),
                             is_feasible ? 1 : 0),
          "fddp_set_candidate");
  }

  std::vector<VectorXd> get_xs() const {  // element 0 (B = 1: the problem)
    VectorXd a((size_t)dims_.B * (dims_.T + 1) * dims_.nx);
    check(fddp_get_xs(h_.get(), a.data(), 0), "fddp_get_xs");
    std::vector<VectorXd> out;
    for (int t = 0; t <= dims_.T; ++t) out.push_back(VectorXd(a.begin() + t * dims_.nx, a.begin() + (t + 1) * dims_.nx));
    return out;
  }
  std::vector<VectorXd> get_us() const {
    VectorXd a((size_t)dims_.B * dims_.T * dims_.nu_max);
    check(fddp_get_us(h_.get(), a.data(), 0), "fddp_get_us");
    std::vector<VectorXd> out;
    for (int t = 0; t < dims_.T; ++t)
      out.push_back(VectorXd(a.begin() + t * dims_.nu_max, a.begin() + (t + 1) * dims_.nu_max));
    return out;
  }
  const std::vector<fddp_result>& get_results() const { return res_; }  // per batch element
  double get_cost() const { return res_[0].cost; }
  double get_stop() const { return res_[0].stop; }
  std::size_t get_iter() const { return (std::size_t)res_[0].iter; }
  double get_xreg() const { return res_[0].xreg; }
  double get_ureg() const { return res_[0].ureg; }
  double get_steplength() const { return res_[0].steplength; }
  bool get_is_feasible() const { return res_[0].is_feasible != 0; }
  double get_dV() const { return res_[0].dV; }
  double get_dVexp() const { return res_[0].dVexp; }
  std::vector<double> get_d() const { return {res_[0].d0, res_[0].d1}; }

  // thresholds with the reference setter validation (enforced by fddp_set_params)
  void set_th_stop(double v) { params_.th_stop = v; push(); }
  void set_th_acceptstep(double v) { params_.th_acceptstep = v; push(); }
  void set_th_acceptnegstep(double v) { params_.th_acceptnegstep = v; push(); }
  void set_th_grad(double v) { params_.th_grad = v; push(); }
  void set_th_stepdec(double v) { params_.th_stepdec = v; push(); }
  void set_th_stepinc(double v) { params_.th_stepinc = v; push(); }
  void set_regfactor(double v) { params_.regfactor = v; push(); }
  void set_regmin(double v) { params_.regmin = v; push(); }
  void set_regmax(double v) { params_.regmax = v; push(); }
  double get_th_stop() const { return params_.th_stop; }
  fddp_handle* handle() const { return h_.get(); }

 protected:
  void push() {
    const int rc = fddp_set_params(h_.get(), &params_);
    if (rc != FDDP_OK) {
      fddp_get_params(h_.get(), &params_);  // keep the last valid thresholds
      throw Exception(std::string("Invalid argument: ") + fddp_last_error());
    }
  }
  std::shared_ptr<ShootingProblem> problem_;
  std::shared_ptr<fddp_handle> h_;
  fddp_dims dims_;
  fddp_params params_;
  std::vector<fddp_result> res_;
  std::vector<std::shared_ptr<CallbackAbstract> > callbacks_;
  std::vector<int32_t> reported_;
  std::exception_ptr cb_error_;
  std::vector<double> costs_, costs_try_;
  std::vector<int32_t> step_status_;

  // per-knot blocks of element 0 (fddp_get_quantity: [b][t][per])
  std::vector<VectorXd> quantity(int which, int nk, size_t per) const {
    VectorXd a((size_t)dims_.B * nk * per);
    check(fddp_get_quantity(h_.get(), which, a.data()), "fddp_get_quantity");
    std::vector<VectorXd> out;
    for (int t = 0; t < nk; ++t) out.push_back(VectorXd(a.begin() + t * per, a.begin() + (t + 1) * per));
    return out;
  }

 private:
  // fddp_iteration_callback: the C ABI calls it between iterations; no exception may
  // cross the ABI, so one is kept, fddp_solve is told to stop (return 1) and the
  // exception is rethrown after it returns
  static int on_iteration(void* user, int, const fddp_result* results, const int32_t* reported, int B) {
    SolverFDDP* self = static_cast<SolverFDDP*>(user);
    self->res_.assign(results, results + B);
    self->reported_.assign(reported, reported + B);
    if (self->dims_.B == 1 && !reported[0]) return 0;
    try {
      for (const auto& cb : self->callbacks_) (*cb)(*self);
    } catch (...) {  // any exception: kept, rethrown by solve() after fddp_solve returns
      self->cb_error_ = std::current_exception();
      return 1;
    }
    return 0;
  }
};

// CallbackVerbose (core/utils/callbacks.cpp:13-67): one table row per iteration,
// a header every 10 iterations; level 2 adds dV-exp and dV.
class CallbackVerbose : public CallbackAbstract {
 public:
  explicit CallbackVerbose(int level = 1, FILE* out = stdout) : level_(level), out_(out) {}
  // batched: the row of the first element that ran this iteration (reported()), so a
  // finished element 0 does not repeat its last row under later iterations
  void operator()(SolverFDDP& s) override {
    std::size_t e = 0;
    const std::vector<int32_t>& rep = s.reported();
    while (e < rep.size() && !rep[e]) ++e;
    if (!rep.empty() && e == rep.size()) return;
    if (rep.empty()) e = 0;
    const fddp_result& r = s.get_results()[e];
    if (r.iter % 10 == 0)
      std::fprintf(out_, "iter \t cost \t      stop \t    grad \t  xreg \t      ureg \t step \t feas%s\n",
                   level_ == 2 ? " \tdV-exp \t      dV" : "");
    std::fprintf(out_, "%4d  %.5e  %.5e  %.5e  %.5e  %.5e   %.4f     %d", r.iter, r.cost, r.stop, -r.d1, r.xreg,
                 r.ureg, r.steplength, r.is_feasible ? 1 : 0);
    if (level_ == 2) std::fprintf(out_, "  %.5e  %.5e", r.dVexp, r.dV);
    std::fprintf(out_, "\n");
  }

 private:
  int level_;
  FILE* out_;
};

// SolverBoxFDDP (box-fddp.cpp:15-164): box-QP gains on limited knots once
// feasible, clamped controls in the forward pass; th_stop = 5e-5 (:28).
class SolverBoxFDDP : public SolverFDDP {
 public:
  explicit SolverBoxFDDP(std::shared_ptr<ShootingProblem> problem, int device = 0) : SolverFDDP(problem, device) {
    check(fddp_set_solver_kind(h_.get(), FDDP_SOLVER_BOXFDDP), "fddp_set_solver_kind");
    params_.th_stop = 5e-5;
    push();
  }
};

}  // namespace crocoddyl_amd

#endif  // CROCODDYL_AMD_SOLVER_FDDP_HIP_HPP_
