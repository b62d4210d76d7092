// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// Standalone driver of the CPU oracle (fddp_oracle.cpp compiled in): reads a
// packed problem written by tools/dump_problem.py and times the bench protocol
// (the same warm start solved with solve(maxiter=1, reg_init=0.1) each step,
// benchmark/bipedal_walk_optctrl.py:36-43). It exists to diagnose host-specific
// builds of the oracle (e.g. -march=native) outside Python: a fault prints the
// backtrace of the faulting thread (glibc backtrace, addresses for addr2line).
//
// usage: cpu_driver PROBLEM_FILE THREADS STEPS [MODE (2 batch-parallel, 1 knot-parallel)]
// ============================================================================
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/fddp_hip.h"

extern "C" {
struct oracle_handle;
int oracle_create(const fddp_dims*, const fddp_knot_desc*, const double*, int64_t, oracle_handle**);
void oracle_destroy(oracle_handle*);
int oracle_set_threading(oracle_handle*, int, int);
int oracle_set_x0(oracle_handle*, const double*);
int oracle_set_candidate(oracle_handle*, const double*, const double*, int);
int oracle_solve(oracle_handle*, int, int, double, fddp_result*);
const char* oracle_last_error(void);
}

static void on_fault(int sig) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  const char msg[] = "cpu_driver: fatal signal, backtrace:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

template <class T>
static bool rd(FILE* f, T* p, size_t n) {
  return fread(p, sizeof(T), n, f) == n;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s PROBLEM_FILE THREADS STEPS [MODE]\n", argv[0]);
    return 2;
  }
  signal(SIGSEGV, on_fault);
  signal(SIGBUS, on_fault);
  signal(SIGILL, on_fault);
  signal(SIGFPE, on_fault);
  const int threads = atoi(argv[2]), steps = atoi(argv[3]), mode = argc > 4 ? atoi(argv[4]) : 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) {
    perror("open");
    return 2;
  }
  int32_t dm[5];
  int64_t nk = 0, np = 0;
  if (!rd(f, dm, 5) || !rd(f, &nk, 1)) return 3;
  fddp_dims d{dm[0], dm[1], dm[2], dm[3], dm[4]};
  std::vector<fddp_knot_desc> kd(nk);
  if (!rd(f, kd.data(), nk) || !rd(f, &np, 1)) return 3;
  std::vector<double> pool(np), x0((size_t)d.B * d.nx);
  if (!rd(f, pool.data(), np) || !rd(f, x0.data(), x0.size())) return 3;
  int32_t has_xs = 0, has_us = 0;
  std::vector<double> xs, us;
  if (!rd(f, &has_xs, 1)) return 3;
  if (has_xs) {
    xs.resize((size_t)d.B * (d.T + 1) * d.nx);
    if (!rd(f, xs.data(), xs.size())) return 3;
  }
  if (!rd(f, &has_us, 1)) return 3;
  if (has_us) {
    us.resize((size_t)d.B * d.T * d.nu_max);
    if (!rd(f, us.data(), us.size())) return 3;
  }
  fclose(f);
  oracle_handle* h = nullptr;
  if (oracle_create(&d, kd.data(), pool.data(), np, &h)) {
    fprintf(stderr, "oracle_create: %s\n", oracle_last_error());
    return 4;
  }
  oracle_set_threading(h, mode, threads);
  oracle_set_x0(h, x0.data());
  std::vector<fddp_result> res(d.B);
  const double* xp = has_xs ? xs.data() : nullptr;
  const double* up = has_us ? us.data() : nullptr;
  oracle_set_candidate(h, xp, up, 0);
  oracle_solve(h, 1, 0, 0.1, res.data());  // warm-up
  long iters = 0;
  const auto t0 = std::chrono::steady_clock::now();
  for (int s = 0; s < steps; ++s) {
    oracle_set_candidate(h, xp, up, 0);
    oracle_solve(h, 1, 0, 0.1, res.data());
    for (const auto& r : res) iters += r.n_iter_run;
  }
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("{\"iters\": %ld, \"seconds\": %.4f, \"it_per_s\": %.3f, \"threads\": %d, \"mode\": %d, \"B\": %d}\n", iters, dt,
         iters / dt, threads, mode, d.B);
  oracle_destroy(h);
  return 0;
}
