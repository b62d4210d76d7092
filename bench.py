"""Benchmark: FDDP iterations/s + MPC solves/s, Talos walking (contact dynamics) T=100, B=1024 per GPU.

One step = one warm-started solve of every batch element on this GPU,
SolverFDDP::solve(xs, us, maxiter=1, isFeasible=false, regInit=0.1) — the
reference's benchmark unit. Two protocols:
  fixed (default): the same warm start every step (default state, quasi-static
      controls), exactly the loop of benchmark/bipedal_walk_optctrl.py:36-43 and
      quadrupedal-gaits-optctrl.cpp:60-64; the warm start is kept in HBM.
  shift: a receding horizon — the gait knots rotate one knot (circularAppend,
      shooting.hxx:235-281), x0 <- xs[1] and xs/us shift on device, then the solve.
Each step runs exactly one FDDP iteration per element (calc, calcDiff + gaps,
backward Riccati sweep, line search), so FDDP iterations/s == MPC solves/s.

Multi-GPU: one process per GPU, the batch axis is sharded (each rank owns B
independent problems: weak scaling, no collective inside the solve), and the
solved trajectories are collected with one RCCL all-gather at the end of the
timed region (crocoddyl_amd/dist.py). Under torchrun the ranks come from its
environment; `python bench.py --gpus N` without one starts the N ranks itself
(launch_ranks) and relays rank 0's line.

Prints one JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "FDDP iterations/sec + MPC solves/sec, Talos contact T=100, batch=1024"
FP64_PEAK_TFLOPS = 78.6  # MI355X dense FP64 (vector == matrix rate on gfx950), datasheet


def backward_flops_per_knot(n, m):
    """F = 4n^3 + 6n^2 m + 4n m^2 + m^3/3 + 6n^2 + 6nm + 4m^2 (reference op sequence)."""
    return 4 * n ** 3 + 6 * n * n * m + 4 * n * m * m + m ** 3 / 3 + 6 * n * n + 6 * n * m + 4 * m * m


HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md


def rollout_bytes_per_knot_trial(nx, n, m, psz):
    """One knot of one line-search trial (fddp.cpp:149-225): reads xs, us, fs, Vxx fs,
    K (m x n), k and the knot's parameter block (psz doubles); writes xs_try, us_try,
    xnext and the knot cost."""
    return 8 * ((nx + m + 2 * n + m * n + m + psz) + (2 * nx + m + 1))


def calc_diff_bytes_per_knot(nx, n, m, psz):
    """One knot of calcDiff (euler.hxx:83-131 + the DAM): reads x, u and the parameter
    block; writes Fx, Fu, Lxx, Lxu, Luu, Lx, Lu, xnext and the knot cost."""
    return 8 * ((nx + m + psz) + (2 * n * n + 2 * n * m + m * m + n + m + nx + 1))


def mean_param_doubles(problem):
    """Mean parameter-block size over the knots (multibody blocks carry it in their
    header; 0 for the fixed-size kinds, whose blocks are the derivatives themselves)."""
    knots, pool = problem._packed()
    sizes = [int(pool[off + 3]) if kind in (4, 5, 6) else 0 for kind, _, off, _ in knots]
    return float(np.mean(sizes))


def backward_bytes_per_knot(n, m):
    """reads Fx, Lxx, Fu, Lxu, Luu, Lx, fs, Lu; writes K, k, Qu, Quuk, Vx, Vxx·fs."""
    return 8 * ((2 * n * n + 2 * n * m + m * m + 2 * n + m) + (m * n + 2 * m + 2 * n + m))


BOX_LIMIT = 1.0  # --solver boxfddp on configs without an effort table: |u_i| <= 1


BOX_PRESOLVE = 20  # --solver boxfddp: solve(maxiter=20, regInit=0.1) once from the warm start (untimed), then
# every step restarts from that feasible iterate with solve(xs_f, us_f, 1, isFeasible=true, 0.1):
# the box QP (box-fddp.cpp:48-79, only taken when feasible) runs on every knot of every step


def box_limits(config, nu):
    """--solver boxfddp control bounds (lb, ub) of a running knot with nu controls: on
    Talos (C5) the robot's effortLimit on the actuated joints (ActuationModelFloatingBase:
    u = tau[6:]), as examples/bipedal_walk_ubound.py:16-18 bounds the controls. (That
    example halves the limits of Talos' legs alone; on the full body the halved ankle-roll
    limit is below the single-support torque and no step is ever accepted.) Elsewhere
    |u_i| <= BOX_LIMIT."""
    if config.startswith("C5"):
        from crocoddyl_amd import robots
        lim = robots.sample_talos().effortLimit[6:]
        if lim.size == nu:
            return -lim, lim.copy()
    return np.full(nu, -BOX_LIMIT), np.full(nu, BOX_LIMIT)


def box_text(config):
    return ("u within the code-built Talos effortLimit (the bipedal_walk_ubound.py pattern; limits parity unpinned)"
            if config.startswith("C5")
            else f"|u| <= {BOX_LIMIT}")


def synthetic_kind(cfg):
    from crocoddyl_amd import synthetic
    return synthetic.CONFIGS[cfg][0]


def cpu_share():
    """The CPUs this process may use: the affinity mask and the cgroup CPU quota
    (cgroup v2 cpu.max, or v1 cfs_quota_us / cfs_period_us). threads = the smaller."""
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(p)
    except Exception:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / p
        except Exception:
            pass
    threads = aff if quota is None else max(1, min(aff, int(quota)))
    return threads, aff, quota


def cpu_baseline(cfg, T, seed, protocol, target_s=12.0, box=False):
    """Time the CPU oracle (C++ port of the reference solver, OpenMP) on this host, on
    a bounded sample of the same workload and protocol. Runs in a child process
    (the oracle is test infrastructure: never loaded into the benchmarking process)."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-child", cfg, str(T), str(seed),
           str(target_s), "1" if box else "0", protocol]
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    except subprocess.TimeoutExpired:
        return {"error": "timeout"}
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode == 0 and lines:
        return json.loads(lines[-1])
    return {"error": f"exit {p.returncode}: {p.stderr[-400:]}"}


def _cpu_baseline_child(cfg, T, seed, target_s, box, protocol):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import helpers
    import oracle_lib

    # -march=native build of the oracle for this host (built here, in /tmp) with ROCm's
    # clang++ and libomp (gcc 11's native build crashes on AVX-512 hosts: oracle/Makefile)
    out = os.path.join("/tmp", f"oracle_native_{os.getpid()}")
    cxx = "/opt/rocm/llvm/bin/clang++"
    oracle_lib.build(out_dir=out, arch="-march=native", cxx=cxx, ldflags="-Wl,-rpath,/opt/rocm/llvm/lib")
    oracle_lib._lib = oracle_lib.lib(os.path.join(out, "liboracle.so"))
    flags = f"{cxx} -O3 -march=native"
    threads, aff, quota = cpu_share()

    from crocoddyl_amd import _abi, synthetic
    import ctypes as C

    kind = synthetic.CONFIGS[cfg][0]

    def make(Bs, mode=2):
        S = helpers.setup(cfg, T=T, B=Bs, seed=seed)
        d = S["dims"]
        o = oracle_lib.Oracle(S["dims"], S["knots"], S["pool"], S["x0s"], threads=threads, mode=mode)
        if box:
            o.set_solver_kind(_abi.SOLVER_BOXFDDP)
            lo, hi = box_limits(cfg, d.nu_max)
            o.set_control_limits(np.ascontiguousarray(np.broadcast_to(lo, (d.B, d.T, d.nu_max))),
                                 np.ascontiguousarray(np.broadcast_to(hi, (d.B, d.T, d.nu_max))))
            p = oracle_lib.default_params()
            p.th_stop = 5e-5
            o.set_params(p)
        xs_w, us_w = warm_start_arrays(cfg, S["running"], S["x0s"], d)
        o.set_candidate(xs_w, us_w, False)
        st = {"o": o, "knots": list(S["knots"]), "xs": xs_w, "us": us_w, "B": Bs}
        if protocol == "shift":
            o.solve(maxiter=5)
        if protocol == "feasible":
            o.solve(maxiter=BOX_PRESOLVE, reg_init=0.1)
            st["xs"], st["us"] = o.xs(), o.us()
        o.phase_times(reset=True)
        return st

    def timed(st, steps):
        """element-iterations and seconds of `steps` benchmark steps (CLOCK_MONOTONIC)."""
        o = st["o"]
        t0 = time.perf_counter()
        it = 0
        for _ in range(steps):
            if protocol == "shift":
                st["knots"] = st["knots"][1:T] + st["knots"][:1] + st["knots"][T:]
                kd = (_abi.KnotDesc * len(st["knots"]))(*[_abi.KnotDesc(*k) for k in st["knots"]])
                o.L.oracle_set_knots(o.h, kd, _abi.dptr(o.pool), o.pool.size)
                o.mpc_shift()
            else:
                o.set_candidate(st["xs"], st["us"], protocol == "feasible")
            r = o.solve(maxiter=1, is_feasible=protocol == "feasible", reg_init=0.1)
            it += sum(x.n_iter_run for x in r)
        return it, time.perf_counter() - t0

    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    # batch-parallel (OpenMP over elements): the main figure. A calibration solve sizes
    # the batch so one repeat of `steps` steps takes ~target_s / (reps + 1); one warm-up
    # repeat, then the median of `reps` timed repeats (median of >= 5)
    reps, steps = 5, 2
    cal = make(threads)
    it, dt = timed(cal, 1)
    Bs = int(max(threads, min(1024, target_s / (reps + 1) * (it / max(dt, 1e-9)) / steps)))
    Bs = max(threads, (Bs // threads) * threads)
    st = make(Bs)
    timed(st, 1)  # warm-up
    st["o"].phase_times(reset=True)
    runs = [timed(st, steps) for _ in range(reps)]
    rates = sorted(i / d for i, d in runs)
    it, dt = sum(i for i, _ in runs), sum(d for _, d in runs)
    ph = st["o"].phase_times(reset=True)
    per_knot_us = {k: round(v / max(it, 1) / (T + 1) * 1e6, 3) for k, v in ph.items()}
    # reference-faithful (WITH_MULTITHREADING: OpenMP over knots inside calc / calcDiff,
    # shooting.hxx:143-145,176-178; elements one after another): a smaller sample
    cal1 = make(1, mode=1)
    it1, dt1 = timed(cal1, 1)
    B1 = int(max(1, min(256, target_s / 3 / 4 * (it1 / max(dt1, 1e-9)) / steps)))
    st1 = make(B1, mode=1)
    timed(st1, 1)
    runs1 = [timed(st1, steps) for _ in range(3)]
    rates1 = sorted(i / d for i, d in runs1)
    v2, v1 = rates[len(rates) // 2], rates1[len(rates1) // 2]
    share = f"affinity {aff} CPUs, cgroup quota {'none' if quota is None else round(quota, 2)}"
    print(json.dumps({"value": max(v1, v2), "unit": "FDDP iterations/s", "cores": threads, "kind": "port",
                      "host_cpus": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota,
                      "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"), "cpu_model": cpu_model,
                      "build": f"{flags} -fopenmp",
                      "modes": {"batch_parallel": round(v2, 2), "knot_parallel": round(v1, 2)},
                      "repeats_it_per_s": {"batch_parallel": [round(r, 2) for r in rates],
                                           "knot_parallel": [round(r, 2) for r in rates1]},
                      "per_knot_thread_us": dict(per_knot_us, note="thread time per knot per FDDP iteration "
                                                 "(forward: all line-search trials of the iteration), batch-parallel "
                                                 "mode, summed over threads / (element-iterations x (T+1))"),
                      "sample": f"{cfg} T={T}, protocol {protocol}, solve(maxiter=1, reg_init=0.1) per element per "
                                f"step: batch-parallel {Bs} elements, 1 warm-up + {reps} timed repeats of {steps} "
                                f"steps ({it} element-iterations in {dt:.1f} s; value = the median repeat), "
                                f"knot-parallel {B1} elements, 1 warm-up + 3 repeats; value = the faster mode's "
                                f"median. oracle/fddp_oracle.cpp {flags} -fopenmp, {threads} threads ({share}) of "
                                f"{os.cpu_count()} host CPUs ({cpu_model})"
                                f"{', SolverBoxFDDP ' + box_text(cfg) if box else ''}"}), flush=True)


def lib_sha256():
    """sha256 (first 16 hex digits) of the libfddp_hip.so this process runs"""
    import hashlib
    from crocoddyl_amd._lib import LIB_PATH
    with open(LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def load_pmc(cfg, lib_hash):
    """The HBM / MFMA counters of `cfg` in profiles/pmc_backward.json (tools/prof_summary.py),
    used only when they were collected on this very library build: the entry's lib_sha256
    must equal the running library's (and its tag CROCODDYL_AMD_PMC_TAG, when set).
    Returns (entry or None, provenance dict for the roofline)."""
    want_tag = os.environ.get("CROCODDYL_AMD_PMC_TAG")
    try:
        e = json.load(open(os.path.join(ROOT, "profiles", "pmc_backward.json"))).get(cfg)
    except Exception:
        e = None
    prov = {"source": "profiles/pmc_backward.json", "lib_sha256": lib_hash}
    if e is None:
        return None, dict(prov, status="absent: no counters for this config")
    prov.update(tag=e.get("tag"), profiled_lib_sha256=e.get("lib_sha256"))
    if e.get("lib_sha256") != lib_hash:
        return None, dict(prov, status="refused: counters collected on another library build (traffic = null)")
    if want_tag and e.get("tag") != want_tag:
        return None, dict(prov, status=f"refused: tag {e.get('tag')} != CROCODDYL_AMD_PMC_TAG={want_tag}")
    return e, dict(prov, status="matched")


def warm_start_arrays(config, running, x0s, dims):
    """The warm start of every element as dense (B, T+1, nx) / (B, T, nu_max) arrays.
    Gaits: the reference benchmark's (bipedal_walk_optctrl.py:29-32,
    quadrupedal-gaits-optctrl.cpp:51-57): the default state at every knot, each knot's
    quasi-static controls. The arm on contact dynamics: x0 at every knot (state.zero(),
    the stretched arm, is a singular configuration of the gripper contact). Otherwise
    None (state.zero() / zeros, setCandidate's defaults)."""
    from crocoddyl_amd import synthetic
    kind = synthetic.CONFIGS[config][0]
    B, T, nx, m = dims.B, dims.T, dims.nx, dims.nu_max
    if kind in ("gait_biped", "gait_quadruped"):
        xs_w, us_w = synthetic.gait_warm_start(config, running, x0s[0])
        xs = np.ascontiguousarray(np.broadcast_to(np.asarray(xs_w)[None], (B, T + 1, nx)))
        us = np.zeros((B, T, m))
        for t, u in enumerate(us_w):
            us[:, t, :u.size] = u
        return xs, us
    if kind == "multibody_contact":
        return np.ascontiguousarray(np.repeat(x0s[:, None, :], T + 1, axis=1)), None
    return None, None


def make_shard_solver(config, B, rank, dev, box=False, T=None, presolve=True):
    """Rank `rank`'s shard of the job: B problems of `config` (seeded per rank, so
    every rank owns distinct problems) on GPU `dev`, with the config's warm start set
    as the candidate (solver.warm = (xs, us) host arrays). presolve: then
    solve(maxiter=5) once, the starting point of the receding-horizon protocol."""
    from crocoddyl_amd import ShootingProblem, SolverBoxFDDP, SolverFDDP, synthetic
    T = synthetic.CONFIGS[config][3] if T is None else T
    seed = synthetic.seed_of(config) + 1000 * rank
    x0s, running, terminal = synthetic.build(config, T=T, B=B, seed=seed)
    if box:
        for md in set(running):
            md.u_lb, md.u_ub = box_limits(config, md.nu)
    problem = ShootingProblem(x0s, running, terminal, device=dev)
    solver = SolverBoxFDDP(problem) if box else SolverFDDP(problem)
    solver.warm = warm_start_arrays(config, running, x0s, problem._dims())
    solver.setCandidate(solver.warm[0] if solver.warm[0] is not None else [],
                        solver.warm[1] if solver.warm[1] is not None else [], False)
    if presolve:
        solver.solve_from_candidate(maxiter=5)
    return solver


def mpc_step(solver, mpc_iters, rotate=False):
    """One receding-horizon MPC solve of every element: the gait knots rotated one
    knot (ShootingProblem::circularAppend of the first running model, shooting.hxx:
    235-281) when `rotate`, the device shift of x0 / xs / us, then a warm-started
    solve(maxiter=mpc_iters, regInit=0.1)."""
    if rotate:
        p = solver.problem
        p.circularAppend(p.runningModels[0])
    solver.mpcShift()
    solver.solve_from_candidate(maxiter=mpc_iters, isFeasible=False, regInit=0.1)


class FixedWarmStart:
    """The reference benchmark's step (bipedal_walk_optctrl.py:36-43,
    quadrupedal-gaits-optctrl.cpp:60-64): solve(xs, us, MAXITER, false, 0.1) from the
    same warm start every time. The warm start lives in HBM (device tensors) and is
    re-applied on the solver's stream before each solve."""

    def __init__(self, solver, dev):
        import torch
        self.solver = solver
        xs, us = solver.warm
        self.xs = None if xs is None else torch.from_numpy(xs).to(f"cuda:{dev}")
        self.us = None if us is None else torch.from_numpy(us).to(f"cuda:{dev}")
        torch.cuda.synchronize(dev)

    def __call__(self, mpc_iters):
        self.solver.setCandidate_device(None if self.xs is None else self.xs.data_ptr(),
                                        None if self.us is None else self.us.data_ptr(), False)
        self.solver.solve_from_candidate(maxiter=mpc_iters, isFeasible=False, regInit=0.1)


class FeasibleRestart:
    """--solver boxfddp's step: solve(xs_f, us_f, 1, isFeasible=true, 0.1) from the iterate
    of an untimed solve(maxiter=BOX_PRESOLVE) from the warm start (the box QP only runs on
    feasible iterates, box-fddp.cpp:48-51). `start`: (xs, us) device tensors to restart
    from (default: this solver's presolved iterate)."""

    def __init__(self, solver, dev, start=None):
        import torch
        self.solver = solver
        if start is None:
            solver.solve_from_candidate(maxiter=BOX_PRESOLVE, regInit=0.1)
            self.feasible = float(np.mean(np.asarray(solver.isFeasible, float)))
            start = (torch.from_numpy(np.ascontiguousarray(solver.xs)).to(f"cuda:{dev}"),
                     torch.from_numpy(np.ascontiguousarray(solver.us)).to(f"cuda:{dev}"))
        self.xs, self.us = start
        torch.cuda.synchronize(dev)

    def __call__(self, mpc_iters):
        self.solver.setCandidate_device(self.xs.data_ptr(), self.us.data_ptr(), True)
        self.solver.solve_from_candidate(maxiter=mpc_iters, isFeasible=True, regInit=0.1)


def line_search_trials(solver):
    """Trials per element of the last line search: alpha = 2^-k accepted after k + 1."""
    sl = np.atleast_1d(np.asarray(solver.stepLength, float))
    return np.round(-np.log2(np.clip(sl, 2.0 ** -12, 1.0))) + 1


def trials_summary(trials):
    return {"mean": round(float(trials.mean()), 2), "max": int(trials.max()),
            "hist": np.bincount(trials.astype(int), minlength=11)[1:].tolist()}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv, timeout=None):
    """`bench.py --gpus N` without a torchrun environment: start N fresh worker
    processes of this script, one per GPU (RANK / LOCAL_RANK / WORLD_SIZE /
    LOCAL_WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in their environment), wait
    for all of them, and relay rank 0's stdout (the JSON line). The parent touches no
    GPU (nothing here imports torch) and execs nothing: the ranks are children. Ranks
    other than 0 have their stdout sent to stderr, as do rank 0's non-JSON lines, so
    the job's stdout is the one line. If a rank
    fails, the others are stopped (by their own PIDs) and its exit code is returned."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(), text=True))
    t0 = time.time()
    out = []
    import threading

    def pump():  # relay rank 0's stdout as it comes: its JSON line to stdout, the rest (library chatter) to stderr
        for line in procs[0].stdout:
            out.append(line)
            dst = sys.stdout if line.startswith("{") else sys.stderr
            dst.write(line)
            dst.flush()
    th = threading.Thread(target=pump, daemon=True)
    th.start()
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad or (timeout and time.time() - t0 > timeout):
            rc = bad[0] if bad else 124
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        if all(c == 0 for c in codes):
            break
        time.sleep(0.2)
    th.join(timeout=10)
    if rc == 0 and not any(ln.startswith("{") for ln in out):
        sys.stderr.write("bench.py: rank 0 printed no JSON line\n")
        rc = 1
    return rc


def _launch_selftest(args):
    """--launch-selftest: the N-rank launch path without a GPU (gloo, no solve): every
    rank joins the process group, and rank 0 prints the job's line with the per-rank
    table bench.py records (device, world size), for the CPU launcher test."""
    import torch.distributed as tdist

    from crocoddyl_amd import dist as cdist
    ws, rank, local_rank = cdist.world()
    assert ws == args.gpus, f"world size {ws} != --gpus {args.gpus}"
    cdist.init("gloo")
    rt = cdist.rank_table([local_rank, tdist.get_world_size() if tdist.is_initialized() else 1, os.getpid()], "cpu")
    t, w = cdist.job_time_and_work(0.1 * (rank + 1), 10 * (rank + 1), "cpu")
    if rank == 0:
        print(json.dumps({"n_gpus": ws, "job_time_s": t, "work": w,
                          "ranks": cdist.rank_summary(rt, ["device", "world_size", "pid"])}), flush=True)
    if ws > 1:
        tdist.barrier()
        tdist.destroy_process_group()


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--cpu-baseline-child":
        a = sys.argv[2:]
        _cpu_baseline_child(a[0], int(a[1]), int(a[2]), float(a[3]), a[4] == "1", a[5])
        return
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C5_talos_walk")
    ap.add_argument("--batch", type=int, default=None, help="elements per GPU (default: the config's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--solver", choices=["fddp", "boxfddp"], default="fddp",
                    help="boxfddp: SolverBoxFDDP with control limits (C5: the code-built Talos effortLimit on the "
                         "actuated joints, parity unpinned; elsewhere |u| <= 1); default protocol 'feasible': an untimed "
                         "solve(maxiter=20, regInit=0.1), then every step solve(xs_f, us_f, 1, isFeasible=true, 0.1) "
                         "from that iterate, so the box QP runs on every knot")
    ap.add_argument("--protocol", choices=["fixed", "shift", "feasible"], default=None,
                    help="fixed: the reference benchmark's loop, solve(xs, us, 1, false, 0.1) from the same warm "
                         "start every step (bipedal_walk_optctrl.py:36-43); shift: receding horizon, gait knots "
                         "rotated (circularAppend) + device shift of x0/xs/us, then the warm-started solve")
    ap.add_argument("--secondary-steps", type=int, default=5,
                    help="steps of the other protocol, reported beside the headline (1 GPU only; 0: off)")
    ap.add_argument("--launch-selftest", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--rehearsal", action="store_true",
                    help="allow more ranks than GPUs (ranks share devices, gloo collectives): a rehearsal of the "
                         "N-GPU job, marked as such in the JSON line, n_gpus = the distinct devices used")
    args = ap.parse_args()
    box = args.solver == "boxfddp"
    if args.protocol is None:
        args.protocol = "feasible" if box else "fixed"
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no torchrun environment: this process becomes the launcher of N ranks
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.launch_selftest:
        return _launch_selftest(args)

    import torch

    from crocoddyl_amd import synthetic
    from crocoddyl_amd import dist as cdist

    ws, rank, local_rank = cdist.world()
    assert ws == args.gpus, f"world size {ws} (WORLD_SIZE) != --gpus {args.gpus}"
    # one rank per GPU; on a lease with fewer GPUs than ranks (a rehearsal of the N-GPU
    # job) ranks share devices and the collectives run on gloo (RCCL refuses two ranks
    # on one device)
    ndev = torch.cuda.device_count()
    if ndev < ws and not args.rehearsal:
        sys.stderr.write(f"bench.py: {ws} ranks but {ndev} GPU(s): one rank per GPU is required (pass --rehearsal "
                         "to run the ranks on shared devices, reported as a rehearsal)\n")
        sys.exit(2)
    dev = local_rank % max(ndev, 1)
    backend = os.environ.get("CROCODDYL_AMD_DIST_BACKEND") or ("nccl" if ndev >= ws else "gloo")
    cdist.init(backend, dev)

    kind, d1, nu, T, B0, dt = synthetic.CONFIGS[args.config]
    B = args.batch or B0
    mpc_iters = 1

    def make_stepper(protocol):
        s = make_shard_solver(args.config, B, rank, dev, box, presolve=(protocol == "shift"))
        if protocol == "fixed":
            fw = FixedWarmStart(s, dev)
            return s, (lambda: fw(mpc_iters))
        if protocol == "feasible":
            fr = FeasibleRestart(s, dev)
            s.restart = fr
            return s, (lambda: fr(mpc_iters))
        rotate = kind in ("gait_biped", "gait_quadruped")
        return s, (lambda: mpc_step(s, mpc_iters, rotate=rotate))

    solver, step = make_stepper(args.protocol)
    problem = solver.problem
    n, m, nx = problem.ndx, problem.nu_max, problem.nx

    for _ in range(args.warmup):
        step()
    if ws > 1:
        torch.distributed.barrier()
    solver.synchronize()
    torch.cuda.synchronize(dev)
    solver.get_timing()
    solver.set_timing(True)
    t0 = time.perf_counter()
    iters = 0
    for _ in range(args.steps):
        step()
        iters += int(np.sum(solver.n_iter_run))
    solver.synchronize()
    t_solve = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    if ws > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0  # exactly the K steps, barrier to barrier
    # then, once per job (outside the timed steps; its time and bytes are in `ranks`): the
    # solved trajectories and per-element results, device to device, and the all-gathers
    # (RCCL over xGMI), the only collectives of the batched solve
    gstats = {}
    xs_all, us_all, res_all = cdist.gather_solution(solver, f"cuda:{dev}", gstats)
    torch.cuda.synchronize(dev)
    if ws > 1:
        torch.distributed.barrier()
    solver.set_timing(False)
    timing = solver.get_timing()
    trials = line_search_trials(solver)  # of the last step
    rank_elapsed = elapsed
    elapsed, total_iters = cdist.job_time_and_work(elapsed, iters, f"cuda:{dev}")
    assert xs_all.shape[0] == us_all.shape[0] == res_all.shape[0] == ws * B
    # per-rank diagnostics (outside the timed region): the timed loop's own time, the
    # gather's time and bytes, the rank's iterations; max/min imbalance per column
    names = ["elapsed_s", "solve_s", "gather_s", "iterations", "mean_trials_last_step", "device", "world_size"]
    gws = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1
    rt = cdist.rank_table([rank_elapsed, t_solve, gstats["gather_s"], iters, float(np.mean(trials)), dev, gws],
                          f"cuda:{dev}")
    ranks = dict(cdist.rank_summary(rt, names), backend=cdist.backend(),
                 gather_bytes_sent_per_rank=gstats["gather_bytes_sent"],
                 gather_bytes_received_per_rank=gstats["gather_bytes_received"],
                 gather_GBps_received=round(gstats["gather_bytes_received"] / max(float(rt[:, 2].max()), 1e-12) / 1e9, 3)
                 if ws > 1 else None,
                 note="elapsed_s: this rank's barrier-to-barrier time of the K timed steps (the job time is the "
                      "max); solve_s: the steps before the device synchronisation; gather_s: the all-gathers of xs, "
                      "us and results after the timed steps, once per job (device-synchronised; RCCL "
                      "when every rank has its own GPU, gloo over host copies when ranks share one); device: the "
                      "rank's GPU; world_size: dist.get_world_size() seen by the rank")

    box_bwd = None
    if box and ws == 1 and args.protocol == "feasible":
        # the FDDP backward on the same step: SolverFDDP on the same problems, restarted
        # from the same feasible iterate (FDDP gains: no box QP)
        sf = make_shard_solver(args.config, B, rank, dev, False, presolve=False)
        fr = FeasibleRestart(sf, dev, start=(solver.restart.xs, solver.restart.us))
        fr(mpc_iters)
        sf.synchronize()
        sf.get_timing()
        sf.set_timing(True)
        for _ in range(args.steps):
            fr(mpc_iters)
        sf.synchronize()
        sf.set_timing(False)
        f_ms = sf.get_timing()["backward"][0] / args.steps
        b_ms = timing["backward"][0] / args.steps
        box_bwd = {"backward_ms_boxfddp": round(b_ms, 3), "backward_ms_fddp": round(f_ms, 3),
                   "ratio": round(b_ms / f_ms, 3),
                   "feasible_fraction_after_presolve": solver.restart.feasible,
                   "method": "per-step backward (HIP events) of SolverBoxFDDP and of SolverFDDP on the same "
                             "problems, both restarted from the same feasible iterate with "
                             "solve(xs_f, us_f, 1, isFeasible=true, 0.1)"}
        del sf, fr

    secondary = None
    if ws == 1 and args.secondary_steps > 0 and args.protocol != "feasible":
        other = "shift" if args.protocol == "fixed" else "fixed"
        del xs_all, us_all, res_all
        s2, step2 = make_stepper(other)
        step2()
        s2.synchronize()
        t1 = time.perf_counter()
        it2 = 0
        for _ in range(args.secondary_steps):
            step2()
            it2 += int(np.sum(s2.n_iter_run))
        s2.synchronize()
        el2 = time.perf_counter() - t1
        secondary = {"protocol": other, "steps": args.secondary_steps, "value": round(it2 / el2, 2),
                     "ms_per_step": round(el2 / args.secondary_steps * 1e3, 3),
                     "line_search_trials_last_step": trials_summary(line_search_trials(s2))}
        del s2, step2

    if rank == 0:
        value = total_iters / elapsed
        bwd_ms, bwd_n = timing["backward"]
        avg_bwd_s = bwd_ms / max(bwd_n, 1) / 1e3
        F = backward_flops_per_knot(n, m) * B * T
        Y = backward_bytes_per_knot(n, m) * B * T
        achieved = F / avg_bwd_s / 1e12
        lib_hash = lib_sha256()
        pmc, pmc_prov = load_pmc(args.config, lib_hash)
        roof_bwd = {"kernel": "backward Riccati sweep (bwd_mfma.hpp)", "bound": "mfma", "achieved": round(achieved, 3),
                    "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / FP64_PEAK_TFLOPS, 4),
                    "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
                    "algorithmic_flops_per_launch": F, "algorithmic_bytes_per_launch": Y,
                    "achieved_algorithmic_GBps": round(Y / avg_bwd_s / 1e9, 1),
                    "avg_launch_ms": round(avg_bwd_s * 1e3, 3), "timer": "HIP events on the solver stream"}
        if Y / (HBM_PEAK_GBPS * 1e9) > F / (FP64_PEAK_TFLOPS * 1e12):  # the HBM floor binds (F/Y below the ridge)
            gb = Y / avg_bwd_s / 1e9
            roof_bwd.update(bound="hbm", achieved=round(gb, 1), peak=HBM_PEAK_GBPS, unit="GB/s",
                            frac=round(gb / HBM_PEAK_GBPS, 4),
                            fp64={"achieved": round(achieved, 3), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                                  "frac": round(achieved / FP64_PEAK_TFLOPS, 4)})
        # the knot kernels: algorithmic HBM bytes and FP64 flops (crocoddyl_amd/opcount.py,
        # the reference op sequence); the binding roof is the one with the larger time floor
        psz = mean_param_doubles(problem)
        rooflines = {"backward": (bwd_ms, roof_bwd)}
        kfl = None
        if kind in ("gait_biped", "gait_quadruped", "multibody", "multibody_contact"):
            from crocoddyl_amd import opcount
            kfl = opcount.horizon_flops(problem.runningModels, problem.terminalModel)
        kpm = (pmc or {}).get("kernels", {})

        def knot_roof(name, ms, n_launch, Y, F, traffic, extra):
            t = ms / n_launch / 1e3
            hb = Y / t / 1e9
            r = {"kernel": name, "bound": "hbm", "achieved": round(hb, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                 "frac": round(hb / HBM_PEAK_GBPS, 5), "traffic": traffic, "algorithmic_bytes_per_launch": int(Y)}
            if F:
                fl = F / t / 1e12
                r["fp64"] = {"achieved": round(fl, 3), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                             "frac": round(fl / FP64_PEAK_TFLOPS, 5), "algorithmic_flops_per_launch": int(F),
                             "flop_model": "crocoddyl_amd/opcount.py (reference op sequence, spatial-algebra costs)"}
                if F / (FP64_PEAK_TFLOPS * 1e12) > Y / (HBM_PEAK_GBPS * 1e9):  # FP64 floor binds
                    hb_roof = {k: r[k] for k in ("achieved", "peak", "unit", "frac")}
                    r.update(bound="fp64", achieved=r["fp64"]["achieved"], peak=FP64_PEAK_TFLOPS, unit="TFLOP/s",
                             frac=r["fp64"]["frac"], hbm=hb_roof)
            r.update(extra, avg_launch_ms=round(ms / n_launch, 3), timer="HIP events on the solver stream")
            return r

        fw_ms, fw_n = timing["forward"]
        if fw_n:
            g, nl = solver.line_search_info()
            kt = float(np.sum(trials)) * (T + 1)  # knot-trials of one line search (last step's trials)
            Yf = rollout_bytes_per_knot_trial(nx, n, m, psz) * kt
            fpm = kpm.get("forward") or {}
            rooflines["forward"] = (fw_ms, knot_roof(
                "line-search rollout: forward_kernel" + (f" x {nl} trial groups of {g} + ls_select_kernel"
                                                         if g > 1 else " (serial line search, one dispatch)"),
                fw_ms, fw_n, Yf, kfl[0] * kt if kfl else None,
                # HBM bytes of one line search: every forward dispatch of a timed step (profiles/)
                fpm.get("hbm_bytes_per_step"),
                {"knot_trials_per_launch": int(kt), "trial_group_size": g, "dispatches_per_line_search": nl}))
        cd_ms, cd_n = timing["calcDiff"]
        if cd_n:
            nk = B * (T + 1)
            Yc = calc_diff_bytes_per_knot(nx, n, m, psz) * nk
            rooflines["calcDiff"] = (cd_ms, knot_roof(
                "knot-parallel calcDiff (mb_knot_kernel / calc_diff_kernel) + gaps", cd_ms, cd_n, Yc,
                kfl[1] * nk if kfl else None,
                (kpm.get("mb_calc_diff") or kpm.get("calc_fused") or {}).get("hbm_bytes_per_step"),
                {"knots_per_launch": nk}))
        dominant = max(rooflines, key=lambda k: rooflines[k][0])
        roof = dict(rooflines[dominant][1], dominant_of=sorted(rooflines), pmc=pmc_prov)
        cpu = None
        if ws == 1 and not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(args.config, T, synthetic.seed_of(args.config), args.protocol, box=box)
            except Exception as e:  # reported, never fatal for the GPU number
                cpu = {"error": repr(e)}
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "FDDP iterations/s", "n_gpus": min(ws, max(ndev, 1)),
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": ("synthetic: the reference's Talos walking gait (utils/biped.py createWalkingProblem: 6D foot "
                     "contacts, friction cones, CoM / swing-foot tracking, pseudo-impulse foot switches) on real "
                     "contact dynamics (Euler ∘ ContactFwdDynamics, free-flyer root, nv=38) of a Talos-class robot "
                     "built in code (URDF absent); per-element x0 = half-sitting perturbed on the manifold"
                     if kind == "gait_biped" else
                     "synthetic: the reference's Solo12 trotting gait (utils/quadruped.py createTrottingProblem: 3D "
                     "foot contacts, friction cones, state bounds, impulse foot switches) on real contact dynamics "
                     "(free-flyer root, nv=18) of a Solo12-class robot built in code; per-element x0 perturbed"
                     if kind == "gait_quadruped" else
                     "synthetic: arm-manipulation problem of benchmark/factory/arm.hpp on real multibody knots "
                     "(Euler ∘ FreeFwdDynamics, 7-DoF Talos-class arm model built in code: the URDF is absent), "
                     "per-element x0" if kind == "multibody" else
                     "synthetic: the 7-DoF arm on contact dynamics (Euler ∘ ContactFwdDynamics, gripper "
                     "ContactModel6D with Baumgarte gains, ActuationModelFloatingBase), xReg + uReg costs, "
                     "per-element x0 = bent posture + U[-0.3, 0.3]" if kind == "multibody_contact" else
                     "synthetic: seeded Euler(dt)∘DifferentialActionModelLQR knots at the config's (n, m, T); "
                     "per-element matrices (SURVEY §8d); no robot model (Pinocchio/URDF absent)"),
            "config": {"workload": f"{args.config}: n={n}, m={m}, T={T}, B={B} per GPU, "
                                   + (f"protocol fixed: solve(xs_w, us_w, maxiter={mpc_iters}, isFeasible=false, "
                                      f"reg_init=0.1) from the same HBM-resident warm start every step, as the "
                                      f"reference benchmark (bipedal_walk_optctrl.py:36-43)"
                                      if args.protocol == "fixed" else
                                      f"protocol shift: gait knots rotated (circularAppend), device shift of x0/xs/us, "
                                      f"then solve(maxiter={mpc_iters}, isFeasible=false, reg_init=0.1)"
                                      if args.protocol == "shift" else
                                      f"protocol feasible: solve(xs_f, us_f, {mpc_iters}, isFeasible=true, reg_init=0.1) "
                                      f"from the HBM-resident iterate of an untimed solve(maxiter={BOX_PRESOLVE}, reg_init=0.1) "
                                      f"from the warm start")
                                   + (", SolverBoxFDDP, " + box_text(args.config) if box else ""),
                       "protocol": args.protocol,
                       "global_batch": B * ws, "T": T, "parallelism": f"batch-sharded x{ws}",
                       "solver": "SolverBoxFDDP" if box else "SolverFDDP"},
            "mpc_solves_per_s": round(B * ws * args.steps / elapsed, 2),
            "kernel_ms_per_step": {k: round(v[0] / max(args.steps, 1), 3) for k, v in timing.items()},
            "per_knot_device_us": {k: round(v[0] / max(args.steps, 1) / (B * (T + 1)) * 1e3, 5)
                                   for k, v in timing.items()},
            "ranks": ranks,
            "line_search_trials_last_step": trials_summary(trials),
            "secondary_protocol": secondary,
            **({"box_backward": box_bwd} if box_bwd else {}),
            "lib_sha256": lib_hash,
            "roofline": roof,
            "rooflines": {k: v[1] for k, v in rooflines.items()},
            "cpu_baseline": cpu,
        }
        if cpu and "value" in cpu:
            out["speedup_vs_cpu"] = round(value / cpu["value"], 2)
        if ndev < ws:  # (--rehearsal) not an N-GPU measurement
            out["rehearsal"] = {"ranks": ws, "physical_gpus": ndev,
                                "note": "ranks share GPUs (gloo collectives): a rehearsal of the sharded job, "
                                        "not a multi-GPU throughput"}
        print(json.dumps(out), flush=True)
    if ws > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
