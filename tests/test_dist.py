"""World-size-2 gloo test of the batch-sharded path (CPU): each rank solves
its shard (the CPU oracle stands in for the GPU solver here), the results are
all-gathered with the same helper bench.py uses, and rank 0 checks them
against solving every shard in one process. Also checks the job-time
reduction (max over ranks) and work sum."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_problem(rank):
    import helpers
    return helpers.setup("C2_lqr", T=6, B=3, seed=1234 + rank)


def _worker(rank, ws, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, HERE)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(ws), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import torch

    import oracle_lib
    from crocoddyl_amd import dist as cdist

    cdist.init("gloo")
    S = _shard_problem(rank)
    o = oracle_lib.Oracle(S["dims"], S["knots"], S["pool"], S["x0s"])
    o.set_candidate(None, None, False)
    r = o.solve(maxiter=10)
    xs = torch.from_numpy(o.xs())
    allxs = cdist.gather_rows(xs)
    t, w = cdist.job_time_and_work(0.5 + rank, sum(x.n_iter_run for x in r), "cpu")
    # bench.py's per-rank diagnostics table
    rt = cdist.rank_table([0.5 + rank, 10.0 * (rank + 1)], "cpu")
    summ = cdist.rank_summary(rt, ["elapsed_s", "iterations"])
    if rank == 0:
        q.put((allxs.numpy(), t, w, rt, summ))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("n", [2, 3])
def test_bench_launches_n_ranks(n):
    """`python bench.py --gpus N` with no torchrun environment starts N rank processes
    itself (bench.launch_ranks: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set per child)
    and relays rank 0's one JSON line; here on gloo without a GPU (--launch-selftest)."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launch-selftest"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    r = out["ranks"]
    assert r["world_size"] == [float(n)] * n
    assert r["device"] == [float(i) for i in range(n)]
    assert len(set(r["pid"])) == n
    assert out["job_time_s"] == pytest.approx(0.1 * n)
    assert out["work"] == 10 * n * (n + 1) / 2


def test_bench_rank_refuses_world_size_mismatch():
    """A rank whose WORLD_SIZE disagrees with --gpus stops instead of reporting n_gpus wrong."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-selftest"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "--gpus 2" in p.stderr


def test_shard_bounds():
    from crocoddyl_amd.dist import shard
    for bg in (1, 7, 8, 1024, 8192):
        for ws in (1, 2, 4, 8):
            spans = [shard(bg, ws, r) for r in range(ws)]
            assert sum(c for _, c in spans) == bg
            assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(ws - 1))
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def test_world2_gloo_gather_matches_single_process():
    import oracle_lib
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    allxs, t, w, rt, summ = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = []
    iters = 0
    for rank in range(2):
        S = _shard_problem(rank)
        o = oracle_lib.Oracle(S["dims"], S["knots"], S["pool"], S["x0s"])
        o.set_candidate(None, None, False)
        iters += sum(x.n_iter_run for x in o.solve(maxiter=10))
        ref.append(o.xs())
    np.testing.assert_array_equal(allxs, np.concatenate(ref))
    assert t == pytest.approx(1.5)
    assert w == iters
    np.testing.assert_array_equal(rt, [[0.5, 10.0], [1.5, 20.0]])
    assert summ["elapsed_s"] == [0.5, 1.5] and summ["elapsed_s_max_over_min"] == 3.0
    assert summ["iterations_max_over_min"] == 2.0
