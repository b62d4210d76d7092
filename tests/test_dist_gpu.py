"""The batch-sharded product path on the GPU: two ranks (gloo, world
size 2) each drive libfddp_hip on device 0 through bench.py's own shard / solve /
gather code (make_shard_solver, mpc_step, dist.gather_solution), and the gathered
xs / us / per-element results must equal solving every shard in one process.

Shapes: the C4 trot (T = 60) and the headline C5 Talos walk (T = 100, nx = 77,
nu = 32: the gather moves the xs / us rows at the bench's widths), a few elements
per rank. The box has one GPU, so both ranks share device 0 and the collective runs
on gloo over host copies; the RCCL-over-xGMI all-gather of the 8-GPU job is the same
dist.gather_rows call on device tensors and is unmeasured on hardware here."""
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
STEPS = 2
CASES = [("C4_solo12_trot", 3), ("C5_talos_walk", 2)]

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q, CONFIG, B):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(ws), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import torch

    import bench
    from crocoddyl_amd import dist as cdist

    cdist.init("gloo")
    solver = bench.make_shard_solver(CONFIG, B, rank, 0)
    for _ in range(STEPS):
        bench.mpc_step(solver, 1)
    xs, us, res = cdist.gather_solution(solver, "cuda:0")
    t, w = cdist.job_time_and_work(0.25 * (rank + 1), int(np.sum(solver.n_iter_run)), "cpu")
    if rank == 0:
        q.put((xs.numpy(), us.numpy(), res.numpy(), t, w))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("CONFIG,B", CASES)
def test_world2_product_shards_gather_matches_single_process(CONFIG, B):
    import torch.multiprocessing as mp

    sys.path.insert(0, ROOT)
    import bench
    from crocoddyl_amd import dist as cdist

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, CONFIG, B)) for r in range(2)]
    for p in procs:
        p.start()
    xs, us, res, t, w = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert xs.shape[0] == us.shape[0] == res.shape[0] == 2 * B
    assert t == pytest.approx(0.5)
    iters = 0
    for rank in range(2):  # each shard again, in this process
        solver = bench.make_shard_solver(CONFIG, B, rank, 0)
        for _ in range(STEPS):
            bench.mpc_step(solver, 1)
        iters += int(np.sum(solver.n_iter_run))
        sl = slice(rank * B, (rank + 1) * B)
        np.testing.assert_allclose(xs[sl], solver.xs, rtol=0, atol=1e-12)
        np.testing.assert_allclose(us[sl], solver.us, rtol=0, atol=1e-12)
        want = np.array([[float(getattr(r, f)) for f in cdist.RESULT_FIELDS] for r in solver._res()])
        np.testing.assert_allclose(res[sl], want, rtol=1e-12, atol=1e-12)
    assert w == iters
    assert np.all(res[:, 0] >= 0)  # statuses gathered as well
