"""Multi-GPU plumbing: one process per GPU, the batch axis sharded.

The B problems of a batch are independent (the reference has no coupling
between problems), so each rank solves its own shard with no
communication during solve(). The only collective is one all-gather of the
solved trajectories at the end (RCCL over xGMI on the GPU box: backend
"nccl"; gloo in the CPU tests).
"""
import os
import time

import numpy as np
import torch
import torch.distributed as dist


def world():
    """(world_size, rank, local_rank) from the torchrun environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend, local_rank=None):
    """Initialise the default process group (MASTER_ADDR/PORT from the env)."""
    ws, rank, lr = world()
    if ws <= 1 or dist.is_initialized():
        return ws, rank
    if backend == "nccl":
        lr = lr if local_rank is None else local_rank
        torch.cuda.set_device(lr)
        dist.init_process_group("nccl", device_id=torch.device("cuda", lr))
    else:
        dist.init_process_group(backend)
    return ws, rank


def backend():
    """The default group's backend ("nccl" = RCCL on ROCm, "gloo"), or None on one process."""
    return dist.get_backend() if dist.is_initialized() else None


def shard(b_global, ws, rank):
    """Contiguous block of batch elements owned by `rank`: (start, count)."""
    base, rem = divmod(b_global, ws)
    start = rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


def gather_rows(local):
    """All-gather equally shaped per-rank tensors along dim 0 (the one
    collective of the batched solve)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return local
    out = torch.empty((dist.get_world_size() * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous())
    return out


# per-element solve results gathered with the trajectories, one row each
RESULT_FIELDS = ("status", "iter", "is_feasible", "n_iter_run", "cost", "stop", "steplength")


def gather_solution(solver, device, stats=None):
    """All-gather every rank's solved shard: (xs (B_all, T+1, nx), us (B_all, T, nu_max),
    results (B_all, len(RESULT_FIELDS))), rows in rank order. The trajectories are
    copied device to device from the solver (no host round trip); with the gloo
    backend (CPU tests) the collective runs on host copies. stats (a dict, optional):
    receives the collectives' wall time on this rank ("gather_s", device-synchronised)
    and bytes ("gather_bytes_sent" = this rank's rows, "gather_bytes_received" = the
    other ranks' rows)."""
    p = solver.problem
    dev = torch.device(device) if not isinstance(device, torch.device) else device
    xs = torch.empty((p.B, p.T + 1, p.nx), dtype=torch.float64, device=dev)
    us = torch.empty((p.B, p.T, p.nu_max), dtype=torch.float64, device=dev)
    solver.xs_device(xs.data_ptr())
    solver.us_device(us.data_ptr())
    res = torch.tensor([[float(getattr(r, f)) for f in RESULT_FIELDS] for r in solver._res()], dtype=torch.float64,
                       device=dev)
    solver.synchronize()
    if dist.is_initialized() and dist.get_backend() == "gloo":
        xs, us, res = xs.cpu(), us.cpu(), res.cpu()
    t0 = time.perf_counter()
    out = gather_rows(xs), gather_rows(us), gather_rows(res)
    if out[0].is_cuda:
        torch.cuda.synchronize(out[0].device)
    if stats is not None:
        ws = dist.get_world_size() if dist.is_initialized() else 1
        nbytes = sum(t.numel() * t.element_size() for t in (xs, us, res))
        stats.update(gather_s=time.perf_counter() - t0, gather_bytes_sent=int(nbytes),
                     gather_bytes_received=int(nbytes * (ws - 1)))
    return out


def rank_table(values, device):
    """All-gather a short per-rank vector of floats: a (world_size, k) numpy array in
    rank order (one row on a single process). Diagnostics only (bench.py's per-rank
    times), outside the timed region."""
    v = torch.tensor([float(x) for x in values], dtype=torch.float64, device=device)
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return v.cpu().numpy()[None]
    if dist.get_backend() == "gloo":
        v = v.cpu()
    return gather_rows(v[None]).cpu().numpy()


def rank_summary(table, names):
    """{name: [per-rank values]} plus the max/min imbalance of each column."""
    out = {}
    for j, n in enumerate(names):
        col = [float(x) for x in table[:, j]]
        out[n] = [round(x, 6) for x in col]
        lo = min(col)
        out[n + "_max_over_min"] = round(max(col) / lo, 4) if lo > 0 else None
    return out


def job_time_and_work(elapsed_s, work, device):
    """Whole-job numbers: the slowest rank's time, the sum of the work."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return float(elapsed_s), float(work)
    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=device)
    w = torch.tensor([float(work)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(w, op=dist.ReduceOp.SUM)
    return float(t.item()), float(w.item())
