"""Multi-GPU trajectory sharding: one process per GPU, torch.distributed (RCCL over xGMI).

The batched solve shards trivially: trajectories are independent and a Newton step has no
exchange.  Each rank owns a contiguous slice of the batch; the only collective
on the solve path is an all-reduce(MAX) of an 8-byte "trajectories still running on this rank"
count every `poll_every` device iterations -- the multi-GPU form of the reference's vmap'd
while_loop predicate ("loop while any lane is active").  Results are all-gathered at the end.

The engine is injectable (`engine_factory`) so the sharding / polling / gather logic is tested
with world_size 2 on CPU (gloo) without a GPU (tests/test_distributed.py).
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np
import torch
import torch.distributed as dist


def shard_bounds(batch: int, world: int, rank: int):
    """Contiguous, balanced slice [lo, hi) of `batch` trajectories for `rank`."""
    base, rem = divmod(batch, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def _comm_device():
    return torch.device("cuda", torch.cuda.current_device()) \
        if dist.get_backend() == "nccl" else torch.device("cpu")


def max_global(local: float) -> float:
    """All-reduce(MAX) of one fp64 scalar (the convergence norm): one 8-byte collective."""
    t = torch.tensor([float(local)], dtype=torch.float64, device=_comm_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def any_active_global(local_active: int) -> bool:
    """All-reduce(MAX) of the local "still running" count: one 8-byte collective."""
    t = torch.tensor([int(local_active)], dtype=torch.int64, device=_comm_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return bool(t.item() > 0)


def sum_global(local: int) -> int:
    t = torch.tensor([int(local)], dtype=torch.int64, device=_comm_device())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def gather_rows(local: np.ndarray, batch: int, world: int) -> np.ndarray:
    """All-gather the per-rank slices (padded to the largest shard) into the full batch."""
    dev = _comm_device()
    maxlen = shard_bounds(batch, world, 0)[1]
    pad = np.zeros((maxlen,) + local.shape[1:], dtype=local.dtype)
    pad[: local.shape[0]] = local
    src = torch.as_tensor(pad, device=dev)
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src)
    out = []
    for r in range(world):
        lo, hi = shard_bounds(batch, world, r)
        out.append(parts[r][: hi - lo].cpu().numpy())
    return np.concatenate(out, axis=0)


def solve_sharded(ocp, controls, initial_state, mode=None, terminal=None,
                  engine_factory: Optional[Callable] = None, poll_every: int = 8,
                  bp0: float = 0.1, persistent: Optional[bool] = None,
                  info: Optional[dict] = None):
    """Batched interior-point solve sharded over the process group.  Every rank passes the FULL
    batch (controls (B, N, nu), initial_state (B, nx)) and gets the full result back:
    (controls*, iterations, kkt_solves).

    persistent (default: when the family / horizon supports it): every rank runs its shard's whole
    solve in one launch (noc_ipm_solve) and the only collective on the solve path is the final
    all-reduce(MAX) of the convergence norm max|Hu| (P:158) -- SURVEY.md §8e's "RCCL only for the
    global convergence-norm all-reduce".  Otherwise the multi-launch loop polls the all-reduced
    "still running" count every `poll_every` iterations.  `info` (a dict) receives
    convergence_norm and not_done (global)."""
    from . import _lib
    mode = _lib.MODE_PAR if mode is None else mode
    if terminal is None:
        from .ipm import default_terminal
        terminal = default_terminal(mode)
    world, rank = dist.get_world_size(), dist.get_rank()
    u = np.asarray(controls, dtype=np.float64)
    x0 = np.asarray(initial_state, dtype=np.float64)
    B, N, _ = u.shape
    lo, hi = shard_bounds(B, world, rank)
    if engine_factory is None:
        from .ipm import BatchedIPM, persistent_supported
        if persistent is None:
            persistent = persistent_supported(ocp.family, N)

        def engine_factory(n, b):
            return BatchedIPM(ocp.family, n, b, persistent=bool(persistent))
    eng = engine_factory(N, max(hi - lo, 0))
    if persistent is None:
        persistent = bool(getattr(eng, "persistent", False))
    if persistent:
        if hi > lo:
            eng.load(u[lo:hi], x0[lo:hi])
            eng.solve_persistent(mode, terminal, bp0)
        norm = max_global(eng.convergence_norm() if hi > lo else 0.0)
        not_done = sum_global(eng.active_count() if hi > lo else 0)
    else:
        if hi > lo:
            eng.load(u[lo:hi], x0[lo:hi])
            eng.init(bp0)
        while True:
            if hi > lo:
                for _ in range(poll_every):
                    eng.step(mode, terminal)
            local = 0 if hi <= lo else eng.active_count()
            if not any_active_global(local):
                break
        norm = max_global(eng.convergence_norm() if hi > lo else 0.0)
        not_done = 0
    if info is not None:
        info.update(convergence_norm=norm, not_done=not_done)
    if hi > lo:
        U, it, solves = (t.cpu().numpy() for t in eng.result())
    else:
        U = np.zeros((0,) + u.shape[1:])
        it = np.zeros(0, dtype=np.int32)
        solves = np.zeros(0, dtype=np.int32)
    return gather_rows(U, B, world), gather_rows(it, B, world), gather_rows(solves, B, world)


def ddp_sharded(ocp, controls, initial_state, ddp_fn: Optional[Callable] = None,
                info: Optional[dict] = None, **kw):
    """Batched interior-point DDP (noc.differential_dynamic_programming.interior_point_ddp, D:189-208)
    sharded over the process group like solve_sharded: every rank passes the FULL batch, solves its
    contiguous slice in one launch, and gets the full (controls*, iterations, passes) back.  No
    collective on the solve path; `info` receives the global backward-pass total and the number of
    trajectories a max_passes cap stopped early (two 8-byte all-reduces).  `ddp_fn(ocp, u, x0,
    return_info=True, **kw) -> (U, its, info)` is injectable for CPU tests."""
    if ddp_fn is None:
        from .differential_dynamic_programming import interior_point_ddp as ddp_fn
    world, rank = dist.get_world_size(), dist.get_rank()
    u = np.asarray(controls, dtype=np.float64)
    x0 = np.asarray(initial_state, dtype=np.float64)
    B = u.shape[0]
    lo, hi = shard_bounds(B, world, rank)
    if hi > lo:
        U, its, inf = ddp_fn(ocp, u[lo:hi], x0[lo:hi], return_info=True, **kw)
        its = np.asarray(its, dtype=np.int32).reshape(-1)
        passes = np.asarray(inf["passes"], dtype=np.int32).reshape(-1)
        capped = int(np.sum(~np.asarray(inf["done"], dtype=bool)))
    else:
        U = np.zeros((0,) + u.shape[1:])
        its = np.zeros(0, dtype=np.int32)
        passes = np.zeros(0, dtype=np.int32)
        capped = 0
    if info is not None:
        info.update(passes_total=sum_global(int(passes.sum())), not_done=sum_global(capped))
    return gather_rows(U, B, world), gather_rows(its, B, world), gather_rows(passes, B, world)
