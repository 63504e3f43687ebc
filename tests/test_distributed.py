"""N>1 path on CPU: world_size-2 gloo process group, fake engine (no GPU needed).  Checks shard
bounds, the all-reduce(MAX) polling termination (a rank whose trajectories finished keeps
participating until every rank is done) and the all-gather reassembly order."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class FakeEngine:
    """Trajectory b needs (b % 5) + 3 device iterations; result u = u0 + b-dependent offset."""

    def __init__(self, N, B):
        self.N, self.B = N, B
        self.steps = 0

    def load(self, u, x0):
        self.u = np.array(u)
        self.x0 = np.array(x0)
        self.need = (np.round(self.x0[:, 0]).astype(int) % 5) + 3

    def init(self, bp0):
        self.steps = 0

    def step(self, mode, terminal):
        self.steps += 1

    def active_count(self):
        return int(np.sum(self.need > self.steps))

    def convergence_norm(self):
        return 1e-5 * float(np.max(self.x0[:, 0])) if len(self.x0) else 0.0

    def result(self):
        import torch
        done_at = np.minimum(self.need, self.steps)
        return (torch.as_tensor(self.u + self.x0[:, :1, None]),
                torch.as_tensor(done_at.astype(np.int32)), torch.as_tensor(self.need.astype(np.int32)))


class FakePersistentEngine(FakeEngine):
    """The whole solve in one call (noc_ipm_solve semantics): no polling."""
    persistent = True

    def solve_persistent(self, mode, terminal, bp0):
        self.steps = int(self.need.max()) if len(self.need) else 0

    def step(self, mode, terminal):  # must not be used on the persistent path
        raise AssertionError("persistent engines are not stepped")


def _worker(rank, world, port, B, q, persistent=False):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from noc import distributed as D
    N, nu = 6, 1
    u = np.arange(B * N, dtype=np.float64).reshape(B, N, nu)
    x0 = np.zeros((B, 2))
    x0[:, 0] = np.arange(B)
    eng = FakePersistentEngine if persistent else FakeEngine
    info = {}
    U, it, solves = D.solve_sharded(None, u, x0, mode=0, terminal=0,
                                    engine_factory=lambda n, b: eng(n, b), poll_every=2,
                                    info=info)
    q.put((rank, U, it, solves, info))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,B", [(2, 7), (2, 8), (2, 1), (8, 37), (8, 4096), (8, 5)])
@pytest.mark.parametrize("persistent", [False, True])
def test_sharded_solve_gloo(world, B, persistent):
    """World 2 and world 8 (the whole node of the north-star curve: 4096 cart-poles over 8 ranks,
    a ragged batch, and fewer trajectories than ranks, so some ranks hold an empty shard)."""
    from noc.distributed import shard_bounds
    spans = [shard_bounds(B, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == B
    assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, q, persistent))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    u = np.arange(B * 6, dtype=np.float64).reshape(B, 6, 1)
    need = (np.arange(B) % 5) + 3
    for rank, U, it, solves, info in res:
        assert np.array_equal(U, u + np.arange(B)[:, None, None])   # order preserved
        assert np.array_equal(solves, need)
        assert np.array_equal(it, need)                            # every trajectory finished
        # the global convergence norm is the all-reduce(MAX) over both ranks' shards
        assert info["convergence_norm"] == pytest.approx(1e-5 * (B - 1))
        assert info["not_done"] == 0


def _fake_ddp(ocp, u, x0, return_info=True):
    """interior_point_ddp stand-in: iterations = 10 + b, passes = 2 (10 + b), u shifted by b."""
    b = np.round(x0[:, 0]).astype(int)
    return (u + b[:, None, None], (10 + b).astype(np.int32),
            dict(passes=(2 * (10 + b)).astype(np.int32), done=b != 3))


def _ddp_worker(rank, world, port, B, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from noc import distributed as D
    u = np.arange(B * 5, dtype=np.float64).reshape(B, 5, 1)
    x0 = np.zeros((B, 2))
    x0[:, 0] = np.arange(B)
    info = {}
    U, it, passes = D.ddp_sharded(None, u, x0, ddp_fn=_fake_ddp, info=info)
    q.put((rank, U, it, passes, info))
    dist.destroy_process_group()


@pytest.mark.parametrize("B", [5, 1])
def test_ddp_sharded_world2_gloo(B):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, world, port, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    b = np.arange(B)
    for rank, U, it, passes, info in res:
        assert np.array_equal(U, np.arange(B * 5, dtype=np.float64).reshape(B, 5, 1) + b[:, None, None])
        assert np.array_equal(it, 10 + b) and np.array_equal(passes, 2 * (10 + b))
        assert info["passes_total"] == int(np.sum(2 * (10 + b)))
        assert info["not_done"] == int(np.sum(b == 3))
