"""The sharded solve with the REAL engine (noc.distributed.solve_sharded + BatchedIPM): a
world-size-2 gloo group launched by torch.distributed.run as child processes, both ranks on
cuda:0, and a world-size-1 RCCL ("nccl") group (the collectives on device tensors); every trajectory's result must be bit-identical to the unsharded solve (persistent kernel
and multi-launch loop).  The rank program is tests/dist_ipm_worker.py."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("name,N,B,persistent,world,backend", [
    ("cartpole", 60, 13, 1, 2, "gloo"), ("pendulum", 40, 9, 0, 2, "gloo"),
    # the RCCL path on hardware: one rank (a one-GPU box cannot give two ranks their own GPUs);
    # the collectives (all-reduce of the convergence norm / running count, all-gather of the
    # results) run on device tensors through RCCL
    ("cartpole", 60, 13, 1, 1, "nccl"), ("pendulum", 40, 9, 0, 1, "nccl")])
def test_sharded_solve_with_real_engine_is_bit_identical(name, N, B, persistent, world, backend):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(HERE, "dist_ipm_worker.py"), name, str(N), str(B), str(persistent)]
    env = dict(os.environ, OMP_NUM_THREADS="1", NOC_DIST_BACKEND=backend)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "SHARD_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
    assert f"world={world} backend={backend}" in r.stdout
