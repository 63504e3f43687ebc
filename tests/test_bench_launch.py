"""bench.py's multi-GPU contract on the CPU (no GPU work: NOC_BENCH_DRYRUN=1, gloo): `bench.py
--gpus N` with no launcher starts N ranks itself and prints ONE line with n_gpus = N; under a
launcher whose world size differs from --gpus it refuses to run (non-zero exit)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(NOC_BENCH_DRYRUN="1", **kw)
    return env


def _lines(out):
    return [json.loads(s) for s in out.splitlines() if s.startswith("{")]


def test_bench_gpus_2_starts_two_ranks():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "2", "--warmup", "1"],
                       env=_env(), capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _lines(p.stdout)
    assert len(lines) == 1, p.stdout            # rank 0 only
    line = lines[0]
    assert line["n_gpus"] == 2 and line["rccl_world_size"] == 2
    assert line["ranks_seen"] == [0, 1]
    assert line["value"] is None and line["dry_run"] is True


def test_bench_refuses_gpus_world_mismatch():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1"],
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0
    assert "refusing" in p.stderr
    assert not _lines(p.stdout)


def test_bench_gpus_1_is_one_process():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--steps", "1"], env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    (line,) = _lines(p.stdout)
    assert line["n_gpus"] == 1 and line["ranks_seen"] == [0]
