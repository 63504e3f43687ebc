"""bench.py's multi-GPU contract on the CPU (no GPU work: NOC_BENCH_DRYRUN=1, gloo): `bench.py
--gpus N` with no launcher starts N ranks itself and prints ONE line with n_gpus = N; under a
launcher whose world size differs from --gpus it refuses to run (non-zero exit)."""
import json
import os
import subprocess
import sys

import pytest

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


def test_bench_gpus_8_is_the_whole_node():
    """--gpus 8 (the north-star curve's last point; the driver's SCALE run): 8 ranks over gloo on
    the CPU, one line, every rank seen."""
    p = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--steps", "2", "--warmup", "1"],
                       env=_env(), capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-2000:]
    (line,) = _lines(p.stdout)
    assert line["n_gpus"] == 8 and line["rccl_world_size"] == 8
    assert line["ranks_seen"] == list(range(8))
    assert line["scaling"] == "strong" and line["config"]["global_batch"] == 4096


def test_bench_gpus_1_is_one_process():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--steps", "1"], env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    (line,) = _lines(p.stdout)
    assert line["n_gpus"] == 1 and line["ranks_seen"] == [0]


def _dump(tmp_path, gpus, extra=(), global_batch=37):
    d = tmp_path / f"w{gpus}_{global_batch}_{len(extra)}"
    d.mkdir()
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(gpus), "--steps", "1",
                        "--global-batch", str(global_batch), "--horizon", "20", *extra],
                       env=_env(NOC_BENCH_DRYRUN_DUMP=str(d)), capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    import numpy as np
    parts = [np.load(d / f"rank{r}_of{gpus}.npz") for r in range(gpus)]
    return parts, _lines(p.stdout)[0]


def test_bench_shards_one_global_batch(tmp_path):
    """every rank of the strong-scaling bench draws the SAME global batch
    (one seed) and keeps its shard_bounds slice, so the N-rank shards concatenate to exactly the
    1-rank inputs (bit for bit) -- the N-rank line solves the 1-rank problem."""
    import numpy as np
    (one,), line1 = _dump(tmp_path, 1)
    assert line1["config"]["global_batch"] == 37 and line1["scaling"] == "strong"
    for gpus in (2, 4, 8):
        parts, line = _dump(tmp_path, gpus)
        assert line["config"]["global_batch"] == 37
        los = [int(q["lo"]) for q in parts]
        assert los == sorted(los) and los[0] == 0
        for k in ("x0", "u0"):
            cat = np.concatenate([q[k] for q in parts])
            assert np.array_equal(cat, one[k]), (gpus, k)


def test_bench_world8_c3_shards(tmp_path):
    """The north-star point itself: c3's 4096 cart-poles over 8 ranks are 8 shards of 512 that
    concatenate bit for bit to the 1-rank batch."""
    import numpy as np
    (one,), _ = _dump(tmp_path, 1, global_batch=4096)
    parts, line = _dump(tmp_path, 8, global_batch=4096)
    assert line["config"]["global_batch"] == 4096 and line["ranks_seen"] == list(range(8))
    assert [len(q["x0"]) for q in parts] == [512] * 8
    for k in ("x0", "u0"):
        assert np.array_equal(np.concatenate([q[k] for q in parts]), one[k]), k


@pytest.mark.parametrize("gpus,batch", [(2, 5), (8, 8192)])
def test_bench_weak_scaling_slices(tmp_path, gpus, batch):
    """--batch B (weak scaling): rank r owns trajectories [rB, (r+1)B) of the global B x world;
    (8, 8192) is BASELINE config c5 (65 536 cart-poles over the 8 GPUs of a node)."""
    import numpy as np
    parts, line = _dump(tmp_path, gpus, ("--batch", str(batch)))
    assert line["scaling"] == "weak" and line["config"]["global_batch"] == gpus * batch
    sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))
    from noc import problems
    x0, u0 = problems.initial_conditions("cartpole", 20, gpus * batch, seed=1234)
    assert np.array_equal(np.concatenate([q["x0"] for q in parts]), x0)
    assert np.array_equal(np.concatenate([q["u0"] for q in parts]), u0)
