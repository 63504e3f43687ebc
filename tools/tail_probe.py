#!/usr/bin/env python3
"""End-to-end tail of the persistent interior-point solve at a batched config (default c3:
cart-pole N=200, B=4096): wall time of noc_ipm_solve (HIP events), the per-trajectory KKT-solve
counts (saved as .npy next to the JSON line) and their distribution -- the straggler that sets the
wall time.  Usage: python tools/tail_probe.py [--problem cartpole --N 200 --B 4096 --out DIR]"""
import argparse, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))
import numpy as np, torch
from noc import problems
from noc.ipm import BatchedIPM

ap = argparse.ArgumentParser()
ap.add_argument("--problem", default="cartpole")
ap.add_argument("--N", type=int, default=200)
ap.add_argument("--B", type=int, default=4096)
ap.add_argument("--seed", type=int, default=11)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "tail"))
a = ap.parse_args()
os.makedirs(a.out, exist_ok=True)
ocp = problems.make_problem(a.problem, a.N)
x0, u0 = problems.initial_conditions(a.problem, a.N, a.B, seed=a.seed)
eng = BatchedIPM(ocp.family, a.N, a.B, persistent=True)
ms = []
for r in range(a.reps + 1):
    eng.load(u0, x0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); eng.solve(); e1.record(); torch.cuda.synchronize()
    if r:
        ms.append(e0.elapsed_time(e1))
# KKT solves actually computed: the retry-cap repeats are accounted without recomputation (§3.4)
solves = eng.t["kkt_solves"].cpu().numpy() - eng.t["repeats"].cpu().numpy()
timeline = {}
if "prof" in os.environ.get("NOC_HIP_LIB", ""):  # per-trajectory start / end (100 MHz stamps)
    import ctypes
    from noc import _lib
    n = a.B
    buf = (ctypes.c_longlong * (2 * n))()
    _lib.load().noc_debug_traj_times(buf, n)
    tt = np.frombuffer(buf, dtype=np.int64).reshape(n, 2).astype(np.float64)
    t0 = tt[:, 0].min()
    start_ms, end_ms = (tt[:, 0] - t0) * 1e-5, (tt[:, 1] - t0) * 1e-5
    np.save(os.path.join(a.out, f"{a.problem}_N{a.N}_B{a.B}{os.environ.get('NOC_PERSIST_HEAVY', '')}_times_ms.npy"),
            np.stack([start_ms, end_ms], 1))
    k = int(solves.argmax())
    z = int(end_ms.argmax())
    order = np.sort(end_ms)
    timeline = {"straggler": {"start_ms": start_ms[k], "end_ms": end_ms[k],
                              "us_per_solve": 1e3 * (end_ms[k] - start_ms[k]) / solves[k]},
                "last_to_end": {"traj": z, "start_ms": start_ms[z], "end_ms": end_ms[z],
                                "solves": int(solves[z])},
                "starts_after_ms": {t: int((start_ms > t).sum()) for t in (1, 5, 10, 20, 30)},
                "ms_when_remaining": {r: float(order[a.B - r - 1]) for r in (2048, 1024, 256, 64, 16, 1)
                                      if r < a.B},
                "us_per_solve_p50": float(np.median(1e3 * (end_ms - start_ms) / solves))}
its = eng.t["total_it"].cpu().numpy()
tag = os.environ.get("TAIL_TAG", os.environ.get("NOC_PERSIST_HEAVY", ""))
tag = f"_h{tag}" if tag else ""
np.save(os.path.join(a.out, f"{a.problem}_N{a.N}_B{a.B}{tag}_solves.npy"), solves)
if getattr(eng, "_order", None) is not None:  # the launch order (descending initial cost)
    np.save(os.path.join(a.out, f"{a.problem}_N{a.N}_B{a.B}{tag}_order.npy"), eng._order.cpu().numpy())
q = np.percentile(solves, [50, 90, 99, 99.9, 100])
print(json.dumps({"problem": a.problem, "N": a.N, "B": a.B, "wall_ms": ms,
                  "kkt_solves_computed": int(solves.sum()), "mean": float(solves.mean()),
                  "p50_p90_p99_p999_max": [float(v) for v in q],
                  "n_over_300": int((solves > 300).sum()), "n_over_400": int((solves > 400).sum()),
                  "argmax": int(solves.argmax()), "mean_iters": float(its.mean()),
                  "env_wide": os.environ.get("NOC_PERSIST_WIDE"), "tag": os.environ.get("TAIL_TAG", os.environ.get("NOC_PERSIST_HEAVY")), "timeline": timeline}), flush=True)
