#!/usr/bin/env python3
"""End-to-end batched interior-point solve timing (device loop), per-kernel breakdown via
rocprofv3 when run under it.  Prints one JSON line."""
import hashlib, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))
import numpy as np
import torch
from noc import problems, _lib
from noc.ipm import BatchedIPM

name = sys.argv[1] if len(sys.argv) > 1 else "cartpole"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 200
B = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
persistent = (sys.argv[4] == "persistent") if len(sys.argv) > 4 else False
lanes = int(sys.argv[5]) if len(sys.argv) > 5 else 0   # 0: the batch-aware policy
ocp = problems.make_problem(name, N)
x0, u0 = problems.initial_conditions(name, N, B, seed=11)
eng = BatchedIPM(ocp.family, N, B, persistent=persistent, lanes=lanes)
if os.environ.get("PROBE_SOLVES"):  # the probe-ordered launch's probe length (A/B only)
    eng.PROBE_SOLVES = int(os.environ["PROBE_SOLVES"])
if os.environ.get("NOC_NO_REPEAT_SKIP") == "1":  # recompute the identical retries at the rp clip
    eng.ws.flags = _lib.WS_NO_REPEAT_SKIP
eng.load(u0, x0)
eng.solve(max_steps=eng.PROBE_SOLVES + 16 if persistent else 16)   # warm-up: kernels loaded (the probe and the resume instance), caches
torch.cuda.synchronize()
eng.load(u0, x0)
t0 = time.perf_counter()
# solve() / solve_persistent() return the KKT solves of the slowest trajectory (accounted retries
# included), not a launch count: the per-solve time below is per KKT solve of that trajectory
slowest = eng.solve_persistent(schedule=os.environ.get("NOC_SCHEDULE", "auto")) if persistent else eng.solve()
torch.cuda.synchronize()
dt = time.perf_counter() - t0
U, its, solves = (t.cpu().numpy() for t in eng.result())
print(json.dumps({"problem": name, "N": N, "B": B, "lanes": eng.lanes, "persistent": persistent,
                  "max_kkt_solves_slowest": slowest,
                  "wall_s": dt, "ms_per_kkt_solve_of_slowest": 1e3 * dt / max(slowest, 1),
                  "total_kkt_solves": int(solves.sum()), "kkt_solves_per_s": float(solves.sum() / dt),
                  "mean_outer_iters": float(its.mean()), "max_kkt_solves": int(solves.max()),
                  "min_kkt_solves": int(solves.min()),
                  "repeats_accounted": int(eng.t["repeats"].sum().item()),
                  "no_repeat_skip": bool(eng.ws.flags & _lib.WS_NO_REPEAT_SKIP),
                  # bit-identity across kernel variants (NOC_PERSIST_WAVES / NOC_PERSIST_QLDS)
                  "u_sha1": hashlib.sha1(np.ascontiguousarray(U).tobytes()).hexdigest()[:16],
                  "env": {k: v for k, v in os.environ.items() if k.startswith("NOC_")}}))
