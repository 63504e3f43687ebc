#!/usr/bin/env python3
"""How well does the state after the first K KKT solves of every trajectory predict its
remaining solves?  c3 persistent solve (cart-pole N=200, B=4096, seed 11): a capped launch
(max_solves = K, cost order), a snapshot of every trajectory's solver state, then the resumed
launch to the end.  Saves the snapshots and the final counts (npz) for an offline
list-scheduling model (profiles/r05/heavy_split/).  GPU only."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))
import numpy as np, torch
from noc import problems
from noc.ipm import BatchedIPM

out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "predict")
os.makedirs(out, exist_ok=True)
N, B = 200, 4096
ocp = problems.make_problem("cartpole", N)
x0, u0 = problems.initial_conditions("cartpole", N, B, seed=11)
eng = BatchedIPM(ocp.family, N, B, persistent=True)
keys = ("kkt_solves", "repeats", "total_it", "it", "inner", "bp", "hu", "cost", "rp", "rinc", "gnorm", "phase")
res = {}
KS = [int(k) for k in os.environ.get("PROBE_KS", "10,20,40").split(",")]
for K in [KS[0]] + KS:  # the first K twice: its first pass warms the kernels up
    eng.load(u0, x0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.solve_persistent(max_solves=K, schedule="cost")
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    snap = {f"K{K}_{k}": eng.t[k].cpu().numpy().copy() for k in keys}
    eng.solve_persistent(resume=True)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    snap[f"K{K}_final_solves"] = eng.t["kkt_solves"].cpu().numpy().copy()
    snap[f"K{K}_final_repeats"] = eng.t["repeats"].cpu().numpy().copy()
    snap[f"K{K}_order"] = eng_order = np.arange(B)
    res.update(snap)
    print(json.dumps({"K": K, "probe_ms": 1e3 * (t1 - t0), "resume_ms": 1e3 * (t2 - t1)}), flush=True)
np.savez_compressed(os.path.join(out, "predict_probe.npz"), **res)
