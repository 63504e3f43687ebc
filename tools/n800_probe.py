#!/usr/bin/env python3
"""Cart-pole B=1 at the runtime-sweep inputs (CR:85-101): time and KKT-solve count of the par
solve per horizon, for the NOC_PERSIST_WAVES setting in the environment."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))
import numpy as np, torch
from noc import problems
from noc.par_interior_point_newton import par_interior_point_optimal_control
from noc.utils import wrap_angle
for ts, n in [(0.0025, 400), (0.00125, 800), (0.001, 1000)]:
    ocp = problems.cartpole(ts)
    x0 = np.array([0.01, float(wrap_angle(-0.01)), 0.01, -0.01])
    u = 0.1 * np.random.default_rng(1).normal(size=(n, 1))
    par_interior_point_optimal_control(ocp, u, x0)
    torch.cuda.synchronize()
    t0 = time.time()
    U, its, info = par_interior_point_optimal_control(ocp, u, x0, return_info=True)
    torch.cuda.synchronize()
    print(json.dumps({"N": n, "waves": os.environ.get("NOC_PERSIST_WAVES", "auto"),
                      "ms": 1e3 * (time.time() - t0), "iters": its,
                      "kkt_solves": int(info["kkt_solves"]), "u_sum": float(np.sum(U))}), flush=True)
