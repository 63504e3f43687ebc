"""Debug tool: compare the persistent and the multi-launch drivers' workspaces after k KKT solves."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))
import numpy as np, torch
from noc import problems, _lib
from noc.ipm import BatchedIPM
name, N, Bt = "cartpole", 200, 64
ocp = problems.make_problem(name, N)
x0, u0 = problems.initial_conditions(name, N, Bt, seed=21)
term = int(sys.argv[1]) if len(sys.argv) > 1 else _lib.TERMINAL_STAGE0
for k in (1, 2, 3, 5, 10):
    ep = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=True)
    ep.load(u0, x0)
    ep.solve_persistent(_lib.MODE_PAR, term, 0.1, max_solves=k)
    em = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=False)
    em.load(u0, x0)
    em.init(0.1)
    for _ in range(k):
        em.step(_lib.MODE_PAR, term)
    torch.cuda.synchronize()
    diffs = {}
    for f in ["x", "u", "P", "A", "B", "Q", "R", "M", "r", "pred", "reg", "rp", "cost", "hu"]:
        a, b = ep.t[f].double(), em.t[f].double()
        diffs[f] = float((a - b).abs().max())
    print(k, {f: f"{v:.1e}" for f, v in diffs.items() if v > 0}, flush=True)
