"""Debug probe (round 5): where do the AB-on and AB-off natural-layout solves differ?"""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "ip-parallel-optimal-control_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np, torch
from noc import lqt, _lib
from lq_cases import rand_lq, oracle_batch
lib = _lib.load()
for (N, L, B, tiled) in [(200, 64, 1024, False), (200, 64, 1024, True), (7, 64, 33, False), (300, 128, 64, False)]:
    case = rand_lq(4200 + N + L + B, B, N, 4, 1)
    g = lambda k: torch.as_tensor(case[k], device="cuda")
    def solve():
        if tiled:
            tb = lqt.to_tiled(g("A"), g("B"), g("Q"), g("R"), g("M"), g("r"), g("P"), L)
            return lqt.kkt_solve_tiled(tb, reg=g("reg"))
        return lqt.kkt_solve(g("A"), g("B"), g("Q"), g("R"), g("M"), g("r"), g("P"), reg=g("reg"), lanes=L)
    on = solve(); lib.noc_debug_set_ablation(64); off = solve(); lib.noc_debug_set_ablation(0)
    torch.cuda.synchronize()
    d = (on.dx - off.dx).abs()
    bad = torch.nonzero(d.amax(dim=2) > 0)
    ref = oracle_batch({k: v[[0, B - 1]] for k, v in case.items()})
    e_on = float(np.max(np.abs(on.dx[[0, B - 1]].cpu().numpy() - ref["dx"])))
    e_off = float(np.max(np.abs(off.dx[[0, B - 1]].cpu().numpy() - ref["dx"])))
    stages = sorted(set(bad[:, 1].tolist()))[:40]
    print(dict(N=N, L=L, B=B, tiled=tiled, maxdiff=float(d.max()), n_bad=len(bad),
               traj_bad=len(set(bad[:, 0].tolist())), first_stages=stages, err_on=e_on, err_off=e_off,
               du=float((on.du - off.du).abs().max()), K=float((on.K - off.K).abs().max()) if on.K is not None and not tiled else None))
