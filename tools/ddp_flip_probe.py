#!/usr/bin/env python3
"""First divergent accept / reject decision of one-stage interior-point DDP (ddp(ocp, u, x0, bp),
D:98-186) between the GPU kernel (noc_ddp_solve_ex, its per-pass decision trace
noc_debug_set_ddp_trace) and the oracle restatement (oracle/noc_oracle.py: ddp), on one input.
Prints both iteration / pass counts, the first pass whose decision (success, iteration, inner
count) differs, both sides' pred, cost, new_cost, gain there, and the margins |pred| / (eps |cost|)
and |new_cost - cost| / (eps |cost|): a decision taken at the resolution of the cost (a few eps)
is a rounding flip; a larger margin would be an algorithmic difference.
Usage: ddp_flip_probe.py [problem N seed bp]   (default: pendulum 20 5 5e-5, tests/test_ddp.py)"""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ip-parallel-optimal-control_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np
import torch
from noc import problems, _lib
from noc import differential_dynamic_programming as D
from oracle import noc_oracle as O, problems as PR

KEYS = ["bp", "it", "inner", "pred", "gain", "success", "rp", "hu", "cost", "new_cost"]


def oracle_problem(name, N):
    return O.NumpyProblem(PR.pendulum_ocp(1.0 / N) if name == "pendulum" else PR.cartpole_ocp(1.0 / N))


def probe(name="pendulum", N=20, seed=5, bp=5e-5):
    ocp = problems.make_problem(name, N) if name != "pendulum" else problems.pendulum(1.0 / N)
    x0, u0 = problems.initial_conditions(name, N, 1, seed=seed)
    lib = _lib.load()
    fn = lib.noc_debug_set_ddp_trace
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    CAP = 8192
    tbuf = torch.zeros(1, CAP, len(KEYS), dtype=torch.float64, device="cuda")
    assert fn(tbuf.data_ptr(), CAP, 1) == 0
    try:
        X, U, its = D.ddp(ocp, u0[0], x0[0], bp)
        torch.cuda.synchronize()
    finally:
        assert fn(None, 0, 0) == 0
    tr = []
    Xr, Ur, itr, passes_r = O.ddp(oracle_problem(name, N), u0[0], x0[0], bp, trace=tr)
    rows = tbuf[0].cpu().numpy()
    g = [dict(zip(KEYS, r)) for r in rows if r[2] >= 1]  # recorded passes (inner >= 1)
    eps = np.finfo(np.float64).eps
    first = None
    for i, (a, b) in enumerate(zip(tr, g)):
        if bool(a["success"]) != bool(b["success"]) or a["it"] != int(b["it"]) or a["inner"] != int(b["inner"]):
            res = lambda d: abs(d["cost"]) * eps
            first = dict(pass_index=i,
                         oracle={k: (float(a[k]) if k != "success" else bool(a[k])) for k in a},
                         gpu={k: (float(b[k]) if k != "success" else bool(b[k])) for k in KEYS},
                         oracle_pred_over_eps_cost=abs(a["pred"]) / res(a),
                         oracle_dcost_over_eps_cost=abs(a["new_cost"] - a["cost"]) / res(a),
                         gpu_pred_over_eps_cost=abs(b["pred"]) / res(b),
                         gpu_dcost_over_eps_cost=abs(b["new_cost"] - b["cost"]) / res(b),
                         rel_diff_cost=abs(a["cost"] - b["cost"]) / res(a),
                         rel_diff_pred=abs(a["pred"] - b["pred"]) / max(abs(a["pred"]), 1e-300))
            break
    # how far apart the two runs were before the flip: max relative pred difference so far
    upto = first["pass_index"] if first else min(len(tr), len(g))
    drift = [abs(a["pred"] - b["pred"]) / max(abs(a["pred"]), 1e-300) for a, b in zip(tr[:upto], g[:upto])]
    return dict(problem=name, N=N, seed=seed, bp=bp, gpu=dict(iterations=int(its), passes=len(g)),
                oracle=dict(iterations=int(itr), passes=int(passes_r)), first_divergence=first,
                max_rel_pred_diff_before=max(drift) if drift else 0.0,
                rel_pred_diff_by_pass=[float(x) for x in drift[-40:]],
                max_abs_dU=float(np.max(np.abs(U - Ur))))


if __name__ == "__main__":
    a = sys.argv[1:]
    out = probe(a[0], int(a[1]), int(a[2]), float(a[3])) if len(a) >= 4 else probe()
    print(json.dumps(out, indent=1, default=float))
