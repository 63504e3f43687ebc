#!/usr/bin/env python3
"""Root cause of a KKT-count flip between the two persistent solvers: the wide
kernel (ipm_wide.hip, 4 waves per trajectory) and the one-wave kernel (ipm_persistent.hip) run the
same reference control flow (P:127-254) but their scans associate differently, so their accept
tests (P:159-173) see different last bits.  This probe records every accept decision of both
kernels (the decision-trace build: `make -C ip-parallel-optimal-control_amd trace-lib`, loaded via
NOC_HIP_LIB) and of the oracle (oracle/noc_oracle.py par loop), finds the first decision where
they differ and prints, for each solver, cost, new_cost, pred, the gain ratio and how far the
actual and predicted reductions are from rounding level:

    ulp_actual = |new_cost - cost| / (eps |cost|)      ulp_pred = |pred| / (eps |cost|)

Usage (GPU): NOC_HIP_LIB=ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_trace.so \\
             python tools/flip_probe.py [--problem cartpole --N 200 --Bt 8 --seed 33 --traj 3]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ip-parallel-optimal-control_amd"), ROOT]
import numpy as np  # noqa: E402

FIELDS = ["bp", "it", "inner", "cost", "new_cost", "pred", "gain", "success", "rp", "rinc", "hu",
          "bwd_ok"]
EPS = np.finfo(np.float64).eps


def gpu_traces(problem, N, Bt, seed, mode, cap):
    import torch
    from noc import problems, _lib
    from noc.ipm import BatchedIPM
    lib = _lib.load()
    fn = lib.noc_debug_set_decision_trace
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    ocp = problems.make_problem(problem, N)
    x0, u0 = problems.initial_conditions(problem, N, Bt, seed=seed)
    out = {}
    for wide in ("1", "0"):
        os.environ["NOC_PERSIST_WIDE"] = wide
        buf = torch.full((Bt, cap, len(FIELDS)), float("nan"), dtype=torch.float64, device="cuda")
        rc = fn(buf.data_ptr(), cap, Bt)
        if rc != 1:
            raise SystemExit("this library has no decision trace: build `make trace-lib` and set "
                             "NOC_HIP_LIB to noc/_lib/libnoc_hip_trace.so")
        eng = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=True)
        eng.load(u0, x0)
        eng.ws.flags = _lib.WS_NO_REPEAT_SKIP  # one record per retry, none accounted
        eng.solve(mode=_lib.MODE_PAR if mode == "par" else _lib.MODE_SEQ)
        torch.cuda.synchronize()
        fn(None, 0, 0)
        U, its, solves = (t.cpu().numpy() for t in eng.result())
        out["wide" if wide == "1" else "one_wave"] = dict(trace=buf.cpu().numpy(), U=U, its=its,
                                                          solves=solves)
    os.environ.pop("NOC_PERSIST_WIDE", None)
    return out, x0, u0


def oracle_trace(problem, N, x0, u0):
    from oracle import noc_oracle as O, problems as PR
    tocp = PR.cartpole_ocp(1.0 / N) if problem == "cartpole" else PR.pendulum_ocp(1.0 / N)
    tr = []
    U, it, solves = O.par_interior_point_optimal_control(O.NumpyProblem(tocp), u0, x0,
                                                         terminal="stage0", trace=tr)
    rec = np.array([[t["bp"], t["it"], t["inner"] - 1, t["cost"], t["new_cost"], t["pred"],
                     t["gain"], float(t["success"]), np.nan, np.nan, t["hu"], np.nan] for t in tr])
    return dict(trace=rec, U=U, its=it, solves=solves)


def describe(rec):
    d = {k: float(v) for k, v in zip(FIELDS, rec)}
    c = abs(d["cost"])
    d["ulp_actual"] = abs(d["new_cost"] - d["cost"]) / (EPS * c) if c else None
    d["ulp_pred"] = abs(d["pred"]) / (EPS * c) if c else None
    return d


def first_divergence(ta, tb):
    n = min(len(ta), len(tb))
    for i in range(n):
        a, b = ta[i], tb[i]
        if np.isnan(a[0]) or np.isnan(b[0]):
            return None
        if a[7] != b[7] or a[1] != b[1] or a[0] != b[0]:
            return i
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problem", default="cartpole")
    ap.add_argument("--N", type=int, default=200)
    ap.add_argument("--Bt", type=int, default=8)
    ap.add_argument("--seed", type=int, default=33)
    ap.add_argument("--traj", type=int, default=3)
    ap.add_argument("--mode", default="par")
    ap.add_argument("--cap", type=int, default=4096)
    ap.add_argument("--no-oracle", action="store_true")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    g, x0, u0 = gpu_traces(args.problem, args.N, args.Bt, args.seed, args.mode, args.cap)
    b = args.traj
    res = {"case": vars(args),
           "solves": {k: g[k]["solves"].tolist() for k in g},
           "iterations": {k: g[k]["its"].tolist() for k in g}}
    tr = {k: g[k]["trace"][b] for k in g}
    if not args.no_oracle and args.mode == "par":
        o = oracle_trace(args.problem, args.N, x0[b], u0[b])
        tr["oracle"] = o["trace"]
        res["oracle"] = {"its": int(o["its"]), "solves": int(o["solves"])}
    names = list(tr)
    res["pairs"] = {}
    for i in range(len(names)):
        for j in range(i + 1, len(names)):
            a, c = names[i], names[j]
            k = first_divergence(tr[a], tr[c])
            entry = {"first_divergent_solve": k}
            if k is not None:
                entry[a] = describe(tr[a][k])
                entry[c] = describe(tr[c][k])
                # relative difference of the decision inputs at that solve
                entry["rel_diff"] = {f: float(abs(tr[a][k][n] - tr[c][k][n]) /
                                              max(abs(tr[c][k][n]), 1e-300))
                                     for n, f in enumerate(FIELDS) if f in ("cost", "new_cost", "pred")}
                entry["context"] = {nm: [describe(r) for r in tr[nm][max(0, k - 2):k + 3]]
                                    for nm in (a, c)}
            res["pairs"][f"{a}|{c}"] = entry
    # the largest gain-ratio decisions that were rounding-level in each solver: where every
    # accept / reject is decided by |actual| < 64 eps |cost|
    for nm in names:
        t = tr[nm][~np.isnan(tr[nm][:, 0])]
        ua = np.abs(t[:, 4] - t[:, 3]) / (EPS * np.abs(t[:, 3]))
        res.setdefault("rounding_level_decisions", {})[nm] = int(np.sum(ua < 64))
    txt = json.dumps(res, indent=1, default=float)
    print(txt)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(txt)


if __name__ == "__main__":
    main()
