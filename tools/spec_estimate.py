#!/usr/bin/env python3
"""How much of a trajectory's serial chain of KKT solves could speculative retries take off?

A rejected trial (P:166-172) re-solves the same linearisation with the next regularisation
rp * r_inc, which is known before the trial is evaluated.  With K waves per trajectory, wave k can
solve and evaluate the k-th next candidate of the failure chain concurrently; the accept decisions
are then replayed in order, so the result is the sequential one bit for bit.  This tool records
every accept decision of the one-wave persistent solver (the decision-trace build:
`make -C ip-parallel-optimal-control_amd trace-lib`, loaded via NOC_HIP_LIB) and counts, per
trajectory, the computed KKT solves (the serial chain today) and the rounds of K candidates the
same decisions would take.

    NOC_HIP_LIB=ip-parallel-optimal-control_amd/noc/_lib/libnoc_hip_trace.so \\
        python tools/spec_estimate.py [--problem cartpole --N 200 --B 512 --seed 11]
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


def rounds(succ_iter, K):
    """Rounds of K speculative candidates for one Newton iteration's accept sequence (every entry
    but the last a rejection)."""
    return -(-len(succ_iter) // K)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problem", default="cartpole")
    ap.add_argument("--N", type=int, default=200)
    ap.add_argument("--B", type=int, default=512)
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--cap", type=int, default=1100)
    args = ap.parse_args()
    import torch
    from noc import problems, _lib
    from noc.ipm import BatchedIPM
    lib = _lib.load()
    fn = lib.noc_debug_set_decision_trace
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    os.environ["NOC_PERSIST_WIDE"] = "0"
    ocp = problems.make_problem(args.problem, args.N)
    x0, u0 = problems.initial_conditions(args.problem, args.N, args.B, seed=args.seed)
    buf = torch.full((args.B, args.cap, len(FIELDS)), float("nan"), dtype=torch.float64, device="cuda")
    if fn(buf.data_ptr(), args.cap, args.B) != 1:
        raise SystemExit("this library has no decision trace (make trace-lib; NOC_HIP_LIB)")
    eng = BatchedIPM(ocp.family, args.N, args.B, lanes=64, persistent=True)
    eng.load(u0, x0)
    eng.solve()
    torch.cuda.synchronize()
    fn(None, 0, 0)
    tr = buf.cpu().numpy()
    _, its, solves = (t.cpu().numpy() for t in eng.result())
    per = []
    for b in range(args.B):
        rec = tr[b]
        rec = rec[~np.isnan(rec[:, 0])]  # computed solves (accounted repeats leave gaps)
        # split into Newton iterations: a record ends its iteration when it succeeded or the
        # iteration hit inner > 500 (P:177-182); bp changes between barrier stages
        seqs, cur = [], []
        for r in rec:
            cur.append(r[7])
            if r[7] == 1.0 or r[2] > 500:
                seqs.append(cur)
                cur = []
        if cur:
            seqs.append(cur)
        row = {"traj": b, "computed": int(len(rec)), "solves": int(solves[b]), "iters": int(len(seqs))}
        for K in (2, 4):
            row[f"rounds{K}"] = int(sum(rounds(s, K) for s in seqs))
        per.append(row)
    comp = np.array([p["computed"] for p in per])
    r2 = np.array([p["rounds2"] for p in per])
    r4 = np.array([p["rounds4"] for p in per])
    hv = int(np.argmax(comp))
    out = {"problem": args.problem, "N": args.N, "B": args.B, "seed": args.seed,
           "computed_max": int(comp.max()), "rounds2_of_heaviest": int(r2[hv]),
           "rounds4_of_heaviest": int(r4[hv]), "rounds2_max": int(r2.max()), "rounds4_max": int(r4.max()),
           "computed_total": int(comp.sum()), "rounds2_total": int(r2.sum()), "rounds4_total": int(r4.sum()),
           "heaviest": per[hv], "top8_computed": sorted(per, key=lambda p: -p["computed"])[:8]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
