#!/usr/bin/env python3
"""The tail schedule of BatchedIPM.solve_persistent (capped launches, then the stragglers gathered
and resumed with speculative candidates) over a few cap ladders: wall time of the whole solve,
(cap, trajectories still running) per capped launch, and the controls' hash (every ladder must
give the same bits).  One JSON line per (B, ladder).

    python tools/tail_caps.py [--problem cartpole --N 200 --B 1024,2048,4096 --seed 11]
"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

LADDERS = ["off", "128,256,384,512", "192,320,480", "256,384,512", "320,480,640"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problem", default="cartpole")
    ap.add_argument("--N", type=int, default=200)
    ap.add_argument("--B", default="1024,2048,4096")
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--ladders", default=";".join(LADDERS))
    args = ap.parse_args()
    from noc import problems
    from noc.ipm import BatchedIPM
    ocp = problems.make_problem(args.problem, args.N)
    for B in (int(b) for b in args.B.split(",")):
        x0, u0 = problems.initial_conditions(args.problem, args.N, B, seed=args.seed)
        for lad in args.ladders.split(";"):
            if lad == "off":
                os.environ["NOC_PERSIST_TAIL"] = "0"
                os.environ.pop("NOC_PERSIST_TAIL_CAPS", None)
            else:
                os.environ["NOC_PERSIST_TAIL"] = "1"
                os.environ["NOC_PERSIST_TAIL_CAPS"] = lad
            eng = BatchedIPM(ocp.family, args.N, B, persistent=True)
            times = []
            for rep in range(3):
                eng.load(u0, x0)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                eng.solve_persistent()
                e1.record()
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1))
            U, its, solves = (t.cpu().numpy() for t in eng.result())
            print(json.dumps({"B": B, "ladder": lad, "ms": times, "tail_log": getattr(eng, "tail_log", None),
                              "total_solves": int(solves.sum()), "max_solves": int(solves.max()),
                              "mean_iters": float(its.mean()),
                              "u_sha1": hashlib.sha1(np.ascontiguousarray(U).tobytes()).hexdigest()[:16]}),
                  flush=True)
    os.environ.pop("NOC_PERSIST_TAIL", None)
    os.environ.pop("NOC_PERSIST_TAIL_CAPS", None)


if __name__ == "__main__":
    main()
