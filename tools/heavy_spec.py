#!/usr/bin/env python3
"""Schedules of one batch of cart-poles in one process, each timed over repeated solves (the
first call of a process also loads the kernel instances it meets): the default (auto), the probe
schedule, and the probe schedule with the costliest H trajectories on two speculative candidates
each (NOC_PERSIST_HEAVY=H, NOC_PERSIST_HEAVY_SPEC=2).  One JSON line per configuration.

    python tools/heavy_spec.py [--B 1024 --N 200 --H 64,128,256,384,512]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1024)
    ap.add_argument("--N", type=int, default=200)
    ap.add_argument("--H", default="64,128,256,384,512")
    ap.add_argument("--reps", type=int, default=4)
    args = ap.parse_args()
    from noc import problems
    from noc.ipm import BatchedIPM
    ocp = problems.make_problem("cartpole", args.N)
    x0, u0 = problems.initial_conditions("cartpole", args.N, args.B, seed=11)
    configs = [("auto", None), ("probe", None)] + [("probe", int(h)) for h in args.H.split(",")]
    for sched, h in configs:
        if h is None:
            os.environ.pop("NOC_PERSIST_HEAVY", None)
            os.environ.pop("NOC_PERSIST_HEAVY_SPEC", None)
        else:
            os.environ["NOC_PERSIST_HEAVY"] = str(h)
            os.environ["NOC_PERSIST_HEAVY_SPEC"] = "2"
        eng = BatchedIPM(ocp.family, args.N, args.B, persistent=True)
        times = []
        for _ in range(args.reps):
            eng.load(u0, x0)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eng.solve_persistent(schedule=sched)
            e1.record()
            torch.cuda.synchronize()
            times.append(round(e0.elapsed_time(e1), 3))
        U = eng.result()[0].cpu().numpy()
        print(json.dumps({"B": args.B, "schedule": sched, "heavy": h, "ms": times,
                          "u_sha1": hashlib.sha1(np.ascontiguousarray(U).tobytes()).hexdigest()[:16]}),
              flush=True)


if __name__ == "__main__":
    main()
