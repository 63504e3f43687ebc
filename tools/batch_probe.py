#!/usr/bin/env python3
"""Per-trajectory cost of the c3 KKT scan vs the number of trajectories resident per launch.

The scan reads every block twice (phase 1 element build, phase 3 in-chunk Riccati) and A, B a
third time (phase 4).  Whether the re-reads hit the memory-side cache depends on how much data
the whole grid streams between a wave's first read and its re-read, so this times the batch as
one launch and as k back-to-back launches of B/k trajectories (HIP events, median of rounds).
Prints one JSON line per variant."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problem", default="cartpole")
    ap.add_argument("--horizon", type=int, default=200)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--splits", default="1,2,4")
    ap.add_argument("--lanes", default="32,64")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    import torch
    from noc import lqt, problems
    from bench import algorithmic_bytes
    N, B = args.horizon, args.batch
    variants = {}
    for L in [int(x) for x in args.lanes.split(",")]:
        for k in [int(x) for x in args.splits.split(",")]:
            parts = []
            for i in range(k):
                blk = problems.make_bench_blocks(args.problem, N=N, batch=B // k, seed=7 + i, lanes=L)
                parts.append((blk["tiled"], blk["reg"]))
                del blk["engine"]
            outs = [lqt.kkt_solve_tiled(tb, reg=reg, want_gains=False) for tb, reg in parts]
            variants[(L, k)] = (parts, outs)
    torch.cuda.synchronize()
    times = {key: [] for key in variants}
    for _ in range(args.rounds):
        for key, (parts, outs) in variants.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                for (tb, reg), o in zip(parts, outs):
                    lqt.kkt_solve_tiled(tb, reg=reg, out=o, want_gains=False)
            e1.record()
            torch.cuda.synchronize()
            times[key].append(e0.elapsed_time(e1) / args.reps)
    tb0 = variants[next(iter(variants))][0][0][0]
    abytes = algorithmic_bytes(tb0.nx, tb0.nu, N, B)
    for (L, k), ts in times.items():
        ts = sorted(ts)
        med = ts[len(ts) // 2]
        feas = min(float(o.feasible.float().mean()) for o in variants[(L, k)][1])
        print(json.dumps({"problem": args.problem, "N": N, "B": B, "lanes": L, "launches": k,
                          "batch_per_launch": B // k, "ms_median": med, "ms_min": ts[0],
                          "traj_kkt_per_s": B / (med * 1e-3),
                          "achieved_GBs": abytes / (med * 1e-3) / 1e9,
                          "feasible_frac": feas}), flush=True)


if __name__ == "__main__":
    main()
