#!/usr/bin/env python3
"""Time the KKT scan kernel per (config, lanes) -- interleaved rounds in one process (median of
rounds), HIP events on the launch stream.  Prints one JSON line per variant."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))
sys.path.insert(0, ROOT)

CONFIGS = {"c2": ("pendulum", 100, 1024), "c3": ("cartpole", 200, 4096),
           "c4": ("linear8", 512, 16384), "c5": ("cartpole", 200, 8192)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c2")
    ap.add_argument("--lanes", default="64,32,16,8")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--layouts", default="tiled,natural")
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    import torch
    from noc import lqt, problems
    from bench import algorithmic_bytes
    for cname in args.configs.split(","):
        name, N, B = CONFIGS[cname]
        times, outs, tbs = {}, {}, {}
        for L in [int(x) for x in args.lanes.split(",")]:
            blk = problems.make_bench_blocks(name, N=N, batch=B, seed=7, lanes=L)
            tb = blk["tiled"]
            nx, nu = tb.nx, tb.nu
            for layout in args.layouts.split(","):
                key = (L, layout)
                times[key] = []
                if layout == "tiled":
                    fn = (lambda tb=tb, reg=blk["reg"], o=None: lqt.kkt_solve_tiled(tb, reg=reg, out=o, want_gains=False))
                else:
                    nat = blk["engine"].natural_blocks()
                    fn = (lambda nat=nat, reg=blk["reg"], L=L, o=None: lqt.kkt_solve(
                        *(nat[k] for k in ("A", "B", "Q", "R", "M", "r", "P")), reg=reg, lanes=L,
                        out=o, want_gains=False))
                outs[key] = fn()
                tbs[key] = fn
            del blk
        torch.cuda.synchronize()
        ref = outs[next(iter(outs))].dx
        for _ in range(args.rounds):
            for key, fn in tbs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    fn(o=outs[key])
                e1.record()
                torch.cuda.synchronize()
                times[key].append(e0.elapsed_time(e1) / args.reps)
        abytes = algorithmic_bytes(nx, nu, N, B)
        for (L, layout), ts in times.items():
            ts = sorted(ts)
            med = ts[len(ts) // 2]
            diff = float((outs[(L, layout)].dx - ref).abs().max())
            print(json.dumps({"config": cname, "problem": name, "N": N, "B": B, "lanes": L,
                              "layout": layout,
                              "ms_median": med, "ms_min": ts[0],
                              "traj_kkt_per_s": B / (med * 1e-3),
                              "achieved_GBs": abytes / (med * 1e-3) / 1e9,
                              "max_abs_dx_diff_vs_first": diff,
                              "feasible_frac": float(outs[(L, layout)].feasible.float().mean())}),
                  flush=True)


if __name__ == "__main__":
    main()
