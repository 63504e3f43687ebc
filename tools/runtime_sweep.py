#!/usr/bin/env python3
"""Timing-harness parity with the reference's examples/pendulum_runtime.py:74-161 and
examples/cartpole_runtime.py:85-170.

Protocol mirrored: for (Ts, N) in zip(Ts, N) with Ts*N = 1 s, x0 as the reference (pendulum
[wrap(0.1), -0.1], cart-pole [0.01, wrap(-0.01), 0.01, -0.01]), u0 = 0.1*normal(horizon, 1); one
warm-up call, then 10 timed calls of the par and seq interior-point solves, each followed by a
device sync (the reference's jax.block_until_ready); mean and median per (Ts, N) written to CSV
files named like the reference's (<problem>_ip_means_par.csv, ..._medians_seq.csv; one column,
pandas layout).  Differences: u0 comes from numpy default_rng(1) (jax.random.PRNGKey(1) is not
available here); `--batch B` optionally solves B copies at once (B = 1 is the reference's
setting).  All three solvers the reference times: par, seq and interior-point DDP (*_ddp.csv).

Usage: python tools/runtime_sweep.py [--problem pendulum|cartpole] [--out DIR] [--runs 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))

TS = [0.05, 0.025, 0.0125, 0.01, 0.005, 0.0025, 0.00125, 0.001]   # PR:74 / CR:85
NS = [20, 40, 80, 100, 200, 400, 800, 1000]                        # PR:75 / CR:86


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problem", default="pendulum", choices=["pendulum", "cartpole"])
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "runtime"))
    ap.add_argument("--runs", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--max-n", type=int, default=1000)
    args = ap.parse_args()
    import pandas as pd
    import torch
    from noc import problems
    from noc.par_interior_point_newton import par_interior_point_optimal_control
    from noc.seq_interior_point_newton import seq_interior_point_optimal_control
    from noc.differential_dynamic_programming import interior_point_ddp
    from noc.utils import wrap_angle

    os.makedirs(args.out, exist_ok=True)
    stats = {k: [] for k in ("par_mean", "par_median", "seq_mean", "seq_median", "ddp_mean",
                             "ddp_median")}
    rows = []
    for ts, n in zip(TS, NS):
        if n > args.max_n:
            break
        ocp = problems.pendulum(ts) if args.problem == "pendulum" else problems.cartpole(ts)
        if args.problem == "pendulum":
            x0 = np.array([float(wrap_angle(0.1)), -0.1])
        else:
            x0 = np.array([0.01, float(wrap_angle(-0.01)), 0.01, -0.01])
        u = 0.1 * np.random.default_rng(1).normal(size=(n, 1))
        if args.batch > 1:
            u = np.repeat(u[None], args.batch, 0)
            x0 = np.repeat(x0[None], args.batch, 0)
        res = {}
        for tag, fn in (("par", par_interior_point_optimal_control),
                        ("seq", seq_interior_point_optimal_control),
                        ("ddp", interior_point_ddp)):
            out = fn(ocp, u, x0)          # warm-up (the reference's first jitted call)
            torch.cuda.synchronize()
            times = []
            for _ in range(args.runs):
                t0 = time.time()
                out = fn(ocp, u, x0)
                torch.cuda.synchronize()
                times.append(time.time() - t0)
            stats[f"{tag}_mean"].append(float(np.mean(times)))
            stats[f"{tag}_median"].append(float(np.median(times)))
            its = np.asarray(out[1])
            res[tag] = {"mean_s": float(np.mean(times)), "median_s": float(np.median(times)),
                        "iterations": int(its.max())}
        rows.append({"Ts": ts, "N": n, "batch": args.batch, **res})
        print(json.dumps(rows[-1]), flush=True)
    p = args.problem
    for tag in ("par", "seq", "ddp"):
        pd.DataFrame(np.array(stats[f"{tag}_mean"])).to_csv(os.path.join(args.out, f"{p}_ip_means_{tag}.csv"))
        pd.DataFrame(np.array(stats[f"{tag}_median"])).to_csv(os.path.join(args.out, f"{p}_ip_medians_{tag}.csv"))
    with open(os.path.join(args.out, f"{p}_runtime.json"), "w") as fh:
        json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
