"""The north-star curve end to end, slice by slice on ONE GPU: `bench.py --slice r/W` for every
rank r of a W-rank strong-scaling run of c3 (cart-pole N = 200, global batch 4096), W = 1, 2, 4, 8.
A W-GPU run is trajectory-sharded with no collective on the data path (noc/distributed.py), so its
wall time is the slowest rank's: the max over the W slices measured here.  Both of the bench's
per-rank figures are collected -- the KKT launch (the metric's step) and the whole interior-point
solve (ipm_solve, the reference's own timing target: examples/cartpole_runtime.py:115-152 times
par_interior_point_optimal_control, noc/par_interior_point_newton.py:228-254) -- and each slice's
limiter is named: its heaviest trajectory's serial chain (max_kkt_solves) vs the slots it fills.

Usage (GPU box): python tools/slice_curve.py [--ws 1,2,4,8] [--out gpurun_out/slices.json]
Every bench call is the driver-reproducible command `python bench.py --slice r/W --no-cpu`.
"""
import argparse
import contextlib
import io
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run_bench(argv):
    import bench
    buf = io.StringIO()
    old = sys.argv
    sys.argv = ["bench.py"] + argv
    try:
        with contextlib.redirect_stdout(buf):
            bench.main()
    finally:
        sys.argv = old
    return json.loads(buf.getvalue().strip().splitlines()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ws", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "slices.json"))
    args = ap.parse_args()
    rows, curve = [], {}
    for W in (int(w) for w in args.ws.split(",")):
        per = []
        for r in range(W):
            t0 = time.time()
            line = run_bench(["--slice", f"{r}/{W}", "--no-cpu", "--steps", str(args.steps)])
            ip = line["ipm_solve"]
            row = {"W": W, "r": r, "trajectories": line["config"]["slice_trajectories"],
                   "kkt_kernel_ms": line["roofline"]["kernel_ms"],
                   "kkt_frac": line["roofline"]["frac"],
                   "ipm_wall_ms": ip["wall_ms"], "kkt_solves_computed": ip["kkt_solves_computed"],
                   "max_kkt_solves": ip["max_kkt_solves"],
                   "mean_newton_iters": ip["mean_newton_iters"],
                   "build_hash": line["build_hash"]}
            per.append(row)
            rows.append(row)
            print(json.dumps(row), f"({time.time() - t0:.1f} s)", flush=True)
        curve[W] = {"ipm_wall_ms_max": max(p["ipm_wall_ms"] for p in per),
                    "kkt_kernel_ms_max": max(p["kkt_kernel_ms"] for p in per),
                    "kkt_solves_computed": sum(p["kkt_solves_computed"] for p in per),
                    "heaviest_traj_solves": max(p["max_kkt_solves"] for p in per)}
    if 1 in curve:
        for W, c in curve.items():
            c["ipm_speedup_vs_1"] = curve[1]["ipm_wall_ms_max"] / c["ipm_wall_ms_max"]
            c["kkt_speedup_vs_1"] = curve[1]["kkt_kernel_ms_max"] / c["kkt_kernel_ms_max"]
    out = {"what": "c3 (cart-pole N=200, global batch 4096) split W ways, every slice measured on "
                   "one GPU by `bench.py --slice r/W`; a W-GPU run's time is the max over its "
                   "slices (no data-path collective)", "slices": rows, "curve": curve}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(curve, indent=1))


if __name__ == "__main__":
    main()
