#!/usr/bin/env python3
"""Interleaved A/B of the KKT scan instances on one set of bench blocks (timing; every variant's
results are exact): "lds" = K, d kept on chip (the round-4 instance), "dma" = the LDS-DMA
instance (K, d through the caller's HBM buffers, phase 3 prefetched into LDS by DMA), "kd_hbm" =
the DMA instance with phase 3's plain register loads (ablation bit 7): K, d through HBM only.
Each variant's 10 launches are one HIP graph, replayed ROUNDS times interleaved; prints the median
per-launch time of every variant (us).  Usage: dma_ab.py [problem N B lanes]"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))
import numpy as np
import torch
from noc import lqt, problems, _lib

name, N, B = (sys.argv[1], int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else ("cartpole", 200, 4096)
lanes = int(sys.argv[4]) if len(sys.argv) > 4 else 0
blk = problems.make_bench_blocks(name, N=N, batch=B, seed=7, lanes=lanes)
tb = blk["tiled"]
L = tb.lanes
lib = _lib.load()
f64 = dict(device="cuda", dtype=torch.float64)
base = lqt.kkt_solve_tiled(tb, reg=blk["reg"], want_gains=True)
K, d = base.K, base.d
outs = {"lds": base._replace(K=None, d=None), "dma": base, "kd_hbm": base}
bits = {"lds": 0, "dma": 0, "kd_hbm": 128}
REPS, ROUNDS = 10, 15
graphs, ref = {}, None
side = torch.cuda.Stream()
for k in outs:
    lib.noc_debug_set_ablation(bits[k])
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        lqt.kkt_solve_tiled(tb, reg=blk["reg"], out=outs[k])
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    dx = outs[k].dx.clone()
    if ref is None:
        ref = dx
    assert torch.equal(dx, ref), k  # every variant computes the same step
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(REPS):
            lqt.kkt_solve_tiled(tb, reg=blk["reg"], out=outs[k])
    graphs[k] = g
lib.noc_debug_set_ablation(0)
times = {k: [] for k in graphs}
for _ in range(ROUNDS):
    for k, g in graphs.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) * 1000.0 / REPS)
print(json.dumps({"problem": name, "N": N, "B": B, "lanes": L,
                  "dma_selected": lqt.gains_buffer_pays(tb.nx, tb.nu, N, B, L),
                  "median_us": {k: float(np.median(v)) for k, v in times.items()},
                  "min_us": {k: float(np.min(v)) for k, v in times.items()}}))
