#!/usr/bin/env python3
"""Attribute KKT-scan kernel time to phases by ablation (timing only; results are wrong while an
ablation bit 0-2 is set).  Interleaved rounds in one process.  Each variant's 10 launches are
captured in one HIP graph and replayed, so the time is the GPU's (kernels + boundaries), not the
Python/ctypes launch path's."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))
import torch
from noc import lqt, problems, _lib

name, N, B = (sys.argv[1], int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else ("cartpole", 200, 4096)
lanes = int(sys.argv[4]) if len(sys.argv) > 4 else 64
blk = problems.make_bench_blocks(name, N=N, batch=B, seed=7, lanes=lanes)
tb = blk["tiled"]
lib = _lib.load()
out = lqt.kkt_solve_tiled(tb, reg=blk["reg"], want_gains=(lanes == 1))
variants = {"full": 0, "streamed": 8, "no_fwd": 2, "no_scan": 1, "no_scan_no_fwd": 3,
            "phase1_only": 5, "phase1+2": 4, "hot_rereads": 16}
if os.environ.get("ABLATE_VARIANTS"):  # e.g. '{"full": 0, "prio_mem": 128}'
    variants = json.loads(os.environ["ABLATE_VARIANTS"])
elif lanes == 1:  # the group solve (kkt_group8_impl.h): backward sweep / forward sweep split
    variants = {"full": 0, "no_fwd": 2, "fwd_only": 64}
REPS = 10
graphs = {}
side = torch.cuda.Stream()
for k, bits in variants.items():   # the ablation bits are read at launch, i.e. at capture
    lib.noc_debug_set_ablation(bits)
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        lqt.kkt_solve_tiled(tb, reg=blk["reg"], out=out)   # warm-up outside the capture
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(REPS):
            lqt.kkt_solve_tiled(tb, reg=blk["reg"], out=out)
    graphs[k] = g
lib.noc_debug_set_ablation(0)
torch.cuda.synchronize()
times = {k: [] for k in variants}
for _ in range(5):
    for k, g in graphs.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record(); torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) / REPS)
print(json.dumps({"problem": name, "N": N, "B": B, "lanes": lanes, "unit": "ms per launch (graph)",
                  **{k: sorted(v)[2] for k, v in times.items()}}))
