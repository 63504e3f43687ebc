#!/usr/bin/env python3
"""Time the lanes=1 group solve split into its backward (par_bwd_pass) and forward
(par_fwd_pass) launches on the c4 blocks, HIP events on the launch stream.  One JSON line."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))
import torch
from noc import lqt, problems

name, N, B = (sys.argv[1], int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else ("linear8", 512, 16384)
blk = problems.make_bench_blocks(name, N=N, batch=B, seed=7, lanes=16, natural=True)
nat = [blk[k] for k in ("A", "B", "Q", "R", "M", "r", "P")]
reg = blk["reg"]
K, d, S, v, pred, feas = lqt.bwd_pass(*nat, reg=reg, lanes=1)
out = lqt.kkt_solve(*nat, reg=reg, lanes=1)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


res = {"problem": name, "N": N, "B": B,
       "full_ms": timed(lambda: lqt.kkt_solve(*nat, reg=reg, lanes=1, out=out)),
       "bwd_ms": timed(lambda: lqt.bwd_pass(*nat, reg=reg, lanes=1)),
       "fwd_ms": timed(lambda: lqt.fwd_pass(nat[0], nat[1], K, d, lanes=1))}
print(json.dumps(res), flush=True)
