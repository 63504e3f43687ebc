#!/usr/bin/env python3
"""Per-phase cycle breakdown of the persistent solver for one trajectory (B = 1) -- needs the
library built with -DNOC_PERSIST_PROFILE (load it via NOC_HIP_LIB).  One JSON line per config."""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))
import numpy as np, torch
from noc import problems, _lib
from noc.ipm import BatchedIPM
lib = _lib.load()
names = ["rollout", "linearize", "costate_blocks", "kkt", "trial", "iterations"]
# round 6 sub-phases (slots 6-14): the trial's costs + reductions, the costate cross-lane scan, the
# KKT scan's phases (kkt_scan_impl.h: NOC_STAMP 1-6)
subs = {6: "trial_costs", 7: "costate_scan", 9: "kkt_elements", 10: "kkt_cross_lane",
        11: "kkt_riccati", 12: "kkt_fwd_scan", 13: "kkt_propagate", 14: "kkt_copy_out"}
# one-wave kernel throughout (B = 1 would run the wide kernel); both block layouts (round 6:
# NOC_PERSIST_STRUCT=1 structure-aware compact blocks, 0 dense)
os.environ["NOC_PERSIST_WIDE"] = "0"
os.environ["NOC_PERSIST_SPEC"] = "1"  # one wave per trajectory (no speculative candidates)
CONFIGS = [("pendulum", 50, 1), ("cartpole", 200, 1), ("cartpole", 200, 512), ("cartpole", 200, 4096)]
for name, N, B, struct in [c + (s,) for c in CONFIGS for s in ("1", "0")]:
    os.environ["NOC_PERSIST_STRUCT"] = struct
    ocp = problems.make_problem(name, N)
    x0, u0 = problems.initial_conditions(name, N, B, seed=11)
    eng = BatchedIPM(ocp.family, N, B, persistent=True)
    eng.load(u0, x0); eng.solve(); torch.cuda.synchronize()
    buf = (ctypes.c_longlong * 16)()
    lib.noc_debug_phase_cycles(buf, 16, 1)
    eng.load(u0, x0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); eng.solve(); e1.record(); torch.cuda.synchronize()
    lib.noc_debug_phase_cycles(buf, 16, 1)
    c = {k: int(buf[i]) for i, k in enumerate(names)}
    c.update({k: int(buf[i]) for i, k in subs.items()})
    its = max(c["iterations"], 1)
    print(json.dumps({"problem": name, "N": N, "B": B, "struct": struct, "ms": e0.elapsed_time(e1),
                      "cycles_per_iteration": {k: c[k] / its for k in names[:5] + list(subs.values())}, "totals": c}), flush=True)
