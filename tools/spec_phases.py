#!/usr/bin/env python3
"""Phase cycles of trajectory 0's whole persistent solve with 1, 2 and 4 speculative candidates
(the profile build, -DNOC_PERSIST_PROFILE, via NOC_HIP_LIB): where a round of candidates spends
its time against one solve.  Slots as tools/persist_phases.py; the KKT sub-phase stamps count every
wave's lane 0 (SPEC times).  One JSON line per (B, SPEC)."""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))
import torch
from noc import problems, _lib
from noc.ipm import BatchedIPM
lib = _lib.load()
names = ["rollout", "linearize", "costate_blocks", "kkt", "trial", "solves_processed", "trial_costs",
         "costate_scan"]
os.environ["NOC_PERSIST_WIDE"] = "0"
for B in (1, 512):
    for spec in ("1", "2", "4"):
        if B * int(spec) > 4 * torch.cuda.get_device_properties(0).multi_processor_count:
            continue
        os.environ["NOC_PERSIST_SPEC"] = spec
        ocp = problems.make_problem("cartpole", 200)
        x0, u0 = problems.initial_conditions("cartpole", 200, B, seed=11)
        eng = BatchedIPM(ocp.family, 200, B, persistent=True)
        eng.load(u0, x0); eng.solve_persistent(); torch.cuda.synchronize()
        buf = (ctypes.c_longlong * 16)()
        lib.noc_debug_phase_cycles(buf, 16, 1)
        eng.load(u0, x0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); eng.solve_persistent(); e1.record(); torch.cuda.synchronize()
        lib.noc_debug_phase_cycles(buf, 16, 1)
        c = {k: int(buf[i]) for i, k in enumerate(names)}
        solves = int(eng.t["kkt_solves"][0].item())
        print(json.dumps({"B": B, "spec": spec, "ms": e0.elapsed_time(e1), "traj0_solves": solves,
                          "traj0_total_cycles": sum(c[k] for k in names[:5]), "totals": c}), flush=True)
