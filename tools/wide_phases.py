#!/usr/bin/env python3
"""Per-phase cycle breakdown of the wide persistent solver (ipm_wide.hip, W waves per trajectory)
beside the one-wave kernel, for one trajectory's workgroup -- needs the library built with
-DNOC_PERSIST_PROFILE (load it via NOC_HIP_LIB).  One JSON line per config; cycles per Newton
iteration of workgroup 0, wave 0 lane 0."""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))
import torch
from noc import problems, _lib
from noc.ipm import BatchedIPM
lib = _lib.load()
names = ["rollout", "linearize", "costate_blocks", "kkt", "trial", "iterations"]
# ipm_wide.hip NOC_WSUB 0-6 (slots 8-14)
wide_subs = {8: "kkt_elements", 9: "kkt_in_wave_scan", 10: "kkt_wave_join", 11: "kkt_riccati",
             12: "kkt_pred_reduce", 13: "kkt_fwd_scan", 14: "kkt_propagate"}
one_subs = {6: "trial_costs", 7: "costate_scan", 9: "kkt_elements", 10: "kkt_cross_lane",
            11: "kkt_riccati", 12: "kkt_fwd_scan", 13: "kkt_propagate", 14: "kkt_copy_out"}
CONFIGS = [("cartpole", 200, 1), ("cartpole", 200, 512)]
for name, N, B in CONFIGS:
    for wide, waves in (("0", "-"), ("1", "2"), ("1", "4")):
        if wide == "1" and B > 256 and waves == "4":
            continue
        os.environ["NOC_PERSIST_WIDE"] = wide
        os.environ["NOC_WIDE_WAVES"] = "2" if waves == "-" else waves
        os.environ["NOC_PERSIST_SPEC"] = "1"
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
        subs = wide_subs if wide == "1" else one_subs
        c.update({k: int(buf[i]) for i, k in subs.items()})
        its = max(c["iterations"], 1)
        print(json.dumps({"problem": name, "N": N, "B": B, "wide": wide, "waves": waves,
                          "ms": e0.elapsed_time(e1),
                          "cycles_per_iteration": {k: round(c[k] / its) for k in names[:5] + list(subs.values())},
                          "totals": c}), flush=True)
