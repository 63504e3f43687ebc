#!/usr/bin/env python3
"""B = 1 latency probe of the whole-solve kernels: the wide (4 waves / trajectory, ipm_wide.hip)
against the one-wave kernel (NOC_PERSIST_WIDE=0|1 per call), per problem / horizon:
  * kernel_ms: HIP events around eng.solve() (the one launch),
  * call_ms: the whole par_interior_point_optimal_control call (host staging included),
  * with the -DNOC_PERSIST_PROFILE library (NOC_HIP_LIB=.../libnoc_hip_prof.so) also the cycles
    per Newton iteration of each phase (workgroup 0).
One JSON line per (problem, N, kernel)."""
import ctypes, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))
import numpy as np, torch
from noc import problems, _lib
from noc.ipm import BatchedIPM
from noc.par_interior_point_newton import par_interior_point_optimal_control

lib = _lib.load()
prof = "prof" in os.environ.get("NOC_HIP_LIB", "")
names = ["rollout", "linearize", "costate_blocks", "kkt", "trial", "iterations"]
sub = ["prepend", "wave_scan", "join", "riccati", "pred_reduce", "fwd_scan", "propagate"]
configs = [("pendulum", 20), ("pendulum", 50), ("pendulum", 100), ("cartpole", 20),
           ("cartpole", 50), ("cartpole", 100), ("cartpole", 200)]
if len(sys.argv) > 1:
    configs = [(a.split(":")[0], int(a.split(":")[1])) for a in sys.argv[1:]]
for name, N in configs:
    ocp = problems.make_problem(name, N)
    x0, u0 = problems.initial_conditions(name, N, 1, seed=11)
    for wide in ("1", "0"):
        os.environ["NOC_PERSIST_WIDE"] = wide
        eng = BatchedIPM(ocp.family, N, 1, persistent=True)
        eng.load(u0, x0); eng.solve(); torch.cuda.synchronize()
        buf = (ctypes.c_longlong * 16)()
        if prof:
            lib.noc_debug_phase_cycles(buf, 16, 1)
        ks = []
        for _ in range(5):
            eng.load(u0, x0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); eng.solve(); e1.record(); torch.cuda.synchronize()
            ks.append(e0.elapsed_time(e1))
        solves = int(eng.t["kkt_solves"][0].item())
        out = {"problem": name, "N": N, "kernel": "wide" if wide == "1" else "one_wave",
               "kernel_ms": float(np.median(ks)), "kkt_solves": solves,
               "us_per_solve": 1e3 * float(np.median(ks)) / max(solves, 1)}
        if prof:
            lib.noc_debug_phase_cycles(buf, 16, 1)
            c = {k: int(buf[i]) for i, k in enumerate(names)}
            its = max(c["iterations"] / 5, 1)
            out["cycles_per_solve"] = {k: round(c[k] / 5 / its) for k in names[:5]}
            if wide == "1":
                out["kkt_sub"] = {k: round(int(buf[8 + i]) / 5 / its) for i, k in enumerate(sub)}
        else:
            par_interior_point_optimal_control(ocp, u0[0], x0[0])
            cs = []
            for _ in range(5):
                torch.cuda.synchronize(); t0 = time.perf_counter()
                par_interior_point_optimal_control(ocp, u0[0], x0[0])
                torch.cuda.synchronize(); cs.append(time.perf_counter() - t0)
            out["call_ms"] = 1e3 * float(np.median(cs))
        print(json.dumps(out), flush=True)
os.environ.pop("NOC_PERSIST_WIDE", None)
