#!/usr/bin/env python3
"""Per-phase timing of the KKT scan kernel under full load, from the phase-stamp build
(`make -C ip-parallel-optimal-control_amd stamps-lib`, loaded through NOC_HIP_LIB).  Lane 0 of
every wave stamps s_memrealtime / s_memtime at the phase boundaries (kkt_scan_impl.h NOC_STAMP);
this prints, over the waves of one launch, the median / p10 / p90 start time of each phase
relative to the earliest wave start (us, 100 MHz realtime) and the median per-wave phase
durations in shader cycles.  Diagnostic only (the stamps themselves cost a little)."""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("NOC_HIP_LIB", os.path.join(ROOT, "ip-parallel-optimal-control_amd", "noc",
                                                  "_lib", "libnoc_hip_stamps.so"))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))
import numpy as np
import torch
from noc import lqt, problems, _lib

name, N, B = (sys.argv[1], int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else ("cartpole", 200, 4096)
lanes = int(sys.argv[4]) if len(sys.argv) > 4 else 0
blk = problems.make_bench_blocks(name, N=N, batch=B, seed=7, lanes=lanes)
tb = blk["tiled"]
lib = _lib.load()
fn = lib.noc_debug_scan_stamps
fn.restype, fn.argtypes = ctypes.c_int, [ctypes.POINTER(ctypes.c_longlong), ctypes.c_int, ctypes.c_int]
out = lqt.kkt_solve_tiled(tb, reg=blk["reg"], want_gains=False)
waves = (B * tb.lanes + 63) // 64
buf = (ctypes.c_longlong * (waves * 16))()
names = ["start", "phase1", "phase2", "phase3", "fwdscan", "propagate", "copyout"]
res = []
for rep in range(5):
    torch.cuda.synchronize()
    assert fn(buf, waves, 1) == 0
    lqt.kkt_solve_tiled(tb, reg=blk["reg"], out=out)
    torch.cuda.synchronize()
    assert fn(buf, waves, 0) == 0
    st = np.frombuffer(buf, dtype=np.int64).reshape(waves, 8, 2)
    rt = (st[:, :7, 0] - st[:, 0, 0].min()) / 100.0    # us
    cyc = np.diff(st[:, :7, 1], axis=1)
    res.append({"kernel_span_us": float(rt[:, 6].max()),
                "start_us": {n: [float(np.percentile(rt[:, i], q)) for q in (10, 50, 90)]
                             for i, n in enumerate(names)},
                "phase_cycles_median": {names[i + 1]: float(np.median(cyc[:, i])) for i in range(6)}})
print(json.dumps({"problem": name, "N": N, "B": B, "lanes": tb.lanes, "runs": res[1:]}, indent=1))
