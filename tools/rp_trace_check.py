"""Every accepted step's regularisation update, checked bit for bit against the reference's
rounding (decision-trace build: NOC_HIP_LIB=ip-parallel-optimal-control_amd/noc/_lib/
libnoc_hip_trace.so).

P:167-173 (S:139-143 for seq's mu): after an accepted trial rp <- clip(rp * max(1/3,
1 - (2 gain - 1) ** 3)).  In JAX `x ** 3` is lax.integer_pow, x * (x * x) -- two roundings -- and
the subtraction rounds once more (oracle/noc_oracle.py: _cube).  A fused multiply-subtract rounds
once, so it differs in the last bit at some gains; the kernels compute the factor without
contraction (noc_internal.h: rp_shrink).  For each kernel (one-wave, wide) and mode this prints
how many accepted updates were checked, how many differ from the two-rounding formula (must be
0) and at how many a fused evaluation would have differed (the check's power).  One JSON line.
"""
import ctypes
import json
import os
import sys
from fractions import Fraction

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))

FIELDS = ["bp", "it", "inner", "cost", "new_cost", "pred", "gain", "success", "rp", "rinc", "hu",
          "bwd_ok"]


def shrink_two_roundings(g):
    c = 2.0 * g - 1.0
    return max(1.0 / 3.0, 1.0 - c * (c * c))


def shrink_fused(g):
    c = 2.0 * g - 1.0
    t = c * c
    return max(1.0 / 3.0, float(Fraction(1) - Fraction(t) * Fraction(c)))  # one rounding


def check(trace, par):
    n = bad = power = 0
    for rec in trace:  # (cap, fields) of one trajectory, NaN past its last solve
        for i in range(len(rec) - 1):
            a, b = rec[i], rec[i + 1]
            if np.isnan(b[0]) or a[7] != 1.0 or a[0] != b[0]:
                continue  # not an accepted step followed by a solve of the same barrier stage
            g, rp = a[6], a[8]
            want = rp * shrink_two_roundings(g)
            fused = rp * shrink_fused(g)
            if par:
                want, fused = min(max(want, 1e-16), 1e16), min(max(fused, 1e-16), 1e16)
            n += 1
            bad += int(b[8] != want)
            power += int(fused != want)
    return n, bad, power


def main():
    import torch
    from noc import problems, _lib
    from noc.ipm import BatchedIPM
    lib = _lib.load()
    fn = lib.noc_debug_set_decision_trace
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    out = {}
    for name, N, Bt in (("pendulum", 60, 64), ("cartpole", 100, 32)):
        ocp = problems.make_problem(name, N)
        x0, u0 = problems.initial_conditions(name, N, Bt, seed=8)
        for mode in ("par", "seq"):
            for wide in ("0", "1"):
                os.environ["NOC_PERSIST_WIDE"] = wide
                cap = 2048
                buf = torch.full((Bt, cap, len(FIELDS)), float("nan"), dtype=torch.float64,
                                 device="cuda")
                if fn(buf.data_ptr(), cap, Bt) != 1:
                    raise SystemExit("no decision trace in this library: NOC_HIP_LIB must be "
                                     "noc/_lib/libnoc_hip_trace.so")
                eng = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=True)
                eng.load(u0, x0)
                eng.ws.flags = _lib.WS_NO_REPEAT_SKIP  # one record per solve
                eng.solve(mode=_lib.MODE_PAR if mode == "par" else _lib.MODE_SEQ)
                torch.cuda.synchronize()
                fn(None, 0, 0)
                n, bad, power = check(buf.cpu().numpy(), mode == "par")
                out[f"{name}_{mode}_{'wide' if wide == '1' else 'one_wave'}"] = dict(
                    checked=n, mismatched=bad, fused_would_differ=power)
    os.environ.pop("NOC_PERSIST_WIDE", None)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
