#!/usr/bin/env python3
"""Root cause of the +-1 iteration tolerance of tests/test_ddp.py (cart-pole N=25): run the oracle
interior-point DDP (oracle/noc_oracle.py, D:98-208) twice -- with its own torch.func derivatives
and with the DEVICE-evaluated derivatives (noc.par_interior_point_newton.compute_derivatives:
the generated family code the DDP kernel uses) -- and compare both traces with each other and the
iteration / pass counts with the GPU DDP.  Prints the first diverging decision (accept / stop)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ip-parallel-optimal-control_amd"), ROOT]
import numpy as np
import torch
from noc import problems
from noc.differential_dynamic_programming import interior_point_ddp
from noc.par_interior_point_newton import compute_derivatives
from noc.costates import final_cost_grad
from oracle import noc_oracle as O, problems as PR


class DeviceDerivs(O.NumpyProblem):
    """The oracle problem with derivatives / terminal gradient from the device kernels."""
    def __init__(self, tocp, ocp):
        super().__init__(tocp)
        self.ocp = ocp

    def derivatives(self, X, U, bp):
        d = compute_derivatives(self.ocp, X, U, bp)
        return tuple(t.cpu().numpy() for t in d)

    def final_grad_hess(self, xN):
        g, h = final_cost_grad(self.ocp, xN, hessian=True)
        return g.cpu().numpy(), h.cpu().numpy()


def run(prob, u0, x0):
    bp, total, passes, trace = 0.1, 0, 0, []
    U = u0
    while bp > 1e-4:
        tr = []
        X, U, it, p = O.ddp(prob, U, x0, bp, trace=tr)
        trace += [dict(bp=bp, **t) for t in tr]
        bp /= 5
        total += it
        passes += p
    return U, total, passes, trace


def main():
    N, Bt = 25, 2
    rng = np.random.default_rng(7 + N)
    u0 = 0.1 * rng.normal(size=(Bt, N, 1))
    x0 = np.array([0.01, -0.01, 0.01, -0.01]) + 0.01 * rng.normal(size=(Bt, 4))
    ocp = problems.make_problem("cartpole", N)
    import ctypes
    from noc import _lib
    lib = _lib.load()
    fn = lib.noc_debug_set_ddp_trace
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    CAP = 4096
    tbuf = torch.zeros(Bt, CAP, 10, dtype=torch.float64, device="cuda")
    assert fn(tbuf.data_ptr(), CAP, Bt) == 0
    Ug, itg, info = interior_point_ddp(ocp, u0, x0, return_info=True)
    torch.cuda.synchronize()
    assert fn(None, 0, 0) == 0
    gtrace = tbuf.cpu().numpy()
    out = []
    for b in range(Bt):
        Ua, ita, pa, ta = run(O.NumpyProblem(PR.cartpole_ocp(1.0 / N)), u0[b], x0[b])
        Ud, itd, pd, td = run(DeviceDerivs(PR.cartpole_ocp(1.0 / N), ocp), u0[b], x0[b])
        first = None
        for i, (a, d) in enumerate(zip(ta, td)):
            if a["success"] != d["success"] or a["it"] != d["it"] or a["bp"] != d["bp"]:
                first = dict(index=i, autodiff=a, device_derivs=d)
                break
        # GPU trace vs the oracle's, pass by pass: the first pass whose decision differs, and
        # the passes around the end of every barrier stage (where |Hu| meets 1e-4)
        keys = ["bp", "it", "inner", "pred", "gain", "success", "rp", "hu", "cost", "new_cost"]
        g = [dict(zip(keys, row)) for row in gtrace[b][: int(info["passes"][b])]]
        first_gpu = None
        for i, (a, gg) in enumerate(zip(ta, g)):
            if bool(a["success"]) != bool(gg["success"]) or a["it"] != gg["it"] or a["bp"] != gg["bp"]:
                first_gpu = dict(index=i, oracle=a, gpu=gg,
                                 oracle_prev=ta[i - 1] if i else None, gpu_prev=g[i - 1] if i else None)
                break
        ends = [i for i in range(len(g) - 1) if g[i + 1]["bp"] != g[i]["bp"]] + [len(g) - 1]
        stage_ends = [dict(pass_index=i, gpu_hu=g[i]["hu"], gpu_it=g[i]["it"], bp=g[i]["bp"]) for i in ends]
        side = [dict(i=i, o_pred=a["pred"], g_pred=gg["pred"], o_gain=a["gain"], g_gain=gg["gain"],
                     o_rp=a["rp"], g_rp=gg["rp"], o_ok=bool(a["success"]), g_ok=bool(gg["success"]),
                     g_hu=gg["hu"]) for i, (a, gg) in enumerate(zip(ta, g))]
        out.append(dict(trajectory=b, gpu=dict(iterations=int(itg[b]), passes=int(info["passes"][b])),
                        oracle_autodiff=dict(iterations=ita, passes=pa),
                        oracle_device_derivatives=dict(iterations=itd, passes=pd),
                        first_divergence=first,
                        first_gpu_vs_oracle_divergence=first_gpu,
                        gpu_stage_ends=stage_ends, side_by_side=side,
                        max_abs_dU_gpu_vs_devderiv=float(np.max(np.abs(Ug[b] - Ud))),
                        max_abs_dU_gpu_vs_autodiff=float(np.max(np.abs(Ug[b] - Ua)))))
    print(json.dumps(out, indent=1, default=float))


if __name__ == "__main__":
    main()
