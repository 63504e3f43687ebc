"""Interior-point DDP -- drop-in for noc/differential_dynamic_programming.py (the reference's third
solver, "D").

`interior_point_ddp(ocp, controls, initial_state) -> (controls*, iterations)` keeps the
reference signature (D:189-208).  The whole barrier schedule runs on the MI355X in one launch
(`noc_ddp_solve`, one wave per trajectory: DDP's backward pass carries the Vx . fxx terms of its
own value gradient, so the recursion is horizon-sequential, not a scan; the stage derivatives are
evaluated lane-parallel).  Differences, all additive:
  * inputs may carry a leading batch axis (controls (B, N, nu), initial_state (B, nx)); the
    result is then batched too -- each trajectory follows its own reference control flow;
  * `ocp.family` must be a registered family with nx <= 4 (noc.problems);
  * return_info=True adds the backward-pass counts (incl. rejected retries) and final states.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .optimal_control_problem import OCP


def interior_point_ddp(ocp: OCP, controls, initial_state, device="cuda", bp0: float = 0.1,
                       max_passes: int = 10 ** 7, return_info: bool = False):
    """D:189-208: barrier 0.1 / 5^k while > 1e-4, ddp (D:98-186) at each barrier value."""
    import torch
    if ocp.family is None:
        raise _lib.NocError("OCP has no registered device family (use noc.problems.*): the HIP "
                            "kernels cannot evaluate Python callables")
    lib = _lib.load_for(ocp.family)
    fam = ocp.family.to_c()
    if not lib.noc_ddp_supported(ctypes.byref(fam)):
        raise _lib.NocError("interior-point DDP supports the registered families with nx <= 4")
    u = np.asarray(controls, dtype=np.float64)
    x0 = np.asarray(initial_state, dtype=np.float64)
    single = u.ndim == 2
    if single:
        u, x0 = u[None], x0[None]
    Bt, N, nu = u.shape
    nx = x0.shape[-1]
    dev = torch.device(device)
    if dev.type != "cuda":
        raise _lib.NocError("the MI355X path has no CPU fallback")
    f64 = dict(device=dev, dtype=torch.float64)
    U = torch.as_tensor(np.ascontiguousarray(u), **f64)
    X0 = torch.as_tensor(np.ascontiguousarray(x0), **f64)
    work = torch.empty(int(lib.noc_ddp_work_doubles(nx, nu, N, Bt)), **f64)
    i32 = dict(device=dev, dtype=torch.int32)
    its, passes, done = (torch.zeros(Bt, **i32) for _ in range(3))
    _lib.check(lib.noc_ddp_solve(ctypes.byref(fam), N, Bt, _lib.ptr(X0), _lib.ptr(U),
                                 _lib.ptr(work), _lib.ptr(its), _lib.ptr(passes), _lib.ptr(done),
                                 float(bp0), int(max_passes), _lib.stream_handle(dev)),
               "noc_ddp_solve", lib)
    Uh, itn = U.cpu().numpy(), its.cpu().numpy()
    info = dict(passes=passes.cpu().numpy(), done=done.cpu().numpy().astype(bool),
                states=work[:Bt * (N + 1) * nx].view(Bt, N + 1, nx).cpu().numpy())
    if single:
        Uh, itn = Uh[0], int(itn[0])
        info = {k: v[0] for k, v in info.items()}
    if return_info:
        return Uh, itn, info
    return Uh, itn
