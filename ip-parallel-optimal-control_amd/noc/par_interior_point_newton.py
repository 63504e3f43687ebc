"""Parallel-in-time interior-point solver -- drop-in for noc/par_interior_point_newton.py.

`par_interior_point_optimal_control(ocp, controls, initial_state) -> (controls*, iterations)`
keeps the reference signature (P:228-254).  Differences, all additive:
  * inputs may carry a leading batch axis (controls (B, N, nu), initial_state (B, nx)); the
    result is then batched too -- each trajectory follows its own reference control flow;
  * the whole loop runs on the MI355X (libnoc_hip.so); `ocp.family` must be a registered family
    (noc.problems) because device code cannot call Python callables;
  * `terminal`: "stage0" (default: the reference par path's terminal Hessian XT = Q[0], P:73 --
    what par_Newton actually feeds its LQT) or "final_cost" (hessian(final_cost), the reference
    seq path S:66).  The default reproduces the reference par loop's iteration counts (e.g.
    cart-pole N=50: 88 outer / 129 KKT solves; with "final_cost": 91 / 135).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .ipm import BatchedIPM
from .optimal_control_problem import OCP

_TERMINAL = {"final_cost": _lib.TERMINAL_FINAL_COST, "stage0": _lib.TERMINAL_STAGE0}


def _run(ocp: OCP, controls, initial_state, mode, terminal="stage0", lanes=0,
         device="cuda", return_info=False):
    if ocp.family is None:
        raise _lib.NocError("OCP has no registered device family (use noc.problems.*): the HIP "
                            "kernels cannot evaluate Python callables")
    u = np.asarray(controls, dtype=np.float64)
    x0 = np.asarray(initial_state, dtype=np.float64)
    single = u.ndim == 2
    if single:
        u, x0 = u[None], x0[None]
    Bt, N, _ = u.shape
    from .ipm import persistent_supported
    # whole solve in one launch when the family / horizon allows it (same results, lanes 64)
    persistent = lanes in (0, 64) and persistent_supported(ocp.family, N)
    eng = BatchedIPM(ocp.family, N, Bt, device=device, lanes=lanes, persistent=persistent)
    eng.load(u, x0)
    steps = eng.solve(mode=mode, terminal=_TERMINAL[terminal])
    U, iters, solves = eng.result()
    U, iters, solves = U.cpu().numpy(), iters.cpu().numpy(), solves.cpu().numpy()
    if single:
        U, iters, solves = U[0], int(iters[0]), int(solves[0])
    if return_info:
        return U, iters, dict(kkt_solves=solves, device_steps=steps)
    return U, iters


def par_interior_point_optimal_control(ocp: OCP, controls, initial_state, terminal="stage0",
                                       lanes: int = 0, device="cuda", return_info=False):
    """P:228-254: barrier 0.1 / 5^k while > 1e-4; Newton with retry loop; returns (u*, iters)."""
    return _run(ocp, controls, initial_state, _lib.MODE_PAR, terminal, lanes, device, return_info)
