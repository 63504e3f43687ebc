"""Sequential-semantics interior-point solver -- drop-in for noc/seq_interior_point_newton.py.

Same signature as the reference (S:180-202).  The Newton logic is the reference's seq one (one
accept/reject per iteration, Quu += mu*I, stop when |Hu| < 1e-4 AND the backward pass is
feasible); the KKT solve itself runs through the same MI355X scan kernels (it has a unique
solution, so only rounding differs from a sequential Riccati sweep).
"""
from __future__ import annotations

from . import _lib
from .optimal_control_problem import OCP
from .par_interior_point_newton import _run


def seq_interior_point_optimal_control(ocp: OCP, controls, initial_state, lanes: int = 0,
                                       device="cuda", return_info=False):
    return _run(ocp, controls, initial_state, _lib.MODE_SEQ, "final_cost", lanes, device,
                return_info)
