"""Sequential-semantics interior-point solver -- drop-in for noc/seq_interior_point_newton.py.

Same public functions and signatures as the reference (S:10-202).  The Newton logic is the
reference's seq one (one accept/reject per iteration, Quu += mu*I, stop when |Hu| < 1e-4 AND the
backward pass is feasible); the KKT solve itself runs through the same MI355X kernels (it has a
unique solution, so only rounding differs from a sequential Riccati sweep).
"""
from __future__ import annotations

import torch

from . import _lib
from .costates import final_cost_grad, seq_costates
from .optimal_control_problem import OCP, Derivatives, LinearizedOCP
from .par_interior_point_newton import (_dev, _run, check_traj_feasibility, compute_derivatives,
                                        compute_lqr_params)

__all__ = ["compute_derivatives", "compute_lqr_params", "bwd_pass", "fwd_pass",
           "check_feasibility", "seq_solution", "newton_oc", "seq_interior_point_optimal_control"]


def _terminal_hessian(final_cost, xN):
    """hessian(final_cost)(xN) (S:66): final_cost is the OCP's callable (carrying its family),
    the OCP itself, or the Hessian array."""
    fam = getattr(final_cost, "family", None)
    if fam is not None:
        class _O:  # noqa: N801 -- the family-bearing stand-in final_cost_grad expects
            family = fam
        return final_cost_grad(_O, xN, hessian=True)[1]
    return _dev(final_cost, "final_cost Hessian")


def bwd_pass(final_cost, xN, lqr: LinearizedOCP, d: Derivatives, rp):
    """S:42-75 -> (gain K (N,nu,nx), ff_gain k (N,nu), dV, feasible); Quu += rp*I."""
    from . import lqt
    P = _terminal_hessian(final_cost, xN)
    r, Q, R, M = (_dev(t) for t in lqr)
    fx, fu = _dev(d.fx), _dev(d.fu)
    single = Q.dim() == 3
    if single:
        r, Q, R, M, fx, fu, P = (t[None] for t in (r, Q, R, M, fx, fu, P))
    reg = torch.as_tensor(rp, dtype=torch.float64, device=Q.device).reshape(-1).expand(Q.shape[0])
    K, k, _, _, dV, feas = lqt.bwd_pass(fx, fu, Q, R, M, r, P.contiguous(), reg=reg.contiguous())
    res = (K, k, dV, feas.bool())
    return tuple(t[0] for t in res) if single else res


def fwd_pass(gain, ff_gain, d: Derivatives):
    """S:78-90: dx_0 = 0, dx_{k+1} = (fx + fu K) dx_k + fu k -> (du, dx)."""
    from . import lqt
    return lqt.fwd_pass(_dev(d.fx), _dev(d.fu), _dev(gain), _dev(ff_gain))


def check_feasibility(ocp: OCP, x, u):
    """S:93-95."""
    return check_traj_feasibility(ocp, x, u)


def seq_solution(ocp: OCP, x, u, bp, rp):
    """S:98-105 -> (dx, du, dV, bp_feasible, ru)."""
    x = _dev(x, "x")
    d = compute_derivatives(ocp, x, u, bp)
    lam = seq_costates(ocp, x[..., -1, :], d)
    ru, Q, R, M = compute_lqr_params(lam, d)
    K, k, dV, feas = bwd_pass(ocp.final_cost, x[..., -1, :], LinearizedOCP(ru, Q, R, M), d, rp)
    du, dx = fwd_pass(K, k, d)
    return dx, du, dV, feas, ru


def newton_oc(ocp: OCP, controls, initial_state, bp):
    """S:108-177: ONE barrier stage of the seq Newton loop -> (states, controls, iterations)."""
    return _run(ocp, controls, initial_state, _lib.MODE_SEQ, "final_cost", one_stage_bp=bp)


def seq_interior_point_optimal_control(ocp: OCP, controls, initial_state, lanes: int = 0,
                                       device="cuda", return_info=False):
    """S:180-202: barrier 0.1 / 5^k while > 1e-4 -> (u*, iterations)."""
    return _run(ocp, controls, initial_state, _lib.MODE_SEQ, "final_cost", lanes, device,
                return_info)
