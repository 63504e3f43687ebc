"""Interior-point DDP -- drop-in for noc/differential_dynamic_programming.py (the reference's third
solver, "D").

`interior_point_ddp(ocp, controls, initial_state) -> (controls*, iterations)` keeps the
reference signature (D:189-208).  The whole barrier schedule runs on the MI355X in one launch
(`noc_ddp_solve`, one wave per trajectory: DDP's backward pass carries the Vx . fxx terms of its
own value gradient, so the recursion is horizon-sequential, not a scan; the stage derivatives are
evaluated lane-parallel).  Differences, all additive:
  * inputs may carry a leading batch axis (controls (B, N, nu), initial_state (B, nx)); the
    result is then batched too -- each trajectory follows its own reference control flow;
  * `ocp.family` must be a registered family (noc.problems, noc.families); nx <= 4 runs the
    one-launch kernel, larger states (nx = 8: the linear double-integrator stack) the same control
    flow as a host loop over the device building blocks below (`_solve_blocks`);
  * return_info=True adds the backward-pass counts (incl. rejected retries) and final states.

The module's building blocks keep the reference names too (D:10-186): compute_derivatives (the
same jax.grad / hessian / jacrev arrays as the Newton solvers', noc_derivatives), bwd_pass (the
second-order backward pass, noc_ddp_bwd_pass), nonlin_rollout (noc_nonlin_rollout),
check_feasibility (noc_check_feasibility) and ddp (one barrier value, noc_ddp_solve_ex with
NOC_DDP_ONE_STAGE).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .optimal_control_problem import OCP, Derivatives
from .par_interior_point_newton import (_dev, _expect_shapes, _family, _shape,
                                        check_traj_feasibility, compute_derivatives,
                                        nonlin_rollout, total_cost)

__all__ = ["compute_derivatives", "bwd_pass", "nonlin_rollout", "check_feasibility", "ddp",
           "interior_point_ddp"]


def check_feasibility(ocp: OCP, x, u):
    """D:93-95 (== P:45-47)."""
    return check_traj_feasibility(ocp, x, u)


def bwd_pass(final_cost, final_state, d: Derivatives, reg_param):
    """D:28-70: the DDP backward pass -> (ffgain k (N, nu), gain K (N, nu, nx), pred_reduction,
    feasible_bwd_pass, Hu (N, nu)).  Vx, Vxx at x_N are grad / hessian of `final_cost` (the OCP's
    callable, carrying its family, or the OCP itself); reg = reg_param * ||cu||_F.  Batched inputs
    (leading B axis) give batched outputs."""
    import torch
    from .costates import final_cost_grad
    fam = getattr(final_cost, "family", None)
    if fam is None:
        raise _lib.NocError("bwd_pass: final_cost must be a registered family's callable (or its "
                            "OCP): grad / hessian come from the device code")

    class _O:  # noqa: N801 -- the family-bearing stand-in final_cost_grad expects
        family = fam
    cus = _shape(d.cu)
    single = len(cus) == 2
    if len(cus) not in (2, 3):
        raise _lib.NocError(f"bwd_pass: d.cu must be (N, nu) or (B, N, nu); got {cus}")
    B, N = (1, cus[0]) if single else (cus[0], cus[1])
    nx, nu = fam.nx, fam.nu
    fields = dict(cx=(nx,), cu=(nu,), cxx=(nx, nx), cuu=(nu, nu), cxu=(nx, nu), fx=(nx, nx),
                  fu=(nx, nu), fxx=(nx, nx, nx), fuu=(nx, nu, nu), fxu=(nx, nx, nu))
    _expect_shapes("bwd_pass", single, B,
                   [("final_state", final_state, (nx,))] +
                   [(f"d.{f}", getattr(d, f), (N,) + fields[f]) for f in Derivatives._fields])
    rps = _shape(reg_param)
    if rps not in ((), (1,)) and rps != (B,):
        raise _lib.NocError(f"bwd_pass: reg_param must be a scalar or one per trajectory ({B},); "
                            f"got {rps}")
    xN = _dev(final_state, "final_state")
    dd = Derivatives(*(_dev(t) for t in d))
    if single:
        xN = xN[None]
        dd = Derivatives(*(t[None] for t in dd))
    Vx, Vxx = final_cost_grad(_O, xN, hessian=True)
    dev = dd.cu.device
    f64 = dict(dtype=torch.float64, device=dev)
    rp = torch.as_tensor(reg_param, **f64).reshape(-1).expand(B).contiguous()
    k, K, pred, Hu = (torch.empty(s, **f64) for s in ((B, N, nu), (B, N, nu, nx), (B,), (B, N, nu)))
    feas = torch.empty(B, dtype=torch.int32, device=dev)
    lib = _lib.for_shape(nx, nu)
    _lib.check(lib.noc_ddp_bwd_pass(nx, nu, N, B, Vx.data_ptr(), Vxx.contiguous().data_ptr(),
                                    rp.data_ptr(), *(getattr(dd, f).data_ptr() for f in
                                                     Derivatives._fields),
                                    k.data_ptr(), K.data_ptr(), pred.data_ptr(), feas.data_ptr(),
                                    Hu.data_ptr(), _lib.stream_handle(dev)),
               "noc_ddp_bwd_pass", lib)
    res = (k, K, pred, feas.bool(), Hu)
    return tuple(t[0] for t in res) if single else res


def ddp(ocp: OCP, controls, initial_state, barrier_param, device="cuda",
        max_passes: int = 10 ** 7):
    """D:98-186: ONE barrier value -- rollout, then DDP iterations with the retry loop until
    |Hu|inf < 1e-4 (or 500 iterations) -> (states, controls, iterations)."""
    X, U, its, _ = _solve(ocp, controls, initial_state, device, float(barrier_param), max_passes,
                          _lib.DDP_ONE_STAGE)
    return X, U, its


def interior_point_ddp(ocp: OCP, controls, initial_state, device="cuda", bp0: float = 0.1,
                       max_passes: int = 10 ** 7, return_info: bool = False):
    """D:189-208: barrier 0.1 / 5^k while > 1e-4, ddp (D:98-186) at each barrier value."""
    X, Uh, itn, info = _solve(ocp, controls, initial_state, device, float(bp0), max_passes, 0)
    if return_info:
        info["states"] = X
        return Uh, itn, info
    return Uh, itn


def _solve(ocp, controls, initial_state, device, bp0, max_passes, flags):
    import torch
    if ocp.family is None:
        raise _lib.NocError("OCP has no registered device family (use noc.problems.*): the HIP "
                            "kernels cannot evaluate Python callables")
    if not (np.isfinite(bp0) and bp0 >= 0.0):  # the rule of noc_ddp_solve_ex, for both paths
        raise _lib.NocError(f"ddp: barrier parameter must be finite and >= 0, got {bp0}")
    lib = _lib.load_for(ocp.family)
    fam = ocp.family.to_c()
    blocks = not lib.noc_ddp_supported(ctypes.byref(fam))
    if blocks and not (lib.noc_family_supported(ctypes.byref(fam))
                       and _lib.for_shape(fam.nx, fam.nu).noc_kkt_supported(fam.nx, fam.nu) == 1):
        raise _lib.NocError("interior-point DDP: family / shape not instantiated in this build")
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
    if blocks:
        Xd, Ud, itd, passd, doned = _solve_blocks(ocp, U, X0, bp0, max_passes, flags)
        X, Uh, itn = Xd.cpu().numpy(), Ud.cpu().numpy(), itd.to(torch.int32).cpu().numpy()
        info = dict(passes=passd.to(torch.int32).cpu().numpy(), done=doned.cpu().numpy())
        if single:
            Uh, itn, X = Uh[0], int(itn[0]), X[0]
            info = {k: v[0] for k, v in info.items()}
        return X, Uh, itn, info
    work = torch.empty(int(lib.noc_ddp_work_doubles(nx, nu, N, Bt)), **f64)
    i32 = dict(device=dev, dtype=torch.int32)
    its, passes, done = (torch.zeros(Bt, **i32) for _ in range(3))
    _lib.check(lib.noc_ddp_solve_ex(ctypes.byref(fam), N, Bt, _lib.ptr(X0), _lib.ptr(U),
                                    _lib.ptr(work), _lib.ptr(its), _lib.ptr(passes),
                                    _lib.ptr(done), float(bp0), int(max_passes), int(flags),
                                    _lib.stream_handle(dev)),
               "noc_ddp_solve_ex", lib)
    Uh, itn = U.cpu().numpy(), its.cpu().numpy()
    X = work[:Bt * (N + 1) * nx].view(Bt, N + 1, nx).cpu().numpy()
    info = dict(passes=passes.cpu().numpy(), done=done.cpu().numpy().astype(bool))
    if single:
        Uh, itn, X = Uh[0], int(itn[0]), X[0]
        info = {k: v[0] for k, v in info.items()}
    return X, Uh, itn, info


def _solve_blocks(ocp, U, X0, bp0, max_passes, flags):
    """D:98-208 for the families the one-launch kernel does not instantiate (nx > 4: its lanes
    hold the value Hessian and the stage blocks in registers): the same control flow, every
    trajectory its own (masked updates), as a host loop over the device building blocks --
    noc_derivatives, noc_ddp_bwd_pass, noc_nonlin_rollout, noc_check_feasibility, noc_total_cost.
    One host synchronisation per retry (the loop conditions).  Returns final states, controls,
    iterations, backward passes (retries included) and done (not stopped by max_passes), all on
    the device."""
    import torch
    Bt, N, nu = U.shape
    nx = X0.shape[-1]
    dev = U.device
    f64 = dict(dtype=torch.float64, device=dev)
    i64 = dict(dtype=torch.int64, device=dev)

    def sel(m, a, b):  # per-trajectory select
        return torch.where(m.view(-1, *([1] * (a.dim() - 1))), a, b)

    zK, zk = torch.zeros(Bt, N, nu, nx, **f64), torch.zeros(Bt, N, nu, **f64)
    u = U.clone()
    x = torch.zeros(Bt, N + 1, nx, **f64)
    total_it, passes = torch.zeros(Bt, **i64), torch.zeros(Bt, **i64)
    capped = torch.zeros(Bt, dtype=torch.bool, device=dev)
    one_stage = bool(flags & _lib.DDP_ONE_STAGE)
    inf = torch.full((Bt,), float("inf"), **f64)
    bp = float(bp0)
    while (one_stage or bp > 1e-4) and not bool(capped.all()):  # barrier schedule (D:189-208)
        run = ~capped
        nom = torch.zeros(Bt, N + 1, nx, **f64)
        nom[:, 0] = X0
        xr, _ = nonlin_rollout(ocp, zK, zk, nom, u)  # rollout of the controls (D:101): zero gains
        x = sel(run, xr, x)
        reg_param, reg_inc = torch.ones(Bt, **f64), torch.full((Bt,), 2.0, **f64)  # D:102-103
        hu, it = torch.ones(Bt, **f64), torch.zeros(Bt, **i64)
        active = run.clone()
        while bool(active.any()):  # DDP iterations (D:105-170)
            cost = total_cost(ocp, x, u, bp)  # D:108
            d = compute_derivatives(ocp, x, u, bp)  # D:112
            rp, r_inc = reg_param.clone(), reg_inc.clone()
            inner = torch.zeros(Bt, **i64)
            tx, tu, hn = x.clone(), u.clone(), hu.clone()
            retry = active.clone()
            while bool(retry.any()):  # retry loop (D:114-152)
                k, K, pred, feas, Hu = bwd_pass(ocp, x[:, -1], d, rp)
                xt, ut = nonlin_rollout(ocp, K, k, x, u)
                new_cost = torch.where(check_traj_feasibility(ocp, xt, ut),
                                       total_cost(ocp, xt, ut, bp), inf)  # D:121-125
                gain = (new_cost - cost) / pred
                succ = (gain > 0) & feas
                c = 2.0 * gain - 1.0  # x ** 3 as lax.integer_pow: c * (c * c), then 1 - it
                rp_new = torch.where(succ, rp * torch.clamp(1.0 - c * (c * c), min=1.0 / 3.0),
                                     rp * reg_inc)  # D:129-133: the outer reg_inc
                r_inc_new = torch.where(succ, torch.full_like(r_inc, 2.0), 2.0 * r_inc)
                rp = torch.where(retry, rp_new.clamp(1e-16, 1e16), rp)
                r_inc = torch.where(retry, r_inc_new, r_inc)
                tx, tu = sel(retry, xt, tx), sel(retry, ut, tu)
                hn = torch.where(retry, Hu.abs().amax(dim=(1, 2)), hn)  # D:120
                inner += retry.long()
                passes += retry.long()
                cap_now = retry & (passes >= max_passes)
                capped |= cap_now
                retry = retry & ~(succ | (inner > 500) | cap_now)
            # the last trial becomes the nominal trajectory, accepted or not (D:154)
            x, u = sel(active, tx, x), sel(active, tu, u)
            reg_param = torch.where(active, rp, reg_param)
            reg_inc = torch.where(active, r_inc, reg_inc)
            hu = torch.where(active, hn, hu)
            it += active.long()
            active = active & ~((hu < 1e-4) | (it > 500) | capped)  # D:167-170
        total_it += torch.where(run, it, torch.zeros_like(it))  # D:196
        bp = bp / 5.0
        if one_stage:
            break
    return x, u, total_it, passes, ~capped
