"""Parallel-in-time interior-point solver -- drop-in for noc/par_interior_point_newton.py.

Every public function of the reference module is here with its signature (P:13-254):
compute_derivatives, compute_lqr_params, check_traj_feasibility, noc_to_lqt, nonlin_rollout,
par_Newton, newton_oc, par_interior_point_optimal_control.  They run on the MI355X: the building blocks as
batched HIP kernels (noc_derivatives, noc_costates, noc_lqr_params, noc_kkt_solve), the loops as
the persistent whole-solve kernel (noc_ipm_solve) or the launch-per-phase driver.

Differences, all additive:
  * inputs may carry a leading batch axis (controls (B, N, nu), initial_state (B, nx), states
    (B, N+1, nx)); the result is then batched too -- each trajectory follows its own reference
    control flow (jax.vmap semantics);
  * `ocp.family` must be a registered family (noc.problems built-ins or noc.families
    .register_family) because device code cannot call Python callables;
  * `terminal`: "stage0" (default: the reference par path's terminal Hessian XT = Q[0], P:73 --
    what par_Newton actually feeds its LQT) or "final_cost" (hessian(final_cost), the reference
    seq path S:66).  The default reproduces the reference par loop's iteration counts (e.g.
    cart-pole N=50: 88 outer / 129 KKT solves; with "final_cost": 91 / 135).
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np
import torch

from . import _lib
from .ipm import BatchedIPM
from .optimal_control_problem import OCP, Derivatives

_TERMINAL = {"final_cost": _lib.TERMINAL_FINAL_COST, "stage0": _lib.TERMINAL_STAGE0}


def _family(ocp: OCP):
    if getattr(ocp, "family", None) is None:
        raise _lib.NocError("OCP has no registered device family (noc.problems / noc.families): "
                            "the HIP kernels cannot evaluate Python callables")
    return ocp.family


def _dev(t, name="array"):
    if isinstance(t, torch.Tensor):
        _lib.require_device(t, name)
        return t.to(torch.float64).contiguous()
    return torch.as_tensor(np.ascontiguousarray(t, dtype=np.float64), device="cuda")


def _shape(t):
    return tuple(t.shape) if hasattr(t, "shape") else tuple(np.shape(t))


def _expect_shapes(fn: str, single: bool, B, items):
    """Raise NocError unless every (name, array, shape) of `items` has exactly `shape` (with the
    leading batch axis B prepended when the call is batched).  Run on the host BEFORE any pointer
    reaches a kernel: a mis-shaped input must raise, not make the device read or write out of
    bounds (e.g. states without the terminal row, unbatched gains with batched states)."""
    bad = []
    for name, t, shp in items:
        want = tuple(shp) if single else (B,) + tuple(shp)
        got = _shape(t)
        if got != want:
            bad.append(f"{name} {got} (expected {want})")
    if bad:
        raise _lib.NocError(f"{fn}: mis-shaped input: " + "; ".join(bad))


def compute_derivatives(ocp: OCP, states, controls, bp) -> Derivatives:
    """P:13-28: per-stage grad / hessian of stage_cost and jacrev / second derivatives of the
    dynamics at (x_k, u_k), k < N (noc_derivatives).  states (N+1, nx), controls (N, nu) (or
    batched), bp a scalar or one per trajectory."""
    fam = _family(ocp)
    nx, nu = fam.nx, fam.nu
    # every size from the states, the controls checked against them on the host, before anything
    # reaches the device
    xs = _shape(states)
    single = len(xs) == 2
    B = 1 if single else (xs[0] if len(xs) == 3 else -1)
    N = xs[-2] - 1 if len(xs) in (2, 3) else -1
    _expect_shapes("compute_derivatives", single, B,
                   [("states", states, (N + 1, nx)), ("controls", controls, (N, nu))])
    x, u = _dev(states, "states"), _dev(controls, "controls")
    if single:
        x, u = x[None], u[None]
    bpt = torch.as_tensor(bp, dtype=torch.float64, device=x.device).reshape(-1)
    if bpt.numel() not in (1, B):
        raise _lib.NocError(f"compute_derivatives: bp needs 1 or {B} values, got {bpt.numel()}")
    bpt = bpt.expand(B).contiguous()
    f64 = dict(dtype=torch.float64, device=x.device)
    shapes = dict(cx=(nx,), cu=(nu,), cxx=(nx, nx), cuu=(nu, nu), cxu=(nx, nu), fx=(nx, nx),
                  fu=(nx, nu), fxx=(nx, nx, nx), fuu=(nx, nu, nu), fxu=(nx, nx, nu))
    out = {k: torch.empty((B, N) + s, **f64) for k, s in shapes.items()}
    lib = _lib.load_for(fam)
    _lib.check(lib.noc_derivatives(ctypes.byref(fam.to_c()), N, B, x.data_ptr(), u.data_ptr(),
                                   bpt.data_ptr(), *(out[k].data_ptr() for k in Derivatives._fields),
                                   _lib.stream_handle(x.device)), "noc_derivatives", lib)
    d = Derivatives(*(out[k] for k in Derivatives._fields))
    return Derivatives(*(t[0] for t in d)) if single else d


def compute_lqr_params(lagrange_multipliers, d: Derivatives):
    """P:31-42: ru = cu + fu' l, Q = cxx + l.fxx, R = cuu + l.fuu, M = cxu + l.fxu with
    l = lambda[1:] (noc_lqr_params)."""
    # sizes from lambda (N+1, nx) and cu (N, nu); lambda and every Derivatives field checked
    # against them on the host, before anything reaches the device
    ls, cus = _shape(lagrange_multipliers), _shape(d.cu)
    single = len(ls) == 2
    B = 1 if single else (ls[0] if len(ls) == 3 else -1)
    N = ls[-2] - 1 if len(ls) in (2, 3) else -1
    nx = ls[-1] if len(ls) in (2, 3) else -1
    nu = cus[-1] if len(cus) >= 1 else -1
    shapes = dict(cx=(nx,), cu=(nu,), cxx=(nx, nx), cuu=(nu, nu), cxu=(nx, nu), fx=(nx, nx),
                  fu=(nx, nu), fxx=(nx, nx, nx), fuu=(nx, nu, nu), fxu=(nx, nx, nu))
    _expect_shapes("compute_lqr_params", single, B,
                   [("lagrange_multipliers", lagrange_multipliers, (N + 1, nx))] +
                   [(k, getattr(d, k), (N,) + shapes[k]) for k in Derivatives._fields])
    lam = _dev(lagrange_multipliers, "lagrange_multipliers")
    dd = Derivatives(*(_dev(t) for t in d))
    if single:
        lam = lam[None]
        dd = Derivatives(*(t[None] for t in dd))
    f64 = dict(dtype=torch.float64, device=lam.device)
    ru, Q, R, M = (torch.empty(B, N, *s, **f64) for s in ((nu,), (nx, nx), (nu, nu), (nx, nu)))
    lib = _lib.load()
    _lib.check(lib.noc_lqr_params(nx, nu, N, B, lam.data_ptr(), *(getattr(dd, k).data_ptr() for k in
                                  ("cu", "cxx", "cuu", "cxu", "fu", "fxx", "fuu", "fxu")),
                                  ru.data_ptr(), Q.data_ptr(), R.data_ptr(), M.data_ptr(),
                                  _lib.stream_handle(lam.device)), "noc_lqr_params", lib)
    res = (ru, Q, R, M)
    return tuple(t[0] for t in res) if single else res


def check_traj_feasibility(ocp: OCP, x, u):
    """P:45-47: all(constraints(x_k, u_k) <= 0) over k < N (x[:-1] paired with u) with the
    family's whole constraint vector -- the built-ins' box on u, a registered family's traced
    constraints(x, u) including state constraints (noc_check_feasibility, one wave per
    trajectory).  x (N+1, nx), u (N, nu) -> a 0-d bool tensor; batched (B, N+1, nx), (B, N, nu)
    -> (B,) bool."""
    fam = _family(ocp)
    x, u = _dev(x, "x"), _dev(u, "u")
    single = u.dim() == 2
    if single:
        x, u = x[None], u[None]
    if x.dim() != 3 or u.dim() != 3 or x.shape[0] != u.shape[0] or x.shape[1] != u.shape[1] + 1 \
            or x.shape[2] != fam.nx or u.shape[2] != fam.nu:
        raise _lib.NocError(f"check_traj_feasibility: need x (B, N+1, {fam.nx}) and u (B, N, "
                            f"{fam.nu}); got {tuple(x.shape)} and {tuple(u.shape)}")
    B, N = u.shape[0], u.shape[1]
    if N == 0:  # jnp.all of an empty constraint array
        ok = torch.ones(B, dtype=torch.bool, device=u.device)
        return ok[0] if single else ok
    ok = torch.empty(B, dtype=torch.int32, device=u.device)
    lib = _lib.load_for(fam)
    _lib.check(lib.noc_check_feasibility(ctypes.byref(fam.to_c()), N, B, x.data_ptr(),
                                         u.data_ptr(), ok.data_ptr(),
                                         _lib.stream_handle(u.device)),
               "noc_check_feasibility", lib)
    ok = ok.bool()
    return ok[0] if single else ok


def total_cost(ocp: OCP, states, controls, bp):
    """ocp.total_cost(states, controls, bp) on the device (PR:53-56, CR:48-51, LD:45-48; a
    registered family's own traced costs): final_cost(x_N) + sum_k stage_cost(x_k, u_k, bp)
    (noc_total_cost, one wave per trajectory).  states (N+1, nx), controls (N, nu) -> a 0-d
    tensor; batched -> (B,); bp a scalar or one per trajectory."""
    fam = _family(ocp)
    us = _shape(controls)
    single = len(us) == 2
    if len(us) not in (2, 3):
        raise _lib.NocError(f"total_cost: controls must be (N, nu) or (B, N, nu); got {us}")
    B, N = (1, us[0]) if single else (us[0], us[1])
    _expect_shapes("total_cost", single, B, [("states", states, (N + 1, fam.nx)),
                                             ("controls", controls, (N, fam.nu))])
    if N == 0:
        raise _lib.NocError("total_cost: need a horizon N >= 1")
    x, u = _dev(states, "states"), _dev(controls, "controls")
    if single:
        x, u = x[None], u[None]
    bpt = torch.as_tensor(bp, dtype=torch.float64, device=u.device).reshape(-1).expand(B).contiguous()
    cost = torch.empty(B, dtype=torch.float64, device=u.device)
    lib = _lib.load_for(fam)
    _lib.check(lib.noc_total_cost(ctypes.byref(fam.to_c()), N, B, x.data_ptr(), u.data_ptr(),
                                  bpt.data_ptr(), cost.data_ptr(), _lib.stream_handle(u.device)),
               "noc_total_cost", lib)
    return cost[0] if single else cost


def nonlin_rollout(ocp: OCP, gain, ffgain, nominal_states, nominal_controls):
    """P:87-104 (== D:73-90): x_hat_0 = x_0, u_hat = u + k + K (x_hat - x), x_hat+ =
    dynamics(x_hat, u_hat) -> (new_states (N+1, nx), new_controls (N, nu)); batched inputs
    (leading B axis) give batched outputs (noc_nonlin_rollout, one thread per trajectory)."""
    fam = _family(ocp)
    us = _shape(nominal_controls)
    single = len(us) == 2
    if len(us) not in (2, 3):
        raise _lib.NocError(f"nonlin_rollout: nominal_controls must be (N, nu) or (B, N, nu); got {us}")
    B, N = (1, us[0]) if single else (us[0], us[1])
    nx, nu = fam.nx, fam.nu
    _expect_shapes("nonlin_rollout", single, B, [("gain", gain, (N, nu, nx)),
                                                 ("ffgain", ffgain, (N, nu)),
                                                 ("nominal_states", nominal_states, (N + 1, nx)),
                                                 ("nominal_controls", nominal_controls, (N, nu))])
    K, k = _dev(gain, "gain"), _dev(ffgain, "ffgain")
    x, u = _dev(nominal_states, "nominal_states"), _dev(nominal_controls, "nominal_controls")
    if single:
        K, k, x, u = K[None], k[None], x[None], u[None]
    xn, un = torch.empty_like(x), torch.empty_like(u)
    lib = _lib.load_for(fam)
    _lib.check(lib.noc_nonlin_rollout(ctypes.byref(fam.to_c()), N, B, K.data_ptr(), k.data_ptr(),
                                      x.data_ptr(), u.data_ptr(), xn.data_ptr(), un.data_ptr(),
                                      _lib.stream_handle(u.device)), "noc_nonlin_rollout", lib)
    return (xn[0], un[0]) if single else (xn, un)


def noc_to_lqt(ru, Q, R, M, A, B):
    """P:50-84: the paroc tracking-form LQT of the Newton step (references r, s by the two
    per-stage solves; terminal XT = Q[0], HT = I, rT = 0).  Needs Q invertible, like the
    reference; the solvers here never use this form (noc_kkt_solve takes the canonical blocks)."""
    from .lqt import LQT
    ru, Q, R, M, A, B = (_dev(t) for t in (ru, Q, R, M, A, B))
    XinvM = torch.linalg.solve(Q, M)
    s = -torch.linalg.solve(R - M.transpose(-1, -2) @ XinvM, ru.unsqueeze(-1)).squeeze(-1)
    r = -(XinvM @ s.unsqueeze(-1)).squeeze(-1)
    T, nx, nu = Q.shape[-3], Q.shape[-1], R.shape[-1]
    eye = lambda n: torch.eye(n, dtype=torch.float64, device=Q.device).expand(*Q.shape[:-2], n, n)
    zeros = torch.zeros(*Q.shape[:-1], dtype=torch.float64, device=Q.device)
    return LQT(A, B, zeros, Q[..., 0, :, :], torch.eye(nx, dtype=torch.float64, device=Q.device)
               .expand(*Q.shape[:-3], nx, nx), torch.zeros(*Q.shape[:-3], nx, dtype=torch.float64,
                                                           device=Q.device),
               Q, eye(nx), r, R, eye(nu), s, M)


def par_Newton(nominal_states, d: Derivatives, reg_param, ru, Q, R, M):
    """P:107-124: reg = reg_param * ||cu||_F added to R, the LQT's bwd + fwd pass from dx_0 = 0
    with terminal Hessian XT = Q[0] -> (dx, du, pred_reduction, feasible, ru).  One fused KKT
    launch (noc_kkt_solve) instead of noc_to_lqt + par_bwd_pass + par_fwd_pass."""
    from . import lqt
    ru, Q, R, M = (_dev(t) for t in (ru, Q, R, M))
    fx, fu, cu = _dev(d.fx), _dev(d.fu), _dev(d.cu)
    single = Q.dim() == 3
    if single:
        ru, Q, R, M, fx, fu, cu = (t[None] for t in (ru, Q, R, M, fx, fu, cu))
    gnorm = torch.linalg.vector_norm(cu.flatten(1), dim=1)
    reg = (torch.as_tensor(reg_param, dtype=torch.float64, device=Q.device).reshape(-1) * gnorm)
    P = Q[:, 0].contiguous()
    out = lqt.kkt_solve(fx, fu, Q, R, M, ru, P, reg=reg.contiguous(), want_gains=False)
    res = (out.dx, out.du, out.pred, out.feasible.bool(), ru)
    return tuple(t[0] for t in res) if single else res


# Engines of small solves are kept between calls (the reference's timing harness calls the solver
# at B = 1 over and over: the workspace allocation and its zero fill were part of every call's
# host cost).  Every solve starts from the controls / initial state it loads -- the persistent
# kernel and noc_ipm_init reset the whole solver state -- so a reused engine gives the results of
# a fresh one.  Keyed by the family's descriptor bytes, so an edited family gets a new engine, and
# by the calling thread, so cached engines are never shared across threads (the cache dict itself
# is guarded by a lock).
_ENGINES: "dict" = {}
_ENGINES_LOCK = threading.Lock()
_ENGINE_CACHE_MAX = 8
_ENGINE_CACHE_STAGES = 1 << 16  # Bt * N at most: B = 1 up to N = 65536, B = 64 at N = 1000


def _engine(fam, N, Bt, lanes, device):
    from .ipm import persistent_supported
    # whole solve in one launch when the family / horizon allows it (same results, lanes 64)
    persistent = lanes in (0, 64) and persistent_supported(fam, N)
    if Bt * N > _ENGINE_CACHE_STAGES:
        return BatchedIPM(fam, N, Bt, device=device, lanes=lanes, persistent=persistent)
    # per thread: an engine is a workspace, so two threads solving the same shape must not share
    # one (the reference's functions have no shared state)
    key = (id(fam), bytes(fam.to_c()), getattr(fam, "lib_path", None), N, Bt, lanes, persistent,
           str(torch.device(device)), threading.get_ident())
    with _ENGINES_LOCK:
        eng = _ENGINES.pop(key, None)
    if eng is None:
        eng = BatchedIPM(fam, N, Bt, device=device, lanes=lanes, persistent=persistent)
        eng._family_ref = fam  # keeps id(fam) from being reused while the entry lives
    with _ENGINES_LOCK:
        _ENGINES[key] = eng  # most recently used last
        while len(_ENGINES) > _ENGINE_CACHE_MAX:
            _ENGINES.pop(next(iter(_ENGINES)))
    return eng


def _run(ocp: OCP, controls, initial_state, mode, terminal="stage0", lanes=0,
         device="cuda", return_info=False, one_stage_bp=None):
    fam = _family(ocp)
    u = np.asarray(controls, dtype=np.float64)
    x0 = np.asarray(initial_state, dtype=np.float64)
    single = u.ndim == 2
    if single:
        u, x0 = u[None], x0[None]
    Bt, N, _ = u.shape
    eng = _engine(fam, N, Bt, lanes, device)
    eng.ws.flags = _lib.WS_ONE_STAGE if one_stage_bp is not None else 0
    eng.load(u, x0)
    bp0 = 0.1 if one_stage_bp is None else float(one_stage_bp)
    steps = eng.solve(mode=mode, terminal=_TERMINAL[terminal], bp0=bp0)
    U, iters, solves, X = eng.host_result()  # straight to the host, two copies
    if single:
        U, iters, solves, X = U[0], int(iters[0]), int(solves[0]), X[0]
    if one_stage_bp is not None:
        return X, U, iters
    if return_info:
        return U, iters, dict(kkt_solves=solves, device_steps=steps)
    return U, iters


def newton_oc(ocp: OCP, controls, initial_state, barrier_param, terminal="stage0"):
    """P:127-225: ONE barrier stage -- rollout, then Newton iterations with the retry loop until
    |Hu|inf < 1e-4 (or 1000 iterations) -> (states, controls, iterations)."""
    return _run(ocp, controls, initial_state, _lib.MODE_PAR, terminal, one_stage_bp=barrier_param)


def par_interior_point_optimal_control(ocp: OCP, controls, initial_state, terminal="stage0",
                                       lanes: int = 0, device="cuda", return_info=False):
    """P:228-254: barrier 0.1 / 5^k while > 1e-4; Newton with retry loop; returns (u*, iters)."""
    return _run(ocp, controls, initial_state, _lib.MODE_PAR, terminal, lanes, device, return_info)
