"""Batched LQ (KKT) solves on the MI355X -- the drop-in for `paroc` as used by the reference.

Reference call sites replaced:
  * noc/par_interior_point_newton.py:119-123 (par_Newton: noc_to_lqt -> par_bwd_pass -> par_fwd_pass)
  * examples/linear_mpc_parallel.py:64-75 (LQT(...), par_bwd_pass(lqt), par_fwd_pass(lqt, x0, Kx, d))

Two levels of API:
  * `kkt_solve(...)`: the canonical stage form used by the interior-point Newton step
    (include/noc_hip.h), batched over a leading trajectory axis; one fused HIP launch.
  * `LQT` + `par_bwd_pass` / `par_fwd_pass` / `seq_bwd_pass` / `seq_fwd_pass`: paroc's 13-field
    tracking form (field order from LM:64 and P:69-83), batched or not.  The tracking form is
    converted to the canonical form on the device (a few batched einsums), then the same HIP
    kernels run.  The "seq" names are kept for API compatibility and run the same kernels.

All tensors are torch fp64 CUDA tensors; calls are asynchronous on the current stream.
"""
from __future__ import annotations

from typing import NamedTuple, Optional

import torch

from . import _lib


class KKTResult(NamedTuple):
    dx: torch.Tensor          # (Bt, N+1, nx)
    du: torch.Tensor          # (Bt, N, nu)
    pred: torch.Tensor        # (Bt,)  sum of dV (noc/seq_interior_point_newton.py:63,75)
    feasible: torch.Tensor    # (Bt,) int32, all Quu > 0 (S:52-53)
    K: Optional[torch.Tensor]  # (Bt, N, nu, nx), None if want_gains=False
    d: Optional[torch.Tensor]  # (Bt, N, nu), None if want_gains=False
    S: Optional[torch.Tensor]  # (Bt, N+1, nx, nx) or None
    v: Optional[torch.Tensor]  # (Bt, N+1, nx) or None


def _c(t, name):
    if t is None:
        return None
    _lib.require_device(t, name)
    if t.dtype != torch.float64:
        raise _lib.NocError(f"{name}: expected float64, got {t.dtype}")
    return t.contiguous()


def _batched(*ts):
    """Accept unbatched (N, ...) inputs like the reference; returns (squeeze flag, tensors)."""
    A = ts[0]
    if A.dim() == 3:
        return True, [None if t is None else t.unsqueeze(0) for t in ts]
    return False, list(ts)


def pick_lanes(nx: int, nu: int, N: int, B: int) -> int:
    """Batch-aware lanes per trajectory for B trajectories (noc_kkt_pick_lanes)."""
    lib = _lib.for_shape(nx, nu)
    L = lib.noc_kkt_pick_lanes(nx, nu, N, B)
    _lib.check(0 if L > 0 else L, "noc_kkt_pick_lanes", lib)
    return L


def gains_on_chip(nx: int, nu: int, N: int, lanes: int = 0) -> bool:
    """True if the fused solve keeps K, d in LDS (noc_kkt_gains_on_chip), so they may be omitted."""
    return _lib.for_shape(nx, nu).noc_kkt_gains_on_chip(nx, nu, N, lanes) == 1


def kkt_solve(A, B, Q, R, M, r, P, reg=None, x0=None, q=None, c=None, p=None, active=None,
              lanes: int = 0, want_value: bool = False, out: Optional[KKTResult] = None,
              want_gains: bool = True) -> KKTResult:
    """Batched fused KKT solve (bwd + fwd).  Shapes (leading batch Bt optional):
    A (Bt,N,nx,nx) B (Bt,N,nx,nu) Q (Bt,N,nx,nx) R (Bt,N,nu,nu) M (Bt,N,nx,nu) r (Bt,N,nu)
    P (Bt,nx,nx) reg (Bt,) x0/p (Bt,nx) q/c (Bt,N,nx) active (Bt,) int32.
    want_gains=False: par_Newton's outputs only (dx, du, pred, feasible); K, d are then kept on
    chip when they fit (gains_on_chip) and returned as None."""
    squeeze, (A, B, Q, R, M, r, P, x0, q, c, p) = _batched(A, B, Q, R, M, r, P, x0, q, c, p)
    if squeeze and reg is not None and reg.dim() == 0:
        reg = reg.reshape(1)
    A, B, Q, R, M, r, P = (_c(t, n) for t, n in zip((A, B, Q, R, M, r, P), "A B Q R M r P".split()))
    x0, q, c, p, reg = _c(x0, "x0"), _c(q, "q"), _c(c, "c"), _c(p, "p"), _c(reg, "reg")
    Bt, N, nx, _ = A.shape
    nu = B.shape[-1]
    dev = A.device
    if active is not None:
        active = active.to(device=dev, dtype=torch.int32).contiguous()
    lanes = lanes or pick_lanes(nx, nu, N, Bt)
    if out is None:
        f64 = dict(device=dev, dtype=torch.float64)
        gains = want_gains or not gains_on_chip(nx, nu, N, lanes)
        out = KKTResult(
            torch.empty(Bt, N + 1, nx, **f64), torch.empty(Bt, N, nu, **f64),
            torch.empty(Bt, **f64), torch.empty(Bt, device=dev, dtype=torch.int32),
            torch.empty(Bt, N, nu, nx, **f64) if gains else None,
            torch.empty(Bt, N, nu, **f64) if gains else None,
            torch.empty(Bt, N + 1, nx, nx, **f64) if want_value else None,
            torch.empty(Bt, N + 1, nx, **f64) if want_value else None)
    lib = _lib.for_shape(nx, nu)
    rc = lib.noc_kkt_solve(nx, nu, N, Bt, lanes, *(_lib.ptr(t) for t in (
        A, B, Q, R, M, r, q, c, P, p, x0, reg, active,
        out.dx, out.du, out.pred, out.feasible, out.K, out.d, out.S, out.v)),
        _lib.stream_handle(dev))
    _lib.check(rc, "noc_kkt_solve", lib)
    if squeeze:
        out = KKTResult(*(None if t is None else t[0] for t in out))
    return out


# ------------------------------------------------------------------------------------------------
# tiled ("lane-interleaved") layout: the KKT scan's native HBM layout (include/noc_hip.h)
# ------------------------------------------------------------------------------------------------
def tiled_numel(N: int, Bt: int, lanes: int, E: int) -> int:
    return int(_lib.load().noc_tiled_doubles(N, Bt, lanes, E))


def tile(t: torch.Tensor, lanes: int, sym: bool = False) -> torch.Tensor:
    """Natural (Bt, N, ...) field -> flat tiled buffer.  sym=True packs an (n x n) symmetric
    field (upper triangle)."""
    t = _c(t, "field")
    Bt, N = t.shape[0], t.shape[1]
    if sym:
        n = t.shape[-1]
        E, sym_n = n * (n + 1) // 2, n
    else:
        E, sym_n = int(t[0, 0].numel()), 0
    out = torch.empty(tiled_numel(N, Bt, lanes, E), dtype=torch.float64, device=t.device)
    _lib.check(_lib.load().noc_relayout(0, E, sym_n, N, Bt, lanes, t.data_ptr(), out.data_ptr(),
                                        _lib.stream_handle(t.device)), "noc_relayout")
    return out


def untile(buf: torch.Tensor, shape, lanes: int, sym: bool = False) -> torch.Tensor:
    """Inverse of `tile`: flat tiled buffer -> natural tensor of `shape` = (Bt, N, ...)."""
    Bt, N = shape[0], shape[1]
    if sym:
        n = shape[-1]
        E, sym_n = n * (n + 1) // 2, n
    else:
        E = 1
        for d in shape[2:]:
            E *= d
        sym_n = 0
    out = torch.empty(shape, dtype=torch.float64, device=buf.device)
    _lib.check(_lib.load().noc_relayout(1, E, sym_n, N, Bt, lanes, buf.data_ptr(), out.data_ptr(),
                                        _lib.stream_handle(buf.device)), "noc_relayout")
    return out


class TiledBlocks(NamedTuple):
    """LQ blocks of Bt trajectories x N stages in the tiled layout of `lanes`."""
    A: torch.Tensor
    B: torch.Tensor
    Q: torch.Tensor        # packed symmetric
    R: torch.Tensor        # packed symmetric
    M: torch.Tensor
    r: torch.Tensor
    P: torch.Tensor        # natural (Bt, nx, nx)
    nx: int
    nu: int
    N: int
    Bt: int
    lanes: int


def to_tiled(A, B, Q, R, M, r, P, lanes: int) -> TiledBlocks:
    Bt, N, nx, _ = A.shape
    nu = B.shape[-1]
    return TiledBlocks(tile(A, lanes), tile(B, lanes), tile(Q, lanes, sym=True),
                       tile(R, lanes, sym=True), tile(M, lanes), tile(r, lanes), _c(P, "P"),
                       nx, nu, N, Bt, lanes)


def kkt_solve_tiled(tb: TiledBlocks, reg=None, x0=None, active=None, want_value=False,
                    out: Optional[KKTResult] = None, want_gains: bool = True) -> KKTResult:
    """Fused KKT solve on tiled blocks (the layout the interior-point workspace produces).
    K, d of the result are flat tiled buffers (None if want_gains=False and they fit on chip);
    dx, du, S, v natural."""
    Bt, N, nx, nu, L = tb.Bt, tb.N, tb.nx, tb.nu, tb.lanes
    dev = tb.A.device
    if out is None:
        f64 = dict(device=dev, dtype=torch.float64)
        gains = want_gains or not gains_on_chip(nx, nu, N, L)
        out = KKTResult(
            torch.empty(Bt, N + 1, nx, **f64), torch.empty(Bt, N, nu, **f64),
            torch.empty(Bt, **f64), torch.empty(Bt, device=dev, dtype=torch.int32),
            torch.empty(tiled_numel(N, Bt, L, nu * nx), **f64) if gains else None,
            torch.empty(tiled_numel(N, Bt, L, nu), **f64) if gains else None,
            torch.empty(Bt, N + 1, nx, nx, **f64) if want_value else None,
            torch.empty(Bt, N + 1, nx, **f64) if want_value else None)
    if active is not None:
        active = active.to(device=dev, dtype=torch.int32).contiguous()
    lib = _lib.for_shape(nx, nu)
    rc = lib.noc_kkt_solve_tiled(nx, nu, N, Bt, L, *(_lib.ptr(t) for t in (
        tb.A, tb.B, tb.Q, tb.R, tb.M, tb.r, None, None, tb.P, None, _c(x0, "x0"), _c(reg, "reg"),
        active, out.dx, out.du, out.pred, out.feasible, out.K, out.d, out.S, out.v)),
        _lib.stream_handle(dev))
    _lib.check(rc, "noc_kkt_solve_tiled", lib)
    return out


def bwd_pass(A, B, Q, R, M, r, P, reg=None, q=None, c=None, p=None, active=None, lanes=0):
    """Backward pass only -> (K, d, S, v, pred, feasible) (paroc.par_bwd_pass semantics)."""
    squeeze, (A, B, Q, R, M, r, P, q, c, p) = _batched(A, B, Q, R, M, r, P, q, c, p)
    A, B, Q, R, M, r, P = (_c(t, n) for t, n in zip((A, B, Q, R, M, r, P), "A B Q R M r P".split()))
    q, c, p, reg = _c(q, "q"), _c(c, "c"), _c(p, "p"), _c(reg, "reg")
    Bt, N, nx, _ = A.shape
    nu = B.shape[-1]
    f64 = dict(device=A.device, dtype=torch.float64)
    K = torch.empty(Bt, N, nu, nx, **f64)
    d = torch.empty(Bt, N, nu, **f64)
    S = torch.empty(Bt, N + 1, nx, nx, **f64)
    v = torch.empty(Bt, N + 1, nx, **f64)
    pred = torch.empty(Bt, **f64)
    feas = torch.empty(Bt, device=A.device, dtype=torch.int32)
    if active is not None:
        active = active.to(device=A.device, dtype=torch.int32).contiguous()
    lib = _lib.for_shape(nx, nu)
    rc = lib.noc_par_bwd_pass(nx, nu, N, Bt, lanes, *(_lib.ptr(t) for t in (
        A, B, Q, R, M, r, q, c, P, p, reg, active, K, d, S, v, pred, feas)),
        _lib.stream_handle(A.device))
    _lib.check(rc, "noc_par_bwd_pass", lib)
    res = (K, d, S, v, pred, feas)
    return tuple(t[0] for t in res) if squeeze else res


def fwd_pass(A, B, K, d, x0=None, c=None, active=None, lanes=0):
    """Forward pass only -> (du, dx) (paroc.par_fwd_pass semantics)."""
    squeeze, (A, B, K, d, x0, c) = _batched(A, B, K, d, x0, c)
    A, B, K, d = _c(A, "A"), _c(B, "B"), _c(K, "K"), _c(d, "d")
    x0, c = _c(x0, "x0"), _c(c, "c")
    Bt, N, nx, _ = A.shape
    nu = B.shape[-1]
    f64 = dict(device=A.device, dtype=torch.float64)
    du = torch.empty(Bt, N, nu, **f64)
    dx = torch.empty(Bt, N + 1, nx, **f64)
    if active is not None:
        active = active.to(device=A.device, dtype=torch.int32).contiguous()
    lib = _lib.for_shape(nx, nu)
    rc = lib.noc_par_fwd_pass(nx, nu, N, Bt, lanes, *(_lib.ptr(t) for t in (
        A, B, c, x0, K, d, active, du, dx)), _lib.stream_handle(A.device))
    _lib.check(rc, "noc_par_fwd_pass", lib)
    return (du[0], dx[0]) if squeeze else (du, dx)


# ------------------------------------------------------------------------------------------------
# paroc-compatible tracking-form LQT (field order: LM:64, P:69-83)
# ------------------------------------------------------------------------------------------------
class LQT(NamedTuple):
    """paroc.lqt_problem.LQT: dynamics x+ = F x + L u + c; stage cost
    1/2 (Hx - r)'X(Hx - r) + 1/2 (Zu - s)'U(Zu - s) + (Hx - r)'M(Zu - s); terminal cost
    1/2 (HT x - rT)'XT(HT x - rT).  (Convention consistent with noc_to_lqt, P:62-66.)"""
    F: torch.Tensor
    L: torch.Tensor
    c: torch.Tensor
    XT: torch.Tensor
    HT: torch.Tensor
    rT: torch.Tensor
    X: torch.Tensor
    H: torch.Tensor
    r: torch.Tensor
    U: torch.Tensor
    Z: torch.Tensor
    s: torch.Tensor
    M: torch.Tensor


def lqt_to_canonical(lqt: LQT):
    """Expand the tracking form into (A, B, Q, R, M, r, q, c, P, p) (batched einsums)."""
    H, Z, X, U, Mt = lqt.H, lqt.Z, lqt.X, lqt.U, lqt.M
    t = lambda x: x.transpose(-1, -2)
    Q = t(H) @ X @ H
    R = t(Z) @ U @ Z
    M = t(H) @ Mt @ Z
    rr, ss = lqt.r.unsqueeze(-1), lqt.s.unsqueeze(-1)
    q = -(t(H) @ (X @ rr + Mt @ ss)).squeeze(-1)
    r = -(t(Z) @ (U @ ss + t(Mt) @ rr)).squeeze(-1)
    P = t(lqt.HT) @ lqt.XT @ lqt.HT
    p = -(t(lqt.HT) @ (lqt.XT @ lqt.rT.unsqueeze(-1))).squeeze(-1)
    return lqt.F, lqt.L, Q, R, M, r, q, lqt.c, P, p


def _aff(t):
    return None if t is None or not bool(torch.any(t != 0)) else t.contiguous()


def par_bwd_pass(lqt: LQT, lanes: int = 0):
    """paroc.par_bwd_pass(lqt) -> (Kx, d, S, v, pred_reduction, feasible); du = Kx dx + d."""
    A, B, Q, R, M, r, q, c, P, p = lqt_to_canonical(lqt)
    K, d, S, v, pred, feas = bwd_pass(A.contiguous(), B.contiguous(), Q.contiguous(),
                                      R.contiguous(), M.contiguous(), r.contiguous(), P.contiguous(),
                                      q=_aff(q), c=_aff(c), p=_aff(p), lanes=lanes)
    return K, d, S, v, pred, feas.bool()


def par_fwd_pass(lqt: LQT, x0, Kx, d, lanes: int = 0):
    """paroc.par_fwd_pass(lqt, x0, Kx, d) -> (u, x)."""
    return fwd_pass(lqt.F.contiguous(), lqt.L.contiguous(), Kx, d, x0=x0.contiguous(),
                    c=_aff(lqt.c), lanes=lanes)


def seq_bwd_pass(lqt: LQT):
    """paroc.seq_bwd_pass(lqt) -> (Kx, d, S, v) (LM:74).  Same solution; same HIP kernels."""
    K, d, S, v, _, _ = par_bwd_pass(lqt)
    return K, d, S, v


def seq_fwd_pass(lqt: LQT, x0, Kx, d):
    """paroc.seq_fwd_pass(lqt, x0, Kx, d) -> (u, x) (LM:75)."""
    return par_fwd_pass(lqt, x0, Kx, d)


# ------------------------------------------------------------------------------------------------
# closed-loop MPC (examples/linear_mpc_parallel.py:67-84)
# ------------------------------------------------------------------------------------------------
def mpc_loop(lqt: LQT, x0, steps: int, lanes: int = 0, graph: bool = True, chunk: int = 50):
    """`par_mpc_loop` under `lax.scan` (LM:67-84): every MPC step solves the LQT from the current
    state (par_bwd_pass + par_fwd_pass, here the fused KKT kernel with x0 = current state) and
    applies the first control: u_t = u_par[0], x_{t+1} = x_par[1].

    x0: (nx,) or (Bm, nx) -- a batch of independent MPC instances sharing the LQT.  Returns
    (xs, us) of shapes (steps, [Bm,] nx) and (steps, [Bm,] nu), like the reference's scan outputs.
    graph=True captures `chunk` consecutive steps in one HIP graph (torch.cuda.CUDAGraph) and
    replays it, so a 5000-step loop costs 100 graph launches instead of 5000 x (solve + copies)."""
    single = x0.dim() == 1
    xcur = (x0.unsqueeze(0) if single else x0).to(torch.float64).contiguous().clone()
    Bm, nx = xcur.shape
    A, B, Q, R, M, r, q, c, P, p = lqt_to_canonical(lqt)
    if lanes == 0 and A.shape[0] <= 32:
        lanes = 1  # MPC horizons are short (LM: T = 5): the horizon-sequential group solve
    exp = lambda t: None if t is None else t.unsqueeze(0).expand(Bm, *t.shape).contiguous()
    A, B, Q, R, M, r, P = (exp(t) for t in (A, B, Q, R, M, r, P))
    q, c, p = exp(_aff(q)), exp(_aff(c)), exp(_aff(p))
    N, nu = A.shape[1], B.shape[-1]
    out = kkt_solve(A, B, Q, R, M, r, P, x0=xcur, q=q, c=c, p=p, lanes=lanes, want_gains=False)
    xs = torch.empty(steps, Bm, nx, dtype=torch.float64, device=xcur.device)
    us = torch.empty(steps, Bm, nu, dtype=torch.float64, device=xcur.device)

    def one_step(xs_t, us_t):
        kkt_solve(A, B, Q, R, M, r, P, x0=xcur, q=q, c=c, p=p, lanes=lanes, out=out)
        us_t.copy_(out.du[:, 0])
        xs_t.copy_(out.dx[:, 1])
        xcur.copy_(out.dx[:, 1])

    t = 0
    if graph and steps >= chunk:
        stg_x = torch.empty(chunk, Bm, nx, dtype=torch.float64, device=xcur.device)
        stg_u = torch.empty(chunk, Bm, nu, dtype=torch.float64, device=xcur.device)
        side = torch.cuda.Stream(device=xcur.device)
        side.wait_stream(torch.cuda.current_stream(xcur.device))
        with torch.cuda.stream(side):  # warm-up on a side stream before capture (torch idiom)
            one_step(stg_x[0], stg_u[0])
        torch.cuda.current_stream(xcur.device).wait_stream(side)
        xcur.copy_((x0.unsqueeze(0) if single else x0).to(torch.float64))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(chunk):
                one_step(stg_x[i], stg_u[i])
        while t + chunk <= steps:
            g.replay()
            xs[t:t + chunk].copy_(stg_x)
            us[t:t + chunk].copy_(stg_u)
            t += chunk
    while t < steps:
        one_step(xs[t], us[t])
        t += 1
    if single:
        return xs[:, 0], us[:, 0]
    return xs, us
