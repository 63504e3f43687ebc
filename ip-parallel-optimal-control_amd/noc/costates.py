"""Costates -- drop-in for the reference's noc/costates.py (C:6-54).

lambda_N = grad(final_cost)(x_N), lambda_k = cx_k + fx_k' lambda_{k+1}.  `par_costates` is the
reference's associative-scan form (C:34-40) and `seq_costates` its sequential lax.scan (C:43-54);
both run as batched HIP kernels (noc_costates: a chunked affine scan over a wave per trajectory,
or one recursion per trajectory).  `combine_fc`, `par_init` and `par_scan` are the reference's
scan helpers (C:6-31), kept with the same semantics on torch tensors (batched over leading axes).

Inputs may be numpy arrays or torch tensors, with an optional leading batch axis (then every
trajectory is solved independently, jax.vmap style); the result is a CUDA tensor.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .optimal_control_problem import OCP, Derivatives


def _dev(t, name="array"):
    if isinstance(t, torch.Tensor):
        _lib.require_device(t, name)
        return t.to(torch.float64).contiguous()
    return torch.as_tensor(np.ascontiguousarray(t, dtype=np.float64), device="cuda")


def final_cost_grad(ocp: OCP, final_state, hessian: bool = False):
    """grad(ocp.final_cost)(x_N) on the device (and hessian(final_cost) with hessian=True) for a
    registered family: (B, nx) [, (B, nx, nx)] for batched x_N (B, nx), else unbatched."""
    fam = getattr(ocp, "family", None)
    if fam is None:
        raise _lib.NocError("OCP has no registered device family (noc.problems / noc.families)")
    xN = _dev(final_state, "final_state")
    single = xN.dim() == 1
    xN = xN.reshape(-1, fam.nx).contiguous()
    B = xN.shape[0]
    g = torch.empty(B, fam.nx, dtype=torch.float64, device=xN.device)
    h = torch.empty(B, fam.nx, fam.nx, dtype=torch.float64, device=xN.device) if hessian else None
    lib = _lib.load_for(fam)
    _lib.check(lib.noc_final_cost_derivs(ctypes.byref(fam.to_c()), B, xN.data_ptr(), g.data_ptr(),
                                         _lib.ptr(h), _lib.stream_handle(xN.device)),
               "noc_final_cost_derivs", lib)
    if single:
        return (g[0], h[0]) if hessian else g[0]
    return (g, h) if hessian else g


def costates(lamda_T, cx, fx, sequential: bool = False):
    """Batched costate recursion from lambda_N: lamda_T (B, nx), cx (B, N, nx), fx (B, N, nx, nx)
    -> lambda (B, N+1, nx) (no batch axis in -> none out)."""
    cx, fx, lT = _dev(cx, "cx"), _dev(fx, "fx"), _dev(lamda_T, "lamda_T")
    single = cx.dim() == 2
    if single:
        cx, fx, lT = cx[None], fx[None], lT[None]
    B, N, nx = cx.shape
    lam = torch.empty(B, N + 1, nx, dtype=torch.float64, device=cx.device)
    lib = _lib.load()
    _lib.check(lib.noc_costates(nx, N, B, lT.contiguous().data_ptr(), cx.data_ptr(),
                                fx.data_ptr(), lam.data_ptr(), 1 if sequential else 0,
                                _lib.stream_handle(cx.device)), "noc_costates", lib)
    return lam[0] if single else lam


def par_costates(ocp: OCP, final_state, d: Derivatives):
    """C:34-40: lambda_N = grad(final_cost)(x_N), then the affine associative scan."""
    return costates(final_cost_grad(ocp, final_state), d.cx, d.fx, sequential=False)


def seq_costates(ocp: OCP, final_state, d: Derivatives):
    """C:43-54: the same recursion as a sequential scan."""
    return costates(final_cost_grad(ocp, final_state), d.cx, d.fx, sequential=True)


def combine_fc(elem1, elem2):
    """C:6-12: (F_ij, c_ij) o (F_jk, c_jk) = (F_jk F_ij, F_jk c_ij + c_jk)."""
    Fij, cij = elem1
    Fjk, cjk = elem2
    return Fjk @ Fij, (Fjk @ cij.unsqueeze(-1)).squeeze(-1) + cjk


def par_init(F, c, x0):
    """C:19-31: element 0 becomes the constant map (0, F_0 x0 + c_0)."""
    F, c, x0 = _dev(F), _dev(c), _dev(x0)
    tF = F.clone()
    tc = c.clone()
    tF[..., 0, :, :] = 0.0
    tc[..., 0, :] = (F[..., 0, :, :] @ x0.unsqueeze(-1)).squeeze(-1) + c[..., 0, :]
    return tF, tc


def par_scan(elems):
    """C:15-16: inclusive associative scan of combine_fc along the stage axis (-3 for F, -2 for
    c), Hillis-Steele in log2(N) vectorised steps."""
    F, c = elems
    F, c = F.clone(), c.clone()
    N = F.shape[-3]
    d = 1
    while d < N:
        nF, nc = combine_fc((F[..., :-d, :, :], c[..., :-d, :]), (F[..., d:, :, :], c[..., d:, :]))
        F = torch.cat((F[..., :d, :, :], nF), dim=-3)
        c = torch.cat((c[..., :d, :], nc), dim=-2)
        d *= 2
    return F, c
