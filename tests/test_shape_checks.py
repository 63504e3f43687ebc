"""Host-side shape validation of the drop-in building blocks (CPU, no kernel is launched).

total_cost, nonlin_rollout (P:87-104 / D:73-90) and the DDP bwd_pass (D:28-70) hand raw device
pointers to their kernels; a caller mistake (states without the terminal row, unbatched gains
beside batched states, a Derivatives field of the wrong horizon) must raise NocError on the host
instead of letting the kernel read or write out of bounds.  The checks run before any array is
moved to the device, so numpy inputs exercise them here without a GPU.
"""
import numpy as np
import pytest

from noc import _lib, problems
from noc import differential_dynamic_programming as ddp_mod
from noc import par_interior_point_newton as par
from noc.optimal_control_problem import Derivatives

N, B = 6, 3


def _cartpole():
    return problems.cartpole(0.05)


def _derivs(nx, nu, batch=None):
    lead = (N,) if batch is None else (batch, N)
    shp = dict(cx=(nx,), cu=(nu,), cxx=(nx, nx), cuu=(nu, nu), cxu=(nx, nu), fx=(nx, nx),
               fu=(nx, nu), fxx=(nx, nx, nx), fuu=(nx, nu, nu), fxu=(nx, nx, nu))
    return Derivatives(*(np.zeros(lead + shp[f]) for f in Derivatives._fields))


@pytest.mark.parametrize("xs,us", [
    ((N, 4), (N, 1)),            # states without the terminal row
    ((N + 1, 3), (N, 1)),        # wrong state dimension
    ((B, N + 1, 4), (N, 1)),     # batched states, unbatched controls
    ((N + 1, 4), (B, N, 1)),     # unbatched states, batched controls
    ((B + 1, N + 1, 4), (B, N, 1)),  # batch sizes disagree
    ((B, N + 1, 4), (B, N, 2)),  # wrong control dimension
])
def test_total_cost_rejects_mis_shaped_inputs(xs, us):
    with pytest.raises(_lib.NocError, match="total_cost"):
        par.total_cost(_cartpole(), np.zeros(xs), np.zeros(us), 0.1)


@pytest.mark.parametrize("Ks,ks,xs,us", [
    ((N, 1, 4), (N, 1), (N + 1, 4), (B, N, 1)),          # unbatched gains, batched controls
    ((B, N, 1, 4), (B, N, 1), (B, N, 4), (B, N, 1)),     # states without the terminal row
    ((B, N, 4, 1), (B, N, 1), (B, N + 1, 4), (B, N, 1)),  # gain transposed
    ((B, N - 1, 1, 4), (B, N, 1), (B, N + 1, 4), (B, N, 1)),  # gain of a shorter horizon
    ((B, N, 1, 4), (B, N), (B, N + 1, 4), (B, N, 1)),    # ffgain without its nu axis
])
def test_nonlin_rollout_rejects_mis_shaped_inputs(Ks, ks, xs, us):
    with pytest.raises(_lib.NocError, match="nonlin_rollout"):
        par.nonlin_rollout(_cartpole(), np.zeros(Ks), np.zeros(ks), np.zeros(xs), np.zeros(us))


@pytest.mark.parametrize("field", list(Derivatives._fields))
def test_ddp_bwd_pass_rejects_any_mis_shaped_derivative(field):
    ocp = _cartpole()
    d = _derivs(4, 1, batch=B)
    bad = np.zeros(getattr(d, field).shape[:-1] + (getattr(d, field).shape[-1] + 1,))
    d = d._replace(**{field: bad})
    with pytest.raises(_lib.NocError, match="bwd_pass"):
        ddp_mod.bwd_pass(ocp, np.zeros((B, 4)), d, 1e-3)


def test_ddp_bwd_pass_rejects_mis_shaped_final_state_and_reg():
    ocp = _cartpole()
    with pytest.raises(_lib.NocError, match="final_state"):
        ddp_mod.bwd_pass(ocp, np.zeros((B, 5)), _derivs(4, 1, batch=B), 1e-3)
    with pytest.raises(_lib.NocError, match="final_state"):
        ddp_mod.bwd_pass(ocp, np.zeros(4), _derivs(4, 1, batch=B), 1e-3)  # unbatched x_N
    with pytest.raises(_lib.NocError, match="reg_param"):
        ddp_mod.bwd_pass(ocp, np.zeros((B, 4)), _derivs(4, 1, batch=B), np.ones(B + 1))


@pytest.mark.parametrize("xs,us", [
    ((N + 1, 4), (B, N, 1)),     # unbatched states, batched controls (N would read as B)
    ((B, N + 1, 4), (N, 1)),     # batched states, unbatched controls
    ((B, N, 4), (B, N, 1)),      # states without the terminal row
    ((B, N + 1, 3), (B, N, 1)),  # wrong state dimension
    ((B, N + 1, 4), (B + 1, N, 1)),  # batch sizes disagree
])
def test_compute_derivatives_rejects_mis_shaped_inputs(xs, us):
    with pytest.raises(_lib.NocError, match="compute_derivatives"):
        par.compute_derivatives(_cartpole(), np.zeros(xs), np.zeros(us), 0.1)


@pytest.mark.parametrize("field", list(Derivatives._fields))
def test_compute_lqr_params_rejects_any_mis_shaped_derivative(field):
    d = _derivs(4, 1, batch=B)
    bad = np.zeros(getattr(d, field).shape[:-1] + (getattr(d, field).shape[-1] + 1,))
    with pytest.raises(_lib.NocError, match="compute_lqr_params"):
        par.compute_lqr_params(np.zeros((B, N + 1, 4)), d._replace(**{field: bad}))


def test_compute_lqr_params_rejects_mis_shaped_lambda():
    for lam in (np.zeros((B, N, 4)), np.zeros((N + 1, 4)), np.zeros((B + 1, N + 1, 4))):
        with pytest.raises(_lib.NocError, match="compute_lqr_params"):
            par.compute_lqr_params(lam, _derivs(4, 1, batch=B))


def test_well_shaped_inputs_pass_the_host_checks():
    """Correct shapes get past the checks: the next thing that happens is the device transfer,
    which on a CPU-only host raises for the missing GPU, never a shape error."""
    ocp = _cartpole()
    calls = [
        lambda: par.total_cost(ocp, np.zeros((B, N + 1, 4)), np.zeros((B, N, 1)), 0.1),
        lambda: par.nonlin_rollout(ocp, np.zeros((N, 1, 4)), np.zeros((N, 1)), np.zeros((N + 1, 4)),
                                   np.zeros((N, 1))),
        lambda: ddp_mod.bwd_pass(ocp, np.zeros(4), _derivs(4, 1), 1e-3),
        lambda: par.compute_derivatives(ocp, np.zeros((B, N + 1, 4)), np.zeros((B, N, 1)), 0.1),
        lambda: par.compute_lqr_params(np.zeros((N + 1, 4)), _derivs(4, 1)),
    ]
    for call in calls:
        try:
            call()
        except _lib.NocError as e:
            assert "mis-shaped" not in str(e) and "must be" not in str(e), e
        except (RuntimeError, AssertionError, OSError):
            pass  # no GPU / no HIP runtime here: past the shape checks
