"""GPU parity of the reference's public building blocks (noc.par_interior_point_newton,
noc.seq_interior_point_newton, noc.costates) against the oracle restatement (oracle/noc_oracle.py,
torch.func autodiff).  Tolerances (fp64): derivatives / costates / LQ blocks 1e-10 relative;
KKT steps 1e-10; one-stage Newton loops identical iteration counts, iterates 1e-6."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def _case(name, N, B, seed):
    from noc import problems
    from oracle import noc_oracle as O, problems as PR
    if name == "actuated_pendulum":
        from custom_families import actuated_pendulum, actuated_pendulum_torch
        ocp, prob = actuated_pendulum(1.0 / N), O.NumpyProblem(actuated_pendulum_torch(1.0 / N))
        rng = np.random.default_rng(seed)
        x0 = np.array([0.1, -0.1, 0.0]) + 0.01 * rng.normal(size=(B, 3))
        u0 = 0.1 * rng.normal(size=(B, N, 1))
    else:
        ocp = problems.make_problem(name, N)
        prob = O.NumpyProblem(PR.pendulum_ocp(1.0 / N) if name == "pendulum" else PR.cartpole_ocp(1.0 / N))
        x0, u0 = problems.initial_conditions(name, N, B, seed=seed)
    X = np.stack([O.rollout(prob.dynamics, u0[b], x0[b]) for b in range(B)])
    return ocp, prob, x0, u0, X


FAMS = ["pendulum", "cartpole", "actuated_pendulum"]


@pytest.mark.parametrize("name", FAMS)
def test_derivatives_costates_lqr_params(name):
    from noc.par_interior_point_newton import compute_derivatives, compute_lqr_params
    from noc.costates import par_costates, seq_costates
    from oracle import noc_oracle as O
    N, B = 37, 3
    ocp, prob, x0, u0, X = _case(name, N, B, 3)
    bp = np.array([0.1, 0.02, 0.004])
    d = compute_derivatives(ocp, X, u0, bp)
    lp = par_costates(ocp, torch.as_tensor(X[:, -1], device="cuda"), d)
    ls = seq_costates(ocp, X[:, -1], d)
    ru, Q, R, M = compute_lqr_params(ls, d)
    torch.cuda.synchronize()
    for b in range(B):
        ref = prob.derivatives(X[b], u0[b], bp[b])
        for k, r in zip(d._fields, ref):
            assert _rel(getattr(d, k)[b].cpu(), r) < 1e-10, k
        lamT, _ = prob.final_grad_hess(X[b, -1])
        lam = O.seq_costates(lamT, ref[0], ref[5])
        assert _rel(ls[b].cpu(), lam) < 1e-12 and _rel(lp[b].cpu(), lam) < 1e-10
        rr, Qr, Rr, Mr = O.compute_lqr_params(lam, *(ref[i] for i in (1, 2, 3, 4, 6, 7, 8, 9)))
        for got, want in ((ru, rr), (Q, Qr), (R, Rr), (M, Mr)):
            assert _rel(got[b].cpu(), want) < 1e-10
    # unbatched call, the reference signature
    d1 = compute_derivatives(ocp, X[0], u0[0], bp[0])
    assert d1.fx.shape == (N, ocp.family.nx, ocp.family.nx)
    assert torch.equal(d1.fxx, d.fxx[0])


@pytest.mark.parametrize("name", ["pendulum", "cartpole"])
def test_par_newton_and_noc_to_lqt(name):
    """par_Newton (P:107-124: reg = rp ||cu||_F, XT = Q[0]) against the seq Riccati with the same
    blocks; noc_to_lqt's tracking form through par_bwd_pass / par_fwd_pass gives the same step."""
    from noc import lqt
    from noc.par_interior_point_newton import (compute_derivatives, compute_lqr_params,
                                               noc_to_lqt, par_Newton)
    from noc.costates import par_costates
    from oracle import noc_oracle as O
    N, B = 30, 2
    ocp, prob, x0, u0, X = _case(name, N, B, 5)
    d = compute_derivatives(ocp, X, u0, 0.1)
    lam = par_costates(ocp, X[:, -1], d)
    ru, Q, R, M = compute_lqr_params(lam, d)
    rp = 0.7
    dx, du, pred, feas, hu = par_Newton(torch.as_tensor(X, device="cuda"), d, rp, ru, Q, R, M)
    torch.cuda.synchronize()
    for b in range(B):
        reg = rp * float(np.linalg.norm(d.cu[b].cpu().numpy()))
        rdx, rdu, rpred, rfeas = O.kkt_solve(d.fx[b].cpu().numpy(), d.fu[b].cpu().numpy(),
                                             Q[b].cpu().numpy(), R[b].cpu().numpy(),
                                             M[b].cpu().numpy(), ru[b].cpu().numpy(),
                                             Q[b, 0].cpu().numpy(), reg)[:4]
        assert _rel(dx[b].cpu(), rdx) < 1e-10 and _rel(du[b].cpu(), rdu) < 1e-10
        assert abs(pred[b].item() - rpred) <= 1e-10 * max(1.0, abs(rpred))
        assert bool(feas[b]) == bool(rfeas)
    assert torch.equal(hu, ru)
    # the LQT detour of the reference (needs Q invertible, as P:62-66 does)
    for b in range(B):
        reg = rp * torch.linalg.vector_norm(d.cu[b])
        Rr = R[b] + reg * torch.eye(1, dtype=torch.float64, device="cuda")
        L = noc_to_lqt(ru[b], Q[b], Rr, M[b], d.fx[b], d.fu[b])
        Kx, dd, S, v, pr, fe = lqt.par_bwd_pass(L)
        u_l, x_l = lqt.par_fwd_pass(L, torch.zeros(ocp.family.nx, dtype=torch.float64, device="cuda"), Kx, dd)
        torch.cuda.synchronize()
        assert _rel(x_l.cpu(), dx[b].cpu()) < 1e-8 and _rel(u_l.cpu(), du[b].cpu()) < 1e-8


@pytest.mark.parametrize("name", FAMS)
@pytest.mark.parametrize("mode", ["par", "seq"])
def test_newton_oc_single_barrier_stage(name, mode):
    """newton_oc (P:127-225 / S:108-177): one barrier stage from a rollout -> (x, u, iterations)
    identical to the oracle's stage loop."""
    from noc import par_interior_point_newton as PN, seq_interior_point_newton as SN
    from oracle import noc_oracle as O
    N, B = 40, 2
    ocp, prob, x0, u0, X = _case(name, N, B, 7)
    bp = 0.02
    fn = PN.newton_oc if mode == "par" else SN.newton_oc
    Xg, Ug, its = fn(ocp, u0, x0, bp)
    for b in range(B):
        if mode == "par":
            Xr, Ur, itr, _ = O.par_newton_oc(prob, u0[b], x0[b], bp, terminal="stage0")
        else:
            Xr, Ur, itr = O.seq_newton_oc(prob, u0[b], x0[b], bp)
        assert its[b] == itr
        assert np.max(np.abs(Ug[b] - Ur)) < 1e-6 and np.max(np.abs(Xg[b] - Xr)) < 1e-6
    # unbatched: the reference signature
    x1, u1, it1 = fn(ocp, u0[0], x0[0], bp)
    assert u1.shape == (N, 1) and x1.shape == (N + 1, ocp.family.nx) and it1 == its[0]


@pytest.mark.parametrize("name", ["pendulum", "actuated_pendulum"])
def test_seq_solution_bwd_fwd(name):
    """S:98-105 seq_solution = derivatives + seq_costates + lqr params + bwd_pass (Quu += rp I,
    hessian(final_cost)) + fwd_pass, against the oracle's seq_solution."""
    from noc.seq_interior_point_newton import seq_solution, check_feasibility
    from oracle import noc_oracle as O
    N, B = 25, 2
    ocp, prob, x0, u0, X = _case(name, N, B, 11)
    dx, du, dV, feas, ru = seq_solution(ocp, X, u0, 0.1, 0.5)
    torch.cuda.synchronize()
    for b in range(B):
        rdx, rdu, rdV, rfeas, rru = O.seq_solution(prob, X[b], u0[b], 0.1, 0.5)
        assert _rel(dx[b].cpu(), rdx) < 1e-10 and _rel(du[b].cpu(), rdu) < 1e-10
        assert abs(dV[b].item() - rdV) <= 1e-10 * max(1.0, abs(rdV))
        assert bool(feas[b]) == bool(rfeas) and _rel(ru[b].cpu(), rru) < 1e-10
    assert bool(check_feasibility(ocp, X[0], u0[0]))
    assert not bool(check_feasibility(ocp, X[0], u0[0] + 100.0))
