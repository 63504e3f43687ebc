"""GPU parity of a family registered at run time (noc.families.register_family; the family
library is pre-built by __graft_entry__.build()): the actuated pendulum of
tests/custom_families.py -- nx = 3, nu = 1, a KKT shape the default library does not have.
Oracle: the same problem restated in torch with torch.func autodiff (oracle/noc_oracle.py loops).
Tolerances as tests/test_ipm_gpu.py: blocks 1e-10 relative; solves identical iteration and
KKT-solve counts, controls 1e-6; KKT step 1e-10."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from custom_families import actuated_pendulum, actuated_pendulum_torch  # noqa: E402
from lq_cases import rand_lq, oracle_batch  # noqa: E402

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def _inputs(N, B, seed):
    rng = np.random.default_rng(seed)
    x0 = np.array([0.1, -0.1, 0.0]) + 0.01 * rng.normal(size=(B, 3))
    u0 = 0.1 * rng.normal(size=(B, N, 1))
    return x0, u0


@pytest.mark.parametrize("lanes", [64, 16])
def test_custom_family_linearisation_matches_autodiff(lanes):
    from noc import _lib
    from noc.ipm import BatchedIPM
    from oracle import noc_oracle as O
    N, B = 50, 3
    ocp = actuated_pendulum(1.0 / N)
    x0, u0 = _inputs(N, B, 5)
    eng = BatchedIPM(ocp.family, N, B, lanes=lanes)
    eng.load(u0, x0)
    eng.init(bp0=0.1)
    eng.prepare(mode=_lib.MODE_PAR, terminal=_lib.TERMINAL_FINAL_COST)
    nat = eng.natural_blocks()
    torch.cuda.synchronize()
    prob = O.NumpyProblem(actuated_pendulum_torch(1.0 / N))
    X = eng.t["x"].cpu().numpy()
    for b in range(B):
        assert _rel(X[b], O.rollout(prob.dynamics, u0[b], x0[b])) < 1e-12
        L = O.linearize(prob, X[b], u0[b], 0.1)
        for k in ("A", "B", "Q", "R", "M", "r", "P"):
            assert _rel(nat[k][b].cpu().numpy(), L[k]) < 1e-10, k
        cost = prob.total_cost(X[b], u0[b], 0.1)
        assert abs(eng.t["cost"][b].item() - cost) <= 1e-12 * abs(cost)


@pytest.mark.parametrize("mode", ["par", "seq"])
def test_custom_family_solve_matches_oracle(mode):
    from noc.par_interior_point_newton import par_interior_point_optimal_control
    from noc.seq_interior_point_newton import seq_interior_point_optimal_control
    from oracle import noc_oracle as O
    N = 40
    ocp = actuated_pendulum(1.0 / N)
    x0, u0 = _inputs(N, 2, 9)
    prob = O.NumpyProblem(actuated_pendulum_torch(1.0 / N))
    if mode == "par":
        U, its, info = par_interior_point_optimal_control(ocp, u0, x0, return_info=True)
    else:
        U, its = seq_interior_point_optimal_control(ocp, u0, x0)
    for b in range(2):
        if mode == "par":
            Ur, itr, sr = O.par_interior_point_optimal_control(prob, u0[b], x0[b], terminal="stage0")
            assert info["kkt_solves"][b] == sr
        else:
            Ur, itr = O.seq_interior_point_optimal_control(prob, u0[b], x0[b])
        assert its[b] == itr
        assert np.max(np.abs(U[b] - Ur)) < 1e-6


def test_custom_family_persistent_equals_multilaunch_and_ddp_runs():
    from noc import _lib
    from noc.ipm import BatchedIPM
    from noc.differential_dynamic_programming import interior_point_ddp
    N, B = 60, 8
    ocp = actuated_pendulum(1.0 / N)
    x0, u0 = _inputs(N, B, 13)
    res = []
    for persistent in (True, False):
        eng = BatchedIPM(ocp.family, N, B, lanes=64, persistent=persistent)
        eng.load(u0, x0)
        eng.solve()
        torch.cuda.synchronize()
        res.append([t.cpu().numpy() for t in eng.result()] + [eng.t["phase"].cpu().numpy()])
    (Up, itp, sp, php), (Um, itm, sm, phm) = res
    assert np.all(php == _lib.PHASE_DONE) and np.array_equal(itp, itm) and np.array_equal(sp, sm)
    assert np.max(np.abs(Up - Um)) <= 1e-12 * max(1.0, float(np.max(np.abs(Um))))
    U, its, info = interior_point_ddp(ocp, u0, x0, return_info=True)
    assert info["done"].all() and np.all(np.isfinite(U))


@pytest.mark.parametrize("lanes", [64, 32, 8])
def test_kkt_solve_on_the_custom_shape(lanes):
    """lqt.kkt_solve on (nx, nu) = (3, 1) routes to the family's build (for_shape)."""
    from noc import lqt, _lib
    actuated_pendulum(0.02)
    _lib.load_for(actuated_pendulum(0.02).family)
    case = rand_lq(31 + lanes, 4, 45, 3, 1, affine=True)
    ref = oracle_batch(case)
    dev = lambda k: None if k not in case else torch.as_tensor(case[k], dtype=torch.float64, device="cuda")
    out = lqt.kkt_solve(*(dev(k) for k in ("A", "B", "Q", "R", "M", "r", "P")), reg=dev("reg"),
                        x0=dev("x0"), q=dev("q"), c=dev("c"), p=dev("p"), lanes=lanes,
                        want_value=True)
    torch.cuda.synchronize()
    for k in ("dx", "du", "K", "d", "S", "v", "pred"):
        assert _rel(getattr(out, k).cpu().numpy(), ref[k]) < 1e-10, k


# ------------------------------------------------------------------------------------------------
# a family with the reference OCP's own kind of callables: traced stage / final costs (a quartic
# term) and a STATE constraint (cart within +-X_LIMIT) inside the log barrier
# ------------------------------------------------------------------------------------------------
def _tl_inputs(N, B, seed):
    from noc import problems
    return problems.initial_conditions("cartpole", N, B, seed=seed)


def test_traced_cost_linearisation_matches_autodiff():
    """compute_derivatives (P:13-28) of the traced costs: every derivative array of the
    Derivatives type (cx, cu, cxx, cuu, cxu) and the LQ blocks against torch.func on the torch
    restatement, at 1e-10; the final-cost gradient / Hessian; the total cost."""
    from noc import _lib
    from noc.ipm import BatchedIPM
    from noc.par_interior_point_newton import compute_derivatives
    from oracle import noc_oracle as O
    import custom_families as CF
    N, B = 50, 3
    ocp = CF.cartpole_track_limit(1.0 / N)
    x0, u0 = _tl_inputs(N, B, 3)
    eng = BatchedIPM(ocp.family, N, B, lanes=64)
    eng.load(u0, x0)
    eng.init(bp0=0.1)
    eng.prepare(mode=_lib.MODE_PAR, terminal=_lib.TERMINAL_FINAL_COST)
    nat = eng.natural_blocks()
    torch.cuda.synchronize()
    prob = O.NumpyProblem(CF.cartpole_track_limit_torch(1.0 / N))
    X = eng.t["x"].cpu().numpy()
    d = compute_derivatives(ocp, X, u0, 0.1)
    for b in range(B):
        assert _rel(X[b], O.rollout(prob.dynamics, u0[b], x0[b])) < 1e-12
        ref = prob.derivatives(X[b], u0[b], 0.1)
        for k, got in enumerate(d):
            assert _rel(got[b].cpu().numpy(), ref[k]) < 1e-10, k
        L = O.linearize(prob, X[b], u0[b], 0.1)
        for k in ("A", "B", "Q", "R", "M", "r", "P"):
            assert _rel(nat[k][b].cpu().numpy(), L[k]) < 1e-10, k
        cost = prob.total_cost(X[b], u0[b], 0.1)
        assert abs(eng.t["cost"][b].item() - cost) <= 1e-12 * abs(cost)
        assert abs(ocp.total_cost(X[b], u0[b], 0.1) - cost) <= 1e-12 * abs(cost)


def test_traced_cost_state_constraint_solve_matches_oracle():
    """The whole par interior-point solve (P:228-254, persistent kernel) of the track-limited
    cart-pole: identical outer iterations and KKT solves per trajectory as the oracle loop on the
    torch restatement, controls within 1e-6; the state constraint holds on the solver's states
    and is active (the cart reaches the limit: the swing-up wants more track)."""
    from noc.par_interior_point_newton import par_interior_point_optimal_control
    from oracle import noc_oracle as O
    import custom_families as CF
    N, B = 50, 2
    ocp = CF.cartpole_track_limit(1.0 / N)
    x0, u0 = _tl_inputs(N, B, 3)
    U, its, info = par_interior_point_optimal_control(ocp, u0, x0, return_info=True)
    prob = O.NumpyProblem(CF.cartpole_track_limit_torch(1.0 / N))
    for b in range(B):
        Ur, itr, sr = O.par_interior_point_optimal_control(prob, u0[b], x0[b], terminal="stage0")
        assert its[b] == itr and info["kkt_solves"][b] == sr, (b, its[b], itr, info["kkt_solves"][b], sr)
        assert np.max(np.abs(U[b] - Ur)) < 1e-6


def test_traced_cost_state_constraint_active_and_respected():
    """On the solver's own states (x + dx of the kept steps, P:184) the trial feasibility test
    (P:45-47, with the state constraint) held at every accepted step: |cart| <= X_LIMIT, and the
    optimum presses against it.  The multi-launch loop gives the same iterates."""
    from noc import _lib
    from noc.ipm import BatchedIPM
    import custom_families as CF
    N, B = 50, 4
    ocp = CF.cartpole_track_limit(1.0 / N)
    x0, u0 = _tl_inputs(N, B, 3)
    res = []
    for persistent in (True, False):
        eng = BatchedIPM(ocp.family, N, B, lanes=64, persistent=persistent)
        eng.load(u0, x0)
        eng.solve()
        torch.cuda.synchronize()
        res.append([t.cpu().numpy() for t in eng.result()] + [eng.t["x"].cpu().numpy()])
    (Up, itp, sp, Xp), (Um, itm, sm, Xm) = res
    assert np.array_equal(itp, itm) and np.array_equal(sp, sm)
    assert np.max(np.abs(Up - Um)) <= 1e-12 * max(1.0, float(np.max(np.abs(Um))))
    xc = np.abs(Xp[:, :-1, 0])
    assert np.all(xc <= CF.X_LIMIT) and np.all(xc.max(axis=1) > 0.9 * CF.X_LIMIT)


def test_traced_cost_family_ddp_matches_oracle():
    """Interior-point DDP (D:28-208) on the traced-cost, state-constrained cart-pole: the DDP
    record carries the stage cost's full Hessian (cxx, cuu, cxu, D:43-45) from the generated
    code, so a registered family's own cost runs through DDP too.  Against the oracle DDP on the
    torch restatement (torch.func derivatives): as tests/test_ddp.py -- iterations and backward
    passes within one, controls 1e-5, cost 1e-9 relative; the state constraint holds."""
    from noc.differential_dynamic_programming import interior_point_ddp
    from oracle import noc_oracle as O
    import custom_families as CF
    N, B = 30, 2
    ocp = CF.cartpole_track_limit(1.0 / N)
    x0, u0 = _tl_inputs(N, B, 5)
    U, its, info = interior_point_ddp(ocp, u0, x0, return_info=True)
    assert info["done"].all()
    prob = O.NumpyProblem(CF.cartpole_track_limit_torch(1.0 / N))
    for b in range(B):
        Ur, itr, pr = O.interior_point_ddp(prob, u0[b], x0[b])
        assert abs(int(its[b]) - itr) <= 1, (b, int(its[b]), itr)
        assert abs(int(info["passes"][b]) - pr) <= 1, (b, int(info["passes"][b]), pr)
        assert np.max(np.abs(U[b] - Ur)) < 1e-5, b
        X = O.rollout(prob.dynamics, U[b], x0[b])
        c = prob.total_cost(X, U[b], 0.8e-4)
        cr = prob.total_cost(O.rollout(prob.dynamics, Ur, x0[b]), Ur, 0.8e-4)
        assert abs(c - cr) <= 1e-9 * max(1.0, abs(cr)), b
        assert np.all(np.abs(X[:-1, 0]) <= CF.X_LIMIT)


def test_traced_cost_family_supports_ddp_and_rejects_mixed_costs():
    from noc import _lib
    from noc import families
    import custom_families as CF
    ocp = CF.cartpole_track_limit(1.0 / 50)
    lib = _lib.load_for(ocp.family)
    import ctypes
    assert lib.noc_ddp_supported(ctypes.byref(ocp.family.to_c())) == 1
    with pytest.raises(_lib.NocError):
        families.register_family("bad", CF.cartpole_ode, 4, 1, dt=0.02,
                                 stage_cost=CF.track_limit_stage_cost, build=False)
    with pytest.raises(_lib.NocError):
        families.register_family("bad", CF.cartpole_ode, 4, 1, dt=0.02, wx=[1.0] * 4,
                                 stage_cost=CF.track_limit_stage_cost,
                                 final_cost=CF.track_limit_final_cost, build=False)


def _host_feasible(ocp, X, U):
    """P:45-47 evaluated with the OCP's own host callables: all(constraints(x_k, u_k) <= 0), k < N."""
    return bool(all(np.all(np.asarray(ocp.constraints(X[k], U[k])) <= 0) for k in range(len(U))))


def test_check_traj_feasibility_state_constraint():
    """check_traj_feasibility / check_feasibility (P:45-47, S:93-95) evaluate the family's whole
    constraint vector on the device (noc_check_feasibility): a state beyond X_LIMIT is infeasible,
    the solver's own states are feasible -- batched and unbatched, equal to the OCP's host
    callables; a u beyond the box and a NaN state are infeasible; x_N is not tested (x[:-1])."""
    from noc.ipm import BatchedIPM
    from noc.par_interior_point_newton import check_traj_feasibility
    from noc.seq_interior_point_newton import check_feasibility
    import custom_families as CF
    N, B = 50, 4
    ocp = CF.cartpole_track_limit(1.0 / N)
    x0, u0 = _tl_inputs(N, B, 3)
    eng = BatchedIPM(ocp.family, N, B, lanes=64, persistent=True)
    eng.load(u0, x0)
    eng.solve()
    torch.cuda.synchronize()
    U, X = eng.result()[0].cpu().numpy(), eng.t["x"].cpu().numpy()
    cases = [X.copy() for _ in range(4)]
    cases[1][1, 17, 0] = CF.X_LIMIT + 1e-3       # cart beyond the track limit
    cases[2][2, 0, 0] = -(CF.X_LIMIT + 0.25)     # at stage 0
    cases[3][3, 9, 2] = np.nan                   # NaN compares false
    Uc = [U.copy() for _ in range(4)]
    Uc[0][0, N - 1, 0] = 50.5                    # the u box, last stage
    tail = X.copy()
    tail[:, N, 0] = 10.0                         # x_N is outside x[:-1]: still feasible
    for Xc, Ucase in list(zip(cases, Uc)) + [(tail, U)]:
        want = np.array([_host_feasible(ocp, Xc[b], Ucase[b]) for b in range(B)])
        for fn in (check_traj_feasibility, check_feasibility):
            got = fn(ocp, Xc, Ucase).cpu().numpy()
            assert got.dtype == np.bool_ and np.array_equal(got, want), (got, want)
            for b in range(B):
                one = fn(ocp, Xc[b], Ucase[b])
                assert one.dim() == 0 and bool(one) == want[b]
    assert np.all(np.array([_host_feasible(ocp, X[b], U[b]) for b in range(B)]))
    assert not _host_feasible(ocp, cases[1][1], U[1])


def test_check_traj_feasibility_builtin_box():
    """The built-ins' constraint is the u box (|u| <= u_bound): the device verdict equals the host
    callables' at random feasible / infeasible controls, for the pendulum and cart-pole."""
    from noc import problems
    from noc.par_interior_point_newton import check_traj_feasibility
    rng = np.random.default_rng(7)
    for name, ocp, N in (("pendulum", problems.pendulum(0.01), 100),
                         ("cartpole", problems.cartpole(0.005), 200)):
        B = 70
        x0, u = problems.initial_conditions(name, N, B, seed=4)
        X = rng.normal(size=(B, N + 1, ocp.family.nx))
        ub = ocp.family.u_bound
        u = np.clip(u, -0.9 * ub, 0.9 * ub)
        hit = rng.integers(0, N, size=B)
        for b in range(0, B, 3):
            u[b, hit[b], 0] = (1 if b % 2 else -1) * ub * 1.0001
        want = np.array([_host_feasible(ocp, X[b], u[b]) for b in range(B)])
        assert 0 < want.sum() < B
        assert np.array_equal(check_traj_feasibility(ocp, X, u).cpu().numpy(), want)
