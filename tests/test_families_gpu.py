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
