"""GPU parity against the COMMITTED golden fixtures (tests/golden/*.npz), no live oracle.

golden_v1.npz (tests/golden/make_golden.py: lq_fixtures, ipm_fixtures):
  lq_<nx>x<nu>_N<N>_{newton,aff}: random LQ problems and their KKT steps (symmetrised seq Riccati,
  cross-checked against the dense KKT solve at generation time); cart20: one cart-pole
  linearisation (P:13-42) at a random iterate; pend50: the whole par / seq interior-point solves
  of BASELINE config c1 (pendulum N=50, terminal = hessian(final_cost)).
golden_v2.npz (newton_block_fixtures): the real first-Newton-step LQ blocks of the c2 (pendulum
  N=100) and c3 (cart-pole N=200) problems and their KKT steps by the FAITHFUL sequential Riccati
  of S:42-90 (Vxx unsymmetrised, inv(Quu)).

Tolerances (fp64, stated): KKT outputs 1e-10 max-relative, identical `feasible`; linearisation
blocks 1e-10; whole solves: identical iteration / KKT-solve counts, controls 1e-6 absolute.
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu
RTOL = 1e-10
HERE = os.path.dirname(os.path.abspath(__file__))


def _load(name):
    return np.load(os.path.join(HERE, "golden", name), allow_pickle=False)


def dev(x):
    return None if x is None else torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64,
                                                  device="cuda")


def relerr(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


LQ_TAGS = [f"lq_{nx}x{nu}_N{N}_{kind}" for nx, nu, N in [(2, 1, 50), (4, 1, 120), (8, 4, 48)]
           for kind in ("newton", "aff")]


@pytest.mark.parametrize("tag", LQ_TAGS)
@pytest.mark.parametrize("lanes", [64, 32, 8, 1])
def test_kkt_matches_committed_lq_fixtures(tag, lanes):
    from noc import lqt
    g = _load("golden_v1.npz")
    inp = lambda k: dev(g[f"{tag}/in/{k}"]) if f"{tag}/in/{k}" in g.files else None
    out = lambda k: g[f"{tag}/out/{k}"]
    res = lqt.kkt_solve(inp("A"), inp("B"), inp("Q"), inp("R"), inp("M"), inp("r"), inp("P"),
                        reg=inp("reg"), x0=inp("x0"), q=inp("q"), c=inp("c"), p=inp("p"),
                        lanes=lanes, want_value=True)
    torch.cuda.synchronize()
    for k in ("dx", "du", "K", "d", "S", "v", "pred"):
        got = getattr(res, k).cpu().numpy()
        assert relerr(got, out(k)) < RTOL, (k, relerr(got, out(k)))
    assert np.array_equal(res.feasible.cpu().numpy().astype(bool), out("feasible").astype(bool))


@pytest.mark.parametrize("tag", ["pend100", "cart200"])
@pytest.mark.parametrize("lanes", [0, 64, 32, 16])
def test_kkt_matches_faithful_seq_riccati_on_real_newton_blocks(tag, lanes):
    """The c2 / c3 problems' real Newton blocks (golden_v2) through noc_kkt_solve: dx, du, K, d,
    pred against the faithful S:42-90 restatement's committed outputs."""
    from noc import lqt
    g = _load("golden_v2.npz")
    f = lambda k: g[f"{tag}/{k}"]
    res = lqt.kkt_solve(*(dev(f(k)) for k in ("A", "B", "Q", "R", "M", "r", "P")),
                        reg=dev(f("reg")), lanes=lanes)
    torch.cuda.synchronize()
    for k in ("dx", "du", "K", "d", "pred"):
        got = getattr(res, k).cpu().numpy()
        assert relerr(got, f(k)) < RTOL, (k, relerr(got, f(k)))
    assert np.array_equal(res.feasible.cpu().numpy().astype(bool), f("feasible").astype(bool))


@pytest.mark.parametrize("tag,name,N", [("pend100", "pendulum", 100), ("cart200", "cartpole", 200)])
@pytest.mark.parametrize("lanes", [64, 32])
def test_device_linearisation_and_fused_step_match_committed_fixtures(tag, name, N, lanes):
    """Rollout + linearisation + costates + LQ blocks on the device (BatchedIPM.prepare, the
    P:133-153 path) from the fixture's (u0, x0), then the tiled KKT solve the interior-point
    loop runs: blocks, reg = ||cu||_F and the step against the committed vectors."""
    from noc import lqt, problems, _lib
    from noc.ipm import BatchedIPM
    g = _load("golden_v2.npz")
    f = lambda k: g[f"{tag}/{k}"]
    ocp = problems.make_problem(name, N)
    eng = BatchedIPM(ocp.family, N, 2, lanes=lanes)
    eng.load(f("u0"), f("x0"))
    eng.init(bp0=0.1)
    eng.prepare(mode=_lib.MODE_PAR, terminal=_lib.TERMINAL_FINAL_COST)
    nat = eng.natural_blocks()
    torch.cuda.synchronize()
    assert relerr(eng.t["x"].cpu().numpy(), f("x")) < 1e-12
    for k in ("A", "B", "Q", "R", "M", "r", "P"):
        assert relerr(nat[k].cpu().numpy(), f(k)) < RTOL, (k, relerr(nat[k].cpu().numpy(), f(k)))
    assert relerr(eng.t["reg"].cpu().numpy(), f("reg")) < 1e-12
    res = lqt.kkt_solve_tiled(eng.tiled_blocks(), reg=eng.t["reg"], want_gains=False)
    torch.cuda.synchronize()
    for k in ("dx", "du", "pred"):
        got = getattr(res, k).cpu().numpy()
        assert relerr(got, f(k)) < RTOL, (k, relerr(got, f(k)))


def test_cartpole_linearisation_matches_committed_cart20():
    from noc import problems, _lib
    from noc.ipm import BatchedIPM
    g = _load("golden_v1.npz")
    f = lambda k: g[f"cart20/{k}"]
    N = 20
    eng = BatchedIPM(problems.cartpole(1.0 / N).family, N, 1, lanes=64)
    eng.load(f("u")[None], f("x")[0][None])
    eng.init(bp0=0.1)
    eng.prepare(mode=_lib.MODE_PAR, terminal=_lib.TERMINAL_FINAL_COST)
    nat = eng.natural_blocks()
    torch.cuda.synchronize()
    assert relerr(eng.t["x"][0].cpu().numpy(), f("x")) < 1e-12
    for k in ("A", "B", "Q", "R", "M", "r", "P"):
        assert relerr(nat[k][0].cpu().numpy(), f(k)) < RTOL, k
    assert relerr(eng.t["lam"][0].cpu().numpy(), f("lam")) < RTOL
    assert abs(eng.t["cost"][0].item() - float(f("cost"))) <= 1e-12 * abs(float(f("cost")))
    assert abs(eng.t["gnorm"][0].item() - np.linalg.norm(f("cu"))) <= 1e-12 * np.linalg.norm(f("cu"))


def test_pendulum_solves_match_committed_pend50():
    """BASELINE c1 (pendulum N=50, B=1): par (terminal = hessian(final_cost), as the fixture) and
    seq solves against the committed iteration counts and controls."""
    from noc import problems
    from noc.par_interior_point_newton import par_interior_point_optimal_control
    from noc.seq_interior_point_newton import seq_interior_point_optimal_control
    g = _load("golden_v1.npz")
    f = lambda k: g[f"pend50/{k}"]
    ocp = problems.pendulum(1.0 / 50)
    U, it, info = par_interior_point_optimal_control(ocp, f("u0"), f("x0"), terminal="final_cost",
                                                     return_info=True)
    assert it == int(f("par_iters")) and info["kkt_solves"] == int(f("par_kkt_solves"))
    assert np.max(np.abs(U - f("par_u"))) < 1e-6
    Us, its = seq_interior_point_optimal_control(ocp, f("u0"), f("x0"))
    assert its == int(f("seq_iters"))
    assert np.max(np.abs(Us - f("seq_u"))) < 1e-6
