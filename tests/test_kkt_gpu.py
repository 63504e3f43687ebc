"""GPU parity of the batched KKT scan (libnoc_hip.so) against the numpy oracle.

Oracle: oracle/noc_oracle.kkt_solve, the restatement of seq_interior_point_newton bwd_pass /
fwd_pass (noc/seq_interior_point_newton.py:42-90).  Tolerance (stated, fp64): max relative error
1e-10 on dx, du, K, d, S, v and pred; `feasible` identical.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from lq_cases import rand_lq, oracle_batch  # noqa: E402

pytestmark = pytest.mark.gpu
RTOL = 1e-10


def dev(x):
    return None if x is None else torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64,
                                                  device="cuda")


def relerr(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def run_kkt(case, lanes, want_value=True):
    from noc import lqt
    g = lambda k: dev(case.get(k))
    res = lqt.kkt_solve(g("A"), g("B"), g("Q"), g("R"), g("M"), g("r"), g("P"), reg=g("reg"),
                        x0=g("x0"), q=g("q"), c=g("c"), p=g("p"), lanes=lanes,
                        want_value=want_value)
    torch.cuda.synchronize()
    return {k: (None if v is None else v.cpu().numpy()) for k, v in res._asdict().items()}


@pytest.mark.parametrize("nx,nu", [(2, 1), (4, 1), (8, 4)])
@pytest.mark.parametrize("lanes", [128, 64, 32, 16, 8, 1])
@pytest.mark.parametrize("N", [1, 7, 50, 200])
@pytest.mark.parametrize("affine", [False, True])
def test_kkt_matches_oracle(nx, nu, lanes, N, affine):
    """lanes 64..8: parallel-in-time scan in one wave; 128: two waves per trajectory joined
    through LDS (nx <= 4); lanes 1: horizon-sequential nx-lane group solve."""
    if lanes == 128 and nx == 8:
        pytest.skip("two-wave segments are instantiated for nx <= 4 (test_two_wave_nx8_rejected)")
    case = rand_lq(1000 * nx + N + lanes + int(affine), 5, N, nx, nu, affine=affine)
    ref = oracle_batch(case)
    out = run_kkt(case, lanes)
    for k in ["dx", "du", "K", "d", "S", "v"]:
        assert relerr(out[k], ref[k]) < RTOL, (k, relerr(out[k], ref[k]))
    assert relerr(out["pred"], ref["pred"]) < RTOL
    assert np.array_equal(out["feasible"].astype(bool), ref["feasible"].astype(bool))


def test_two_wave_nx8_rejected():
    """lanes = 128 is not instantiated for nx = 8: an error, not a silent fallback."""
    from noc import lqt, _lib
    case = rand_lq(8, 2, 20, 8, 4)
    g = lambda k: dev(case.get(k))
    with pytest.raises(_lib.NocError):
        lqt.kkt_solve(g("A"), g("B"), g("Q"), g("R"), g("M"), g("r"), g("P"), reg=g("reg"),
                      lanes=128)


@pytest.mark.parametrize("lanes", [64, 128])
def test_kkt_infeasible_flag(lanes):
    case = rand_lq(7, 4, 30, 4, 1)
    case["R"][1, 10] = -50.0   # Quu < 0 at stage 10 of trajectory 1
    case["R"][3, 29] = -50.0
    ref = oracle_batch(case)
    out = run_kkt(case, lanes)
    assert list(out["feasible"]) == [1, 0, 1, 0]
    assert list(ref["feasible"].astype(int)) == [1, 0, 1, 0]
    ok = [0, 2]
    assert relerr(out["dx"][ok], ref["dx"][ok]) < RTOL


@pytest.mark.parametrize("lanes", [0, 1, 32, 64, 128])
def test_kkt_active_mask_leaves_inactive_untouched(lanes):
    from noc import lqt
    case = rand_lq(11, 6, 40, 4, 1)
    g = lambda k: dev(case.get(k))
    Bt, N = 6, 40
    out = lqt.KKTResult(*(torch.full(s, 7.0, dtype=torch.float64, device="cuda") for s in
                          [(Bt, N + 1, 4), (Bt, N, 1), (Bt,)]),
                        torch.full((Bt,), 7, dtype=torch.int32, device="cuda"),
                        torch.zeros(Bt, N, 1, 4, dtype=torch.float64, device="cuda"),
                        torch.zeros(Bt, N, 1, dtype=torch.float64, device="cuda"), None, None)
    active = torch.tensor([1, 0, 1, 0, 0, 1], dtype=torch.int32, device="cuda")
    lqt.kkt_solve(g("A"), g("B"), g("Q"), g("R"), g("M"), g("r"), g("P"), reg=g("reg"),
                  active=active, out=out, lanes=lanes)
    torch.cuda.synchronize()
    ref = oracle_batch(case)
    dx = out.dx.cpu().numpy()
    for b in range(Bt):
        if active[b]:
            assert relerr(dx[b], ref["dx"][b]) < RTOL
        else:
            assert np.all(dx[b] == 7.0) and out.pred[b].item() == 7.0


@pytest.mark.parametrize("nx,nu", [(2, 1), (4, 1), (8, 4)])
@pytest.mark.parametrize("bwd_lanes,fwd_lanes", [(16, 32), (1, 1), (1, 64), (8, 1), (128, 64),
                                               (64, 128), (128, 128)])
def test_split_bwd_fwd_entry_points(nx, nu, bwd_lanes, fwd_lanes):
    """par_bwd_pass / par_fwd_pass split; the scan and the group solve interoperate through K, d."""
    from noc import lqt
    if nx == 8 and 128 in (bwd_lanes, fwd_lanes):
        pytest.skip("two-wave segments are instantiated for nx <= 4")
    case = rand_lq(5 + nx, 3, 37, nx, nu, affine=True)
    g = lambda k: dev(case.get(k))
    ref = oracle_batch(case)
    K, d, S, v, pred, feas = lqt.bwd_pass(g("A"), g("B"), g("Q"), g("R"), g("M"), g("r"), g("P"),
                                          reg=g("reg"), q=g("q"), c=g("c"), p=g("p"),
                                          lanes=bwd_lanes)
    du, dx = lqt.fwd_pass(g("A"), g("B"), K, d, x0=g("x0"), c=g("c"), lanes=fwd_lanes)
    torch.cuda.synchronize()
    assert relerr(K.cpu(), ref["K"]) < RTOL
    assert relerr(S.cpu(), ref["S"]) < RTOL
    assert relerr(v.cpu(), ref["v"]) < RTOL
    assert relerr(pred.cpu(), ref["pred"]) < RTOL
    assert relerr(dx.cpu(), ref["dx"]) < RTOL
    assert relerr(du.cpu(), ref["du"]) < RTOL


def test_lqt_tracking_form_adapter():
    """paroc LQT (LM:64) -> canonical -> HIP; compare with the oracle on the expanded form."""
    from noc import lqt
    from oracle import noc_oracle as O
    rng = np.random.default_rng(3)
    N, nx, nu = 25, 4, 1
    case = rand_lq(3, 1, N, nx, nu)
    H = np.eye(nx) + 0.1 * rng.normal(size=(N, nx, nx))
    Z = np.ones((N, nu, nu))
    rr = rng.normal(size=(N, nx))
    ss = rng.normal(size=(N, nu))
    X, U, Mt = case["Q"][0], case["R"][0], case["M"][0]
    XT, HT, rT = case["P"][0], np.eye(nx), rng.normal(size=nx)
    c = 0.1 * rng.normal(size=(N, nx))
    x0 = rng.normal(size=nx)
    L = lqt.LQT(*(dev(t) for t in (case["A"][0], case["B"][0], c, XT, HT, rT, X, H, rr, U, Z, ss, Mt)))
    Kx, d, S, v, pred, feas = lqt.par_bwd_pass(L)
    u, x = lqt.par_fwd_pass(L, dev(x0), Kx, d)
    # expanded canonical form on the host
    Q = np.einsum("kji,kjl,klm->kim", H, X, H)
    M = np.einsum("kji,kjl,klm->kim", H, Mt, Z)
    R = np.einsum("kji,kjl,klm->kim", Z, U, Z)
    q = -np.einsum("kji,kj->ki", H, np.einsum("kij,kj->ki", X, rr) + np.einsum("kij,kj->ki", Mt, ss))
    r = -np.einsum("kji,kj->ki", Z, np.einsum("kij,kj->ki", U, ss) + np.einsum("kji,kj->ki", Mt, rr))
    P = HT.T @ XT @ HT
    p = -HT.T @ XT @ rT
    ddx, ddu, _ = O.dense_kkt(case["A"][0], case["B"][0], Q, R, M, r, P, 0.0, x0, q, c, p)
    torch.cuda.synchronize()
    assert relerr(x.cpu(), ddx) < 1e-9
    assert relerr(u.cpu(), ddu) < 1e-9
    assert bool(feas)


@pytest.mark.parametrize("nx,nu,lanes", [(nx, nu, L) for nx, nu in [(2, 1), (4, 1), (8, 4)]
                                          for L in (64, 32, 16, 8)] + [(8, 4, 1), (2, 1, 128),
                                                                       (4, 1, 128)])
@pytest.mark.parametrize("N", [1, 13, 200])
def test_tiled_layout_kkt_matches_oracle(nx, nu, lanes, N):
    """The tiled layout the IPM workspace uses: lane-interleaved for the scan (lanes 8-64),
    grouped records of 8 trajectories for the group solve (lanes 1); Q/R packed."""
    from noc import lqt
    case = rand_lq(77 * nx + N + lanes, 5, N, nx, nu)
    ref = oracle_batch(case)
    g = lambda k: dev(case[k])
    tb = lqt.to_tiled(g("A"), g("B"), g("Q"), g("R"), g("M"), g("r"), g("P"), lanes)
    out = lqt.kkt_solve_tiled(tb, reg=g("reg"), want_value=True)
    torch.cuda.synchronize()
    for k in ["dx", "du", "S", "v", "pred"]:
        assert relerr(getattr(out, k).cpu(), ref[k]) < RTOL, k
    K = lqt.untile(out.K, (5, N, nu, nx), lanes)
    d = lqt.untile(out.d, (5, N, nu), lanes)
    assert relerr(K.cpu(), ref["K"]) < RTOL and relerr(d.cpu(), ref["d"]) < RTOL
    assert np.array_equal(out.feasible.cpu().numpy().astype(bool), ref["feasible"].astype(bool))


@pytest.mark.parametrize("lanes", [128, 64, 16, 1])
def test_tile_untile_roundtrip(lanes):
    from noc import lqt
    rng = np.random.default_rng(0)
    for shape, sym in [((3, 37, 4, 4), False), ((3, 37, 4, 1), False), ((3, 37, 1), False),
                       ((3, 37, 8, 8), True), ((2, 5, 2, 2), True)]:
        x = rng.normal(size=shape)
        if sym:
            x = x + np.swapaxes(x, -1, -2)
        t = dev(x)
        back = lqt.untile(lqt.tile(t, lanes, sym=sym), shape, lanes, sym=sym)
        assert torch.equal(back.cpu(), torch.as_tensor(x))


def test_cartpole_blocks_full_size_properties():
    """BASELINE config c3 size (N=200, B=4096): realistic cart-pole Newton blocks produced by the
    device linearisation in the tiled layout.  Checks (size-independent): dynamics consistency
    dx_{k+1} = A dx_k + B du_k on all trajectories, oracle parity on a strided sample of 16
    trajectories, all feasible, and tiled == natural-layout solve."""
    from noc import lqt
    from noc.problems import make_bench_blocks
    blocks = make_bench_blocks("cartpole", N=200, batch=4096, seed=0, natural=True)
    res = lqt.kkt_solve_tiled(blocks["tiled"], reg=blocks["reg"])
    nat = lqt.kkt_solve(blocks["A"], blocks["B"], blocks["Q"], blocks["R"], blocks["M"],
                        blocks["r"], blocks["P"], reg=blocks["reg"], lanes=64)
    torch.cuda.synchronize()
    dx, du = res.dx, res.du
    pred_dx = torch.einsum("bkij,bkj->bki", blocks["A"], dx[:, :-1]) + \
        torch.einsum("bkij,bkj->bki", blocks["B"], du)
    scale = dx.abs().max().item()
    assert (pred_dx - dx[:, 1:]).abs().max().item() <= 1e-12 * max(1.0, scale)
    assert (nat.dx - dx).abs().max().item() <= 1e-12 * max(1.0, scale)
    sample = list(range(0, 4096, 256))
    case = {k: blocks[k][sample].cpu().numpy() for k in ["A", "B", "Q", "R", "M", "r", "P", "reg"]}
    ref = oracle_batch(case)
    assert relerr(dx[sample].cpu(), ref["dx"]) < RTOL
    assert relerr(du[sample].cpu(), ref["du"]) < RTOL
    assert relerr(res.pred[sample].cpu(), ref["pred"]) < RTOL
    assert bool(torch.all(res.feasible == 1))


@pytest.mark.parametrize("nx,nu,N,lanes", [(2, 1, 100, 64), (4, 1, 200, 32), (4, 1, 200, 64),
                                           (4, 1, 50, 8), (8, 4, 40, 64), (4, 1, 200, 128),
                                           (2, 1, 100, 128), (4, 1, 300, 128)])
@pytest.mark.parametrize("affine", [False, True])
def test_kkt_without_gains_matches_oracle(nx, nu, N, lanes, affine):
    """par_Newton's outputs only (want_gains=False): K, d stay in LDS between the backward and
    forward phases when they fit (noc_kkt_gains_on_chip), else go through the K/d workspace."""
    from noc import lqt
    case = rand_lq(77 + N + lanes + nx, 6, N, nx, nu, affine=affine)
    ref = oracle_batch(case)
    g = lambda k: dev(case.get(k))
    res = lqt.kkt_solve(g("A"), g("B"), g("Q"), g("R"), g("M"), g("r"), g("P"), reg=g("reg"),
                        x0=g("x0"), q=g("q"), c=g("c"), p=g("p"), lanes=lanes, want_gains=False)
    torch.cuda.synchronize()
    assert (res.K is None) == lqt.gains_on_chip(nx, nu, N, lanes)
    for k in ["dx", "du", "pred"]:
        got = getattr(res, k).cpu().numpy()
        assert relerr(got, ref[k]) < RTOL, (k, relerr(got, ref[k]))
    assert np.array_equal(res.feasible.cpu().numpy().astype(bool), ref["feasible"].astype(bool))


@pytest.mark.parametrize("N,lanes", [(64, 64), (100, 64), (128, 64), (64, 32), (65, 32),
                                     (100, 128), (256, 128), (257, 128)])
@pytest.mark.parametrize("affine", [False, True])
@pytest.mark.parametrize("gains", [False, True])
def test_register_cached_chunk_equals_streamed(N, lanes, affine, gains):
    """nx = 2 with chunks of <= 2 stages runs the register-cached scan (one load pass).  It must
    match the oracle and be bit-identical to the streamed scan (ablation bit 3 forces the latter;
    same arithmetic, only where the blocks are read from differs).  N=65/L=32 mixes chunks of 3
    (streamed: cmax > 2) as the negative control."""
    from noc import lqt, _lib
    case = rand_lq(5000 + N + lanes + int(affine), 7, N, 2, 1, affine=affine)
    ref = oracle_batch(case)
    g = lambda k: dev(case.get(k))
    args = (g("A"), g("B"), g("Q"), g("R"), g("M"), g("r"), g("P"))
    kw = dict(reg=g("reg"), x0=g("x0"), q=g("q"), c=g("c"), p=g("p"), lanes=lanes,
              want_gains=gains)
    lib = _lib.load()
    try:
        cached = lqt.kkt_solve(*args, **kw)
        lib.noc_debug_set_ablation(8)
        streamed = lqt.kkt_solve(*args, **kw)
    finally:
        lib.noc_debug_set_ablation(0)
    torch.cuda.synchronize()
    for k in ["dx", "du", "pred"]:
        assert relerr(getattr(cached, k).cpu(), ref[k]) < RTOL, k
        assert torch.equal(getattr(cached, k), getattr(streamed, k)), k
    if gains:
        assert torch.equal(cached.K, streamed.K) and torch.equal(cached.d, streamed.d)
        assert relerr(cached.K.cpu(), ref["K"]) < RTOL
    assert torch.equal(cached.feasible, streamed.feasible)


def test_group_solve_linear8_blocks_properties():
    """c4 family (four stacked RK4 double integrators, nx=8, nu=4) at N=512 with a reduced batch:
    the horizon-sequential group solve (lanes=1) against the oracle on a sample, dynamics
    consistency on every trajectory, and agreement with the parallel scan (lanes=16)."""
    from noc import lqt
    from noc.problems import make_bench_blocks
    blocks = make_bench_blocks("linear8", N=512, batch=512, seed=3, natural=True)
    nat = [blocks[k] for k in ("A", "B", "Q", "R", "M", "r", "P")]
    res = lqt.kkt_solve(*nat, reg=blocks["reg"], lanes=1)
    scan = lqt.kkt_solve(*nat, reg=blocks["reg"], lanes=16)
    torch.cuda.synchronize()
    dx, du = res.dx, res.du
    pred_dx = torch.einsum("bkij,bkj->bki", blocks["A"], dx[:, :-1]) + \
        torch.einsum("bkij,bkj->bki", blocks["B"], du)
    scale = max(1.0, dx.abs().max().item())
    assert (pred_dx - dx[:, 1:]).abs().max().item() <= 1e-12 * scale
    assert (scan.dx - dx).abs().max().item() <= 1e-9 * scale
    sample = list(range(0, 512, 64))
    case = {k: blocks[k][sample].cpu().numpy() for k in ["A", "B", "Q", "R", "M", "r", "P", "reg"]}
    ref = oracle_batch(case)
    assert relerr(dx[sample].cpu(), ref["dx"]) < RTOL
    assert relerr(du[sample].cpu(), ref["du"]) < RTOL
    assert relerr(res.pred[sample].cpu(), ref["pred"]) < RTOL
    assert bool(torch.all(res.feasible == 1))


@pytest.mark.parametrize("name,N,B,lanes", [("linear8", 512, 16384, 1), ("cartpole", 200, 65536, 32),
                                           ("pendulum", 100, 1024, 0), ("cartpole", 200, 4096, 0),
                                           ("cartpole", 200, 512, 0)])
def test_full_size_bench_blocks_properties(name, N, B, lanes):
    """The bench path at BASELINE full sizes where the oracle cannot run on every trajectory:
    c2 (pendulum, N=100, B=1024: the batch-aware pick = 64 lanes, register-cached chunks), c3
    (cart-pole, N=200, B=4096: 32 lanes), c4 (linear8, N=512, B=16384, group solve on the grouped
    layout) and c5's global batch on ONE GPU (cart-pole, N=200, B=65536 = 8 x 8192: 64-bit
    indexing of the tiled layout), and the 8-GPU shard of the north-star curve (cart-pole, N=200,
    512 per GPU: the pick = 128 lanes, two waves per trajectory).  Properties:
    dx_{k+1} = A dx_k + B du_k on every trajectory, all feasible, finite pred, and oracle parity
    on a strided sample of 8 trajectories including the last one."""
    from noc import lqt
    from noc.problems import make_bench_blocks
    blocks = make_bench_blocks(name, N=N, batch=B, seed=5, lanes=lanes)
    res = lqt.kkt_solve_tiled(blocks["tiled"], reg=blocks["reg"], want_gains=False)
    torch.cuda.synchronize()
    nat = blocks["engine"].natural_blocks()
    dx, du = res.dx, res.du
    scale = max(1.0, dx.abs().max().item())
    for lo in range(0, B, 4096):  # chunked: the einsum temporaries stay small
        hi = lo + 4096
        pred_dx = torch.einsum("bkij,bkj->bki", nat["A"][lo:hi], dx[lo:hi, :-1]) + \
            torch.einsum("bkij,bkj->bki", nat["B"][lo:hi], du[lo:hi])
        assert (pred_dx - dx[lo:hi, 1:]).abs().max().item() <= 1e-12 * scale, lo
    assert bool(torch.all(res.feasible == 1))
    assert bool(torch.all(torch.isfinite(res.pred)))
    sample = list(range(0, B, B // 8))[:7] + [B - 1]
    case = {k: nat[k][sample].cpu().numpy() for k in ["A", "B", "Q", "R", "M", "r", "P"]}
    case["reg"] = blocks["reg"][sample].cpu().numpy()
    ref = oracle_batch(case)
    assert relerr(dx[sample].cpu(), ref["dx"]) < RTOL
    assert relerr(du[sample].cpu(), ref["du"]) < RTOL
    assert relerr(res.pred[sample].cpu(), ref["pred"]) < RTOL


def test_nontemporal_phase3_instance_is_bit_identical():
    """The L = 32 scan of a batch whose blocks exceed 1.5x the memory-side cache runs the instance
    that reads phase 3's Q, R, M, r non-temporally (kkt_nt3 in csrc/noc_internal.h) -- a cache
    policy, not an arithmetic change.  The first 4096 trajectories of an 8192-trajectory batch (577
    MB of blocks: that instance) equal the same 4096 solved as a batch of their own (288 MB: the
    default instance) bit for bit, and the 8192 match the oracle on a sample."""
    from noc import lqt
    from noc.problems import make_bench_blocks
    B, H = 8192, 4096
    blocks = make_bench_blocks("cartpole", N=200, batch=B, seed=9, lanes=32)
    nat = blocks["engine"].natural_blocks()
    full = lqt.kkt_solve_tiled(blocks["tiled"], reg=blocks["reg"], want_gains=False)
    half_tb = lqt.to_tiled(*(nat[k][:H] for k in ("A", "B", "Q", "R", "M", "r", "P")), lanes=32)
    half = lqt.kkt_solve_tiled(half_tb, reg=blocks["reg"][:H], want_gains=False)
    torch.cuda.synchronize()
    for k in ("dx", "du", "pred", "feasible"):
        assert torch.equal(getattr(full, k)[:H], getattr(half, k)), k
    sample = [0, 3000, 4095, 4096, 6001, B - 1]
    case = {k: nat[k][sample].cpu().numpy() for k in ["A", "B", "Q", "R", "M", "r", "P"]}
    case["reg"] = blocks["reg"][sample].cpu().numpy()
    ref = oracle_batch(case)
    assert relerr(full.dx[sample].cpu(), ref["dx"]) < RTOL
    assert relerr(full.du[sample].cpu(), ref["du"]) < RTOL


def _lm_lqt(T):
    """examples/linear_mpc_parallel.py:24-64: RK4 double integrator (step 0.001), Q = P =
    diag(1e2, 1), R = 0.1, tracking zero."""
    from noc import problems
    fam = problems.double_integrators(1, 0.001).family
    A = np.repeat(np.asarray(fam.A, dtype=np.float64).reshape(1, 2, 2), T, 0)
    B = np.repeat(np.asarray(fam.B, dtype=np.float64).reshape(1, 2, 1), T, 0)
    Q = np.repeat(np.diag([1e2, 1.0])[None], T, 0)
    R = np.repeat(0.1 * np.eye(1)[None], T, 0)
    return A, B, Q, R


@pytest.mark.parametrize("graph", [True, False])
@pytest.mark.parametrize("batched", [False, True])
def test_mpc_loop_matches_oracle_closed_loop(graph, batched):
    """LM:67-84 par_mpc_loop under lax.scan: each step solves the LQT from the current state and
    applies u_par[0]; x_{t+1} = x_par[1].  Oracle: the sequential Riccati solve per step."""
    from noc import lqt
    from oracle import noc_oracle as O
    T, steps = 5, 120
    A, B, Q, R = _lm_lqt(T)
    eye = lambda n: np.repeat(np.eye(n)[None], T, 0)
    L = lqt.LQT(*(dev(t) for t in (A, B, np.zeros((T, 2)), np.diag([1e2, 1.0]), np.eye(2),
                                    np.zeros(2), Q, eye(2), np.zeros((T, 2)), R, eye(1),
                                    np.zeros((T, 1)), np.zeros((T, 2, 1)))))
    x0s = np.array([[2.0, 1.0], [-1.0, 0.5], [0.3, -2.0]]) if batched else np.array([2.0, 1.0])
    xs, us = lqt.mpc_loop(L, dev(x0s), steps, graph=graph, chunk=50)
    torch.cuda.synchronize()
    xs, us = xs.cpu().numpy(), us.cpu().numpy()
    for b, x0 in enumerate(np.atleast_2d(x0s)):
        x = x0.copy()
        for t in range(steps):
            dx, du = O.kkt_solve(A, B, Q, R, np.zeros((T, 2, 1)), np.zeros((T, 1)),
                                 np.diag([1e2, 1.0]), 0.0, x0=x)[:2]
            got_x = xs[t, b] if batched else xs[t]
            got_u = us[t, b] if batched else us[t]
            assert np.max(np.abs(got_u - du[0])) <= 1e-9 * max(1.0, np.abs(du[0]).max()), t
            assert np.max(np.abs(got_x - dx[1])) <= 1e-10 * max(1.0, np.abs(dx[1]).max()), t
            x = dx[1]


@pytest.mark.parametrize("lanes", [64, 128, 16])
def test_nx2_indefinite_state_cost(lanes):
    """nx = 2 combines use the closed-form 2 x 2 solve (small_linalg.h: solve2_closed) with no
    pivoting or threshold check.  With an indefinite state cost Q (as cxx + lambda.fxx, or a traced
    user cost, can be) the value Hessians are indefinite and det(I + C1 J2) is no longer >= 1;
    the step must still match the oracle at 1e-10 wherever the KKT system is well posed
    (all Quu > 0), and the feasibility flags must agree."""
    # (shift, R boost): all well posed with ~60 % indefinite stage costs; a mix of well-posed
    # and indefinite-Quu trajectories (flags must agree)
    for shift, boost, min_ok in ((0.4, 4.0, 10), (0.6, 2.0, 2)):
        case = rand_lq(77 + lanes, 10, 60, 2, 1)
        case["Q"] = case["Q"] - shift * np.eye(2)  # eigenvalues of H's state block start at 0.1
        case["R"] = case["R"] + boost
        assert np.mean(np.linalg.eigvalsh(case["Q"]).min(axis=-1) < 0) > 0.5
        ref = oracle_batch(case)
        out = run_kkt(case, lanes)
        assert np.array_equal(out["feasible"].astype(bool), ref["feasible"].astype(bool))
        ok = np.flatnonzero(ref["feasible"].astype(bool))
        assert ok.size >= min_ok, ref["feasible"]
        for k in ("dx", "du", "K", "d", "S", "v"):
            assert relerr(out[k][ok], ref[k][ok]) < RTOL, (k, relerr(out[k][ok], ref[k][ok]))
        assert relerr(out["pred"][ok], ref["pred"][ok]) < RTOL


def test_kkt_random_shapes_match_oracle():
    """Property form of the parity test (hypothesis, derandomized so every box draws the same 100
    cases): any shape of the build, any horizon 1-260 (ragged chunks, N < lanes), any batch 1-9
    (partly filled workgroups, the 512-register instance at one wave per SIMD), any lane count
    incl. the batch-aware pick (0) and the group solve (1), affine terms on or off."""
    from hypothesis import HealthCheck, given, settings, strategies as st

    @settings(max_examples=100, deadline=None, derandomize=True, database=None,
              suppress_health_check=list(HealthCheck))
    @given(shape=st.sampled_from([(2, 1), (4, 1), (8, 4)]), N=st.integers(1, 260),
           B=st.integers(1, 9), lanes=st.sampled_from([0, 1, 8, 16, 32, 64, 128]),
           affine=st.booleans(), seed=st.integers(0, 2 ** 20))
    def check(shape, N, B, lanes, affine, seed):
        nx, nu = shape
        if lanes == 128 and nx == 8:
            lanes = 64
        case = rand_lq(seed, B, N, nx, nu, affine=affine)
        ref = oracle_batch(case)
        out = run_kkt(case, lanes)
        for k in ["dx", "du", "K", "d", "S", "v", "pred"]:
            assert relerr(out[k], ref[k]) < RTOL, (k, shape, N, B, lanes, affine, seed)
        assert np.array_equal(out["feasible"].astype(bool), ref["feasible"].astype(bool))

    check()


@pytest.mark.parametrize("N,lanes,B,affine", [(200, 64, 1024, False), (200, 32, 2048, False),
                                              (7, 64, 33, True), (250, 64, 1000, True),
                                              (1, 32, 5, False), (65, 32, 9, True)])
@pytest.mark.parametrize("tiled", [True, False])
def test_ab_slots_equal_rereads(N, lanes, B, affine, tiled):
    """The 512-register instances (L = 32 / 64 with waves <= SIMDs) park A, B of the first chunk
    slots in LDS in phase 1 and read them back in phases 3 and 4 instead of re-reading them.
    Ablation bit 6 turns the slots off.  Every output bit-identical, tiled and natural layout,
    affine or not.  (Until round 6 the natural layout differed in the last bits, 1.6e-15: the
    compiler fused the symmetrisation 0.5 (Q_ij + Q_ji) into the first Riccati product in one
    path only -- six v_fmac_f64 with 0.5 in the slot path's BIG instances against six
    v_mul_f64 in the other; csrc/small_linalg.h gload_sym now keeps that product opaque.)  Both
    match the oracle on a sample.  Covers ragged chunks (N % L), affine terms and N < L."""
    from noc import lqt, _lib
    case = rand_lq(4200 + N + lanes + B, B, N, 4, 1, affine=affine)
    g = lambda k: dev(case.get(k))
    lib = _lib.load()

    def solve():
        if tiled and not affine:
            tb = lqt.to_tiled(g("A"), g("B"), g("Q"), g("R"), g("M"), g("r"), g("P"), lanes)
            return lqt.kkt_solve_tiled(tb, reg=g("reg"), want_value=True)
        return lqt.kkt_solve(g("A"), g("B"), g("Q"), g("R"), g("M"), g("r"), g("P"), reg=g("reg"),
                             x0=g("x0"), q=g("q"), c=g("c"), p=g("p"), lanes=lanes, want_value=True)
    try:
        parked = solve()
        lib.noc_debug_set_ablation(64)
        reread = solve()
    finally:
        lib.noc_debug_set_ablation(0)
    torch.cuda.synchronize()
    exact = tiled and not affine  # the tiled K, d buffers

    def same(x, y, k):
        assert torch.equal(x, y), k

    for k in ("dx", "du", "pred", "S", "v"):
        same(getattr(parked, k), getattr(reread, k), k)
    assert torch.equal(parked.feasible, reread.feasible)
    if exact:  # the tiled K, d buffers have padding slots nobody writes
        gains = lambda r: (lqt.untile(r.K, (B, N, 1, 4), lanes), lqt.untile(r.d, (B, N, 1), lanes))
    else:
        gains = lambda r: (r.K, r.d)
    for x, y in zip(gains(parked), gains(reread)):
        same(x, y, "K/d")
    sample = sorted({0, B // 2, B - 1})
    ref = oracle_batch({k: v[sample] for k, v in case.items()})
    for k in ("dx", "du", "pred"):
        assert relerr(getattr(parked, k)[sample].cpu(), ref[k]) < RTOL, k
