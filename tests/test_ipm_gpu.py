"""GPU parity of the device linearisation and of the whole batched interior-point solve against
the oracle (oracle/noc_oracle.py restating P:127-254 and S:108-202; derivatives by torch.func
autodiff, oracle/problems.py).

Tolerances (fp64, stated): LQ blocks 1e-10 relative; full solves: identical outer-iteration and
KKT-solve counts, final cost relative 1e-8, controls 1e-6 absolute (the step sequence is the same;
only rounding differs).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def _oracle_problem(name, N):
    from oracle import problems as PR, noc_oracle as O
    if name == "pendulum":
        return O.NumpyProblem(PR.pendulum_ocp(1.0 / N))
    if name == "cartpole":
        return O.NumpyProblem(PR.cartpole_ocp(1.0 / N))
    raise ValueError(name)


@pytest.mark.parametrize("name,N", [("pendulum", 50), ("cartpole", 40)])
def test_device_linearisation_matches_autodiff_oracle(name, N):
    from noc.problems import make_bench_blocks
    from oracle import noc_oracle as O
    blk = make_bench_blocks(name, N=N, batch=3, seed=5, natural=True)
    torch.cuda.synchronize()
    prob = _oracle_problem(name, N)
    X = blk["x"].cpu().numpy()
    U = blk["u"].cpu().numpy()
    eng = blk["engine"]
    for b in range(3):
        ref_x = O.rollout(prob.dynamics, U[b], X[b, 0])
        assert _rel(X[b], ref_x) < 1e-12
        L = O.linearize(prob, X[b], U[b], 0.1)
        for k in ["A", "B", "Q", "R", "M", "r", "P"]:
            assert _rel(blk[k][b].cpu().numpy(), L[k]) < 1e-10, (k, _rel(blk[k][b].cpu(), L[k]))
        cost = prob.total_cost(X[b], U[b], 0.1)
        assert abs(eng.t["cost"][b].item() - cost) <= 1e-12 * abs(cost)
        assert abs(eng.t["hu"][b].item() - np.max(np.abs(L["r"]))) <= 1e-12
        assert abs(eng.t["gnorm"][b].item() - np.linalg.norm(L["cu"])) <= 1e-12 * np.linalg.norm(L["cu"])


def test_pendulum_par_solve_matches_oracle():
    """BASELINE config c1 (pendulum N=50, B=1): same iterations / KKT solves as the oracle."""
    from noc import problems
    from noc.par_interior_point_newton import par_interior_point_optimal_control
    from oracle import noc_oracle as O
    N = 50
    ocp = problems.pendulum(1.0 / N)
    u0 = 0.1 * np.random.default_rng(1).normal(size=(N, 1))
    x0 = np.array([0.1, -0.1])
    U, it, info = par_interior_point_optimal_control(ocp, u0, x0, return_info=True)
    prob = _oracle_problem("pendulum", N)
    Ur, itr, solves_r = O.par_interior_point_optimal_control(prob, u0, x0, terminal="stage0")
    assert it == itr == 70
    assert info["kkt_solves"] == solves_r == 87
    c = prob.total_cost(O.rollout(prob.dynamics, U, x0), U, 0.0)
    cr = prob.total_cost(O.rollout(prob.dynamics, Ur, x0), Ur, 0.0)
    assert abs(c - cr) <= 1e-8 * abs(cr)
    assert np.max(np.abs(U - Ur)) < 1e-6


@pytest.mark.parametrize("lanes", [8, 16, 32])
def test_multilaunch_solve_at_every_scan_width_matches_oracle(lanes):
    """The multi-launch device loop at the narrower scan widths the batch-aware lanes policy
    (noc_kkt_pick_lanes) chooses for large batches: same counts and iterates as the oracle."""
    from noc import problems
    from noc.par_interior_point_newton import par_interior_point_optimal_control
    from oracle import noc_oracle as O
    N = 50
    ocp = problems.pendulum(1.0 / N)
    u0 = 0.1 * np.random.default_rng(1).normal(size=(N, 1))
    x0 = np.array([0.1, -0.1])
    U, it, info = par_interior_point_optimal_control(ocp, u0, x0, lanes=lanes, return_info=True)
    prob = _oracle_problem("pendulum", N)
    Ur, itr, solves_r = O.par_interior_point_optimal_control(prob, u0, x0, terminal="stage0")
    assert it == itr == 70
    assert info["kkt_solves"] == solves_r == 87
    assert np.max(np.abs(U - Ur)) < 1e-6


def test_pendulum_seq_solve_matches_oracle():
    from noc import problems
    from noc.seq_interior_point_newton import seq_interior_point_optimal_control
    from oracle import noc_oracle as O
    N = 50
    ocp = problems.pendulum(1.0 / N)
    u0 = 0.1 * np.random.default_rng(1).normal(size=(N, 1))
    x0 = np.array([0.1, -0.1])
    U, it = seq_interior_point_optimal_control(ocp, u0, x0)
    prob = _oracle_problem("pendulum", N)
    Ur, itr = O.seq_interior_point_optimal_control(prob, u0, x0)
    assert it == itr == 79
    assert np.max(np.abs(U - Ur)) < 1e-6


def test_batched_solve_equals_individual_oracle_runs():
    """vmap semantics: every trajectory of a batch follows its own reference control flow."""
    from noc import problems
    from noc.par_interior_point_newton import par_interior_point_optimal_control
    from oracle import noc_oracle as O
    N, Bt = 30, 4
    ocp = problems.pendulum(1.0 / N)
    x0, u0 = problems.initial_conditions("pendulum", N, Bt, seed=9)
    U, its, info = par_interior_point_optimal_control(ocp, u0, x0, return_info=True)
    prob = _oracle_problem("pendulum", N)
    for b in range(Bt):
        Ur, itr, sr = O.par_interior_point_optimal_control(prob, u0[b], x0[b], terminal="stage0")
        assert its[b] == itr and info["kkt_solves"][b] == sr
        assert np.max(np.abs(U[b] - Ur)) < 1e-6


def test_cartpole_par_solve_matches_oracle():
    from noc import problems
    from noc.par_interior_point_newton import par_interior_point_optimal_control
    from oracle import noc_oracle as O
    N = 40
    ocp = problems.cartpole(1.0 / N)
    x0, u0 = problems.initial_conditions("cartpole", N, 1, seed=3)
    U, it, info = par_interior_point_optimal_control(ocp, u0[0], x0[0], return_info=True)
    prob = _oracle_problem("cartpole", N)
    Ur, itr, sr = O.par_interior_point_optimal_control(prob, u0[0], x0[0], terminal="stage0")
    assert it == itr and info["kkt_solves"] == sr
    c = prob.total_cost(O.rollout(prob.dynamics, U, x0[0]), U, 0.0)
    cr = prob.total_cost(O.rollout(prob.dynamics, Ur, x0[0]), Ur, 0.0)
    assert abs(c - cr) <= 1e-8 * abs(cr)


def test_final_cost_terminal_option_matches_oracle():
    """terminal="final_cost" (hessian(final_cost) as in the seq path, S:66) instead of the par
    path's default XT = Q[0] (P:73)."""
    from noc import problems
    from noc.par_interior_point_newton import par_interior_point_optimal_control
    from oracle import noc_oracle as O
    N = 30
    ocp = problems.pendulum(1.0 / N)
    u0 = 0.1 * np.random.default_rng(1).normal(size=(N, 1))
    x0 = np.array([0.1, -0.1])
    U, it = par_interior_point_optimal_control(ocp, u0, x0, terminal="final_cost")
    prob = _oracle_problem("pendulum", N)
    Ur, itr, _ = O.par_interior_point_optimal_control(prob, u0, x0, terminal="final_cost")
    assert it == itr
    assert np.max(np.abs(U - Ur)) < 1e-6


def test_linear_demo_known_answer():
    """examples/linear_demo_cuda.py (LD:19-62): unconstrained LQR, one exact Newton step solves
    it; compare with the dense KKT solution of the same LQ problem."""
    from noc import problems
    from noc.par_interior_point_newton import par_interior_point_optimal_control
    from oracle import noc_oracle as O
    N = 40
    ocp = problems.double_integrators(1, 0.1)
    x0 = np.array([2.0, 1.0])
    u0 = np.zeros((N, 1))
    U, it = par_interior_point_optimal_control(ocp, u0, x0)
    fam = ocp.family
    A = np.repeat(fam.A[None], N, 0)
    B = np.repeat(fam.B[None], N, 0)
    Q = np.repeat(np.diag(fam.wx)[None], N, 0)
    R = np.repeat(np.diag(fam.wu)[None], N, 0)
    M = np.zeros((N, 2, 1))
    r = np.zeros((N, 1))
    _, du, _ = O.dense_kkt(A, B, Q, R, M, r, np.diag(fam.wf), 0.0, x0)
    assert np.max(np.abs(U - du)) < 1e-8


@pytest.mark.parametrize("name,N,Bt", [("pendulum", 60, 16), ("cartpole", 200, 64)])
@pytest.mark.parametrize("mode", ["par", "seq"])
def test_persistent_solve_equals_multilaunch_loop(name, N, Bt, mode, monkeypatch):
    """noc_ipm_solve (whole solve in one launch, one wave per trajectory) against the multi-launch
    device loop at the same lanes (64): same arithmetic, so identical counters and iterates.
    (The one-wave kernel is forced: small batches default to the wide kernel.)"""
    monkeypatch.setenv("NOC_PERSIST_WIDE", "0")
    from noc import problems, _lib
    from noc.ipm import BatchedIPM
    ocp = problems.make_problem(name, N)
    x0, u0 = problems.initial_conditions(name, N, Bt, seed=21)
    m = _lib.MODE_PAR if mode == "par" else _lib.MODE_SEQ
    res = []
    for persistent in (True, False):
        eng = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=persistent)
        eng.load(u0, x0)
        eng.solve(mode=m)
        torch.cuda.synchronize()
        res.append([t.cpu().numpy() for t in eng.result()] + [eng.t["phase"].cpu().numpy()])
    (Up, itp, sp, php), (Um, itm, sm, phm) = res
    assert np.array_equal(itp, itm) and np.array_equal(sp, sm)
    assert np.all(php == _lib.PHASE_DONE) and np.all(phm == _lib.PHASE_DONE)
    assert np.max(np.abs(Up - Um)) <= 1e-12 * max(1.0, float(np.max(np.abs(Um))))


@pytest.mark.parametrize("name,mode", [("pendulum", "par"), ("cartpole", "par"),
                                       ("cartpole", "seq")])
def test_persistent_states_in_lds_equal_workspace(name, mode, monkeypatch):
    """The one-wave persistent solver with x, u resident in LDS for the whole solve (the default
    where it fits) against the same solver on the workspace copies
    (NOC_PERSIST_XLDS=0): the same arithmetic on the same values, so identical counters and
    bit-identical controls and states; also across a capped launch and its resume."""
    monkeypatch.setenv("NOC_PERSIST_WIDE", "0")
    from noc import problems, _lib
    from noc.ipm import BatchedIPM
    N, Bt = 60, 48
    ocp = problems.make_problem(name, N)
    x0, u0 = problems.initial_conditions(name, N, Bt, seed=17)
    m = _lib.MODE_PAR if mode == "par" else _lib.MODE_SEQ
    res = []
    for xlds in ("1", "0"):
        monkeypatch.setenv("NOC_PERSIST_XLDS", xlds)
        eng = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=True)
        eng.load(u0, x0)
        eng.solve_persistent(mode=m, max_solves=40)      # capped mid-solve ...
        eng.solve_persistent(mode=m, resume=True)        # ... and resumed to the end
        torch.cuda.synchronize()
        res.append([t.cpu().numpy() for t in eng.result()] + [eng.t["x"].cpu().numpy()])
    (Ul, itl, sl, Xl), (Uw, itw, sw, Xw) = res
    assert np.array_equal(itl, itw) and np.array_equal(sl, sw)
    assert np.array_equal(Ul, Uw) and np.array_equal(Xl, Xw)


def _struct_problem(name, N, Bt):
    """(ocp, x0, u0) of a built-in family (c2 / c3 shapes) or a registered one (parametrised cost:
    the actuated pendulum, nx = 3; traced cost: the track-limited cart-pole)."""
    from noc import problems
    if name in ("pendulum", "cartpole"):
        return (problems.make_problem(name, N),) + tuple(problems.initial_conditions(name, N, Bt, seed=31))
    import custom_families as CF
    if name == "actuated_pendulum":
        rng = np.random.default_rng(7)
        x0 = np.array([0.1, -0.1, 0.0]) + 0.01 * rng.normal(size=(Bt, 3))
        return CF.actuated_pendulum(1.0 / N), x0, 0.1 * rng.normal(size=(Bt, N, 1))
    return (CF.cartpole_track_limit(1.0 / N),) + tuple(problems.initial_conditions("cartpole", N, Bt, seed=3))


@pytest.mark.parametrize("name,N,Bt,mode", [
    ("pendulum", 100, 1024, "par"),        # c2
    ("cartpole", 200, 4096, "par"),        # c3: probe launch capped at 32 solves + resume
    ("cartpole", 60, 96, "seq"),
    ("actuated_pendulum", 50, 64, "par"),  # registered, parametrised cost, nx = 3
    ("cartpole_track_limit", 60, 64, "par"),  # registered, traced cost with a state constraint
])
def test_structured_blocks_equal_dense_instance(name, N, Bt, mode, monkeypatch):
    """The persistent solver's structure-aware blocks (csrc/block_struct.h: only the variable
    entries of A, B, Q, R, M in the workspace, the constant ones rebuilt from literals and the
    family's parameters, products with structural zeros skipped) against the dense instance
    (NOC_PERSIST_STRUCT=0): bit-identical controls and states, identical counters."""
    monkeypatch.setenv("NOC_PERSIST_WIDE", "0")
    from noc import _lib
    from noc.ipm import BatchedIPM
    ocp, x0, u0 = _struct_problem(name, N, Bt)
    m = _lib.MODE_PAR if mode == "par" else _lib.MODE_SEQ
    res = []
    for struct in ("1", "0"):
        monkeypatch.setenv("NOC_PERSIST_STRUCT", struct)
        eng = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=True)
        eng.load(u0, x0)
        eng.solve(mode=m)
        torch.cuda.synchronize()
        res.append([t.cpu().numpy() for t in eng.result()] + [eng.t["x"].cpu().numpy(),
                                                             eng.t["phase"].cpu().numpy()])
    (Us, its, ss, Xs, phs), (Ud, itd, sd, Xd, phd) = res
    assert np.all(phs == _lib.PHASE_DONE) and np.all(phd == _lib.PHASE_DONE)
    assert np.array_equal(its, itd) and np.array_equal(ss, sd)
    assert np.array_equal(Us, Ud) and np.array_equal(Xs, Xd)


def test_structured_resume_after_launch_per_phase_driver(monkeypatch):
    """A SOLVE resume of the persistent solver recomputes the blocks instead of reading the
    workspace's: after the launch-per-phase driver (dense blocks in the workspace) it continues
    exactly like a persistent solve capped at the same point (compact blocks)."""
    monkeypatch.setenv("NOC_PERSIST_WIDE", "0")
    from noc import problems, _lib
    from noc.ipm import BatchedIPM
    N, Bt = 80, 32
    ocp = problems.make_problem("cartpole", N)
    x0, u0 = problems.initial_conditions("cartpole", N, Bt, seed=12)
    ref = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=True)
    ref.load(u0, x0)
    ref.solve_persistent(schedule="index")
    eng = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=False)
    eng.load(u0, x0)
    eng.init(0.1)
    for _ in range(3):  # a few device iterations leave trajectories mid-retry (phase SOLVE) too
        eng.step(_lib.MODE_PAR, _lib.TERMINAL_STAGE0)
    eng.solve_persistent(resume=True)
    torch.cuda.synchronize()
    a, b = ref.result(), eng.result()
    assert np.array_equal(a[1].cpu().numpy(), b[1].cpu().numpy())
    assert np.array_equal(a[2].cpu().numpy(), b[2].cpu().numpy())
    assert _rel(b[0].cpu().numpy(), a[0].cpu().numpy()) < 1e-12


@pytest.mark.parametrize("wide", ["0", "1"])
def test_persistent_solve_respects_solve_cap(wide, monkeypatch):
    """A trajectory that reaches max_solves stops (phase != DONE) -- every wave exits (the one-wave
    and the wide kernel)."""
    monkeypatch.setenv("NOC_PERSIST_WIDE", wide)
    from noc import problems, _lib
    from noc.ipm import BatchedIPM
    N, Bt = 50, 8
    ocp = problems.pendulum(1.0 / N)
    x0, u0 = problems.initial_conditions("pendulum", N, Bt, seed=4)
    eng = BatchedIPM(ocp.family, N, Bt, persistent=True)
    eng.load(u0, x0)
    eng.solve_persistent(max_solves=5)
    torch.cuda.synchronize()
    assert np.all(eng.t["kkt_solves"].cpu().numpy() == 5)
    assert np.all(eng.t["phase"].cpu().numpy() != _lib.PHASE_DONE)


def test_multilaunch_max_steps_caps_running_trajectories():
    """The multi-launch loop's max_steps: trajectories that finished below the cap do not hold
    the loop open (the cap is tested on the still-running ones), so a capped solve stops with
    slow trajectories unfinished at or past the cap while the fast ones are done with exactly
    their uncapped results."""
    from noc import problems, _lib
    from noc.ipm import BatchedIPM
    N, Bt = 50, 32
    ocp = problems.cartpole(1.0 / N)
    x0, u0 = problems.initial_conditions("cartpole", N, Bt, seed=4)
    eng = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=False)
    eng.load(u0, x0)
    eng.solve()
    torch.cuda.synchronize()
    U_full, _, s_full = (t.cpu().numpy() for t in eng.result())
    cap = int(np.sort(s_full)[Bt // 4]) + 1  # a quarter of the batch finishes below the cap
    assert int(s_full.max()) > cap + 8 * 2, s_full  # ... and some run well past it (seeded)
    eng.load(u0, x0)
    eng.solve(max_steps=cap)
    torch.cuda.synchronize()
    U, _, s = (t.cpu().numpy() for t in eng.result())
    phase = eng.t["phase"].cpu().numpy()
    done, running = phase == _lib.PHASE_DONE, phase != _lib.PHASE_DONE
    assert done.any() and running.any()
    assert np.all(s[running] >= cap)
    assert np.array_equal(s[done], s_full[done]) and np.array_equal(U[done], U_full[done])


@pytest.mark.parametrize("name,N,Bt,mode", [
    ("pendulum", 60, 16, "par"), ("pendulum", 60, 16, "seq"),
    ("pendulum", 20, 4, "par"),      # N < 64: most lanes of every wave own no stage
    ("cartpole", 200, 8, "par"), ("cartpole", 200, 8, "seq"),
    ("cartpole", 300, 3, "par"),     # N > 256: two stages on some lanes
    ("linear2", 100, 5, "par"),
])
@pytest.mark.parametrize("waves", ["4", "2"])
def test_wide_solve_matches_one_wave_kernel(name, N, Bt, mode, waves, monkeypatch):
    """The wide whole-solve kernel (ipm_wide.hip: four -- or, NOC_WIDE_WAVES=2, two -- waves per
    trajectory, compact blocks in LDS) against
    the one-wave kernel on the same inputs: identical outer iterations per trajectory, identical
    KKT solves and controls within 1e-8 relative (the scans associate differently, so not
    bit-identical) -- except where an accept test (P:159-173) is decided below the resolution of
    the cost itself.

    Root cause of the one such case (cartpole N=200 seed 33 trajectory 3, 685 vs 185 solves;
    tools/flip_probe.py, profiles/r03/flip/): at bp = 0.1, Newton iteration 65, |Hu| = 3.4e-7,
    the predicted reduction is -5.6e-13 = 0.35 eps |cost| (cost 7234.93).  The one-wave kernel
    (and the oracle) evaluate the trial cost one ulp below the cost -> gain 1.61, accepted; the
    wide kernel evaluates it exactly equal -> gain -0, rejected; rp then grows, every retry is a
    sub-ulp step, and the retry cap keeps the last trial (500 more solves, same iteration count).
    So a flip is allowed only when the decision-trace build (make trace-lib) reproduces both
    kernels' solve counts and shows, at the first decision where they differ, |pred| and
    |new_cost - cost| within 4 eps |cost| in BOTH kernels: a rounding-level decision, not a
    difference in the algorithm."""
    import json
    import os
    import subprocess
    import sys
    from noc import problems, _lib
    from noc.ipm import BatchedIPM
    if name == "linear2":  # box-constrained double integrator (the LINEAR family's log barrier)
        ocp = problems.double_integrators(1, 0.01, constrained=True)
        x0 = np.random.default_rng(33).normal(size=(Bt, 2))
        u0 = np.zeros((Bt, N, 1))
    else:
        ocp = problems.make_problem(name, N)
        x0, u0 = problems.initial_conditions(name, N, Bt, seed=33)
    m = _lib.MODE_PAR if mode == "par" else _lib.MODE_SEQ
    monkeypatch.setenv("NOC_WIDE_WAVES", waves)
    res = []
    for wide in ("1", "0"):
        monkeypatch.setenv("NOC_PERSIST_WIDE", wide)
        eng = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=True)
        eng.load(u0, x0)
        eng.solve(mode=m)
        torch.cuda.synchronize()
        res.append([t.cpu().numpy() for t in eng.result()] + [eng.t["phase"].cpu().numpy()])
    (Uw, itw, sw, phw), (Un, itn, sn, phn) = res
    assert np.array_equal(itw, itn), (itw, itn)
    assert np.all(phw == _lib.PHASE_DONE)
    flip = sw != sn
    same = ~flip
    assert np.max(np.abs(Uw[same] - Un[same])) <= 1e-8 * max(1.0, float(np.max(np.abs(Un))))
    if not flip.any():
        return
    assert name in ("pendulum", "cartpole"), f"{name}: flip with no decision-trace case: {sw} {sn}"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    tlib = os.path.join(root, "ip-parallel-optimal-control_amd", "noc", "_lib", "libnoc_hip_trace.so")
    assert os.path.exists(tlib), "decision-trace build missing (make trace-lib / build())"
    eps = np.finfo(np.float64).eps
    for b in np.flatnonzero(flip):
        out = os.path.join(root, "gpurun_out", f"flip_{name}_{N}_{mode}_{b}_w{waves}.json")
        os.makedirs(os.path.dirname(out), exist_ok=True)
        env = dict(os.environ, NOC_HIP_LIB=tlib)
        env.pop("NOC_PERSIST_WIDE", None)
        subprocess.run([sys.executable, os.path.join(root, "tools", "flip_probe.py"), "--problem",
                        name, "--N", str(N), "--Bt", str(Bt), "--seed", "33", "--traj", str(b),
                        "--mode", mode, "--no-oracle", "--out", out],
                       check=True, env=env, capture_output=True, timeout=240)
        with open(out) as fh:
            d = json.load(fh)
        # the trace build makes the product build's decisions
        assert d["solves"]["wide"] == sw.tolist() and d["solves"]["one_wave"] == sn.tolist()
        pair = d["pairs"]["wide|one_wave"]
        assert pair["first_divergent_solve"] is not None
        for k in ("wide", "one_wave"):
            r = pair[k]
            assert abs(r["pred"]) <= 4 * eps * abs(r["cost"]), (k, r)
            assert abs(r["new_cost"] - r["cost"]) <= 4 * eps * abs(r["cost"]), (k, r)
        assert pair["wide"]["success"] != pair["one_wave"]["success"]
        # the kept trial after the retry cap is a sub-ulp step: the same optimum
        assert np.max(np.abs(Uw[b] - Un[b])) <= 1e-6 * max(1.0, float(np.max(np.abs(Un))))


@pytest.mark.parametrize("heavy,hspec,beyond", [("1", "0", True), ("64", "0", True), ("64", "2", True),
                                                ("96", "2", False)])
def test_heavy_first_split_gives_identical_results(heavy, hspec, beyond, monkeypatch):
    """The probe-ordered resume of a batch larger than one wave per SIMD with its first `heavy`
    launch-order entries on the one-wave instance and the rest on the two-wave instance,
    concurrently on two streams (NOC_PERSIST_HEAVY, ipm_persistent.hip: solve_split): every
    trajectory's controls, states and counters are bit-identical to the single two-wave launch."""
    monkeypatch.setenv("NOC_PERSIST_WIDE", "0")
    from noc.ipm import BatchedIPM
    simds = 4 * torch.cuda.get_device_properties(0).multi_processor_count
    # beyond one wave per SIMD: the two-wave instance, split engaged; else (hspec = 2 only) at one
    # wave per SIMD, the rest on the one-wave instance
    N, Bt = 30, (simds + 77 if beyond else simds - 100)
    ocp, x0, u0 = _resume_case("cartpole", N, Bt, seed=6)
    keys = ("u", "x", "kkt_solves", "total_it", "phase", "bp", "rp", "rinc", "repeats")
    res = {}
    monkeypatch.setenv("NOC_PERSIST_HEAVY_SPEC", hspec)  # 2: the heavy launch speculates
    for h in ("0", heavy):
        monkeypatch.setenv("NOC_PERSIST_HEAVY", h)
        eng = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=True)
        eng.load(u0, x0)
        eng.solve_persistent(schedule="probe")
        torch.cuda.synchronize()
        res[h] = {k: eng.t[k].cpu().numpy().copy() for k in keys}
    for k in keys:
        assert np.array_equal(res["0"][k], res[heavy][k]), k


@pytest.mark.parametrize("spec", ["2", "4"])
@pytest.mark.parametrize("N,Bt,mode,seed", [(200, 512, "par", 11), (60, 40, "seq", 3), (200, 24, "par", 5)])
def test_speculative_candidates_equal_one_wave(spec, N, Bt, mode, seed, monkeypatch):
    """Speculative retries (ipm_persistent.hip: SPEC waves per trajectory, wave k solving the
    k-th candidate of the regularisation's failure chain, the accept tests replayed in solve
    order) against the one-wave solver: controls, states and every counter bit-identical, for a
    whole solve and for one capped at a solve count that falls inside a round of candidates and
    then resumed (on the speculative resume instance).  The first case is the c3 8-GPU slice size
    (512 cart-poles, N = 200), with accounted repeats at the rp clip."""
    monkeypatch.setenv("NOC_PERSIST_WIDE", "0")
    from noc import _lib
    from noc.ipm import BatchedIPM
    ocp, x0, u0 = _resume_case("cartpole", N, Bt, seed=seed)
    m = _lib.MODE_PAR if mode == "par" else _lib.MODE_SEQ
    keys = ("u", "x", "kkt_solves", "total_it", "phase", "bp", "rp", "rinc", "repeats", "cost",
            "inner", "it", "hu", "gnorm")

    def run(s, cap=None):
        monkeypatch.setenv("NOC_PERSIST_SPEC", s)
        eng = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=True)
        eng.load(u0, x0)
        if cap is None:
            eng.solve_persistent(mode=m, schedule="index")
        else:
            eng.solve_persistent(mode=m, schedule="index", max_solves=cap)
            eng.solve_persistent(mode=m, schedule="index", resume=True)
        torch.cuda.synchronize()
        return {k: eng.t[k].cpu().numpy().copy() for k in keys}

    ref = run("1")
    assert np.all(ref["phase"] == _lib.PHASE_DONE)
    for cap in (None, 37):
        got = run(spec, cap)
        for k in keys:
            assert np.array_equal(ref[k], got[k]), (k, cap)
    if N == 200 and Bt == 512:
        assert int(ref["repeats"].sum()) > 0  # the rp-clip accounting is exercised


@pytest.mark.parametrize("extra,caps", [("half", "20,40,60,90,130,180,250,350,500"),
                                        ("full", "20,40,60,90,130,180,250,350,500")])
def test_tail_schedule_equals_plain_launch(extra, caps, monkeypatch):
    """BatchedIPM.solve_persistent's tail schedule (launches capped at NOC_PERSIST_TAIL_CAPS, then
    the trajectories still running gathered into a small workspace and resumed with speculative
    candidates) against the plain schedule: controls, states and counters bit-identical.  Batches
    just beyond half the SIMDs and at one wave per SIMD exactly (the c3 4-GPU slice's shape)."""
    monkeypatch.setenv("NOC_PERSIST_WIDE", "0")
    from noc.ipm import BatchedIPM
    simds = 4 * torch.cuda.get_device_properties(0).multi_processor_count
    N = 60
    Bt = simds // 2 + 77 if extra == "half" else simds
    ocp, x0, u0 = _resume_case("cartpole", N, Bt, seed=9)
    # (not "repeats": the count of retries accounted without recomputation depends on where the
    # caps fall -- a resume inside a run of identical retries at the rp clip computes its first
    # solve -- while the solve counts, states and controls do not)
    keys = ("u", "x", "kkt_solves", "total_it", "phase", "bp", "rp", "rinc", "cost", "inner", "it",
            "hu", "gnorm")
    res, logs = {}, {}
    for tail in ("0", "1"):
        monkeypatch.setenv("NOC_PERSIST_TAIL", tail)
        monkeypatch.setenv("NOC_PERSIST_TAIL_CAPS", caps)
        eng = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=True)
        eng.load(u0, x0)
        eng.solve_persistent()
        torch.cuda.synchronize()
        res[tail] = {k: eng.t[k].cpu().numpy().copy() for k in keys}
        logs[tail] = getattr(eng, "tail_log", None)
    assert logs["1"], "the tail schedule did not run"
    assert any(2 * r <= simds for _, r in logs["1"]) or logs["1"][-1][1] == 0, logs["1"]
    for k in keys:
        assert np.array_equal(res["0"][k], res["1"][k]), k


def test_rp_update_rounds_like_the_reference():
    """The regularisation update after an accepted step, rp * max(1/3, 1 - (2 gain - 1) ** 3)
    (P:167-173, S:139-143), rounds like the reference: the cube as lax.integer_pow, c * (c * c),
    then the subtraction -- no fused multiply-subtract (noc_internal.h: rp_shrink; the oracle's
    _cube).  Checked bit for bit on every accepted step of par and seq solves of both persistent
    kernels from the decision-trace build (tools/rp_trace_check.py), which must also contain
    gains where a fused evaluation would have rounded differently."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    tlib = os.path.join(root, "ip-parallel-optimal-control_amd", "noc", "_lib", "libnoc_hip_trace.so")
    assert os.path.exists(tlib), "decision-trace build missing (make trace-lib / build())"
    env = dict(os.environ, NOC_HIP_LIB=tlib)
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "rp_trace_check.py")],
                       check=True, env=env, capture_output=True, text=True, timeout=240)
    res = json.loads(r.stdout.strip().splitlines()[-1])
    for k, v in res.items():
        assert v["checked"] > 20 and v["mismatched"] == 0, (k, v)
    assert sum(v["fused_would_differ"] for v in res.values()) > 0, res


def _resume_case(name, N, Bt, seed=5):
    from noc import problems
    ocp = problems.make_problem(name, N)
    x0, u0 = problems.initial_conditions(name, N, Bt, seed=seed)
    return ocp, x0, u0


@pytest.mark.parametrize("wide", ["0", "1"])
@pytest.mark.parametrize("name,N,Bt,mode,caps", [
    ("pendulum", 60, 16, "par", (5, 37, 60)),
    ("pendulum", 60, 16, "seq", (3, 50)),
    ("cartpole", 200, 6, "par", (1, 90, 91, 180)),
])
def test_capped_then_resumed_solve_equals_uninterrupted(name, N, Bt, mode, caps, wide, monkeypatch):
    """noc_ipm_solve stopped by max_solves and continued with NOC_WS_RESUME (as often as the caps
    say) gives exactly the uninterrupted solve: identical counters and controls, bit for bit --
    for the one-wave kernel (its blocks stay in the workspace) and the wide kernel (it recomputes
    them from the workspace states with the same arithmetic)."""
    monkeypatch.setenv("NOC_PERSIST_WIDE", wide)
    from noc import _lib
    from noc.ipm import BatchedIPM
    ocp, x0, u0 = _resume_case(name, N, Bt)
    m = _lib.MODE_PAR if mode == "par" else _lib.MODE_SEQ
    ref = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=True)
    ref.load(u0, x0)
    ref.solve_persistent(mode=m)
    eng = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=True)
    eng.load(u0, x0)
    for i, cap in enumerate(caps):
        eng.solve_persistent(mode=m, max_solves=cap, resume=i > 0)
        torch.cuda.synchronize()
        assert int(eng.t["kkt_solves"].max().item()) <= cap
    eng.solve_persistent(mode=m, resume=True)
    torch.cuda.synchronize()
    for k in ("u", "x", "kkt_solves", "total_it", "phase", "bp", "rp"):
        a, b = eng.t[k].cpu().numpy(), ref.t[k].cpu().numpy()
        assert np.array_equal(a, b), (k, np.max(np.abs(a.astype(float) - b.astype(float))))
    assert np.all(eng.t["phase"].cpu().numpy() == _lib.PHASE_DONE)


@pytest.mark.parametrize("wide", ["0", "1"])
def test_retry_repeats_accounted_bit_identical(wide, monkeypatch):
    """The identical retries at the rp clip (noc_internal.h par_retry_repeats: a rejected trial at
    rp = 1e16 leaves every input of the next par_Newton call unchanged, so the rest of the retry
    loop P:151-188 repeats it until the cap) are accounted without recomputation: same controls,
    states and counters bit for bit as recomputing every retry (NOC_WS_NO_REPEAT_SKIP), also when
    max_solves caps a solve inside such a run and NOC_WS_RESUME continues it."""
    monkeypatch.setenv("NOC_PERSIST_WIDE", wide)
    from noc import _lib
    from noc.ipm import BatchedIPM
    N, Bt = 200, 256
    ocp, x0, u0 = _resume_case("cartpole", N, Bt, seed=11)
    keys = ("u", "x", "kkt_solves", "total_it", "it", "inner", "phase", "bp", "rp", "rinc", "hu")

    def run(flags, caps=()):
        eng = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=True)
        eng.ws.flags = flags
        eng.load(u0, x0)
        for i, cap in enumerate(caps):
            eng.solve_persistent(max_solves=cap, resume=i > 0)
        eng.solve_persistent(resume=bool(caps))
        torch.cuda.synchronize()
        return {k: eng.t[k].cpu().numpy().copy() for k in keys + ("repeats",)}

    full = run(_lib.WS_NO_REPEAT_SKIP)
    skip = run(0)
    capped = run(0, caps=(150, 300, 450, 600, 750))
    assert full["repeats"].sum() == 0
    assert skip["repeats"].sum() >= 400, skip["repeats"].sum()  # the batch has retry-cap runs
    assert np.all(skip["phase"] == _lib.PHASE_DONE)
    for k in keys:
        assert np.array_equal(skip[k], full[k]), k
        assert np.array_equal(capped[k], full[k]), k


def test_cost_ordered_launch_gives_identical_results():
    """noc_ipm_solve with a launch order (ws.order: descending initial cost, BatchedIPM
    schedule="cost") only changes which trajectory starts when: every trajectory's controls,
    states and counters are bit-identical to the index-order launch."""
    from noc.ipm import BatchedIPM
    N, Bt = 60, 96
    ocp, x0, u0 = _resume_case("cartpole", N, Bt, seed=4)
    keys = ("u", "x", "kkt_solves", "total_it", "phase", "bp", "rp", "rinc", "repeats")
    res = {}
    for sched in ("index", "cost"):
        eng = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=True)
        eng.load(u0, x0)
        if sched == "cost":
            order = eng.launch_order(0, 1, 0.1).cpu().numpy()
            assert sorted(order.tolist()) == list(range(Bt)) and order.tolist() != list(range(Bt))
        eng.solve_persistent(schedule=sched)
        torch.cuda.synchronize()
        res[sched] = {k: eng.t[k].cpu().numpy().copy() for k in keys}
    for k in keys:
        assert np.array_equal(res["index"][k], res["cost"][k]), k


@pytest.mark.parametrize("probe", [1, 7, 10])
def test_probe_ordered_launch_gives_identical_results(probe):
    """schedule="probe" (the default beyond the resident waves): a capped launch of every
    trajectory's first PROBE_SOLVES KKT solves, then the rest resumed by descending total cost --
    bit-identical to the single index-order launch (a capped-and-resumed solve equals the
    uninterrupted one); the resumed launch really is reordered."""
    from noc.ipm import BatchedIPM
    N, Bt = 60, 96
    ocp, x0, u0 = _resume_case("cartpole", N, Bt, seed=8)
    keys = ("u", "x", "kkt_solves", "total_it", "phase", "bp", "rp", "rinc", "repeats", "it")
    res = {}
    for sched in ("index", "probe"):
        eng = BatchedIPM(ocp.family, N, Bt, lanes=64, persistent=True)
        eng.PROBE_SOLVES = probe
        eng.load(u0, x0)
        eng.solve_persistent(schedule=sched)
        torch.cuda.synchronize()
        res[sched] = {k: eng.t[k].cpu().numpy().copy() for k in keys}
        if sched == "probe":
            order = eng._order.cpu().numpy()
            assert sorted(order.tolist()) == list(range(Bt)) and order.tolist() != list(range(Bt))
    assert (res["index"]["phase"] == 3).all()
    for k in keys:
        assert np.array_equal(res["index"][k], res["probe"][k]), k


def test_linear8_ipm_uses_group_solve_and_is_exact():
    """Four stacked double integrators (nx=8, nu=4; the c4 family): the IPM workspace defaults to
    the grouped layout + horizon-sequential group solve (lanes 1); the unconstrained LQ problem is
    solved exactly by one Newton step -- compare with the dense KKT solution per trajectory."""
    from noc import problems
    from noc.ipm import BatchedIPM
    from oracle import noc_oracle as O
    N, Bt = 24, 11   # a partial last record of the grouped layout
    ocp = problems.double_integrators(4, 0.01)
    fam = ocp.family
    x0, u0 = problems.initial_conditions("linear8", N, Bt, seed=5)
    eng = BatchedIPM(fam, N, Bt)
    assert eng.lanes == 1
    eng.load(u0, x0)
    eng.solve()
    torch.cuda.synchronize()
    U = eng.result()[0].cpu().numpy()
    A = np.repeat(np.asarray(fam.A, np.float64).reshape(1, 8, 8), N, 0)
    B = np.repeat(np.asarray(fam.B, np.float64).reshape(1, 8, 4), N, 0)
    Q = np.repeat(np.diag(fam.wx)[None], N, 0)
    R = np.repeat(np.diag(fam.wu)[None], N, 0)
    for b in range(Bt):
        _, du, _ = O.dense_kkt(A, B, Q, R, np.zeros((N, 8, 4)), np.zeros((N, 4)),
                               np.diag(fam.wf), 0.0, x0[b])
        assert np.max(np.abs(U[b] - du)) < 1e-8 * max(1.0, np.abs(du).max())


@pytest.mark.parametrize("name,N,par_its,par_solves,seq_its,cost", [
    ("pendulum", 50, 70, 87, 79, 178.3114456),
    ("pendulum", 100, 69, 85, 80, 354.2079694),
    ("cartpole", 50, 88, 129, 124, 1842.144564),
    ("cartpole", 200, 129, 212, 144, 7341.298845),
])
def test_solver_reproduces_survey_restatement_numbers(name, N, par_its, par_solves, seq_its, cost):
    """Pins the GPU solver (persistent kernel, B = 1, the reference's harness setting) to the
    numbers SURVEY.md §6 measured with an independent fp64 restatement of S and P: outer
    iterations, KKT solves and the final cost at bp = 0 (u0 = 0.1 N(0,1), numpy seed 1; x0 as
    PR:90 / CR:101; Ts N = 1 s)."""
    from noc import problems
    from noc.par_interior_point_newton import par_interior_point_optimal_control
    from noc.seq_interior_point_newton import seq_interior_point_optimal_control
    from noc.utils import wrap_angle
    ocp = problems.pendulum(1.0 / N) if name == "pendulum" else problems.cartpole(1.0 / N)
    x0 = (np.array([0.1, -0.1]) if name == "pendulum"
          else np.array([0.01, float(wrap_angle(-0.01)), 0.01, -0.01]))
    u0 = 0.1 * np.random.default_rng(1).normal(size=(N, 1))
    U, it, info = par_interior_point_optimal_control(ocp, u0, x0, return_info=True)
    assert (it, info["kkt_solves"]) == (par_its, par_solves)
    prob = _oracle_problem(name, N)
    from oracle import noc_oracle as O
    c = prob.total_cost(O.rollout(prob.dynamics, U, x0), U, 0.0)
    assert abs(c - cost) <= 1e-6 * abs(cost)
    Us, its = seq_interior_point_optimal_control(ocp, u0, x0)
    assert its == seq_its


@pytest.mark.parametrize("name,N,Bt,lanes", [("pendulum", 60, 24, 64), ("cartpole", 100, 40, 32)])
def test_two_stream_overlap_equals_single_stream_loop(name, N, Bt, lanes):
    """The two-stream loop (rollouts on a second stream beside the Newton step, the default once
    Bt*N >= 256k) forced on at a small size: a trajectory whose barrier stage ends is marked
    ROLLOUT_PENDING by the trial and only promoted to ROLLOUT after the main stream waited on the
    roll event, so it must give the same counters and bit-identical iterates as the single-stream
    loop (the rollout could otherwise read controls the trial is still writing)."""
    from noc import problems, _lib
    from noc.ipm import BatchedIPM
    ocp = problems.make_problem(name, N)
    x0, u0 = problems.initial_conditions(name, N, Bt, seed=33)
    res = []
    for overlap in (True, False):
        eng = BatchedIPM(ocp.family, N, Bt, lanes=lanes, overlap=overlap)
        eng.load(u0, x0)
        eng.solve(poll_every=4)
        torch.cuda.synchronize()
        res.append([t.cpu().numpy() for t in eng.result()] + [eng.t["phase"].cpu().numpy()])
    (Uo, ito, so, pho), (Us, its, ss, phs) = res
    assert np.all(pho == _lib.PHASE_DONE) and np.all(phs == _lib.PHASE_DONE)
    assert np.array_equal(ito, its) and np.array_equal(so, ss)
    assert np.array_equal(Uo, Us)


def test_ipm_step_rejects_mismatched_lanes():
    import ctypes
    from noc import problems, _lib
    from noc.ipm import BatchedIPM
    ocp = problems.pendulum(1.0 / 20)
    eng = BatchedIPM(ocp.family, 20, 2, lanes=64)
    lib = _lib.load()
    rc = lib.noc_ipm_step(ctypes.byref(eng.fam_c), ctypes.byref(eng.ws), _lib.MODE_PAR,
                          _lib.TERMINAL_STAGE0, 32, _lib.stream_handle())
    assert rc != 0 and b"lanes" in lib.noc_last_error()


@pytest.mark.parametrize("mode", ["par", "seq"])
def test_cached_engine_gives_fresh_engine_results(mode, monkeypatch):
    """Small solves reuse their engine between calls (par_interior_point_newton._engine): a call on
    a reused engine -- after a solve of other inputs, after a capped newton_oc on it -- returns
    exactly what a call on a fresh engine returns."""
    from noc import problems
    from noc import par_interior_point_newton as P
    from noc.seq_interior_point_newton import seq_interior_point_optimal_control
    solve = P.par_interior_point_optimal_control if mode == "par" else seq_interior_point_optimal_control
    N = 40
    ocp = problems.cartpole(1.0 / N)
    x0, u0 = problems.initial_conditions("cartpole", N, 2, seed=21)
    P._ENGINES.clear()
    fresh = [solve(ocp, u0[b], x0[b]) for b in range(2)]
    assert len(P._ENGINES) == 1
    P._ENGINES.clear()
    P.newton_oc(ocp, u0[1], x0[1], 0.1)  # leaves a one-stage engine state behind
    again = [solve(ocp, u0[b], x0[b]) for b in (1, 0)][::-1]
    for (Uf, itf), (Ua, ita) in zip(fresh, again):
        assert itf == ita and np.array_equal(Uf, Ua)
    monkeypatch.setattr(P, "_ENGINE_CACHE_STAGES", 0)  # no caching at all
    nocache = [solve(ocp, u0[b], x0[b]) for b in range(2)]
    for (Uf, itf), (Un, itn) in zip(fresh, nocache):
        assert itf == itn and np.array_equal(Uf, Un)


def test_random_solves_match_oracle():
    """Property form of the solver parity tests (hypothesis, derandomized: every box draws the same
    12 cases): pendulum or cart-pole, horizon 5-40, batch 1-2, par or seq, random initial states
    and controls of the BASELINE distributions -- Newton iterations and (par) KKT solves equal to
    the oracle's, controls within 1e-6, final cost within 1e-8."""
    from hypothesis import HealthCheck, given, settings, strategies as st
    from noc import problems
    from noc.par_interior_point_newton import par_interior_point_optimal_control
    from noc.seq_interior_point_newton import seq_interior_point_optimal_control
    from oracle import noc_oracle as O

    @settings(max_examples=12, deadline=None, derandomize=True, database=None,
              suppress_health_check=list(HealthCheck))
    @given(name=st.sampled_from(["pendulum", "cartpole"]), N=st.integers(5, 40),
           B=st.integers(1, 2), par=st.booleans(), seed=st.integers(0, 2 ** 20))
    def check(name, N, B, par, seed):
        ocp = problems.make_problem(name, N)
        x0, u0 = problems.initial_conditions(name, N, B, seed=seed)
        prob = _oracle_problem(name, N)
        if par:
            U, its, info = par_interior_point_optimal_control(ocp, u0, x0, return_info=True)
        else:
            U, its = seq_interior_point_optimal_control(ocp, u0, x0)
        for b in range(B):
            if par:
                Ur, itr, sr = O.par_interior_point_optimal_control(prob, u0[b], x0[b],
                                                                   terminal="stage0")
                assert info["kkt_solves"][b] == sr, (name, N, B, par, seed, b)
            else:
                Ur, itr = O.seq_interior_point_optimal_control(prob, u0[b], x0[b])
            assert its[b] == itr, (name, N, B, par, seed, b, its[b], itr)
            assert np.max(np.abs(U[b] - Ur)) < 1e-6
            c = prob.total_cost(O.rollout(prob.dynamics, U[b], x0[b]), U[b], 0.0)
            cr = prob.total_cost(O.rollout(prob.dynamics, Ur, x0[b]), Ur, 0.0)
            assert abs(c - cr) <= 1e-8 * max(1.0, abs(cr))

    check()
