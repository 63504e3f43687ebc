"""Generate the committed golden fixtures (test infrastructure).

The reference cannot run here (pure JAX; jax/jaxlib/paroc absent, no network), so the fixtures
are produced by the oracle restatement (oracle/noc_oracle.py) and cross-checked at generation
time against the dense KKT solve.  They pin the oracle against regressions and give the GPU
tests fixed vectors that do not depend on re-running the oracle.  Run from the repo root:
    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from lq_cases import rand_lq, oracle_batch  # noqa: E402
from oracle import noc_oracle as O, problems as PR  # noqa: E402


def lq_fixtures():
    out = {}
    for nx, nu, N in [(2, 1, 50), (4, 1, 120), (8, 4, 48)]:
        for aff in (False, True):
            tag = f"lq_{nx}x{nu}_N{N}_{'aff' if aff else 'newton'}"
            case = rand_lq(7 + nx * 100 + N + int(aff), 2, N, nx, nu, affine=aff)
            ref = oracle_batch(case)
            for b in range(2):
                g = lambda k: None if k not in case else case[k][b]
                ddx, ddu, _ = O.dense_kkt(g("A"), g("B"), g("Q"), g("R"), g("M"), g("r"), g("P"),
                                          g("reg"), g("x0"), g("q"), g("c"), g("p"))
                assert np.max(np.abs(ddx - ref["dx"][b])) < 1e-10 * max(1, np.abs(ddx).max())
                assert np.max(np.abs(ddu - ref["du"][b])) < 1e-10 * max(1, np.abs(ddu).max())
            for k, v in case.items():
                out[f"{tag}/in/{k}"] = v
            for k, v in ref.items():
                out[f"{tag}/out/{k}"] = np.asarray(v)
    return out


def ipm_fixtures():
    out = {}
    N = 50
    prob = O.NumpyProblem(PR.pendulum_ocp(1.0 / N))
    u0 = 0.1 * np.random.default_rng(1).normal(size=(N, 1))
    x0 = np.array([0.1, -0.1])
    U, it, solves = O.par_interior_point_optimal_control(prob, u0, x0)
    Us, its = O.seq_interior_point_optimal_control(prob, u0, x0)
    out.update({"pend50/u0": u0, "pend50/x0": x0, "pend50/par_u": U,
                "pend50/par_iters": np.array(it), "pend50/par_kkt_solves": np.array(solves),
                "pend50/seq_u": Us, "pend50/seq_iters": np.array(its),
                "pend50/par_cost": np.array(prob.total_cost(O.rollout(prob.dynamics, U, x0), U, 0.0))})
    # one linearisation of cart-pole (N=20) at a random iterate: the LQ blocks of the first step
    N = 20
    prob = O.NumpyProblem(PR.cartpole_ocp(1.0 / N))
    rng = np.random.default_rng(4)
    u = 0.1 * rng.normal(size=(N, 1))
    x0 = np.array([0.01, 2 * np.pi - 0.01, 0.01, -0.01])
    X = O.rollout(prob.dynamics, u, x0)
    L = O.linearize(prob, X, u, 0.1)
    out.update({"cart20/u": u, "cart20/x": X})
    for k in ("A", "B", "Q", "R", "M", "r", "P", "cu", "lam"):
        out[f"cart20/{k}"] = L[k]
    out["cart20/cost"] = np.array(prob.total_cost(X, u, 0.1))
    return out


def newton_block_fixtures():
    """golden_v2: the LQ blocks of a real first Newton step (bp = 0.1, rp = 1, so
    reg = ||cu||_F, P:116-118) of the BASELINE problems -- pendulum N=100 (c2) and cart-pole
    N=200 (c3), two trajectories each from the SURVEY §8d input distributions -- linearised by
    the autodiff oracle (P:13-42), and the KKT step of each computed by the FAITHFUL sequential
    Riccati (S:42-90: Vxx propagated unsymmetrised, inv(Quu), eigh test), checked against the
    dense KKT solve at generation time.  The GPU tests compare the HIP path with these committed
    vectors directly (no live oracle)."""
    out = {}
    cases = [("pend100", PR.pendulum_ocp(1.0 / 100), 100, "pendulum"),
             ("cart200", PR.cartpole_ocp(1.0 / 200), 200, "cartpole")]
    for tag, tocp, N, name in cases:
        prob = O.NumpyProblem(tocp)
        rng = np.random.default_rng(2024 + N)
        if name == "pendulum":
            x0s = np.array([0.1, -0.1]) + 0.01 * rng.normal(size=(2, 2))
        else:
            x0s = np.array([0.01, 2 * np.pi - 0.01, 0.01, -0.01]) + 0.01 * rng.normal(size=(2, 4))
        u0s = 0.1 * rng.normal(size=(2, N, 1))
        blocks = {k: [] for k in ("x", "A", "B", "Q", "R", "M", "r", "P", "reg", "dx", "du", "pred",
                                  "feasible", "K", "d")}
        for b in range(2):
            X = O.rollout(prob.dynamics, u0s[b], x0s[b])
            L = O.linearize(prob, X, u0s[b], 0.1)
            reg = float(np.linalg.norm(L["cu"]))
            dx, du, pred, feas, K, d, S, v = O.kkt_solve(L["A"], L["B"], L["Q"], L["R"], L["M"],
                                                         L["r"], L["P"], reg, symmetrize=False)
            ddx, ddu, _ = O.dense_kkt(L["A"], L["B"], L["Q"], L["R"], L["M"], L["r"], L["P"], reg)
            assert np.max(np.abs(ddx - dx)) < 1e-10 * max(1, np.abs(ddx).max())
            assert np.max(np.abs(ddu - du)) < 1e-10 * max(1, np.abs(ddu).max())
            for k, val in (("x", X), ("reg", reg), ("dx", dx), ("du", du), ("pred", pred),
                           ("feasible", feas), ("K", K), ("d", d)):
                blocks[k].append(np.asarray(val))
            for k in ("A", "B", "Q", "R", "M", "r", "P"):
                blocks[k].append(L[k])
        out[f"{tag}/u0"] = u0s
        out[f"{tag}/x0"] = x0s
        for k, vals in blocks.items():
            out[f"{tag}/{k}"] = np.stack(vals)
    return out


if __name__ == "__main__":
    data = {}
    data.update(lq_fixtures())
    data.update(ipm_fixtures())
    path = os.path.join(HERE, "golden_v1.npz")
    if "--v2-only" not in sys.argv:
        np.savez_compressed(path, **data)
        print("wrote", path, os.path.getsize(path), "bytes,", len(data), "arrays")
    data2 = newton_block_fixtures()
    path2 = os.path.join(HERE, "golden_v2.npz")
    np.savez_compressed(path2, **data2)
    print("wrote", path2, os.path.getsize(path2), "bytes,", len(data2), "arrays")
