"""Seeded LQ problem generators shared by the CPU and GPU parity tests (test infrastructure)."""
import numpy as np


def rand_lq(seed, Bt, N, nx, nu, affine=False, spread=0.5):
    rng = np.random.default_rng(seed)
    # well-conditioned dynamics: a near-orthogonal map (spectral radius ~0.98) plus small noise,
    # like a discretised ODE; purely random A makes long-horizon KKT systems exponentially
    # ill-conditioned for every solver, which tests nothing.
    G0 = rng.normal(size=(Bt, N, nx, nx))
    Qo, _ = np.linalg.qr(G0)
    A = 0.98 * Qo + 0.1 * spread * rng.normal(size=(Bt, N, nx, nx)) / np.sqrt(nx)
    B = rng.normal(size=(Bt, N, nx, nu))
    G = rng.normal(size=(Bt, N, nx + nu, nx + nu))
    H = np.einsum("bkij,bklj->bkil", G, G) / (nx + nu) + 0.1 * np.eye(nx + nu)
    Q, M, R = H[..., :nx, :nx].copy(), H[..., :nx, nx:].copy(), H[..., nx:, nx:].copy()
    r = rng.normal(size=(Bt, N, nu))
    GP = rng.normal(size=(Bt, nx, nx))
    P = np.einsum("bij,bkj->bik", GP, GP) / nx + np.eye(nx)
    reg = np.abs(rng.normal(size=Bt)) * 0.3
    out = dict(A=A, B=B, Q=Q, R=R, M=M, r=r, P=P, reg=reg)
    if affine:
        out.update(x0=rng.normal(size=(Bt, nx)), q=rng.normal(size=(Bt, N, nx)),
                   c=rng.normal(size=(Bt, N, nx)) * 0.1, p=rng.normal(size=(Bt, nx)))
    return out


def oracle_batch(case, symmetrize=True):
    from oracle import noc_oracle as O
    Bt = case["A"].shape[0]
    res = []
    for b in range(Bt):
        g = lambda k: None if k not in case else case[k][b]
        res.append(O.kkt_solve(case["A"][b], case["B"][b], case["Q"][b], case["R"][b],
                               case["M"][b], case["r"][b], case["P"][b], case["reg"][b],
                               g("x0"), g("q"), g("c"), g("p"), symmetrize=symmetrize))
    keys = ["dx", "du", "pred", "feasible", "K", "d", "S", "v"]
    return {k: np.stack([np.asarray(r[i]) for r in res]) for i, k in enumerate(keys)}
