"""Test infrastructure: a numpy model of the HIP chunked wave-scan (csrc/kkt_scan.hip), lane by lane.

It mirrors the kernel's four phases exactly (chunk assignment, in-chunk prepend, Hillis-Steele
cross-lane scan with shuffle-down semantics, in-chunk Riccati with the true boundary, forward
affine scan) so that the algorithm can be validated on the CPU against the oracle.  Value
convention: V(x) = 1/2 x'Jx + nu'x (nu = -eta of the paper's convention).
"""
import numpy as np


def chunk_bounds(N, L):
    base, rem = divmod(N, L)
    starts, lens = [], []
    for l in range(L):
        n = base + (1 if l < rem else 0)
        starts.append(l * base + min(l, rem))
        lens.append(n)
    return starts, lens


def _ldl_solve(W, rhs):
    return np.linalg.solve(W, rhs)


def prepend(acc, A, B, Q, R, M, r, q, c):
    Aa, ba, Ca, nua, Ja = acc
    JA = Ja @ A
    JB = Ja @ B
    g = Ja @ c + nua
    W = R + B.T @ JB
    Qux = M.T + JB.T @ A
    Qu = r + B.T @ g
    K = -_ldl_solve(W, Qux)
    k = -_ldl_solve(W, Qu)
    Jn = Q + A.T @ JA + Qux.T @ K
    nun = q + A.T @ g + Qux.T @ k
    F = A + B @ K
    f = B @ k + c
    AB = Aa @ B
    Cn = Ca + AB @ _ldl_solve(W, AB.T)
    bn = Aa @ f + ba
    An = Aa @ F
    return (An, bn, Cn, nun, 0.5 * (Jn + Jn.T))


def combine(e1, e2):
    A1, b1, C1, nu1, J1 = e1
    A2, b2, C2, nu2, J2 = e2
    nx = A1.shape[0]
    X = np.eye(nx) + C1 @ J2
    Z = np.linalg.solve(X, np.hstack([A1, (b1 - C1 @ nu2)[:, None], C1]))
    TA, Tb, TC = Z[:, :nx], Z[:, nx], Z[:, nx + 1:]
    A = A2 @ TA
    b = A2 @ Tb + b2
    C = A2 @ TC @ A2.T + C2
    nu = TA.T @ (nu2 + J2 @ b1) + nu1
    J = TA.T @ (J2 @ A1) + J1
    return (A, b, 0.5 * (C + C.T), nu, 0.5 * (J + J.T))


def model_kkt(A, B, Q, R, M, r, P, reg=0.0, x0=None, q=None, c=None, p=None, L=64):
    N, nx, nu = B.shape
    q = np.zeros((N, nx)) if q is None else q
    c = np.zeros((N, nx)) if c is None else c
    p = np.zeros(nx) if p is None else p
    x0 = np.zeros(nx) if x0 is None else x0
    Rr = R + reg * np.eye(nu)
    starts, lens = chunk_bounds(N, L)
    # phase 1
    elems = []
    for l in range(L):
        if l == L - 1:
            acc = (np.zeros((nx, nx)), np.zeros(nx), np.zeros((nx, nx)), p.copy(), P.copy())
        else:
            acc = (np.eye(nx), np.zeros(nx), np.zeros((nx, nx)), np.zeros(nx), np.zeros((nx, nx)))
        for s in range(starts[l] + lens[l] - 1, starts[l] - 1, -1):
            acc = prepend(acc, A[s], B[s], Q[s], Rr[s], M[s], r[s], q[s], c[s])
        elems.append(acc)
    # phase 2: reverse inclusive Hillis-Steele (lane l <- l (x) l+d)
    d = 1
    while d < L:
        elems = [combine(elems[l], elems[l + d]) if l + d < L else elems[l] for l in range(L)]
        d *= 2
    # phase 3
    K = np.zeros((N, nu, nx)); kk = np.zeros((N, nu))
    S = np.zeros((N + 1, nx, nx)); v = np.zeros((N + 1, nx))
    S[N], v[N] = P, p
    pred = 0.0
    feas = True
    maps = []
    for l in range(L):
        if l == L - 1:
            Sc, vc = P.copy(), p.copy()
        else:
            Sc, vc = elems[l + 1][4].copy(), elems[l + 1][3].copy()
        Phi, phi = np.eye(nx), np.zeros(nx)
        for s in range(starts[l] + lens[l] - 1, starts[l] - 1, -1):
            SA, SB = Sc @ A[s], Sc @ B[s]
            g = Sc @ c[s] + vc
            Quu = Rr[s] + B[s].T @ SB
            Qux = M[s].T + SB.T @ A[s]
            Qu = r[s] + B[s].T @ g
            feas = feas and bool(np.all(np.linalg.eigvalsh(Quu) > 0))
            K[s] = -np.linalg.solve(Quu, Qux)
            kk[s] = -np.linalg.solve(Quu, Qu)
            pred += kk[s] @ Qu + 0.5 * kk[s] @ Quu @ kk[s]
            Sn = Q[s] + A[s].T @ SA + Qux.T @ K[s]
            vc = q[s] + A[s].T @ g + Qux.T @ kk[s]
            Sc = 0.5 * (Sn + Sn.T)
            S[s], v[s] = Sc, vc
            F = A[s] + B[s] @ K[s]
            f = B[s] @ kk[s] + c[s]
            phi = phi + Phi @ f
            Phi = Phi @ F
        maps.append((Phi, phi))
    # phase 4: forward inclusive scan, lane 0 map made constant
    Phi0, phi0 = maps[0]
    maps[0] = (np.zeros((nx, nx)), Phi0 @ x0 + phi0)
    d = 1
    while d < L:
        maps = [(maps[l][0] @ maps[l - d][0], maps[l][0] @ maps[l - d][1] + maps[l][1])
                if l - d >= 0 else maps[l] for l in range(L)]
        d *= 2
    dx = np.zeros((N + 1, nx)); du = np.zeros((N, nu))
    for l in range(L):
        x = x0.copy() if l == 0 else maps[l - 1][1].copy()
        for s in range(starts[l], starts[l] + lens[l]):
            dx[s] = x
            du[s] = K[s] @ x + kk[s]
            x = A[s] @ x + B[s] @ du[s] + c[s]
        if l == L - 1:
            dx[N] = x
    return dx, du, pred, feas, K, kk, S, v
