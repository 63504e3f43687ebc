"""ORACLE (test infrastructure only) -- numpy fp64 restatement of the reference's Newton step.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker.  The product path never imports it.

**Parity unpinned**: the reference (pure JAX, /root/reference/noc) ships no tests or golden vectors
and cannot run here (no jax / jaxlib / paroc).  Every function below cites the reference line it
restates; the restatement is cross-validated by two independent oracles (a dense KKT solve and a
from-scratch associative-scan restatement of paroc's par_bwd_pass/par_fwd_pass), see
tests/test_oracle.py.

Abbreviations: S = noc/seq_interior_point_newton.py, P = noc/par_interior_point_newton.py,
C = noc/costates.py, U = noc/utils.py, D = noc/differential_dynamic_programming.py.

LQ sub-problem conventions (shared with the HIP kernel, include/noc_hip.h)
-------------------------------------------------------------------------
stage k (0 <= k < N):  1/2 x'Qx + x'Mu + 1/2 u'(R + reg I)u + r'u + q'x,  x+ = A x + B u + c
terminal:              1/2 x'P x + p'x
initial state:         x_0 = x0  (the Newton step uses x0 = 0, c = q = p = 0: P:72, P:121-123)
value function:        V_k(x) = 1/2 x'S_k x + v_k'x + const   (S = Vxx, v = Vx of S:45-64)
gains:                 du_k = K_k dx_k + d_k                     (S:89)
pred:                  sum_k d_k'Qu_k + 1/2 d_k'Quu_k d_k        (S:63,75)
feasible:              all_k  Quu_k > 0 (positive definite)       (S:52-53,75)
"""
from __future__ import annotations

import numpy as np

# ----------------------------------------------------------------------------------------------
# utilities (U:57-63)
# ----------------------------------------------------------------------------------------------



def _cube(c):
    """(2 gain - 1) ** 3 of S:141 / P:169 / D:131 as JAX evaluates it: `x ** 3` with a Python int
    is lax.integer_pow, lowered by repeated squaring to x * (x * x) -- two roundings, which can
    differ from numpy's pow(x, 3.0) in the last bit (and the device kernels multiply the same
    way).  A last-bit difference in rp steers every later step."""
    return c * (c * c)

def rollout(dynamics, controls: np.ndarray, x0: np.ndarray) -> np.ndarray:
    """U:57-63 -- sequential x_{k+1} = f(x_k, u_k); returns (N+1, nx)."""
    xs = [np.asarray(x0, dtype=np.float64)]
    for u in controls:
        xs.append(np.asarray(dynamics(xs[-1], u), dtype=np.float64))
    return np.stack(xs)


def seq_costates(lam_T: np.ndarray, cx: np.ndarray, fx: np.ndarray) -> np.ndarray:
    """C:43-54 -- lambda_k = cx_k + fx_k' lambda_{k+1}; returns (N+1, nx)."""
    N = cx.shape[0]
    lam = np.zeros((N + 1, lam_T.shape[0]))
    lam[N] = lam_T
    for k in range(N - 1, -1, -1):
        lam[k] = cx[k] + fx[k].T @ lam[k + 1]
    return lam


def compute_lqr_params(lam: np.ndarray, cu, cxx, cuu, cxu, fu, fxx, fuu, fxu):
    """S:28-39 == P:31-42 -- ru = cu + fu' l, Q = cxx + l.fxx, R = cuu + l.fuu, M = cxu + l.fxu
    with l = lambda[1:]."""
    l = lam[1:]
    ru = cu + np.einsum("kij,ki->kj", fu, l)
    Q = cxx + np.einsum("ki,kijl->kjl", l, fxx)
    R = cuu + np.einsum("ki,kijl->kjl", l, fuu)
    M = cxu + np.einsum("ki,kijl->kjl", l, fxu)
    return ru, Q, R, M


# ----------------------------------------------------------------------------------------------
# sequential Riccati KKT solve (S:42-90), generalised with c, q, p, x0 for the LQT entry point
# ----------------------------------------------------------------------------------------------


def riccati_bwd(A, B, Q, R, M, r, P, reg=0.0, q=None, c=None, p=None, symmetrize=False):
    """S:42-75 bwd_pass.  Returns (K, d, S, v, pred, feasible).

    Quu gets reg*I (S:51 adds rp*I to Quu; P:116-118 adds reg*I to R -- identical).
    Uses inv(Quu) exactly like S:58-62 and the eigh convexity test of S:52-53.
    symmetrize=False is the faithful restatement: Vxx is propagated unsymmetrised (S:62), whose
    antisymmetric rounding error can grow along long horizons (measured: 6e-4 drift from the exact
    KKT solution at nx=8, nu=4, N=200; tests/test_oracle.py).  symmetrize=True replaces Vxx by
    its symmetric part every stage (the numerically stable variant used as the parity reference
    where the faithful one drifts).
    """
    N, nx, nu = B.shape
    K = np.zeros((N, nu, nx))
    d = np.zeros((N, nu))
    S = np.zeros((N + 1, nx, nx))
    v = np.zeros((N + 1, nx))
    S[N] = P
    v[N] = 0.0 if p is None else p
    pred = 0.0
    feasible = True
    I = np.eye(nu)
    for k in range(N - 1, -1, -1):
        Vxx, Vx = S[k + 1], v[k + 1]
        g = Vx + (Vxx @ c[k] if c is not None else 0.0)
        Qxx = Q[k] + A[k].T @ Vxx @ A[k]
        Quu = R[k] + B[k].T @ Vxx @ B[k] + reg * I
        eig = np.linalg.eigvalsh(Quu)
        feasible = feasible and bool(np.all(eig > 0))
        Qxu = M[k] + A[k].T @ Vxx @ B[k]
        Qu = r[k] + B[k].T @ g
        Qx = A[k].T @ g + (q[k] if q is not None else 0.0)
        Quu_inv = np.linalg.inv(Quu)
        kk = -Quu_inv @ Qu
        KK = -Quu_inv @ Qxu.T
        v[k] = Qx - Qu @ Quu_inv @ Qxu.T
        S[k] = Qxx - Qxu @ Quu_inv @ Qxu.T
        if symmetrize:
            S[k] = 0.5 * (S[k] + S[k].T)
        pred += kk @ Qu + 0.5 * kk @ Quu @ kk
        K[k], d[k] = KK, kk
    return K, d, S, v, pred, feasible


def riccati_fwd(A, B, K, d, x0=None, c=None):
    """S:78-90 fwd_pass (dx_0 = x0, default 0).  Returns (du (N,nu), dx (N+1,nx))."""
    N, nx, nu = B.shape
    dx = np.zeros((N + 1, nx))
    if x0 is not None:
        dx[0] = x0
    du = np.zeros((N, nu))
    for k in range(N):
        du[k] = K[k] @ dx[k] + d[k]
        dx[k + 1] = (A[k] + B[k] @ K[k]) @ dx[k] + B[k] @ d[k] + (c[k] if c is not None else 0.0)
    return du, dx


def kkt_solve(A, B, Q, R, M, r, P, reg=0.0, x0=None, q=None, c=None, p=None, symmetrize=False):
    """bwd + fwd: returns (dx, du, pred, feasible, K, d, S, v)."""
    K, d, S, v, pred, feas = riccati_bwd(A, B, Q, R, M, r, P, reg, q, c, p, symmetrize)
    du, dx = riccati_fwd(A, B, K, d, x0, c)
    return dx, du, pred, feas, K, d, S, v


# ----------------------------------------------------------------------------------------------
# independent oracle 1: dense KKT solve of the same LQ problem
# ----------------------------------------------------------------------------------------------


def dense_kkt(A, B, Q, R, M, r, P, reg=0.0, x0=None, q=None, c=None, p=None):
    """Assemble and solve the full KKT system; returns (dx (N+1,nx), du (N,nu), objective)."""
    N, nx, nu = B.shape
    nX = (N + 1) * nx
    nZ = nX + N * nu
    H = np.zeros((nZ, nZ))
    g = np.zeros(nZ)
    xi = lambda k: slice(k * nx, (k + 1) * nx)
    ui = lambda k: slice(nX + k * nu, nX + (k + 1) * nu)
    for k in range(N):
        H[xi(k), xi(k)] += Q[k]
        H[xi(k), ui(k)] += M[k]
        H[ui(k), xi(k)] += M[k].T
        H[ui(k), ui(k)] += R[k] + reg * np.eye(nu)
        g[ui(k)] += r[k]
        if q is not None:
            g[xi(k)] += q[k]
    H[xi(N), xi(N)] += P
    if p is not None:
        g[xi(N)] += p
    nE = (N + 1) * nx
    E = np.zeros((nE, nZ))
    e = np.zeros(nE)
    E[0:nx, xi(0)] = np.eye(nx)
    e[0:nx] = 0.0 if x0 is None else x0
    for k in range(N):
        row = slice((k + 1) * nx, (k + 2) * nx)
        E[row, xi(k + 1)] = np.eye(nx)
        E[row, xi(k)] = -A[k]
        E[row, ui(k)] = -B[k]
        e[row] = 0.0 if c is None else c[k]
    KKT = np.block([[H, E.T], [E, np.zeros((nE, nE))]])
    rhs = np.concatenate([-g, e])
    sol = np.linalg.solve(KKT, rhs)
    z = sol[:nZ]
    obj = 0.5 * z @ H @ z + g @ z
    return z[:nX].reshape(N + 1, nx), z[nX:].reshape(N, nu), obj


# ----------------------------------------------------------------------------------------------
# independent oracle 2: associative-scan restatement of paroc.par_bwd_pass / par_fwd_pass
# (Saerkkae & Garcia-Fernandez temporal-parallel LQ; call sites P:120-123, LM:68-69)
# ----------------------------------------------------------------------------------------------


def stage_element(A, B, Q, R, M, r, reg=0.0, q=None, c=None):
    """Element (Ae, be, Ce, eta, J) of one stage; V = 1/2 x'Jx - eta'x convention."""
    nx = A.shape[0]
    Rr = R + reg * np.eye(R.shape[0])
    Ri = np.linalg.inv(Rr)
    c = np.zeros(nx) if c is None else c
    q = np.zeros(nx) if q is None else q
    Ae = A - B @ Ri @ M.T
    be = c - B @ Ri @ r
    Ce = B @ Ri @ B.T
    eta = M @ Ri @ r - q
    J = Q - M @ Ri @ M.T
    return Ae, be, Ce, eta, J


def combine(e1, e2):
    """e_ij (x) e_jk -> e_ik (associative)."""
    A1, b1, C1, n1, J1 = e1
    A2, b2, C2, n2, J2 = e2
    nx = A1.shape[0]
    T = np.linalg.inv(np.eye(nx) + C1 @ J2)
    TA = T @ A1
    A = A2 @ TA
    b = A2 @ T @ (b1 + C1 @ n2) + b2
    C = A2 @ T @ C1 @ A2.T + C2
    n = TA.T @ (n2 - J2 @ b1) + n1
    J = TA.T @ J2 @ A1 + J1
    return A, b, C, n, J


def scan_bwd(A, B, Q, R, M, r, P, reg=0.0, q=None, c=None, p=None, tree=False):
    """Reverse associative scan -> value functions S_k, v_k (k = 0..N)."""
    N, nx, _ = A.shape
    elems = [stage_element(A[k], B[k], Q[k], R[k], M[k], r[k], reg,
                           None if q is None else q[k], None if c is None else c[k])
             for k in range(N)]
    term = (np.zeros((nx, nx)), np.zeros(nx), np.zeros((nx, nx)),
            -(np.zeros(nx) if p is None else p), P)
    elems.append(term)
    suffix = [None] * (N + 1)
    if not tree:
        acc = elems[N]
        suffix[N] = acc
        for k in range(N - 1, -1, -1):
            acc = combine(elems[k], acc)
            suffix[k] = acc
    else:  # Hillis-Steele order -- exercises associativity
        cur = list(elems)
        d = 1
        while d < N + 1:
            cur = [combine(cur[i], cur[i + d]) if i + d <= N else cur[i] for i in range(N + 1)]
            d *= 2
        suffix = cur
    S = np.stack([s[4] for s in suffix])
    v = np.stack([-s[3] for s in suffix])
    return S, v


def gains_from_values(A, B, R, M, r, S, v, reg=0.0, c=None):
    N, nx, nu = B.shape
    K = np.zeros((N, nu, nx))
    d = np.zeros((N, nu))
    pred = 0.0
    feas = True
    for k in range(N):
        g = v[k + 1] + (S[k + 1] @ c[k] if c is not None else 0.0)
        Quu = R[k] + reg * np.eye(nu) + B[k].T @ S[k + 1] @ B[k]
        Qux = M[k].T + B[k].T @ S[k + 1] @ A[k]
        Qu = r[k] + B[k].T @ g
        feas = feas and bool(np.all(np.linalg.eigvalsh(Quu) > 0))
        K[k] = -np.linalg.solve(Quu, Qux)
        d[k] = -np.linalg.solve(Quu, Qu)
        pred += d[k] @ Qu + 0.5 * d[k] @ Quu @ d[k]
    return K, d, pred, feas


def scan_fwd(A, B, K, d, x0=None, c=None):
    """Forward affine associative scan (C:6-16 combine_fc pattern) from dx_0 = x0."""
    N, nx, nu = B.shape
    x0 = np.zeros(nx) if x0 is None else x0
    F = [A[k] + B[k] @ K[k] for k in range(N)]
    f = [B[k] @ d[k] + (c[k] if c is not None else 0.0) for k in range(N)]
    # element 0 is constant: x_1 = F0 x0 + f0  (C:19-31 par_init)
    elems = [(np.zeros((nx, nx)), F[0] @ x0 + f[0])] + [(F[k], f[k]) for k in range(1, N)]
    cur = list(elems)
    dd = 1
    while dd < N:
        cur = [(cur[i][0] @ cur[i - dd][0], cur[i][0] @ cur[i - dd][1] + cur[i][1])
               if i - dd >= 0 else cur[i] for i in range(N)]
        dd *= 2
    dx = np.vstack([x0] + [e[1] for e in cur])
    du = np.stack([K[k] @ dx[k] + d[k] for k in range(N)])
    return du, dx


# ----------------------------------------------------------------------------------------------
# Newton step and loops
# ----------------------------------------------------------------------------------------------


class NumpyProblem:
    """Adapter over oracle.problems.TorchOCP giving numpy-level access to the callables."""

    def __init__(self, tocp):
        from oracle import problems as pr
        self.t = tocp
        self.pr = pr
        self.nx, self.nu = tocp.nx, tocp.nu

    def dynamics(self, x, u):
        return self.pr.dynamics_np(self.t, x, u)

    def derivatives(self, X, U, bp):
        return self.pr.compute_derivatives(self.t, X, U, bp)

    def final_grad_hess(self, xN):
        return self.pr.final_grad_hess(self.t, xN)

    def total_cost(self, X, U, bp):
        return self.pr.total_cost_np(self.t, X, U, bp)

    def feasible(self, X, U):
        return bool(np.all(self.pr.constraints_np(self.t, X[:-1], U) <= 0))


def linearize(prob: NumpyProblem, X, U, bp):
    """S:98-101 / P:145-149: derivatives, costates, LQ blocks.  Returns a dict of blocks."""
    cx, cu, cxx, cuu, cxu, fx, fu, fxx, fuu, fxu = prob.derivatives(X, U, bp)
    lam_T, P = prob.final_grad_hess(X[-1])
    lam = seq_costates(lam_T, cx, fx)
    ru, Q, R, M = compute_lqr_params(lam, cu, cxx, cuu, cxu, fu, fxx, fuu, fxu)
    return dict(A=fx, B=fu, Q=Q, R=R, M=M, r=ru, P=P, cu=cu, lam=lam)


def seq_solution(prob, X, U, bp, rp):
    """S:98-105: (dx, du, dV, bp_feasible, Hu)."""
    L = linearize(prob, X, U, bp)
    K, d, _, _, pred, feas = riccati_bwd(L["A"], L["B"], L["Q"], L["R"], L["M"], L["r"], L["P"], rp)
    du, dx = riccati_fwd(L["A"], L["B"], K, d)
    return dx, du, pred, feas, L["r"]


def seq_newton_oc(prob, U, x0, bp, max_iter=100000):
    """S:108-177 -- one accept/reject per iteration; stops when |Hu|inf < 1e-4 AND bwd feasible."""
    X = rollout(prob.dynamics, U, x0)
    mu, nu_ = 1.0, 2.0
    t = 0
    Hu_norm, bpf = 1.0, True
    while not (Hu_norm < 1e-4 and bpf) and t < max_iter:
        cost = prob.total_cost(X, U, bp)
        dx, du, pred, bpf, Hu = seq_solution(prob, X, U, bp, mu)
        Hu_norm = float(np.max(np.abs(Hu)))
        tU, tX = U + du, X + dx
        new_cost = prob.total_cost(tX, tU, bp) if prob.feasible(tX, tU) else np.inf
        with np.errstate(all="ignore"):
            gain = (new_cost - cost) / pred
        accept = bool(gain > 0) and bpf
        if accept:
            mu = mu * max(1.0 / 3.0, 1.0 - _cube(2.0 * gain - 1.0))
            nu_ = 2.0
            X, U = tX, tU
        else:
            mu = mu * nu_
            nu_ = 2 * nu_
        t += 1
    return X, U, t


def seq_interior_point_optimal_control(prob, U, x0):
    """S:180-202 barrier schedule 0.1 / 5^k while bp > 1e-4."""
    bp, total = 0.1, 0
    while bp > 1e-4:
        _, U, it = seq_newton_oc(prob, U, x0, bp)
        bp /= 5
        total += it
    return U, total


def par_newton_oc(prob, U, x0, bp, terminal="final_cost", trace=None):
    """P:127-225 semantics (the KKT solve itself is unique; see module docstring).

    terminal="final_cost": terminal Hessian = hessian(final_cost)(x_N) (S:66, the build default).
    terminal="stage0":     the reference's par quirk XT = Q[0] (P:73).
    Returns (X, U, outer_iterations, kkt_solves).
    """
    X = rollout(prob.dynamics, U, x0)
    rp, r_inc = 1.0, 2.0
    it, solves = 0, 0
    Hu_norm = 1.0
    while not (Hu_norm < 1e-4 or it > 1000):
        cost = prob.total_cost(X, U, bp)
        L = linearize(prob, X, U, bp)
        P = L["P"] if terminal == "final_cost" else L["Q"][0]
        gnorm = float(np.linalg.norm(L["cu"]))
        inner = 0
        success = False
        while True:
            reg = rp * gnorm                                            # P:116-118
            K, d, _, _, pred, feas = riccati_bwd(L["A"], L["B"], L["Q"], L["R"], L["M"], L["r"],
                                                 P, reg)
            du, dx = riccati_fwd(L["A"], L["B"], K, d)
            solves += 1
            tU, tX = U + du, X + dx
            Hn = float(np.max(np.abs(L["r"])))
            new_cost = prob.total_cost(tX, tU, bp) if prob.feasible(tX, tU) else np.inf
            with np.errstate(all="ignore"):
                gain = (new_cost - cost) / pred
            success = bool(gain > 0.0) and feas
            if success:
                rp = rp * max(1.0 / 3.0, 1.0 - _cube(2.0 * gain - 1.0))
                r_inc = 2.0
            else:
                rp = rp * r_inc
                r_inc = 2 * r_inc
            rp = min(max(rp, 1e-16), 1e16)                              # P:173
            inner += 1
            if trace is not None:
                trace.append(dict(it=it, inner=inner, reg=reg, pred=pred, gain=gain,
                                  success=success, rp=rp, cost=cost, new_cost=new_cost, hu=Hn,
                                  bp=bp))
            if success or inner > 500:                                  # P:177-182
                break
        X, U, Hu_norm = tX, tU, Hn                                      # P:184-188
        it += 1
    return X, U, it, solves


def par_interior_point_optimal_control(prob, U, x0, terminal="final_cost", trace=None):
    """P:228-254.  Returns (U*, total outer Newton iterations, total KKT solves).  trace: a
    list that receives one dict per KKT solve (par_newton_oc)."""
    bp, total, solves = 0.1, 0, 0
    while bp > 1e-4:
        _, U, it, s = par_newton_oc(prob, U, x0, bp, terminal, trace)
        bp /= 5
        total += it
        solves += s
    return U, total, solves


# ----------------------------------------------------------------------------------------------
# interior-point DDP (D:28-208): sequential second-order backward pass + nonlinear rollout
# ----------------------------------------------------------------------------------------------
def ddp_bwd_pass(Vx_T, Vxx_T, derivs, reg_param):
    """D:28-70.  reg = reg_param * ||cu||_F; Q-function with the second-order dynamics terms
    Vx . fxx (tensordot over the output axis); eigh(Quu) > 0 feasibility; LU solves.
    Returns (ffgain k (N,nu), gain K (N,nu,nx), pred_reduction, feasible, Hu = Qu (N,nu))."""
    cx, cu, cxx, cuu, cxu, fx, fu, fxx, fuu, fxu = derivs
    N, nu = cu.shape
    nx = cx.shape[1]
    reg = reg_param * float(np.linalg.norm(cu))                         # D:34-35
    Vx, Vxx = np.asarray(Vx_T, dtype=np.float64), np.asarray(Vxx_T, dtype=np.float64)
    k = np.zeros((N, nu))
    K = np.zeros((N, nu, nx))
    Hu = np.zeros((N, nu))
    dV = np.zeros(N)
    feasible = True
    for t in range(N - 1, -1, -1):                                      # lax.scan(reverse=True)
        Qx = cx[t] + fx[t].T @ Vx                                       # D:41
        Qu = cu[t] + fu[t].T @ Vx                                       # D:42
        Qxx = cxx[t] + fx[t].T @ Vxx @ fx[t] + np.tensordot(Vx, fxx[t], axes=1)   # D:43
        Qxu = cxu[t] + fx[t].T @ Vxx @ fu[t] + np.tensordot(Vx, fxu[t], axes=1)   # D:44
        Quu = cuu[t] + fu[t].T @ Vxx @ fu[t] + np.tensordot(Vx, fuu[t], axes=1)   # D:45
        Quu = Quu + reg * np.eye(nu)                                    # D:46
        feasible &= bool(np.all(np.linalg.eigvalsh(Quu) > 0))           # D:47-48
        k[t] = -np.linalg.solve(Quu, Qu)                                # D:50
        K[t] = -np.linalg.solve(Quu, Qxu.T)                             # D:51
        dV[t] = -0.5 * Qu @ np.linalg.solve(Quu, Qu)                    # D:53
        Vx = Qx - Qu @ np.linalg.solve(Quu, Qxu.T)                      # D:54
        Vxx = Qxx - Qxu @ np.linalg.solve(Quu, Qxu.T)                   # D:55
        Hu[t] = Qu
    return k, K, float(dV.sum()), feasible, Hu                          # D:61-70


def ddp_nonlin_rollout(prob, K, k, X, U):
    """D:73-90: u_hat = u + k + K (x_hat - x); x_hat+ = f(x_hat, u_hat) from x_hat_0 = x_0."""
    N = U.shape[0]
    TX = np.zeros_like(X)
    TU = np.zeros_like(U)
    xh = X[0].copy()
    for t in range(N):
        uh = U[t] + k[t] + K[t] @ (xh - X[t])
        TX[t], TU[t] = xh, uh
        xh = prob.dynamics(xh, uh)
    TX[N] = xh
    return TX, TU


def ddp(prob, U, x0, bp, trace=None):
    """D:98-186.  Quirk kept: inside one inner (retry) loop the failure multiplier is the OUTER
    iteration's reg_inc (D:132 closes over it), while r_inc doubles per failure and becomes the
    next outer iteration's reg_inc (D:133, D:154).  The last trial is kept even if the retry cap
    ended the inner loop (D:154).  Returns (X, U, iterations, bwd passes)."""
    X = rollout(prob.dynamics, U, x0)                                   # D:102
    reg_param, reg_inc = 1.0, 2.0                                       # D:102-103
    it, passes, Hu_norm = 0, 0, 1.0
    while not (Hu_norm < 1e-4 or it > 500):                             # D:167-170
        cost = prob.total_cost(X, U, bp)                                # D:109
        derivs = prob.derivatives(X, U, bp)                             # D:112
        Vx_T, Vxx_T = prob.final_grad_hess(X[-1])                       # D:58-59
        rp, r_inc, inner = reg_param, reg_inc, 0
        while True:
            k, K, pred, feas, Hu = ddp_bwd_pass(Vx_T, Vxx_T, derivs, rp)
            passes += 1
            TX, TU = ddp_nonlin_rollout(prob, K, k, X, U)
            Hn = float(np.max(np.abs(Hu)))
            new_cost = prob.total_cost(TX, TU, bp) if prob.feasible(TX, TU) else np.inf
            with np.errstate(all="ignore"):
                gain = (new_cost - cost) / pred
            success = bool(gain > 0) and feas                          # D:128
            if success:
                rp = rp * max(1.0 / 3.0, 1.0 - _cube(2.0 * gain - 1.0))
                r_inc = 2.0
            else:
                rp = rp * reg_inc                                       # outer reg_inc (D:132)
                r_inc = 2 * r_inc
            rp = min(max(rp, 1e-16), 1e16)                              # D:135
            inner += 1
            if trace is not None:
                trace.append(dict(it=it, inner=inner, pred=pred, gain=gain, success=success, rp=rp,
                                  cost=cost, new_cost=new_cost, hu=Hn))
            if success or inner > 500:                                  # D:147-152
                break
        X, U, Hu_norm, reg_param, reg_inc = TX, TU, Hn, rp, r_inc       # D:154-162
        it += 1
    return X, U, it, passes


def interior_point_ddp(prob, U, x0):
    """D:189-208: barrier 0.1 / 5^k while bp > 1e-4.  Returns (U*, total iterations, passes)."""
    bp, total, passes = 0.1, 0, 0
    while bp > 1e-4:
        _, U, it, p = ddp(prob, U, x0, bp)
        bp /= 5
        total += it
        passes += p
    return U, total, passes
