"""Registered problem families (device-side dynamics/costs live in csrc/ipm_kernels.hip).

Each constructor returns the reference's `OCP` (five NumPy-callable functions, same semantics as
the reference examples) with the `family` descriptor the HIP kernels consume:

  pendulum(dt)                      examples/pendulum_runtime.py:19-72   (nx=2, nu=1, |u|<=5)
  cartpole(dt)                      examples/cartpole_runtime.py:18-82   (nx=4, nu=1, |u|<=50)
  double_integrators(n, step, ...)  examples/linear_mpc_parallel.py:24-63 (nx=2n, nu=n; n=1 is
                                    examples/linear_demo_cuda.py:19-62, unconstrained LQR)
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List

import numpy as np

from . import _lib
from .optimal_control_problem import OCP
from .utils import discretize_dynamics, euler, wrap_angle


@dataclass
class Family:
    kind: int
    nx: int
    nu: int
    dt: float = 0.0
    u_bound: float = 0.0          # <= 0: no constraints / no barrier
    wrap_index: int = -1
    goal: List[float] = field(default_factory=list)
    wx: List[float] = field(default_factory=list)
    wu: List[float] = field(default_factory=list)
    wf: List[float] = field(default_factory=list)
    A: np.ndarray = None
    B: np.ndarray = None
    lib_path: str = None          # a registered family's own build (noc.families), else None
    name: str = ""

    def to_c(self) -> _lib.NocFamily:
        c = _lib.NocFamily()
        c.kind, c.nx, c.nu, c.wrap_index = self.kind, self.nx, self.nu, self.wrap_index
        c.dt, c.u_bound = float(self.dt), float(self.u_bound)
        for name in ("goal", "wx", "wu", "wf"):
            arr = getattr(c, name)
            for i, v in enumerate(getattr(self, name)):
                arr[i] = float(v)
        if self.A is not None:
            for i, v in enumerate(np.asarray(self.A, dtype=np.float64).ravel()):
                c.A[i] = v
            for i, v in enumerate(np.asarray(self.B, dtype=np.float64).ravel()):
                c.B[i] = v
        return c


def _box_constraints(bound):
    def constraints(state, control):
        control = np.atleast_1d(control)
        return np.concatenate((control - bound, -control - bound))
    return constraints


def _quadratic_barrier_costs(fam: Family):
    goal, wx, wu, wf = (np.asarray(v, dtype=np.float64) for v in (fam.goal, fam.wx, fam.wu, fam.wf))
    cons = _box_constraints(fam.u_bound)

    def _err(x):
        x = np.array(x, dtype=np.float64, copy=True)
        if fam.wrap_index >= 0:
            x[fam.wrap_index] = wrap_angle(x[fam.wrap_index])
        return x - goal

    def final_cost(state):
        e = _err(state)
        return 0.5 * float(e @ (wf * e))

    def stage_cost(state, action, bp):
        e = _err(state)
        u = np.atleast_1d(action)
        c = 0.5 * float(e @ (wx * e)) + 0.5 * float(u @ (wu * u))
        if fam.u_bound > 0:
            with np.errstate(invalid="ignore", divide="ignore"):
                c -= bp * float(np.sum(np.log(-cons(state, u))))
        return c

    def total_cost(states, controls, bp):
        return final_cost(states[-1]) + sum(stage_cost(x, u, bp) for x, u in zip(states[:-1], controls))

    # the device solvers find the family through the callables too (seq bwd_pass takes
    # ocp.final_cost, S:42-66)
    for fn in (final_cost, stage_cost, total_cost):
        fn.family = fam

    constraints = cons if fam.u_bound > 0 else (lambda state, control: -1.0)
    return constraints, stage_cost, final_cost, total_cost


def pendulum(dt: float) -> OCP:
    """Constrained pendulum, examples/pendulum_runtime.py:19-72 (Euler, PR:88)."""
    fam = Family(kind=_lib.FAMILY_PENDULUM, nx=2, nu=1, dt=dt, u_bound=5.0, wrap_index=0,
                 goal=[np.pi, 0.0], wx=[1e0, 1e-1], wu=[1e-3], wf=[1e0, 1e-1])

    def ode(state, action):
        g, l, m, d = 9.81, 1.0, 1.0, 1e-3
        th, om = state
        a = np.atleast_1d(action)[0]
        return np.array([om, -g / l * np.sin(th) + (a - d * om) / (m * l ** 2)])

    return OCP(euler(ode, dt), *_quadratic_barrier_costs(fam), family=fam)


def cartpole(dt: float) -> OCP:
    """Constrained cart-pole, examples/cartpole_runtime.py:18-82 (Euler, CR:88)."""
    fam = Family(kind=_lib.FAMILY_CARTPOLE, nx=4, nu=1, dt=dt, u_bound=50.0, wrap_index=1,
                 goal=[0.0, np.pi, 0.0, 0.0], wx=[1e0, 1e1, 1e-1, 1e-1], wu=[1e-3],
                 wf=[1e0, 1e1, 1e-1, 1e-1])

    def ode(state, action):
        g, pl, mc, mp = 9.81, 0.5, 10.0, 1.0
        mt = mc + mp
        _, th, xd, thd = state
        a = np.atleast_1d(action)[0]
        s, c = np.sin(th), np.cos(th)
        xdd = (a + mp * s * (pl * thd ** 2 + g * c)) / (mc + mp * s ** 2)
        thdd = (-a * c - mp * pl * thd ** 2 * c * s - mt * g * s) / (pl * mc + pl * mp * s ** 2)
        return np.array([xd, thd, xdd, thdd])

    return OCP(euler(ode, dt), *_quadratic_barrier_costs(fam), family=fam)


def double_integrator_matrices(n_blocks: int, step: float, downsampling: int = 1):
    """A, B of n stacked RK4-discretised double integrators (LM:24-38).  The discretisation is
    affine, so its Jacobians are obtained exactly by probing unit vectors."""
    def ode(state, control):
        return np.array([state[1], control[0]])
    dyn = discretize_dynamics(ode, step, downsampling)
    A1 = np.stack([dyn(np.eye(2)[i], np.zeros(1)) for i in range(2)], axis=1)
    B1 = dyn(np.zeros(2), np.ones(1))[:, None]
    A = np.kron(np.eye(n_blocks), A1)
    B = np.kron(np.eye(n_blocks), B1)
    return A, B


def double_integrators(n_blocks: int = 1, step: float = 0.1, constrained: bool = False,
                       u_bound: float = 5.0) -> OCP:
    """Linear-quadratic family.  n_blocks=1, step=0.1, unconstrained = linear_demo_cuda.py
    (X = diag(1e2, 1), U = 0.1 I, P = X: LD:34-42); n_blocks=4 is BASELINE config c4's nx=8."""
    A, B = double_integrator_matrices(n_blocks, step)
    nx, nu = 2 * n_blocks, n_blocks
    fam = Family(kind=_lib.FAMILY_LINEAR, nx=nx, nu=nu, dt=step,
                 u_bound=u_bound if constrained else 0.0, wrap_index=-1, goal=[0.0] * nx,
                 wx=[1e2, 1e0] * n_blocks, wu=[1e-1] * nu, wf=[1e2, 1e0] * n_blocks, A=A, B=B)

    def dynamics(state, control):
        return A @ np.asarray(state) + B @ np.atleast_1d(control)

    return OCP(dynamics, *_quadratic_barrier_costs(fam), family=fam)


def initial_conditions(name: str, N: int, batch: int, seed: int = 0):
    """Synthetic batched initial states / controls of the BASELINE configs:
    pendulum x0 = [wrap(0.1), -0.1] (PR:90) + 0.01 N(0,1); cart-pole x0 = [0.01, wrap(-0.01),
    0.01, -0.01] (CR:101) + 0.01 N(0,1); u0 = 0.1 N(0,1) (PR:91-92); linear x0 = N(0,1)."""
    rng = np.random.default_rng(seed)
    if name == "pendulum":
        x0 = np.array([wrap_angle(0.1), -0.1]) + 0.01 * rng.normal(size=(batch, 2))
        u0 = 0.1 * rng.normal(size=(batch, N, 1))
    elif name == "cartpole":
        x0 = np.array([0.01, wrap_angle(-0.01), 0.01, -0.01]) + 0.01 * rng.normal(size=(batch, 4))
        u0 = 0.1 * rng.normal(size=(batch, N, 1))
    elif name == "linear8":
        x0 = rng.normal(size=(batch, 8))
        u0 = np.zeros((batch, N, 4))
    else:
        raise ValueError(name)
    return x0, u0


def make_problem(name: str, N: int) -> OCP:
    """Problems of the BASELINE configs with Ts*N = 1 s (PR:74-75, CR:85-86); linear8 uses the
    LM step 0.001 (LM:30)."""
    if name == "pendulum":
        return pendulum(1.0 / N)
    if name == "cartpole":
        return cartpole(1.0 / N)
    if name == "linear8":
        return double_integrators(4, 0.001)
    raise ValueError(name)


def shard_initial_conditions(name: str, N: int, global_batch: int, lo: int, hi: int,
                             seed: int = 0):
    """Trajectories lo..hi-1 of ONE global batch (initial_conditions(name, N, global_batch,
    seed)): every rank of a sharded run draws the same global problem and keeps its slice, so the
    shards of N ranks concatenate to exactly the 1-rank inputs."""
    if not 0 <= lo <= hi <= global_batch:
        raise ValueError(f"shard [{lo}, {hi}) outside the global batch {global_batch}")
    x0, u0 = initial_conditions(name, N, global_batch, seed)
    return x0[lo:hi].copy(), u0[lo:hi].copy()


def make_bench_blocks(name: str, N: int, batch: int, seed: int = 0, device="cuda", lanes: int = 0,
                      natural: bool = False, shard=None):
    """Realistic LQ blocks of the first Newton step (bp = 0.1, rp = 1) of `batch` trajectories,
    produced on the GPU by the HIP linearisation kernels, in the KKT scan's tiled layout
    (`tiled`: noc.lqt.TiledBlocks).  natural=True also returns the natural-layout copies
    (A, B, Q, R, M, r, P) for checks.  `reg`, `x`, `u` are natural.  shard = (global_batch, lo):
    the trajectories lo..lo+batch-1 of one global batch (shard_initial_conditions) instead of a
    batch of its own."""
    from .ipm import BatchedIPM
    from .lqt import pick_lanes
    ocp = make_problem(name, N)
    if shard is None:
        x0, u0 = initial_conditions(name, N, batch, seed)
    else:
        G, lo = shard
        x0, u0 = shard_initial_conditions(name, N, G, lo, lo + batch, seed)
    # one all-active KKT launch over the batch: the batch-aware lanes policy
    lanes = lanes or pick_lanes(ocp.family.nx, ocp.family.nu, N, batch)
    # the interior-point workspace's tiled layout spans one wave (lanes <= 64); two-wave segments
    # (lanes = 128) get the same blocks relaid out on the device
    eng = BatchedIPM(ocp.family, N, batch, device=device, lanes=min(lanes, 64))
    eng.load(u0, x0)
    eng.init(bp0=0.1)
    eng.prepare(mode=_lib.MODE_PAR, terminal=_lib.TERMINAL_FINAL_COST)
    t = eng.t
    if lanes == eng.lanes:
        tiled = eng.tiled_blocks()
    else:
        from .lqt import to_tiled
        nat = eng.natural_blocks()
        tiled = to_tiled(*(nat[k] for k in ("A", "B", "Q", "R", "M", "r", "P")), lanes)
    out = dict(tiled=tiled, reg=t["reg"], x=t["x"], u=t["u"], engine=eng)
    if natural:
        out.update(eng.natural_blocks())
    return out
