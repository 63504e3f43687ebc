"""ORACLE (test infrastructure only) -- problem families restated in torch fp64 on the CPU.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker.  The product path (ip-parallel-optimal-control_amd/noc + libnoc_hip.so)
never imports it.

Parity status: **parity unpinned**.  The reference (casiacob/ip-parallel-optimal-control) is pure
JAX and ships no tests, fixtures or golden vectors; neither jax, jaxlib nor its LQ-solver
dependency `paroc` is installed here, so the reference cannot be executed.  These callables are
line-by-line restatements of the reference problem definitions, written against torch so that
`torch.func.{grad,hessian,jacrev,vmap}` reproduce the reference's JAX autodiff (`P:13-28`).
`torch.remainder` has derivative 1 exactly like `jnp` `%` in `wrap_angle` (`noc/utils.py:8-10`).

Reference anchors
-----------------
* pendulum:   examples/pendulum_runtime.py:19-72  (constraints 19-27, final_cost 30-37,
              transient_cost 40-50, total_cost 53-56, ODE 59-72, x0 90)
* cart-pole:  examples/cartpole_runtime.py:18-82 (constraints 18-24, final_cost 27-33,
              transient_cost 36-45, total_cost 48-51, ODE 54-81, x0 101)
* linear:     examples/linear_mpc_parallel.py:24-63 (RK4 double integrator, Q/R/P weights)
              examples/linear_demo_cuda.py:19-62 (unconstrained LQR through the IPM)
* euler / RK4 / wrap_angle: noc/utils.py:8-54
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable

import numpy as np
import torch
from torch.func import grad, hessian, jacrev, vmap

torch.set_default_dtype(torch.float64)
TWO_PI = 2.0 * math.pi


def wrap_angle(x):
    """noc/utils.py:8-10 -- x mod 2*pi (gradient 1).

    Restates jnp.remainder exactly (lax.rem = C fmod, then + divisor where the signs differ and
    the remainder is non-zero); torch.remainder uses floor-division and can differ in the last ulp.
    """
    r = torch.fmod(x, TWO_PI)
    return torch.where(r < 0, r + TWO_PI, r)


def euler(ode: Callable, dt: float) -> Callable:
    """noc/utils.py:50-54."""
    def dynamics(state, control):
        return state + dt * ode(state, control)
    return dynamics


def runge_kutta(state, action, ode, step):
    """noc/utils.py:13-23."""
    k1 = ode(state, action)
    k2 = ode(state + 0.5 * step * k1, action)
    k3 = ode(state + 0.5 * step * k2, action)
    k4 = ode(state + step * k3, action)
    return state + step / 6.0 * (k1 + 2.0 * k2 + 2.0 * k3 + k4)


def discretize_dynamics(ode: Callable, step: float, downsampling: int) -> Callable:
    """noc/utils.py:26-47 (fori_loop of RK4 steps)."""
    def dynamics(state, action):
        for _ in range(downsampling):
            state = runge_kutta(state, action, ode, step)
        return state
    return dynamics


@dataclass
class TorchOCP:
    """Mirror of noc/optimal_control_problem.py:5-10 (OCP NamedTuple of 5 callables)."""
    dynamics: Callable
    constraints: Callable
    stage_cost: Callable
    final_cost: Callable
    total_cost: Callable
    nx: int
    nu: int
    name: str = ""


# ----------------------------------------------------------------------------------------------
# pendulum -- examples/pendulum_runtime.py:19-72
# ----------------------------------------------------------------------------------------------
def pendulum_ocp(dt: float, u_bound: float = 5.0) -> TorchOCP:
    def constraints(state, control):            # PR:19-27
        c0 = control - u_bound
        c1 = -control - u_bound
        return torch.cat((c0, c1))

    goal = torch.tensor([math.pi, 0.0])
    Wx = torch.diag(torch.tensor([1e0, 1e-1]))
    Wu = torch.diag(torch.tensor([1e-3]))

    def final_cost(state):                       # PR:30-37
        err = torch.stack((wrap_angle(state[0]), state[1])) - goal
        return 0.5 * err @ Wx @ err

    def transient_cost(state, action, bp):       # PR:40-50
        err = torch.stack((wrap_angle(state[0]), state[1])) - goal
        c = 0.5 * err @ Wx @ err
        c = c + 0.5 * action @ Wu @ action
        log_barrier = torch.sum(torch.log(-constraints(state, action)))
        return c - bp * log_barrier

    def total_cost(states, controls, bp):        # PR:53-56
        ct = vmap(transient_cost, in_dims=(0, 0, None))(states[:-1], controls, bp)
        return final_cost(states[-1]) + torch.sum(ct)

    def ode(state, action):                      # PR:59-72
        gravity, length, mass, damping = 9.81, 1.0, 1.0, 1e-3
        position, velocity = state[0], state[1]
        return torch.stack((velocity,
                            -gravity / length * torch.sin(position)
                            + (action[0] - damping * velocity) / (mass * length ** 2)))

    return TorchOCP(euler(ode, dt), constraints, transient_cost, final_cost, total_cost,
                    2, 1, "pendulum")


# ----------------------------------------------------------------------------------------------
# cart-pole -- examples/cartpole_runtime.py:18-82
# ----------------------------------------------------------------------------------------------
def cartpole_ocp(dt: float, u_bound: float = 50.0) -> TorchOCP:
    def constraints(state, control):             # CR:18-24
        c0 = control[0] - u_bound
        c1 = -control[0] - u_bound
        return torch.stack((c0, c1))

    goal = torch.tensor([0.0, math.pi, 0.0, 0.0])
    Wx = torch.diag(torch.tensor([1e0, 1e1, 1e-1, 1e-1]))
    Wu = torch.diag(torch.tensor([1e-3]))

    def _wrapped(state):
        return torch.stack((state[0], wrap_angle(state[1]), state[2], state[3]))

    def final_cost(state):                        # CR:27-33
        e = _wrapped(state) - goal
        return 0.5 * e @ Wx @ e

    def transient_cost(state, action, bp):        # CR:36-45
        e = _wrapped(state) - goal
        c = 0.5 * e @ Wx @ e
        c = c + 0.5 * action @ Wu @ action
        log_barrier = torch.sum(torch.log(-constraints(state, action)))
        return c - bp * log_barrier

    def total_cost(states, controls, bp):         # CR:48-51
        ct = vmap(transient_cost, in_dims=(0, 0, None))(states[:-1], controls, bp)
        return final_cost(states[-1]) + torch.sum(ct)

    def ode(state, action):                       # CR:54-81
        gravity, pole_length, cart_mass, pole_mass = 9.81, 0.5, 10.0, 1.0
        total_mass = cart_mass + pole_mass
        pole_position, cart_velocity, pole_velocity = state[1], state[2], state[3]
        sth, cth = torch.sin(pole_position), torch.cos(pole_position)
        a = action[0]
        cart_acc = (a + pole_mass * sth * (pole_length * pole_velocity ** 2 + gravity * cth)) / (
            cart_mass + pole_mass * sth ** 2)
        pole_acc = (-a * cth - pole_mass * pole_length * pole_velocity ** 2 * cth * sth
                    - total_mass * gravity * sth) / (
            pole_length * cart_mass + pole_length * pole_mass * sth ** 2)
        return torch.stack((cart_velocity, pole_velocity, cart_acc, pole_acc))

    return TorchOCP(euler(ode, dt), constraints, transient_cost, final_cost, total_cost,
                    4, 1, "cartpole")


# ----------------------------------------------------------------------------------------------
# linear double integrators -- examples/linear_mpc_parallel.py:24-63, linear_demo_cuda.py:19-62
# ----------------------------------------------------------------------------------------------
def double_integrator_blocks(n_blocks: int, step: float, downsampling: int = 1):
    """A, B of `n_blocks` stacked RK4-discretised double integrators (LM:24-38).

    Each block is x'' = u (LM:24-27).  The discretisation is affine, so its Jacobian at any point
    is the matrix itself (LM:37-38 evaluate jacfwd at x0).
    """
    def ode1(state, control):
        A = torch.tensor([[0.0, 1.0], [0.0, 0.0]])
        Bm = torch.tensor([[0.0], [1.0]])
        return A @ state + Bm @ control
    dyn1 = discretize_dynamics(ode1, step, downsampling)
    x0 = torch.zeros(2)
    u0 = torch.zeros(1)
    A1 = jacrev(dyn1, 0)(x0, u0)
    B1 = jacrev(dyn1, 1)(x0, u0)
    A = torch.block_diag(*([A1] * n_blocks))
    Bm = torch.block_diag(*([B1] * n_blocks))
    return A.numpy(), Bm.numpy()


def linear_ocp(n_blocks: int, step: float, constrained: bool = False,
               u_bound: float = 5.0) -> TorchOCP:
    """Linear-quadratic family; with constrained=False it is linear_demo_cuda.py's LQR
    (constraints == -1, LD:30-31; stage/final costs LD:34-42)."""
    A_np, B_np = double_integrator_blocks(n_blocks, step)
    A, Bm = torch.from_numpy(A_np), torch.from_numpy(B_np)
    nx, nu = 2 * n_blocks, n_blocks
    X = torch.diag(torch.tensor([1e2, 1e0] * n_blocks))
    U = 1e-1 * torch.eye(nu)

    def dynamics(state, control):
        return A @ state + Bm @ control

    if constrained:
        def constraints(state, control):
            return torch.cat((control - u_bound, -control - u_bound))
    else:
        def constraints(state, control):       # LD:30-31
            return -torch.ones(1)

    def stage_cost(state, control, bp):         # LD:34-37
        c = 0.5 * state @ X @ state + 0.5 * control @ U @ control
        if constrained:
            c = c - bp * torch.sum(torch.log(-constraints(state, control)))
        return c

    def final_cost(state):                       # LD:40-42
        return 0.5 * state @ X @ state

    def total_cost(states, controls, bp):        # LD:45-48
        ct = vmap(stage_cost, in_dims=(0, 0, None))(states[:-1], controls, bp)
        return final_cost(states[-1]) + torch.sum(ct)

    return TorchOCP(dynamics, constraints, stage_cost, final_cost, total_cost, nx, nu,
                    f"linear{nx}")


# ----------------------------------------------------------------------------------------------
# derivative oracle -- restates compute_derivatives (P:13-28 == S:10-25) with torch.func
# ----------------------------------------------------------------------------------------------
def compute_derivatives(ocp: TorchOCP, states: np.ndarray, controls: np.ndarray, bp: float):
    """Returns the 10 Derivatives arrays of noc/optimal_control_problem.py:13-23 as numpy."""
    X = torch.as_tensor(states[:-1])
    U = torch.as_tensor(controls)
    bp_t = torch.tensor(float(bp))

    def body(x, u):
        cx, cu = grad(ocp.stage_cost, (0, 1))(x, u, bp_t)
        cxx = hessian(ocp.stage_cost, 0)(x, u, bp_t)
        cuu = hessian(ocp.stage_cost, 1)(x, u, bp_t)
        cxu = jacrev(jacrev(ocp.stage_cost, 0), 1)(x, u, bp_t)
        fx, fu = jacrev(ocp.dynamics, (0, 1))(x, u)
        fxx = jacrev(jacrev(ocp.dynamics, 0), 0)(x, u)
        fuu = jacrev(jacrev(ocp.dynamics, 1), 1)(x, u)
        fxu = jacrev(jacrev(ocp.dynamics, 0), 1)(x, u)
        return cx, cu, cxx, cuu, cxu, fx, fu, fxx, fuu, fxu

    out = vmap(body)(X, U)
    return tuple(o.detach().numpy() for o in out)


def final_grad_hess(ocp: TorchOCP, xN: np.ndarray):
    x = torch.as_tensor(xN)
    return (grad(ocp.final_cost)(x).numpy(), hessian(ocp.final_cost)(x).numpy())


def dynamics_np(ocp: TorchOCP, x: np.ndarray, u: np.ndarray) -> np.ndarray:
    return ocp.dynamics(torch.as_tensor(x), torch.as_tensor(u)).numpy()


def constraints_np(ocp: TorchOCP, X: np.ndarray, U: np.ndarray) -> np.ndarray:
    return vmap(ocp.constraints)(torch.as_tensor(X), torch.as_tensor(U)).numpy()


def total_cost_np(ocp: TorchOCP, X: np.ndarray, U: np.ndarray, bp: float) -> float:
    return float(ocp.total_cost(torch.as_tensor(X), torch.as_tensor(U), float(bp)))
