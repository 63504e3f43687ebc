"""Host utilities with the reference's names and semantics (noc/utils.py:8-63), numpy fp64.

These are the host-side (NumPy-callable) versions used for problem definition and checks; the
device equivalents (Euler step, rollout, wrap) live in csrc/ipm_kernels.hip.
"""
from typing import Callable

import numpy as np

TWO_PI = 2.0 * np.pi


def wrap_angle(x):
    """x mod 2*pi (noc/utils.py:8-10); numpy's remainder == jnp.remainder semantics."""
    return np.remainder(x, TWO_PI)


def runge_kutta(state, action, ode: Callable, step: float):
    """noc/utils.py:13-23."""
    k1 = ode(state, action)
    k2 = ode(state + 0.5 * step * k1, action)
    k3 = ode(state + 0.5 * step * k2, action)
    k4 = ode(state + step * k3, action)
    return state + step / 6.0 * (k1 + 2.0 * k2 + 2.0 * k3 + k4)


def discretize_dynamics(ode: Callable, simulation_step: float, downsampling: int) -> Callable:
    """noc/utils.py:26-47."""
    def dynamics(state, action):
        for _ in range(downsampling):
            state = runge_kutta(state, action, ode, simulation_step)
        return state
    return dynamics


def euler(ode: Callable, simulation_step: float) -> Callable:
    """noc/utils.py:50-54."""
    def dynamics(state, control):
        return state + simulation_step * ode(state, control)
    return dynamics


def rollout(dynamics: Callable, controls, initial_state):
    """noc/utils.py:57-63 -- (N, nu), (nx,) -> (N+1, nx)."""
    xs = [np.asarray(initial_state, dtype=np.float64)]
    for u in np.asarray(controls, dtype=np.float64):
        xs.append(np.asarray(dynamics(xs[-1], u), dtype=np.float64))
    return np.stack(xs)
