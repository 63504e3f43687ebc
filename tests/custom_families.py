"""User problem families registered through noc.families.register_family for the tests (test
infrastructure; __graft_entry__.build() pre-builds their libraries so the GPU box only loads
them).  Written with numpy exactly like the reference examples' dynamics (PR:59-72), and
restated independently in torch for the autodiff oracle (oracle/problems.py style).

actuated_pendulum (nx=3, nu=1, continuous ODE + Euler): the reference pendulum driven through a
first-order actuator, state (angle, angular velocity, torque), the command u the torque set-point;
a (3, 1) KKT shape the default library does not instantiate.

cartpole_track_limit (nx=4, nu=1): cart-pole with its own traced costs and a state constraint
(see below).
"""
import math

import numpy as np

ACT_PEND = dict(nx=3, nu=1, goal=[math.pi, 0.0, 0.0], wx=[1e0, 1e-1, 1e-2], wu=[1e-3],
                wf=[1e0, 1e-1, 1e-2], u_bound=5.0, wrap_index=0)


def actuated_pendulum_ode(state, action):
    g, length, damping, lag = 9.81, 1.0, 0.1, 0.05
    angle, velocity, torque = state
    a = np.atleast_1d(action)[0]
    return np.hstack((velocity, -g / length * np.sin(angle) - damping * velocity + torque,
                      (a - torque) / lag))


def actuated_pendulum(dt, build=True):
    from noc import families
    return families.register_family("actuated_pendulum", actuated_pendulum_ode, dt=dt,
                                    build=build, **ACT_PEND)


def actuated_pendulum_torch(dt):
    """The same problem restated in torch (oracle/problems.py conventions) for torch.func."""
    import torch
    from oracle import problems as PR
    goal = torch.tensor(ACT_PEND["goal"])
    Wx = torch.diag(torch.tensor(ACT_PEND["wx"]))
    Wf = torch.diag(torch.tensor(ACT_PEND["wf"]))
    Wu = torch.diag(torch.tensor(ACT_PEND["wu"]))
    ub = ACT_PEND["u_bound"]

    def constraints(state, control):
        return torch.cat((control - ub, -control - ub))

    def err(state):
        return torch.stack((PR.wrap_angle(state[0]), state[1], state[2])) - goal

    def final_cost(state):
        e = err(state)
        return 0.5 * e @ Wf @ e

    def stage_cost(state, action, bp):
        e = err(state)
        c = 0.5 * e @ Wx @ e + 0.5 * action @ Wu @ action
        return c - bp * torch.sum(torch.log(-constraints(state, action)))

    def total_cost(states, controls, bp):
        ct = torch.func.vmap(stage_cost, in_dims=(0, 0, None))(states[:-1], controls, bp)
        return final_cost(states[-1]) + torch.sum(ct)

    def ode(state, action):
        g, length, damping, lag = 9.81, 1.0, 0.1, 0.05
        return torch.stack((state[1], -g / length * torch.sin(state[0]) - damping * state[1] + state[2],
                            (action[0] - state[2]) / lag))

    return PR.TorchOCP(PR.euler(ode, dt), constraints, stage_cost, final_cost, total_cost, 3, 1,
                       "actuated_pendulum")


# ------------------------------------------------------------------------------------------------
# cartpole_track_limit (nx=4, nu=1): the reference cart-pole ODE (CR:54-81) with the reference
# OCP's own kind of callables instead of the parametrised cost -- a STATE constraint (the cart
# stays within |x| <= X_LIMIT, besides |u| <= 50) inside the log barrier, and a non-quadratic
# stage cost (a quartic penalty on the pole rate on top of the quadratic tracking), written with
# numpy exactly like CR:18-51 writes them with jnp.  Registered through
# register_family(stage_cost=..., final_cost=..., constraints=...): traced and differentiated
# symbolically for the device.
X_LIMIT = 0.5
_CP_WX = np.array([1e0, 1e1, 1e-1, 1e-1])
_CP_WF = np.array([1e0, 1e1, 1e-1, 1e-1])
_CP_GOAL = np.array([0.0, math.pi, 0.0, 0.0])


def cartpole_ode(state, action):
    g, pl, mc, mp = 9.81, 0.5, 10.0, 1.0
    mt = mc + mp
    _, th, xd, thd = state
    a = np.atleast_1d(action)[0]
    s, c = np.sin(th), np.cos(th)
    xdd = (a + mp * s * (pl * thd ** 2 + g * c)) / (mc + mp * s ** 2)
    thdd = (-a * c - mp * pl * thd ** 2 * c * s - mt * g * s) / (pl * mc + pl * mp * s ** 2)
    return np.hstack((xd, thd, xdd, thdd))


def track_limit_constraints(state, action):
    u = np.atleast_1d(action)
    return np.hstack((u - 50.0, -u - 50.0, state[0] - X_LIMIT, -state[0] - X_LIMIT))


def _cp_err(state):
    return np.hstack((state[0], state[1] % (2.0 * np.pi), state[2], state[3])) - _CP_GOAL


def track_limit_final_cost(state):
    e = _cp_err(state)
    return 0.5 * e @ np.diag(_CP_WF) @ e


def track_limit_stage_cost(state, action, bp):
    e = _cp_err(state)
    u = np.atleast_1d(action)
    c = 0.5 * e @ np.diag(_CP_WX) @ e + 0.5 * 1e-3 * u @ u + 1e-3 * state[3] ** 4
    return c - bp * np.sum(np.log(-track_limit_constraints(state, action)))


def cartpole_track_limit(dt, build=True):
    from noc import families
    return families.register_family("cartpole_track_limit", cartpole_ode, nx=4, nu=1, dt=dt,
                                    stage_cost=track_limit_stage_cost,
                                    final_cost=track_limit_final_cost,
                                    constraints=track_limit_constraints, build=build)


def cartpole_track_limit_torch(dt):
    """The same problem restated in torch (oracle/problems.py conventions) for torch.func."""
    import torch
    from oracle import problems as PR
    goal = torch.tensor(_CP_GOAL)
    Wx, Wf = torch.diag(torch.tensor(_CP_WX)), torch.diag(torch.tensor(_CP_WF))

    def constraints(state, control):
        return torch.cat((control - 50.0, -control - 50.0, state[:1] - X_LIMIT, -state[:1] - X_LIMIT))

    def err(state):
        return torch.stack((state[0], PR.wrap_angle(state[1]), state[2], state[3])) - goal

    def final_cost(state):
        e = err(state)
        return 0.5 * e @ Wf @ e

    def stage_cost(state, action, bp):
        e = err(state)
        c = 0.5 * e @ Wx @ e + 0.5 * 1e-3 * action @ action + 1e-3 * state[3] ** 4
        return c - bp * torch.sum(torch.log(-constraints(state, action)))

    def total_cost(states, controls, bp):
        ct = torch.func.vmap(stage_cost, in_dims=(0, 0, None))(states[:-1], controls, bp)
        return final_cost(states[-1]) + torch.sum(ct)

    def ode(state, action):
        g, pl, mc, mp = 9.81, 0.5, 10.0, 1.0
        mt = mc + mp
        th, xd, thd = state[1], state[2], state[3]
        a = action[0]
        s, c = torch.sin(th), torch.cos(th)
        xdd = (a + mp * s * (pl * thd ** 2 + g * c)) / (mc + mp * s ** 2)
        thdd = (-a * c - mp * pl * thd ** 2 * c * s - mt * g * s) / (pl * mc + pl * mp * s ** 2)
        return torch.stack((xd, thd, xdd, thdd))

    return PR.TorchOCP(PR.euler(ode, dt), constraints, stage_cost, final_cost, total_cost, 4, 1,
                       "cartpole_track_limit")


def build_all(verbose=False):
    """Register (and build once) every test family; returns their OCPs."""
    return [actuated_pendulum(1.0 / 50), cartpole_track_limit(1.0 / 50)]
