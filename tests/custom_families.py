"""User problem families registered through noc.families.register_family for the tests (test
infrastructure; __graft_entry__.build() pre-builds their libraries so the GPU box only loads
them).  Written with numpy exactly like the reference examples' dynamics (PR:59-72), and
restated independently in torch for the autodiff oracle (oracle/problems.py style).

actuated_pendulum (nx=3, nu=1, continuous ODE + Euler): the reference pendulum driven through a
first-order actuator, state (angle, angular velocity, torque), the command u the torque set-point;
a (3, 1) KKT shape the default library does not instantiate.
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


def build_all(verbose=False):
    """Register (and build once) every test family; returns their OCPs."""
    return [actuated_pendulum(1.0 / 50)]
