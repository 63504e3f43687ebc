"""Run-time family registration (noc.families): symbolic tracing of numpy-written dynamics, the
generated device code, and the family's own library build (CPU checks; no launches).  GPU parity
of the registered family's solves: tests/test_families_gpu.py."""
import ctypes

import numpy as np
import pytest
import sympy as sp

from custom_families import ACT_PEND, actuated_pendulum, actuated_pendulum_ode


def test_trace_numpy_dynamics_matches_the_formula():
    from noc import _codegen
    X, U, f = _codegen.trace(actuated_pendulum_ode, 3, 1)
    x0, x1, x2 = X
    u0, = U
    want = [x1, -9.81 * sp.sin(x0) - 0.1 * x1 + x2, (u0 - x2) / 0.05]
    for a, b in zip(f, want):
        assert sp.simplify(a - b) == 0
    # numpy ufuncs are restored on sympy afterwards
    assert not hasattr(sp.Symbol("z"), "arctan2")


def test_trace_rejects_wrong_dimension_and_free_symbols():
    from noc import _codegen
    with pytest.raises(ValueError):
        _codegen.trace(lambda x, u: np.hstack((x[0], u[0])), 3, 1)
    k = sp.Symbol("k")
    with pytest.raises(ValueError):
        _codegen.trace(lambda x, u: np.hstack((x[1], k * x[0], u[0])), 3, 1)


def test_generated_derivatives_match_finite_differences():
    """Evaluate the generated expressions' sympy sources numerically: Jacobian and the
    lambda-contracted Hessian against central differences of the numpy dynamics."""
    from noc import _codegen
    X, U, f = _codegen.trace(actuated_pendulum_ode, 3, 1)
    Z = X + U
    fn = sp.lambdify(Z, f, "numpy")
    J = sp.lambdify(Z, [[sp.diff(fi, z) for z in Z] for fi in f], "numpy")
    rng = np.random.default_rng(0)
    z = rng.normal(size=4)
    h = 1e-6
    Jn = np.array(J(*z), dtype=float)
    for j in range(4):
        e = np.zeros(4)
        e[j] = h
        fd = (np.array(fn(*(z + e))) - np.array(fn(*(z - e)))) / (2 * h)
        assert np.max(np.abs(fd - Jn[:, j])) < 1e-6
    ref = actuated_pendulum_ode(z[:3], z[3:])
    assert np.max(np.abs(np.array(fn(*z)) - ref)) < 1e-12


def test_register_validates_arguments():
    from noc import families, _lib
    bad = dict(ACT_PEND)
    bad["wx"] = [1.0]
    with pytest.raises(_lib.NocError):
        families.register_family("bad", actuated_pendulum_ode, dt=0.02, build=False, **bad)
    with pytest.raises(_lib.NocError):
        families.register_family("bad", actuated_pendulum_ode, dt=0.0, build=False, **ACT_PEND)


def test_host_ocp_callables_follow_the_reference_semantics():
    from noc import utils
    ocp = actuated_pendulum(0.02, build=False)
    x = np.array([0.3, -0.2, 0.5])
    u = np.array([1.5])
    assert np.allclose(ocp.dynamics(x, u), x + 0.02 * actuated_pendulum_ode(x, u))
    e = np.array([utils.wrap_angle(0.3), -0.2, 0.5]) - np.array(ACT_PEND["goal"])
    want = 0.5 * e @ (np.array(ACT_PEND["wx"]) * e) + 0.5 * 1e-3 * 1.5 ** 2 \
        - 0.1 * (np.log(5 - 1.5) + np.log(1.5 + 5))
    assert abs(ocp.stage_cost(x, u, 0.1) - want) < 1e-12
    assert np.all(ocp.constraints(x, u) <= 0)


def test_family_library_builds_loads_and_exports_the_abi():
    """The family's own build: every header symbol, the family supported there (and not in the
    default library), its (3, 1) KKT shape instantiated, persistent solve and DDP available."""
    from noc import _lib
    from test_abi import header_functions
    ocp = actuated_pendulum(0.02)
    lib = _lib.load_for(ocp.family)
    for f in header_functions():
        assert hasattr(lib, f), f
    fam = ocp.family.to_c()
    assert lib.noc_family_supported(ctypes.byref(fam)) == 1
    assert _lib.load().noc_family_supported(ctypes.byref(fam)) == 0
    assert lib.noc_kkt_supported(3, 1) == 1 and _lib.load().noc_kkt_supported(3, 1) == 0
    assert lib.noc_ipm_solve_supported(ctypes.byref(fam), 50, 64) == 1
    assert lib.noc_ddp_supported(ctypes.byref(fam)) == 1
    assert _lib.for_shape(3, 1) is lib
