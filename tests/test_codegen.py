"""Device code generation (noc/_codegen.py): the C printer and the committed built-in families.

The generated right-hand sides / Jacobians / lambda-contracted Hessians are what the kernels
evaluate for the reference's jax.jacrev / jax.hessian (noc/par_interior_point_newton.py:13-28);
their values are checked on the GPU against torch.func autodiff (tests/test_ipm_gpu.py,
tests/test_families_gpu.py).  Here, without a GPU: small integer powers are printed as products
(pow() on the device is the general double-double routine, ~200 instructions -- it dominated the
rollout's dependent chain), and csrc/families_gen.h is exactly what the generator produces.
"""
import os
import sys

import pytest

sp = pytest.importorskip("sympy")

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "ip-parallel-optimal-control_amd")


def test_small_integer_powers_print_as_products():
    from noc._codegen import _ccode
    x, y = sp.symbols("x y", real=True)
    assert _ccode(x ** 2) == "(x*x)"
    assert _ccode(x ** 3) == "(x*x*x)"
    assert _ccode(x ** -2) == "(1.0/(x*x))"
    assert _ccode(1 / x) == "(1.0/(x))"
    assert _ccode((x + y) ** 2) == "((x + y)*(x + y))"
    assert _ccode(sp.sqrt(x)) == "sqrt(x)"
    assert _ccode(x ** sp.Rational(-1, 2)) == "(1.0/sqrt(x))"
    assert _ccode(x ** 9) == "pow(x, 9)" and _ccode(x ** sp.Rational(1, 3)) == "cbrt(x)"  # C99 fallback


def test_products_evaluate_like_the_powers():
    from noc._codegen import _ccode
    x, y = sp.symbols("x y", real=True)
    for e in (x ** 2 * y - 3 * x ** -2, (x + y) ** 3 / (1 + x ** 2), sp.sqrt(x) + x ** sp.Rational(-1, 2)):
        src = _ccode(e).replace("sqrt", "math.sqrt").replace("pow", "math.pow")
        import math
        for xv, yv in ((0.7, -1.3), (2.5, 0.25)):
            got = eval(src, {"math": math, "x": xv, "y": yv})
            want = float(e.subs({x: xv, y: yv}))
            assert abs(got - want) <= 1e-14 * max(1.0, abs(want))


def test_committed_families_gen_is_the_generator_output():
    sys.path.insert(0, os.path.join(PKG, "tools"))
    try:
        import gen_family_derivs
    finally:
        sys.path.pop(0)
    with open(os.path.join(PKG, "csrc", "families_gen.h")) as fh:
        committed = fh.read()
    assert committed == gen_family_derivs.render()
    assert "pow(" not in committed
