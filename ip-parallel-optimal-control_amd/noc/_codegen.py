"""Device code generation for problem families: sympy expressions of an ODE right-hand side (or a
discrete map) -> straight-line fp64 HIP device functions for the value, the Jacobian with respect
to z = [x; u] and the lambda-contracted Hessian sum_i l_i d2 f_i / dz dz, with common
subexpressions eliminated and sin/cos of a state computed once with sincos().

Used by tools/gen_family_derivs.py (the built-in families -> csrc/families_gen.h, committed) and
by noc.families.register_family (user families -> a per-family build of libnoc_hip.so).  This is
what the reference gets from jax.jacrev / jax.hessian on the Python dynamics
(noc/par_interior_point_newton.py:13-28): the derivatives are exact symbolic ones, evaluated on
the device.
"""
from __future__ import annotations

import contextlib

import numpy as np
import sympy as sp
from sympy.printing.c import C99CodePrinter
from sympy.printing.precedence import PRECEDENCE


class _DevicePrinter(C99CodePrinter):
    """sympy's C printer, except that small integer powers become products (x^2 -> (x*x),
    x^-2 -> 1.0/(x*x)) and x^(+-1/2) sqrt: pow() on the device is the general double-double
    exp/log routine -- ~200 instructions per call, which dominated the Euler step of the rollout's
    sequential chain -- where a product is one correctly rounded multiply."""

    def _print_Pow(self, expr, rational=False):
        b, e = expr.base, expr.exp
        if e.is_Integer and 1 <= abs(int(e)) <= 8:
            n = abs(int(e))
            base = self.parenthesize(b, PRECEDENCE["Mul"] + 1)
            prod = "*".join([base] * n) if n > 1 else base
            return f"({prod})" if int(e) > 0 else f"(1.0/({prod}))"
        if e == sp.Rational(1, 2):
            return f"sqrt({self._print(b)})"
        if e == sp.Rational(-1, 2):
            return f"(1.0/sqrt({self._print(b)}))"
        return super()._print_Pow(expr)


    def _print_PyMod(self, expr):
        a, b = expr.args
        return f"noc_pymod({self._print(a)}, {self._print(b)})"


class PyMod(sp.Function):
    """a mod b with the sign of b -- Python's / jnp's `%` (the reference's wrap_angle, U:8-10) --
    with the derivative jax.grad gives it: d/da = 1 (sympy leaves Mod's derivative unevaluated).
    Printed as noc_pymod() (defined in the generated header)."""
    nargs = 2

    def fdiff(self, argindex=1):
        a, b = self.args
        return sp.Integer(1) if argindex == 1 else -sp.floor(a / b)


def _pymod(e):
    """Mod(a, b) -> PyMod(a, b) (differentiable, printed with Python remainder semantics)."""
    return e.replace(lambda t: isinstance(t, sp.Mod), lambda t: PyMod(*t.args))


# device helper of the generated cost code: Python / jnp remainder (sign of the divisor); the
# general fmod routine only outside |a| < 2 |b|: fmod(a, b) == a exactly for |a| < |b| and
# a - sign(a) |b| exactly for |b| <= |a| < 2 |b| (Sterbenz), fmod's own result bit for bit
PYMOD_DEVICE = """NOC_DEV double noc_pymod(double a, double b) {
  double r = a;
  const double fa = fabs(a), fb = fabs(b);
  if (fa >= fb) r = (fa < 2.0 * fb) ? a - copysign(fb, a) : fmod(a, b);
  return (r != 0.0 && ((r < 0.0) != (b < 0.0))) ? r + b : r;
}"""


def _ccode(e) -> str:
    return _DevicePrinter().doprint(e)


def _trig_subst(exprs, X):
    """Replace sin(x_i)/cos(x_i) by symbols computed once with sincos() (shared range reduction:
    the rollout's dependent chain is dominated by fp64 trig)."""
    subs, pre = {}, []
    for xi in X:
        s_, c_ = sp.symbols(f"s_{xi} c_{xi}", real=True)
        if any(e.has(sp.sin(xi)) or e.has(sp.cos(xi)) for e in exprs):
            subs[sp.sin(xi)] = s_
            subs[sp.cos(xi)] = c_
            pre.append(f"  double {s_}, {c_};\n  sincos({xi}, &{s_}, &{c_});")
    return [e.subs(subs) for e in exprs], pre


def emit(name, X, U, f):
    """Device functions {name}_ode(x, u, f), {name}_ode_jac(x, u, J) (J[i][j] = d f_i / d z_j,
    row-major nx x (nx+nu)) and {name}_ode_hess_l(x, u, l, H) ((nx+nu) x (nx+nu), row-major)."""
    Z = list(X) + list(U)
    nz = len(Z)
    nx = len(X)
    lam = sp.symbols(f"l0:{nx}", real=True)
    jac = [[sp.diff(fi, zj) for zj in Z] for fi in f]
    hl = [[sum(lam[i] * sp.diff(f[i], Z[a], Z[b]) for i in range(nx)) for b in range(nz)]
          for a in range(nz)]
    lines = []

    def block(fn_sig, exprs, targets, with_lambda=False):
        exprs, pre = _trig_subst(exprs, X)
        reps, red = sp.cse(exprs, symbols=sp.numbered_symbols("t"))
        lines.append(fn_sig + " {")
        for i in range(nx):
            lines.append(f"  [[maybe_unused]] const double x{i} = x[{i}];")
            if with_lambda:
                lines.append(f"  [[maybe_unused]] const double l{i} = l[{i}];")
        for i in range(len(U)):
            lines.append(f"  [[maybe_unused]] const double u{i} = u[{i}];")
        lines.extend(pre)
        lines.extend(f"  const double {_ccode(s)} = {_ccode(e)};" for s, e in reps)
        lines.extend(f"  {t} = {_ccode(e)};" for t, e in zip(targets, red))
        lines.append("}")

    block(f"NOC_DEV void {name}_ode(const double* x, const double* u, double* f)",
          list(f), [f"f[{i}]" for i in range(nx)])
    block(f"NOC_DEV void {name}_ode_jac(const double* x, const double* u, double* J)",
          [jac[i][j] for i in range(nx) for j in range(nz)],
          [f"J[{i * nz + j}]" for i in range(nx) for j in range(nz)])
    block(f"NOC_DEV void {name}_ode_hess_l(const double* x, const double* u, const double* l, double* H)",
          [hl[a][b] for a in range(nz) for b in range(nz)],
          [f"H[{a * nz + b}]" for a in range(nz) for b in range(nz)], with_lambda=True)
    lines.append(structure(name, "jac", [jac[i][j] for i in range(nx) for j in range(nz)], Z))
    lines.append(f"constexpr signed char {name}_hess_nz[{nz * nz}] = "
                 f"{{{', '.join('0' if hl[a][b] == 0 else '1' for a in range(nz) for b in range(nz))}}};")
    return "\n".join(lines)


def structure(name, what, exprs, args) -> str:
    """The structural pattern of a generated array (csrc/block_struct.h): {name}_{what}_var[k] = 1
    where entry k depends on the arguments, else 0 with its value in {name}_{what}_const[k] -- the
    very literal the device function assigns, so a kernel that folds it in computes the same
    doubles as one that evaluates the function.  A constant that is not a plain number (pi,
    sqrt(2), ...) counts as variable."""
    args = set(args)
    var = [not (sp.sympify(e).is_Number and not (sp.sympify(e).free_symbols & args)) for e in exprs]
    vals = ["0" if v else _ccode(sp.sympify(e)) for v, e in zip(var, exprs)]
    n = len(exprs)
    return "\n".join([
        f"constexpr signed char {name}_{what}_var[{n}] = {{{', '.join('1' if v else '0' for v in var)}}};",
        f"constexpr double {name}_{what}_const[{n}] = {{{', '.join(vals)}}};"])


# numpy ufunc name -> sympy function: numpy applies a ufunc to an object array (or a sympy scalar)
# by calling the element's method of the same name, so while these are attached to sympy.Expr a
# dynamics written with np.sin / np.exp / ... on numpy arrays can be called on sympy symbols.
_UFUNCS = {"sin": sp.sin, "cos": sp.cos, "tan": sp.tan, "arcsin": sp.asin, "arccos": sp.acos,
           "arctan": sp.atan, "sinh": sp.sinh, "cosh": sp.cosh, "tanh": sp.tanh, "exp": sp.exp,
           "log": sp.log, "sqrt": sp.sqrt, "arctan2": None}


@contextlib.contextmanager
def _sympy_ufuncs():
    saved = {k: getattr(sp.Expr, k, None) for k in _UFUNCS}
    try:
        for k, fn in _UFUNCS.items():
            if fn is not None:
                setattr(sp.Expr, k, (lambda f: lambda self: f(self))(fn))
        sp.Expr.arctan2 = lambda self, other: sp.atan2(self, other)
        yield
    finally:
        for k, v in saved.items():
            if v is None:
                if k in sp.Expr.__dict__:
                    delattr(sp.Expr, k)
            else:
                setattr(sp.Expr, k, v)


def trace(fn, nx: int, nu: int):
    """Call fn(x, u) on symbolic state / control arrays (numpy object arrays of sympy symbols
    x0.., u0..) and return (X, U, f) with f the list of nx sympy expressions.  fn may be written
    with numpy (np.sin, np.hstack, @, ...) exactly like the reference examples' dynamics."""
    X = list(sp.symbols(f"x0:{nx}", real=True))
    U = list(sp.symbols(f"u0:{nu}", real=True))
    with _sympy_ufuncs():
        out = fn(np.array(X, dtype=object), np.array(U, dtype=object))
    out = [sp.sympify(e) for e in np.asarray(out, dtype=object).reshape(-1)]
    if len(out) != nx:
        raise ValueError(f"the dynamics returned {len(out)} components, expected nx = {nx}")
    free = set().union(*(e.free_symbols for e in out)) - set(X) - set(U)
    if free:
        raise ValueError(f"the dynamics depend on symbols other than the state / control: {free}")
    return X, U, out


def _block(lines, sig, exprs, targets, X, U, extra=(), ret=None):
    """One straight-line device function: CSE over `exprs`, shared sincos of the states, the
    results assigned to `targets` (or returned: ret = "value" / "all_nonpositive")."""
    exprs, pre = _trig_subst([_pymod(sp.sympify(e)) for e in exprs], X)
    reps, red = sp.cse(exprs, symbols=sp.numbered_symbols("t"))
    lines.append(sig + " {")
    for i in range(len(X)):
        lines.append(f"  [[maybe_unused]] const double x{i} = x[{i}];")
    for i in range(len(U)):
        lines.append(f"  [[maybe_unused]] const double u{i} = u[{i}];")
    lines.extend(pre)
    lines.extend(f"  const double {_ccode(s_)} = {_ccode(e)};" for s_, e in reps)
    if ret == "value":
        lines.append(f"  return {_ccode(red[0])};")
    elif ret == "all_nonpositive":
        conds = " && ".join(f"({_ccode(e)} <= 0.0)" for e in red) or "true"
        lines.append(f"  return {conds};")
    else:
        lines.extend(f"  {t} = {_ccode(e)};" for t, e in zip(targets, red))
    lines.append("}")


def emit_costs(name, X, U, bp, stage, final, cons):
    """Device functions of a user cost (the reference OCP's stage_cost / final_cost / constraints,
    T:5-10, differentiated like P:13-28 does with jax.grad / hessian):
    {name}_stage_cost(x, u, bp), _stage_grad(x, u, bp, cx, cu), _stage_hess(x, u, bp, Q, R, M)
    (Q = d2/dx2, R = d2/du2, M = d2/dxdu, row-major), {name}_final_cost(x), _final_grad(x, g),
    _final_hess(x, H), and {name}_feasible(x, u) = all(constraints(x, u) <= 0) (P:45-47)."""
    nx, nu = len(X), len(U)
    stage, final = _pymod(sp.sympify(stage)), _pymod(sp.sympify(final))
    cx = [sp.diff(stage, xi) for xi in X]
    cu = [sp.diff(stage, ui) for ui in U]
    Q = [sp.diff(stage, X[i], X[j]) for i in range(nx) for j in range(nx)]
    R = [sp.diff(stage, U[i], U[j]) for i in range(nu) for j in range(nu)]
    M = [sp.diff(stage, X[i], U[j]) for i in range(nx) for j in range(nu)]
    g = [sp.diff(final, xi) for xi in X]
    H = [sp.diff(final, X[i], X[j]) for i in range(nx) for j in range(nx)]
    lines = []
    a_xub = "const double* x, const double* u, double bp"
    _block(lines, f"NOC_DEV double {name}_stage_cost({a_xub})", [stage], [], X, U, ret="value")
    _block(lines, f"NOC_DEV void {name}_stage_grad({a_xub}, double* cx, double* cu)",
           cx + cu, [f"cx[{i}]" for i in range(nx)] + [f"cu[{j}]" for j in range(nu)], X, U)
    _block(lines, f"NOC_DEV void {name}_stage_hess({a_xub}, double* Q, double* R, double* M)",
           Q + R + M, [f"Q[{k}]" for k in range(nx * nx)] + [f"R[{k}]" for k in range(nu * nu)] +
           [f"M[{k}]" for k in range(nx * nu)], X, U)
    _block(lines, f"NOC_DEV double {name}_final_cost(const double* x)", [final], [], X, [],
           ret="value")
    _block(lines, f"NOC_DEV void {name}_final_grad(const double* x, double* g)", g,
           [f"g[{i}]" for i in range(nx)], X, [])
    _block(lines, f"NOC_DEV void {name}_final_hess(const double* x, double* H)", H,
           [f"H[{k}]" for k in range(nx * nx)], X, [])
    _block(lines, f"NOC_DEV bool {name}_feasible(const double* x, const double* u)",
           list(cons), [], X, U, ret="all_nonpositive")
    lines.append(structure(name, "cost_hess", Q + R + M, list(X) + list(U) + [bp]))
    return "\n".join(lines)


def trace_costs(stage_cost, final_cost, constraints, nx: int, nu: int):
    """Call the user's stage_cost(x, u, bp), final_cost(x) and constraints(x, u) (numpy, like the
    reference examples' CR:18-51) on symbolic arrays; returns (X, U, bp, stage, final, cons)."""
    X = list(sp.symbols(f"x0:{nx}", real=True))
    U = list(sp.symbols(f"u0:{nu}", real=True))
    bp = sp.Symbol("bp", real=True)
    xa, ua = np.array(X, dtype=object), np.array(U, dtype=object)
    with _sympy_ufuncs():
        stage = sp.sympify(np.asarray(stage_cost(xa, ua, bp), dtype=object).reshape(-1)[0])
        final = sp.sympify(np.asarray(final_cost(xa), dtype=object).reshape(-1)[0])
        cons = [] if constraints is None else \
            [sp.sympify(e) for e in np.asarray(constraints(xa, ua), dtype=object).reshape(-1)]
    for what, es, allowed in (("stage_cost", [stage], set(X) | set(U) | {bp}),
                              ("final_cost", [final], set(X)),
                              ("constraints", cons, set(X) | set(U))):
        free = set().union(set(), *(e.free_symbols for e in es)) - allowed
        if free:
            raise ValueError(f"{what} depends on symbols other than its arguments: {free}")
    return X, U, bp, stage, final, cons
