"""Problem types -- same names, fields and order as the reference (noc/optimal_control_problem.py:5-30).

`OCP` keeps the reference's five callables.  The MI355X path additionally needs to know which
registered device family implements those callables (HIP cannot call Python); that is the
optional 6th field `family` (a `noc.problems.Family`), filled in by the constructors in
`noc.problems`.  `OCP(dynamics, constraints, stage_cost, final_cost, total_cost)` positional
construction works exactly as in the reference.
"""
from typing import Any, Callable, NamedTuple, Optional


class OCP(NamedTuple):
    dynamics: Callable
    constraints: Callable
    stage_cost: Callable
    final_cost: Callable
    total_cost: Callable
    family: Optional[Any] = None


class Derivatives(NamedTuple):
    cx: Any
    cu: Any
    cxx: Any
    cuu: Any
    cxu: Any
    fx: Any
    fu: Any
    fxx: Any
    fuu: Any
    fxu: Any


class LinearizedOCP(NamedTuple):
    r: Any
    Q: Any
    R: Any
    M: Any
