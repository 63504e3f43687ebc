"""noc -- MI355X-native interior-point optimal control (drop-in for casiacob/ip-parallel-optimal-control).

Module layout mirrors the reference package `noc` (optimal_control_problem, utils, costates,
par_interior_point_newton, seq_interior_point_newton, differential_dynamic_programming); the
KKT hot path runs in libnoc_hip.so (hand-written HIP for gfx950) through the C-ABI in
include/noc_hip.h.
"""
__version__ = "0.1.0"
