"""ORACLE (test infrastructure / CPU baseline only): ctypes wrapper of oracle/_build/libkkt_ref.so,
the plain-C restatement of noc/seq_interior_point_newton.py:42-90 (see kkt_ref.c).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libkkt_ref.so")
_lib = None


def build():
    subprocess.run(["make", "-C", HERE], check=True, stdout=subprocess.DEVNULL)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        p = ctypes.c_void_p
        lib.kkt_ref_solve.restype = ctypes.c_int
        lib.kkt_ref_solve.argtypes = [ctypes.c_int] * 5 + [p] * 14
        lib.kkt_ref_max_threads.restype = ctypes.c_int
        _lib = lib
    return _lib


def solve(A, B, Q, R, M, r, P, reg, threads=0):
    """Batched host solve; arrays (Bt, N, ...) float64.  Returns dict dx, du, pred, feasible, K, d."""
    A, B, Q, R, M, r, P, reg = (np.ascontiguousarray(a, dtype=np.float64)
                                for a in (A, B, Q, R, M, r, P, reg))
    Bt, N, nx, _ = A.shape
    nu = B.shape[-1]
    out = dict(dx=np.empty((Bt, N + 1, nx)), du=np.empty((Bt, N, nu)), pred=np.empty(Bt),
               feasible=np.empty(Bt, dtype=np.int32), K=np.empty((Bt, N, nu, nx)),
               d=np.empty((Bt, N, nu)))
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    rc = load().kkt_ref_solve(nx, nu, N, Bt, threads, *(ptr(a) for a in (A, B, Q, R, M, r, P, reg)),
                              *(ptr(out[k]) for k in ("dx", "du", "pred", "feasible", "K", "d")))
    if rc != 0:
        raise RuntimeError(f"kkt_ref_solve rc={rc}")
    return out
