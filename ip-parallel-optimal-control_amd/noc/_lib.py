"""ctypes binding of libnoc_hip.so (the C-ABI declared in include/noc_hip.h).

The product path has no CPU fallback: if the shared library is missing or no GPU is visible,
every compute entry point raises.  Building: `make -C ip-parallel-optimal-control_amd -j8`
(or `python -c "import __graft_entry__ as g; g.build()"` from the repo root).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NOC_HIP_LIB", os.path.join(_HERE, "_lib", "libnoc_hip.so"))

# sources the bench's KKT kernels (kkt_scan_kernel, kkt_group8_kernel) are compiled from: a
# committed PMC traffic figure is valid only for the build it was measured on (source_hash)
_COMMON_SOURCES = ("csrc/small_linalg.h", "csrc/noc_internal.h", "csrc/kkt_shapes.def", "Makefile",
                   "../include/noc_hip.h")
KKT_KERNEL_SOURCES = {
    "kkt_scan": ("csrc/kkt_scan_impl.h", "csrc/kkt_scan_2x1.hip", "csrc/kkt_scan_4x1.hip",
                 "csrc/kkt_scan_4x1_l32.hip", "csrc/kkt_scan_4x1_l32nt.hip",
                 "csrc/kkt_scan_4x1_l128.hip", "csrc/kkt_scan_8x4.hip", "csrc/kkt_scan_8x4_l32.hip",
                 "csrc/kkt_scan_8x4_l16.hip", "csrc/kkt_scan_8x4_l8.hip") + _COMMON_SOURCES,
    "kkt_group8": ("csrc/kkt_group_impl.h", "csrc/kkt_group8_impl.h", "csrc/kkt_group.hip")
    + _COMMON_SOURCES,
}

ABI_VERSION = 5  # include/noc_hip.h NOC_ABI_VERSION
_dp = ctypes.c_void_p  # device pointers are passed as opaque addresses
_i = ctypes.c_int

# name -> (restype, argtypes); mirrors include/noc_hip.h exactly (tests check every symbol)
SIGNATURES = {
    "noc_abi_version": (_i, []),
    "noc_build_hash": (ctypes.c_char_p, []),
    "noc_last_error": (ctypes.c_char_p, []),
    "noc_kkt_supported": (_i, [_i, _i]),
    "noc_kkt_default_lanes": (_i, [_i, _i, _i]),
    "noc_kkt_pick_lanes": (_i, [_i, _i, _i, _i]),
    "noc_kkt_gains_on_chip": (_i, [_i, _i, _i, _i]),
    "noc_debug_set_ablation": (None, [_i]),
    "noc_kkt_solve": (_i, [_i] * 5 + [_dp] * 13 + [_dp] * 8 + [_dp]),
    "noc_kkt_solve_tiled": (_i, [_i] * 5 + [_dp] * 13 + [_dp] * 8 + [_dp]),
    "noc_tiled_doubles": (ctypes.c_longlong, [_i, _i, _i, _i]),
    "noc_relayout": (_i, [_i] * 6 + [_dp, _dp, _dp]),
    "noc_par_bwd_pass": (_i, [_i] * 5 + [_dp] * 12 + [_dp] * 6 + [_dp]),
    "noc_par_fwd_pass": (_i, [_i] * 5 + [_dp] * 7 + [_dp] * 2 + [_dp]),
}

# --- structs of include/noc_hip.h --------------------------------------------------------------
FAMILY_PENDULUM, FAMILY_CARTPOLE, FAMILY_LINEAR, FAMILY_CUSTOM = 1, 2, 3, 4
PHASE_ROLLOUT, PHASE_LINEARIZE, PHASE_SOLVE, PHASE_DONE, PHASE_ROLLED = 0, 1, 2, 3, 4
PHASE_ROLLOUT_PENDING = 5
MODE_PAR, MODE_SEQ = 0, 1
TERMINAL_FINAL_COST, TERMINAL_STAGE0 = 0, 1
DDP_ONE_STAGE = 1  # noc_ddp_solve_ex flags bit: ddp() at one barrier value


class NocFamily(ctypes.Structure):
    _fields_ = [("kind", _i), ("nx", _i), ("nu", _i), ("wrap_index", _i),
                ("dt", ctypes.c_double), ("u_bound", ctypes.c_double),
                ("goal", ctypes.c_double * 8), ("wx", ctypes.c_double * 8),
                ("wu", ctypes.c_double * 4), ("wf", ctypes.c_double * 8),
                ("A", ctypes.c_double * 64), ("B", ctypes.c_double * 32)]


WS_DOUBLE_FIELDS = ["x", "u", "x0", "A", "B", "Q", "R", "M", "r", "P", "cx", "cu", "lc", "lam",
                    "dx", "du", "pred", "K", "d"]
WS_ONE_STAGE = 1  # NocIpmWs.flags bit: stop after one barrier stage (newton_oc)
WS_RESUME = 2  # NocIpmWs.flags bit: noc_ipm_solve continues from the workspace state
WS_NO_REPEAT_SKIP = 4  # NocIpmWs.flags bit: recompute the identical retries at the rp clip
WS_INT_FIELDS = ["feasible", "phase", "kkt_active", "it", "inner", "total_it", "kkt_solves",
                 "repeats"]
WS_STATE_FIELDS = ["bp", "rp", "rinc", "cost", "hu", "gnorm", "reg"]


WS_OPT_FIELDS = ["order"]  # optional pointers, NULL unless set (noc_ipm_ws.order)


class NocIpmWs(ctypes.Structure):
    _fields_ = ([("Bt", _i), ("N", _i), ("lanes", _i), ("flags", _i)]
                + [(f, _dp) for f in WS_DOUBLE_FIELDS]
                + [(f, _dp) for f in WS_INT_FIELDS] + [(f, _dp) for f in WS_OPT_FIELDS]
                + [(f, _dp) for f in WS_STATE_FIELDS])


_fp = ctypes.POINTER(NocFamily)
_wp = ctypes.POINTER(NocIpmWs)
SIGNATURES.update({
    "noc_family_supported": (_i, [_fp]),
    "noc_ipm_init": (_i, [_wp, ctypes.c_double, _dp]),
    "noc_ipm_prepare": (_i, [_fp, _wp, _i, _i, _dp]),
    "noc_ipm_trial": (_i, [_fp, _wp, _i, _dp]),
    "noc_ipm_step": (_i, [_fp, _wp, _i, _i, _i, _dp]),
    "noc_ipm_rollout": (_i, [_fp, _wp, _dp]),
    "noc_ipm_step_main": (_i, [_fp, _wp, _i, _i, _dp]),
    "noc_ipm_promote": (_i, [_wp, _dp]),
    "noc_ipm_solve_supported": (_i, [_fp, _i, _i]),
    "noc_debug_phase_cycles": (_i, [ctypes.POINTER(ctypes.c_longlong), _i, _i]),
    "noc_debug_traj_times": (_i, [ctypes.POINTER(ctypes.c_longlong), _i]),
    "noc_ipm_solve": (_i, [_fp, _wp, _i, _i, ctypes.c_double, _i, _dp]),
    "noc_derivatives": (_i, [_fp, _i, _i] + [_dp] * 13 + [_dp]),
    "noc_final_cost_derivs": (_i, [_fp, _i, _dp, _dp, _dp, _dp]),
    "noc_costates": (_i, [_i, _i, _i, _dp, _dp, _dp, _dp, _i, _dp]),
    "noc_lqr_params": (_i, [_i] * 4 + [_dp] * 13 + [_dp]),
    "noc_check_feasibility": (_i, [_fp, _i, _i, _dp, _dp, _dp, _dp]),
    "noc_total_cost": (_i, [_fp, _i, _i, _dp, _dp, _dp, _dp, _dp]),
    "noc_ddp_work_doubles": (ctypes.c_longlong, [_i, _i, _i, _i]),
    "noc_ddp_supported": (_i, [_fp]),
    "noc_ddp_solve": (_i, [_fp, _i, _i] + [_dp] * 6 + [ctypes.c_double, _i, _dp]),
    "noc_ddp_solve_ex": (_i, [_fp, _i, _i] + [_dp] * 6 + [ctypes.c_double, _i, _i, _dp]),
    "noc_ddp_bwd_pass": (_i, [_i] * 4 + [_dp] * 18 + [_dp]),
    "noc_nonlin_rollout": (_i, [_fp, _i, _i] + [_dp] * 6 + [_dp]),
})

_lib: Optional[ctypes.CDLL] = None
_family_libs = {}   # path -> CDLL of a registered custom family's build (noc.families)
_shape_libs = {}    # (nx, nu) -> CDLL of a custom build that instantiates that KKT shape


class NocError(RuntimeError):
    pass


def tree_build_hash(pkg_root: Optional[str] = None) -> str:
    """sha256 (16 hex digits) of the sources in this tree that libnoc_hip.so is compiled from --
    csrc/*.hip, *.h, *.def and csrc/custom/*.hip in name order, then include/noc_hip.h -- the same
    bytes the Makefile hashes into noc_build_hash()."""
    import glob
    import hashlib
    pkg = pkg_root or os.path.dirname(_HERE)
    rel = sorted(os.path.relpath(f, pkg) for pat in ("csrc/*.hip", "csrc/*.h", "csrc/*.def",
                                                     "csrc/custom/*.hip")
                 for f in glob.glob(os.path.join(pkg, pat)))
    h = hashlib.sha256()
    for f in rel + [os.path.join("..", "include", "noc_hip.h")]:
        with open(os.path.join(pkg, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def verify_build(lib: ctypes.CDLL, pkg_root: Optional[str] = None) -> str:
    """The library's baked-in source hash; NocError if it is not this tree's (a stale binary).
    NOC_ALLOW_STALE_LIB=1 downgrades the refusal (development only: an edited source that is not
    rebuilt yet)."""
    built = lib.noc_build_hash().decode()
    tree = tree_build_hash(pkg_root)
    if built != tree and os.environ.get("NOC_ALLOW_STALE_LIB") != "1":
        raise NocError(f"{getattr(lib, '_name', 'libnoc_hip.so')} was built from other sources "
                       f"(library {built}, tree {tree}); rebuild it: "
                       f"`make -C ip-parallel-optimal-control_amd -j8`")
    return built


def _typed(lib: ctypes.CDLL, pkg_root: Optional[str] = None) -> ctypes.CDLL:
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.noc_abi_version() != ABI_VERSION:
        raise NocError("libnoc_hip.so ABI version mismatch")
    verify_build(lib, pkg_root)
    return lib


def load(path: Optional[str] = None, pkg_root: Optional[str] = None) -> ctypes.CDLL:
    """Load (once) and type the shared library.  Raises NocError if it is missing or was built
    from other sources than this tree's (verify_build; pkg_root: the tree to check against)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise NocError(f"libnoc_hip.so not found at {p}; build it with "
                       f"`make -C ip-parallel-optimal-control_amd -j8`")
    lib = _typed(ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL), pkg_root)
    if path is None:
        _lib = lib
    return lib


def load_for(family) -> ctypes.CDLL:
    """The library that implements `family`: the default build for the built-in families, the
    family's own build (noc.families.register_family) for a registered one."""
    path = getattr(family, "lib_path", None)
    if not path:
        return load()
    lib = _family_libs.get(path)
    if lib is None:
        if not os.path.exists(path):
            raise NocError(f"the library of family '{getattr(family, 'name', '?')}' is not built "
                           f"({path}); call noc.families.register_family(..., build=True)")
        lib = _typed(ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL))
        _family_libs[path] = lib
        _shape_libs.setdefault((int(family.nx), int(family.nu)), lib)
    return lib


def for_shape(nx: int, nu: int) -> ctypes.CDLL:
    """The library whose KKT solve covers (nx, nu): the default build's shapes, else a loaded
    custom family's."""
    lib = load()
    if lib.noc_kkt_supported(int(nx), int(nu)) == 1:
        return lib
    return _shape_libs.get((int(nx), int(nu)), lib)  # the default reports the unsupported shape


def check(rc: int, what: str, lib: Optional[ctypes.CDLL] = None) -> None:
    if rc != 0:
        msg = (lib or load()).noc_last_error().decode(errors="replace")
        raise NocError(f"{what} failed (rc={rc}): {msg}")


def ptr(t) -> Optional[int]:
    """Device address of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def require_device(t, name: str):
    import torch
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise NocError(f"{name}: expected a CUDA (HIP) torch tensor; the MI355X path has no "
                       f"CPU fallback")
    return t


def stream_handle(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream


def source_hash(kernel: str = "kkt_scan") -> str:
    """sha256 (first 16 hex digits) of the sources a KKT kernel is compiled from
    (KKT_KERNEL_SOURCES[kernel], relative to the package root)."""
    import hashlib
    pkg = os.path.dirname(_HERE)
    h = hashlib.sha256()
    for f in KKT_KERNEL_SOURCES[kernel]:
        with open(os.path.join(pkg, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]
