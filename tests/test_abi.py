"""CPU-side checks of the C-ABI: libnoc_hip.so loads, exports every symbol include/noc_hip.h
declares, the ctypes mirror matches the header, and argument validation fails loudly (no compute
calls: there is no GPU here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "noc_hip.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(noc_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_expected_entry_points():
    fns = header_functions()
    for f in ["noc_kkt_solve", "noc_par_bwd_pass", "noc_par_fwd_pass", "noc_ipm_step",
              "noc_ipm_prepare", "noc_ipm_trial", "noc_ipm_init", "noc_abi_version"]:
        assert f in fns


def test_library_exports_every_header_symbol():
    from noc import _lib
    lib = _lib.load()
    for f in header_functions():
        assert hasattr(lib, f), f
        assert f in _lib.SIGNATURES, f"ctypes mirror lacks {f}"
    assert lib.noc_abi_version() == 5


def test_stale_library_is_refused(tmp_path, monkeypatch):
    """Build provenance: libnoc_hip.so carries the sha256 of the sources it was built from
    (noc_build_hash, baked in by the Makefile) and load() refuses it against a tree whose sources
    differ by one byte -- a stale binary cannot pass for the current sources."""
    import shutil
    from noc import _lib
    monkeypatch.delenv("NOC_ALLOW_STALE_LIB", raising=False)
    lib = _lib.load()
    assert lib.noc_build_hash().decode() == _lib.tree_build_hash()
    pkg = os.path.join(ROOT, "ip-parallel-optimal-control_amd")
    copy = tmp_path / "pkg"
    shutil.copytree(os.path.join(pkg, "csrc"), copy / "csrc")
    os.makedirs(tmp_path / "include")
    shutil.copy(HEADER, tmp_path / "include")
    assert _lib.tree_build_hash(str(copy)) == _lib.tree_build_hash()
    _lib.load(_lib.LIB_PATH, pkg_root=str(copy))  # the same sources: accepted
    f = copy / "csrc" / "small_linalg.h"
    f.write_bytes(f.read_bytes() + b" ")
    with pytest.raises(_lib.NocError, match="built from other sources"):
        _lib.load(_lib.LIB_PATH, pkg_root=str(copy))


def test_supported_shapes_and_lanes():
    from noc import _lib
    lib = _lib.load()
    assert lib.noc_kkt_supported(4, 1) == 1
    assert lib.noc_kkt_supported(2, 1) == 1
    assert lib.noc_kkt_supported(8, 4) == 1
    assert lib.noc_kkt_supported(3, 1) == 0
    assert lib.noc_kkt_default_lanes(4, 1, 200) in (8, 16, 32, 64)


def test_batch_aware_lane_policy_picks_the_measured_best():
    """noc_kkt_pick_lanes against the lanes sweep of profiles/r01/session4/lanes_policy/ (MI355X,
    1024 SIMDs -- also the no-device default here): the fastest L of each measured (N, B), or one
    within 4 % of it."""
    from noc import _lib
    lib = _lib.load()
    cases = {  # (nx, nu, N, B): acceptable L (measured best first)
        (4, 1, 50, 4096): (16, 8), (4, 1, 100, 4096): (16, 32), (4, 1, 150, 4096): (32,),
        (4, 1, 200, 4096): (32,), (4, 1, 300, 4096): (64,), (4, 1, 400, 4096): (64,),
        (4, 1, 200, 1024): (32, 64), (4, 1, 200, 16384): (32,),
        (2, 1, 100, 1024): (64,), (2, 1, 100, 4096): (32, 16), (2, 1, 100, 16384): (32,),
        # round 3: the 8-GPU shard of the north-star curve, two waves per trajectory, one wave
        # per SIMD (profiles/r03/two_wave/: 25.7 vs 27.3 us at 64 lanes); the 2-GPU shard keeps 32
        # lanes (profiles/r03/lanes2048/: 53.4 vs 59.2 us at 64); two-wave segments only while the
        # whole batch is resident at one wave per SIMD (B * 2 <= 1024 SIMDs)
        (4, 1, 200, 512): (128,), (4, 1, 200, 2048): (32,), (4, 1, 200, 600): (64,),
    }
    for (nx, nu, N, B), ok in cases.items():
        assert lib.noc_kkt_pick_lanes(nx, nu, N, B) in ok, (nx, nu, N, B)
    assert lib.noc_kkt_pick_lanes(2, 1, 50, 1) == 64      # a lone trajectory takes the whole wave
    assert lib.noc_kkt_pick_lanes(8, 4, 512, 16384) == 1  # nx = 8: the group solve
    assert lib.noc_kkt_pick_lanes(3, 1, 50, 1) == -1      # unsupported shape


def test_gains_on_chip_query_and_required_workspace():
    """K, d may be NULL only where the fused solve keeps them in LDS (20 KB per 64-lane block)."""
    from noc import _lib
    lib = _lib.load()
    assert lib.noc_kkt_gains_on_chip(4, 1, 200, 32) == 1   # c3 default: 2 x 8 KB per wave
    assert lib.noc_kkt_gains_on_chip(2, 1, 100, 64) == 1   # c2
    assert lib.noc_kkt_gains_on_chip(8, 4, 512, 16) == 0   # c4: 147 KB of gains per trajectory
    assert lib.noc_kkt_gains_on_chip(3, 1, 10, 0) == 0     # unsupported shape
    # K = d = NULL with gains that do not fit: rejected before any launch
    rc = lib.noc_kkt_solve(8, 4, 512, 4, 16, *([16] * 6), None, None, 16, None, None, None, None,
                           16, 16, 16, 16, None, None, None, None, None)
    assert rc < 0 and b"noc_kkt_gains_on_chip" in lib.noc_last_error()


def test_argument_errors_are_reported_not_launched():
    from noc import _lib
    lib = _lib.load()
    rc = lib.noc_kkt_solve(3, 1, 10, 4, 0, *([None] * 21), None)
    assert rc < 0 and b"unsupported" in lib.noc_last_error()
    rc = lib.noc_kkt_solve(4, 1, 10, 4, 0, *([None] * 21), None)
    assert rc < 0 and b"NULL" in lib.noc_last_error()
    rc = lib.noc_kkt_solve(4, 1, 0, 4, 0, *([None] * 21), None)
    assert rc < 0 and b"horizon" in lib.noc_last_error()
    rc = lib.noc_kkt_solve(4, 1, 10, 4, 48, *([None] * 21), None)
    assert rc < 0 and b"lanes" in lib.noc_last_error()
    # misaligned pointer is rejected before any launch
    rc = lib.noc_kkt_solve(4, 1, 10, 4, 0, 8, *([16] * 20), None)
    assert rc < 0 and b"aligned" in lib.noc_last_error()


def test_workspace_struct_layout_matches_header():
    from noc import _lib
    text = open(HEADER).read()
    body = re.search(r"typedef struct noc_ipm_ws \{(.*?)\} noc_ipm_ws;", text, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = re.findall(r"\*?\s*\*?(\w+)\s*[,;]", body.replace("*", " "))
    names = [n for n in names if n not in ("int", "double")]
    assert names == [f for f, _ in _lib.NocIpmWs._fields_]
    assert ctypes.sizeof(_lib.NocFamily) == 4 * 4 + 8 * 2 + 8 * (8 + 8 + 4 + 8 + 64 + 32)


def test_family_validation_without_gpu():
    from noc import _lib, problems
    lib = _lib.load()
    for ocp in (problems.pendulum(0.02), problems.cartpole(0.005), problems.double_integrators(4, 0.001),
                problems.double_integrators(1, 0.1)):
        fam = ocp.family.to_c()
        assert lib.noc_family_supported(ctypes.byref(fam)) == 1
    bad = problems.pendulum(0.02).family
    bad.nx = 3
    assert lib.noc_family_supported(ctypes.byref(bad.to_c())) == 0


def test_product_path_fails_loudly_without_gpu():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from noc import _lib, problems
    from noc.par_interior_point_newton import par_interior_point_optimal_control
    import numpy as np
    with pytest.raises(_lib.NocError):
        par_interior_point_optimal_control(problems.pendulum(0.02), np.zeros((50, 1)), np.zeros(2))
    from noc import lqt
    with pytest.raises(_lib.NocError):
        z = torch.zeros(1, 5, 4, 4, dtype=torch.float64)
        lqt.kkt_solve(z, torch.zeros(1, 5, 4, 1, dtype=torch.float64), z,
                      torch.ones(1, 5, 1, 1, dtype=torch.float64),
                      torch.zeros(1, 5, 4, 1, dtype=torch.float64),
                      torch.zeros(1, 5, 1, dtype=torch.float64), torch.eye(4, dtype=torch.float64)[None])


def test_persistent_solve_and_grouped_layout_queries_without_gpu():
    """Capability queries and argument errors of the persistent solver / grouped layout are host
    logic: checked here without a launch."""
    from noc import _lib, problems
    lib = _lib.load()
    cart = problems.cartpole(0.005).family.to_c()
    lin8 = problems.double_integrators(4, 0.001).family.to_c()
    assert lib.noc_ipm_solve_supported(ctypes.byref(cart), 200, 64) == 1
    assert lib.noc_ipm_solve_supported(ctypes.byref(cart), 1000, 64) == 1   # 40 KB of LDS
    assert lib.noc_ipm_solve_supported(ctypes.byref(cart), 2000, 64) == 0   # > 64 KB
    assert lib.noc_ipm_solve_supported(ctypes.byref(cart), 200, 32) == 0    # needs lanes 64
    assert lib.noc_ipm_solve_supported(ctypes.byref(lin8), 512, 64) == 0    # nx = 8: launch loop
    # grouped layout (lanes 1) sizes: whole records of 8 trajectories
    assert lib.noc_tiled_doubles(10, 9, 1, 36) == 16 * 10 * 36
    assert lib.noc_tiled_doubles(10, 16, 1, 64) == 16 * 10 * 64
    assert lib.noc_kkt_default_lanes(8, 4, 512) == 1
    # the grouped tiled layout is only for nx = 8 (before any launch)
    rc = lib.noc_kkt_solve_tiled(4, 1, 10, 8, 1, *([16] * 6), None, None, 16, None, None, None,
                                 None, 16, 16, 16, 16, 16, 16, None, None, None)
    assert rc < 0 and b"grouped" in lib.noc_last_error()
    # persistent solve argument errors are reported, not launched
    ws = _lib.NocIpmWs()
    ws.Bt, ws.N, ws.lanes = 4, 200, 32
    for f in _lib.WS_DOUBLE_FIELDS + _lib.WS_INT_FIELDS + _lib.WS_STATE_FIELDS:
        setattr(ws, f, 16)
    rc = lib.noc_ipm_solve(ctypes.byref(cart), ctypes.byref(ws), 0, 0, 0.1, 100, None)
    assert rc < 0 and b"lanes = 64" in lib.noc_last_error()
    ws.lanes = 64
    rc = lib.noc_ipm_solve(ctypes.byref(cart), ctypes.byref(ws), 0, 0, -1.0, 100, None)
    assert rc < 0 and b"bp0" in lib.noc_last_error()
    rc = lib.noc_ipm_solve(ctypes.byref(cart), ctypes.byref(ws), 0, 0, 0.1, 0, None)
    assert rc < 0 and b"max_solves" in lib.noc_last_error()


def test_ddp_queries_and_argument_errors_without_gpu():
    """noc_ddp_*: workspace size, family support (nx <= 4) and argument validation are host logic."""
    from noc import _lib, problems
    lib = _lib.load()
    # fx fu cx cu | cxx cuu cxu (the stage cost's Hessian) | d2f_i (xx, xu, uu) per i
    rec = 16 + 4 + 4 + 1 + (16 + 1 + 4) + 4 * (16 + 4 + 1)
    assert lib.noc_ddp_work_doubles(4, 1, 200, 3) == 3 * (2 * 201 * 4 + 2 * 200 + 200 * 4 + 200 * rec)
    assert lib.noc_ddp_work_doubles(0, 1, 10, 1) < 0
    for ocp, ok in ((problems.pendulum(0.02), 1), (problems.cartpole(0.005), 1),
                    (problems.double_integrators(1, 0.1), 1),
                    (problems.double_integrators(4, 0.001), 0)):
        assert lib.noc_ddp_supported(ctypes.byref(ocp.family.to_c())) == ok
    pend = problems.pendulum(0.02).family.to_c()
    args = [16, 16, 16, 16, 16, 16]  # 16-byte aligned fake device addresses: never dereferenced
    assert lib.noc_ddp_solve(None, 10, 1, *args, 0.1, 10, None) == -2
    assert lib.noc_ddp_solve(ctypes.byref(pend), 0, 1, *args, 0.1, 10, None) < 0
    assert lib.noc_ddp_solve(ctypes.byref(pend), 10, 1, *args, -0.5, 10, None) < 0
    assert lib.noc_ddp_solve(ctypes.byref(pend), 10, 1, *args, float("nan"), 10, None) < 0
    assert lib.noc_ddp_solve(ctypes.byref(pend), 10, 1, *args, float("inf"), 10, None) < 0
    assert lib.noc_ddp_solve(ctypes.byref(pend), 10, 1, *args, 0.1, 0, None) < 0
    assert lib.noc_ddp_solve(ctypes.byref(pend), 10, 1, None, *args[1:], 0.1, 10, None) == -2
    assert lib.noc_ddp_solve(ctypes.byref(pend), 10, 0, *args, 0.1, 10, None) == 0  # empty batch
    lin8 = problems.double_integrators(4, 0.001).family.to_c()
    assert lib.noc_ddp_solve(ctypes.byref(lin8), 10, 1, *args, 0.1, 10, None) < 0
    assert b"nx <= 4" in lib.noc_last_error()


def test_alignment_checks_use_natural_alignment_for_scalars_and_flags():
    """16-byte alignment is required only for the fp64 fields the kernels access with 16-byte
    vector loads / stores; reg and pred need 8, feasible / active / DDP counters 4.
    B = 0 validates and returns without a launch."""
    from noc import _lib, problems
    lib = _lib.load()
    blocks = [16] * 6  # A, B, Q, R, M, r (fake, never dereferenced)

    def solve(reg=16, pred=16, feasible=16, active=None, A=16):
        return lib.noc_kkt_solve(4, 1, 10, 0, 32, A, *blocks[1:], None, None, 16, None, None, reg,
                                 active, 16, 16, pred, feasible, 16, 16, None, None, None)
    assert solve() == 0
    assert solve(reg=24, pred=40, feasible=20, active=36) == 0   # natural alignment suffices
    assert solve(reg=20) < 0 and b"reg" in lib.noc_last_error()
    assert solve(feasible=18) < 0 and b"feasible" in lib.noc_last_error()
    assert solve(A=24) < 0 and b"16-byte" in lib.noc_last_error()
    pend = problems.pendulum(0.02).family.to_c()
    # x0 / u / work at 8-byte offsets and int32 counters at 4-byte offsets: accepted (empty batch)
    assert lib.noc_ddp_solve(ctypes.byref(pend), 10, 0, 24, 40, 56, 20, 36, 52, 0.1, 10, None) == 0
    assert lib.noc_ddp_solve(ctypes.byref(pend), 10, 0, 20, 40, 56, 20, 36, 52, 0.1, 10, None) < 0
