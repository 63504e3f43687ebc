"""Batched interior-point engine: device workspace + host loop over libnoc_hip.so.

The reference runs one trajectory per call, with its whole solve as nested lax.while_loops
(noc/par_interior_point_newton.py:127-254).  Here B trajectories run at once; every trajectory
carries its own phase / counters / barrier parameter on the device, so each one follows exactly
its own reference control flow (jax.vmap semantics), while the host only launches one fused
iteration (rollout | linearise | costate | assemble | KKT scan | trial) at a time and polls a
single "any trajectory not done" flag every `poll_every` iterations.
"""
from __future__ import annotations

import math
import ctypes
import os
from typing import Optional

import numpy as np
import torch

from . import _lib


def default_terminal(mode: int) -> int:
    """The terminal Hessian the reference uses in each mode: par_Newton's LQT has XT = Q[0]
    (noc/par_interior_point_newton.py:73); the seq bwd_pass uses hessian(final_cost) (S:66)."""
    return _lib.TERMINAL_STAGE0 if mode == _lib.MODE_PAR else _lib.TERMINAL_FINAL_COST


def persistent_supported(family, N: int) -> bool:
    """noc_ipm_solve_supported: the whole-solve kernel handles this family / horizon (lanes 64)."""
    lib = _lib.load_for(family)
    return lib.noc_ipm_solve_supported(ctypes.byref(family.to_c()), int(N), 64) == 1


def carve_zeros(spec, device, dtype, align_bytes: int = 256):
    """{name: shape} -> ({name: zero view}, backing tensor): one allocation, every field starting
    on an align_bytes boundary."""
    per = max(align_bytes // torch.empty((), dtype=dtype).element_size(), 1)
    offs, n = {}, 0
    for k, s in spec.items():
        offs[k] = n
        n += -(-math.prod(s) // per) * per
    buf = torch.zeros(max(n, 1), device=device, dtype=dtype)
    return {k: buf[offs[k]:offs[k] + math.prod(s)].view(s) for k, s in spec.items()}, buf


class BatchedIPM:
    def __init__(self, family, N: int, batch: int, device="cuda", lanes: int = 0,
                 overlap: Optional[bool] = None, persistent: bool = False):
        """persistent=True: solve() runs the whole barrier schedule in one launch
        (noc_ipm_solve, one wave per trajectory; forces lanes = 64)."""
        if not torch.cuda.is_available():
            raise _lib.NocError("no HIP device visible: the MI355X path has no CPU fallback")
        self.family = family
        self.fam_c = family.to_c()
        self.N, self.Bt = int(N), int(batch)
        self.nx, self.nu = family.nx, family.nu
        self.device = torch.device(device)
        lib = _lib.load_for(family)
        self.persistent = bool(persistent)
        if self.persistent:
            if lanes not in (0, 64) or not persistent_supported(family, N):
                raise _lib.NocError("persistent solve needs lanes = 64 and a supported family / "
                                    "horizon (noc_ipm_solve_supported)")
            lanes = 64
        # lanes = 0: the batch-agnostic default.  The batch-aware pick (noc_kkt_pick_lanes) is tuned for
        # all-active launches; inside the loop the active set shrinks and wide segments win
        # (cart-pole N=100 B=4096: 0.124 ms per device step at 64 lanes vs 0.136 at the pick's 16,
        # profiles/r01/session4/ipm_lanes/)
        self.lanes = lanes or lib.noc_kkt_default_lanes(family.nx, family.nu, N)
        if not lib.noc_family_supported(ctypes.byref(self.fam_c)):
            raise _lib.NocError(f"unsupported family kind={family.kind} nx={family.nx} nu={family.nu}")
        Bt, N, nx, nu = self.Bt, self.N, self.nx, self.nu
        f64 = dict(device=self.device, dtype=torch.float64)
        i32 = dict(device=self.device, dtype=torch.int32)
        L = self.lanes
        tiled = lambda E: (int(lib.noc_tiled_doubles(N, Bt, L, E)),)
        # LQ blocks and gains in the KKT scan's tiled layout (Q, R packed symmetric)
        shapes = dict(x=(Bt, N + 1, nx), u=(Bt, N, nu), x0=(Bt, nx), A=tiled(nx * nx),
                      B=tiled(nx * nu), Q=tiled(nx * (nx + 1) // 2), R=tiled(nu * (nu + 1) // 2),
                      M=tiled(nx * nu), r=tiled(nu), P=(Bt, nx, nx), cx=tiled(nx),
                      cu=tiled(nu), lc=tiled(1), lam=(Bt, N + 1, nx), dx=(Bt, N + 1, nx),
                      du=(Bt, N, nu), pred=(Bt,), K=tiled(nu * nx), d=tiled(nu))
        for k in _lib.WS_STATE_FIELDS:
            shapes[k] = (Bt,)
        # one zero-filled allocation per dtype (two fill launches instead of one per field: the
        # host cost of a B = 1 call)
        self.t, self._bufs = {}, []
        for spec, kw in ((shapes, f64), ({k: (Bt,) for k in _lib.WS_INT_FIELDS}, i32)):
            views, buf = carve_zeros(spec, **kw)
            self.t.update(views)
            self._bufs.append(buf)
        ws = _lib.NocIpmWs()
        ws.Bt, ws.N, ws.lanes = Bt, N, L
        for k in _lib.WS_DOUBLE_FIELDS + _lib.WS_INT_FIELDS + _lib.WS_STATE_FIELDS:
            setattr(ws, k, self.t[k].data_ptr())
        self.ws = ws
        self._lib = lib
        # overlapping rollouts on a second stream pays once a Newton step costs more than the
        # extra launch + event overhead (measured: c3 B*N = 819k faster, c2 B*N = 102k slower)
        self.overlap = (Bt * N >= 256 * 1024) if overlap is None else bool(overlap)
        if self.overlap:
            self.roll_stream = torch.cuda.Stream(device=self.device)
            self.ev_roll = torch.cuda.Event()
            self.ev_main = torch.cuda.Event()
            self.ev_main.record(torch.cuda.current_stream(self.device))

    # -------------------------------------------------------------------------------------------
    def load(self, controls, initial_state):
        u = torch.as_tensor(np.asarray(controls, dtype=np.float64)).reshape(self.Bt, self.N, self.nu)
        x0 = torch.as_tensor(np.asarray(initial_state, dtype=np.float64)).reshape(self.Bt, self.nx)
        self.t["u"].copy_(u)
        self.t["x0"].copy_(x0)

    def _stream(self):
        return _lib.stream_handle(self.device)

    def init(self, bp0: float = 0.1):
        _lib.check(self._lib.noc_ipm_init(ctypes.byref(self.ws), float(bp0), self._stream()),
                   "noc_ipm_init", self._lib)
        if self.overlap:  # the roll stream must see load() + init() before its first rollout
            self.ev_main.record(torch.cuda.current_stream(self.device))

    def prepare(self, mode: int, terminal: int):
        _lib.check(self._lib.noc_ipm_prepare(ctypes.byref(self.fam_c), ctypes.byref(self.ws), mode,
                                             terminal, self._stream()), "noc_ipm_prepare", self._lib)

    def step(self, mode: int, terminal: int):
        """One device iteration.  With overlap (default) the rollouts of trajectories that start
        a barrier stage run on a second stream beside the other trajectories' Newton step."""
        if not self.overlap:
            _lib.check(self._lib.noc_ipm_step(ctypes.byref(self.fam_c), ctypes.byref(self.ws),
                                              mode, terminal, self.lanes, self._stream()),
                       "noc_ipm_step", self._lib)
            return
        main = torch.cuda.current_stream(self.device)
        roll = self.roll_stream
        roll.wait_event(self.ev_main)
        _lib.check(self._lib.noc_ipm_rollout(ctypes.byref(self.fam_c), ctypes.byref(self.ws),
                                             roll.cuda_stream), "noc_ipm_rollout", self._lib)
        self.ev_roll.record(roll)
        _lib.check(self._lib.noc_ipm_step_main(ctypes.byref(self.fam_c), ctypes.byref(self.ws),
                                               mode, terminal, main.cuda_stream),
                   "noc_ipm_step_main", self._lib)
        main.wait_event(self.ev_roll)
        _lib.check(self._lib.noc_ipm_promote(ctypes.byref(self.ws), main.cuda_stream),
                   "noc_ipm_promote", self._lib)
        self.ev_main.record(main)

    def active_count(self) -> int:
        return int((self.t["phase"] != _lib.PHASE_DONE).sum().item())

    def convergence_norm(self) -> float:
        """max over this engine's trajectories of |Hu|_inf at their last linearisation (P:158)."""
        return float(self.t["hu"].max().item()) if self.Bt else 0.0

    def all_done(self) -> bool:
        return self.active_count() == 0

    def _resident_slots(self) -> int:
        """Trajectories the one-wave persistent kernel holds at once: 2 waves per SIMD."""
        return 8 * torch.cuda.get_device_properties(self.device).multi_processor_count

    def launch_order(self, mode: int, terminal: int, bp0: float) -> torch.Tensor:
        """Highest initial cost first: the initial total cost (P:142 at bp0, one rollout +
        linearisation, noc_ipm_prepare) is a cheap predictor of how many KKT solves a trajectory
        needs; a batch larger than the resident waves then starts its expected stragglers first
        instead of in index order (longest-processing-time-first list scheduling)."""
        self.init(bp0)
        self.prepare(mode, terminal)
        return torch.argsort(self.t["cost"], descending=True, stable=True).to(torch.int32)

    # KKT solves of the probe launch of schedule="probe" (see solve_persistent); c3 measured
    # 36.3 / 35.7 / 35.0 / 34.5 / 34.5 / 34.4 / 34.3 ms at 6 / 10 / 16 / 24 / 32 / 40 / 56
    # (profiles/r05/probe_order/length/)
    PROBE_SOLVES = 32

    def solve_persistent(self, mode: int = _lib.MODE_PAR, terminal: Optional[int] = None,
                         bp0: float = 0.1, max_solves: int = 10 ** 7, resume: bool = False,
                         schedule: str = "auto"):
        """The whole barrier schedule of every trajectory in ONE launch (noc_ipm_solve).
        Returns the KKT solves of the slowest trajectory (the multi-launch loop's step count).
        terminal=None: the reference's choice for the mode (par: XT = Q[0], P:73; seq: S:66).
        resume=True continues every trajectory from the workspace state a previous (capped)
        solve left (NOC_WS_RESUME); max_solves counts the solves of both.
        schedule: "index" launches trajectory i as workgroup i; "cost" launches them by
        descending initial cost (launch_order, ws.order); "probe" runs every trajectory's first
        PROBE_SOLVES KKT solves in one capped launch (equal jobs: two even rounds at c3) and resumes
        the rest ordered by descending total cost at that point, which predicts the remaining
        solves far better than the initial cost does (c3: correlation 0.86-0.89 after 10-40
        solves vs 0.3; profiles/r05/probe_order/); "auto" = "probe" when
        the batch exceeds the resident waves and this is not a resume.  Every trajectory's result
        is the same either way (independent, deterministic, and a capped-and-resumed solve equals
        an uninterrupted one bit for bit); only the schedule changes."""
        terminal = default_terminal(mode) if terminal is None else terminal
        if schedule not in ("auto", "cost", "index", "probe"):
            raise ValueError(schedule)
        auto = schedule == "auto"
        tail = auto and not resume and self._tail_eligible()
        if auto:
            # the probe order also where the launcher splits off the costliest trajectories onto
            # speculative candidates (cart-pole, #SIMDs < B <= 2 #SIMDs: ipm_persistent.hip
            # heavy_count): 2048 cart-poles 20.4 -> 16.3-16.8 ms (profiles/r06/t/)
            probe = not resume and (self.Bt > self._resident_slots() or self._heavy_split_eligible())
            schedule = "probe" if probe and not tail else "index"
        if schedule == "probe" and not resume:
            k = min(int(self.PROBE_SOLVES), int(max_solves))
            self._launch(mode, terminal, bp0, k, resume=False, order=None)
            if k >= max_solves:
                self._order = None
                return int(self.t["kkt_solves"].max().item()) if self.Bt else 0
            # trajectories already done leave at once; the rest start costliest first
            self._order = torch.argsort(self.t["cost"], descending=True, stable=True).to(torch.int32)
            self._launch(mode, terminal, bp0, max_solves, resume=True, order=self._order)
            return int(self.t["kkt_solves"].max().item()) if self.Bt else 0
        ordered = not resume and schedule == "cost"
        self._order = self.launch_order(mode, terminal, bp0) if ordered else None
        if tail and not ordered:
            self._tail_ladder(mode, terminal, bp0, max_solves, resume, None, 0)
        else:
            self._launch(mode, terminal, bp0, max_solves, resume=resume, order=self._order)
        return int(self.t["kkt_solves"].max().item()) if self.Bt else 0

    # The tail of a batch at one wave per SIMD (cart-pole, #SIMDs / 2 < B <= #SIMDs: the 4-GPU
    # slice of c3; NOC_PERSIST_TAIL=0 turns it off):
    # the launch is capped at solve counts TAIL_CAPS, and once the trajectories
    # still running fit two waves each on the SIMDs, they are gathered into a small workspace and
    # resumed there -- where the solver runs speculative candidates (two or four waves per
    # trajectory, csrc/ipm_persistent.hip: SPEC), so the stragglers' serial chains of rejected
    # trials shorten.  Results, counters and iterates are the uninterrupted solve's bit for bit
    # (capped-and-resumed solves and the candidates both are).  Measured (profiles/r06/o/): 1024
    # cart-poles 13.83-13.91 -> 13.30-13.34 ms with the caps below (cap 256: 205 still running,
    # resumed with four candidates); not at 2 waves per SIMD (2048: equal) nor after the probe
    # launch (4096: 29-31 vs 25 ms -- it breaks the cost-ordered resume), so not there.
    # NOC_PERSIST_TAIL_CAPS="a,b,..." sets the caps.
    TAIL_CAPS = (256, 384, 512)
    _SHARED_FIELDS = ("x", "u", "x0") + tuple(_lib.WS_STATE_FIELDS) + tuple(_lib.WS_INT_FIELDS)

    def _simds(self) -> int:
        return 4 * torch.cuda.get_device_properties(self.device).multi_processor_count

    def _heavy_split_eligible(self) -> bool:
        if os.environ.get("NOC_PERSIST_HEAVY_SPEC") == "0" or os.environ.get("NOC_PERSIST_SPEC") == "1":
            return False
        simds = self._simds()
        return (self.persistent and self.family.kind == _lib.FAMILY_CARTPOLE and self.N <= 320
                and simds < self.Bt <= 2 * simds)

    def _tail_eligible(self) -> bool:
        if os.environ.get("NOC_PERSIST_TAIL", "1") == "0" or os.environ.get("NOC_PERSIST_SPEC") == "1":
            return False
        if os.environ.get("NOC_PERSIST_STRUCT") == "0":
            return False
        simds = self._simds()
        return (self.persistent and self.family.kind == _lib.FAMILY_CARTPOLE and self.N <= 320
                and simds < 2 * self.Bt <= 2 * simds)

    def _tail_caps(self):
        env = os.environ.get("NOC_PERSIST_TAIL_CAPS")
        return tuple(int(c) for c in env.split(",")) if env else self.TAIL_CAPS

    def _tail_ladder(self, mode, terminal, bp0, max_solves, resume, order, done_cap):
        simds = self._simds()
        self.tail_log = []
        for cap in self._tail_caps():
            if cap <= done_cap:
                continue
            if cap >= max_solves:
                break
            self._launch(mode, terminal, bp0, cap, resume=resume, order=order)
            resume = True
            run = torch.nonzero(self.t["phase"] != _lib.PHASE_DONE).flatten()
            R = int(run.numel())
            self.tail_log.append((cap, R))
            if R == 0:
                return
            if 2 * R <= simds:
                self._tail_gather(run, mode, terminal, bp0, max_solves)
                return
        self._launch(mode, terminal, bp0, max_solves, resume=resume, order=order)

    def _tail_gather(self, run, mode, terminal, bp0, max_solves):
        sub = BatchedIPM(self.family, self.N, int(run.numel()), device=self.device, lanes=64,
                         persistent=True)
        for k in self._SHARED_FIELDS:
            sub.t[k].copy_(self.t[k].index_select(0, run))
        sub.ws.flags = self.ws.flags
        sub._launch(mode, terminal, bp0, max_solves, resume=True, order=None)
        for k in self._SHARED_FIELDS:
            self.t[k].index_copy_(0, run, sub.t[k])

    def _launch(self, mode, terminal, bp0, max_solves, resume, order):
        """one noc_ipm_solve (resume: NOC_WS_RESUME; order: ws.order, a permutation or None)"""
        flags = self.ws.flags
        if resume:
            self.ws.flags = flags | _lib.WS_RESUME
        self.ws.order = order.data_ptr() if order is not None else None
        try:
            _lib.check(self._lib.noc_ipm_solve(ctypes.byref(self.fam_c), ctypes.byref(self.ws),
                                               mode, terminal, float(bp0), int(max_solves),
                                               self._stream()), "noc_ipm_solve", self._lib)
        finally:
            self.ws.flags = flags
            self.ws.order = None

    def solve(self, mode: int = _lib.MODE_PAR, terminal: Optional[int] = None,
              bp0: float = 0.1, poll_every: int = 8, max_steps: Optional[int] = None):
        """Run the barrier schedule to completion for every trajectory.  Returns the KKT solves of
        the slowest trajectory (kkt_solves.max(), on both paths).  max_steps caps the KKT solves
        of every trajectory on both paths: the persistent solve stops a trajectory at that many
        solves (resumable); the multi-launch loop stops once every trajectory that is still running
        is at or past the cap (trajectories that finished earlier do not hold it back; one launch
        may account up to 501 identical retries, P:151-188).
        terminal=None: the reference's choice for the mode (par: XT = Q[0], P:73; seq:
        hessian(final_cost), S:66)."""
        terminal = default_terminal(mode) if terminal is None else terminal
        if self.persistent:
            return self.solve_persistent(mode, terminal, bp0,
                                         max_steps if max_steps is not None else 10 ** 7)
        self.init(bp0)
        while True:
            for _ in range(poll_every):
                self.step(mode, terminal)
            if self.all_done():
                break
            if max_steps is not None:
                running = self.t["phase"] != _lib.PHASE_DONE
                if int(self.t["kkt_solves"][running].min().item()) >= max_steps:
                    break
        return int(self.t["kkt_solves"].max().item()) if self.Bt else 0

    def tiled_blocks(self):
        from .lqt import TiledBlocks
        t = self.t
        return TiledBlocks(t["A"], t["B"], t["Q"], t["R"], t["M"], t["r"], t["P"], self.nx,
                           self.nu, self.N, self.Bt, self.lanes)

    def natural_blocks(self):
        """The LQ blocks relaid out to the natural (Bt, N, ...) layout (tests / export)."""
        from .lqt import untile
        Bt, N, nx, nu, L, t = self.Bt, self.N, self.nx, self.nu, self.lanes, self.t
        return dict(A=untile(t["A"], (Bt, N, nx, nx), L), B=untile(t["B"], (Bt, N, nx, nu), L),
                    Q=untile(t["Q"], (Bt, N, nx, nx), L, sym=True),
                    R=untile(t["R"], (Bt, N, nu, nu), L, sym=True),
                    M=untile(t["M"], (Bt, N, nx, nu), L), r=untile(t["r"], (Bt, N, nu), L),
                    P=t["P"])

    # -------------------------------------------------------------------------------------------
    def host_result(self):
        """(u, total_it, kkt_solves, x) as numpy arrays in two device-to-host copies: x and u are
        neighbours in the fp64 workspace allocation, total_it and kkt_solves in the int32 one, so
        each pair leaves as one contiguous span (the per-call host cost of small solves)."""
        out = {}
        for buf, names in ((self._bufs[0], ("x", "u")), (self._bufs[1], ("total_it", "kkt_solves"))):
            es = buf.element_size()
            offs = {k: (self.t[k].data_ptr() - buf.data_ptr()) // es for k in names}
            lo = min(offs.values())
            hi = max(offs[k] + self.t[k].numel() for k in names)
            host = buf[lo:hi].cpu().numpy()
            for k in names:
                out[k] = host[offs[k] - lo:offs[k] - lo + self.t[k].numel()].reshape(self.t[k].shape)
        return out["u"], out["total_it"], out["kkt_solves"], out["x"]

    def result(self):
        return (self.t["u"].clone(), self.t["total_it"].clone(), self.t["kkt_solves"].clone())
