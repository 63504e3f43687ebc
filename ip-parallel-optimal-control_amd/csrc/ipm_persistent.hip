// Persistent batched interior-point solver: the WHOLE barrier schedule of one trajectory in one
// wave64, one launch for the batch (fp64, gfx950).
//
// Replaces par_interior_point_optimal_control / newton_oc (noc/par_interior_point_newton.py:
// 127-254) and, with NOC_MODE_SEQ, seq_interior_point_optimal_control (noc/seq_interior_point_
// newton.py:108-202), for registered families.  Every trajectory runs its own reference control
// flow back to back -- rollout, linearise, costates, LQ blocks, KKT scan, trial / accept /
// regularisation, Newton stop test, barrier schedule -- with no kernel boundary, no host poll and
// no all-trajectory lockstep: a trajectory that needs 850 Newton steps no longer holds 4095 others
// in per-step launches, and the per-step launch overhead is gone.
//
// Same arithmetic and state machine as the multi-launch driver (ipm_kernels.hip + the KKT scan
// kernel at lanes = 64), so both produce identical iterates.  Lane l owns the horizon chunk of
// the tiled layout (workspace lanes must be 64); cross-lane data moves through shuffles, the
// KKT step stays in LDS (kkt_scan_wave with lds_out and dx = du = NULL), and the few hand-offs
// through the workspace (rollout states, pred / feasible, the terminal Hessian) are ordered by a
// workgroup fence (one wave = one workgroup).
#include <hip/hip_runtime.h>
#include <cstdlib>

#include "../../include/noc_hip.h"
#include "block_struct.h"
#include "ipm_family.h"
#include "kkt_scan_impl.h"
#include "noc_internal.h"

namespace noc {

// Per-phase cycle counters of workgroup 0 (timing-only instrumentation; built only with
// -DNOC_PERSIST_PROFILE, read back by noc_debug_phase_cycles): rollout, linearise, costate +
// blocks, KKT scan, trial, number of Newton iterations.
__device__ long long g_phase_cycles[8];  // [6]: the trial's costs + reductions; [7]: the costate scan
// Start / end wall-clock stamps (s_memrealtime, 100 MHz) of every trajectory's persistent solve,
// same builds only (read back by noc_debug_traj_times): the batch's schedule, e.g. when the
// straggler that sets the wall time started and how its neighbours thinned out.
constexpr int kTrajStamps = 16384;
__device__ long long g_traj_times[kTrajStamps][2];
// decision trace (-DNOC_DECISION_TRACE builds only; noc_internal.h)
__device__ DecisionTrace g_dtrace;

namespace {
constexpr int PL = 64;  // lanes per trajectory in the persistent solver

NOC_DEV void wave_fence() { __threadfence_block(); }

// Wave-uniform solver state, parked in LDS across the KKT scan (whose register footprint is the
// kernel's peak) instead of being kept live in VGPRs through it.
struct IpmState {
  double bp, rp, rinc, cost, hu, gnorm;
  int it, inner, total_it, solves;
};
// Speculative candidates (SPEC > 1 waves per trajectory, one candidate regularisation each): the
// scan's reg / pred / feasible of a wave's candidate, and its trial cost, exchanged through LDS.
struct SpecIO {
  double reg, pred, new_cost, pad;
  int feasible, pad2[3];
};

// LDS of one workgroup, in doubles: SPEC regions of KKT slots (lds_slots: one per 64-lane
// segment), SPEC parked states, SPEC SpecIO records (SPEC > 1 only), then SPEC copies of x, u
// (XLDS).  SPEC = 1 is the one-wave layout: [slots][state][x, u].
template <int NX, int NU>
__host__ __device__ constexpr int slot_doubles(int N) { return (N * kd_width<NX, NU>() + NX + 1) & ~1; }
__host__ __device__ constexpr int state_doubles() { return (int)((sizeof(IpmState) + 15) / 16) * 2; }
__host__ __device__ constexpr int specio_doubles(int spec) { return spec > 1 ? (int)(sizeof(SpecIO) / 8) * spec : 0; }
template <int NX, int NU>
NOC_DEV IpmState* state_slot(int N, int spec = 1, int wv = 0) {
  extern __shared__ __attribute__((aligned(16))) double noc_smem[];
  return reinterpret_cast<IpmState*>(noc_smem + spec * slot_doubles<NX, NU>(N) + wv * state_doubles());
}
template <int NX, int NU>
NOC_DEV SpecIO* spec_io(int N, int spec, int wv) {
  extern __shared__ __attribute__((aligned(16))) double noc_smem[];
  return reinterpret_cast<SpecIO*>(noc_smem + spec * (slot_doubles<NX, NU>(N) + state_doubles())) + wv;
}

// XLDS instances: the trajectory's states and controls x[0..N], u[0..N-1] live in LDS for the
// whole solve (the rollout, linearisation, costate sweep, trial and update all read or write
// them; from the workspace each access was a global round trip), copied in at the start and out
// at the end.  Layout behind the KKT slots and the parked state: x [(N+1) NX], u [N NU].
template <int NX, int NU>
__host__ __device__ constexpr int xlds_doubles(int N) { return ((N + 1) * NX + N * NU + 1) & ~1; }
template <int NX, int NU>
__host__ __device__ constexpr int xlds_off(int N, int spec = 1, int wv = 0) {
  return spec * (slot_doubles<NX, NU>(N) + state_doubles()) + specio_doubles(spec) + wv * xlds_doubles<NX, NU>(N);
}

// The KKT scan's block source in the persistent solver: the workspace's compact tiled fields (only
// the variable entries of A, B, Q, R, M; block_struct.h), expanded with the family's constants as
// they are loaded.  BS = BlockStruct<..., false> is the dense layout (the NOC_PERSIST_STRUCT=0
// instance), which loads exactly what ArgsSrc does.
template <class BS, int NX, int NU, int L>
struct CompactSrc {
  using Struct = BS;
  const KKTArgs& a;
  const noc_family& p;
  int traj, l, cmax;
  size_t tN;
  template <int F, bool LAST = false>
  NOC_DEV void field(const double* base, int j, double* full) const {
    constexpr int EV = BS::template nv<F>();
    double v[EV > 0 ? EV : 1];
    if constexpr (EV > 0) tload_pol<EV, L, LAST>(base, traj, j, l, cmax, v);
    BS::template expand<F>(p, v, full);
  }
  // PART / LAST: as load_stage (kkt_scan_impl.h)
  template <int PART, bool LAST = false>
  NOC_DEV void stage_part(int s, int j, double reg, StageData<NX, NU>& st) const {
    constexpr bool REST = PART != 2, WQ = PART != 1, WAB = REST && PART != 3;
    (void)s;
    (void)reg;
    if constexpr (WAB) {
      field<BF_A>(a.A, j, st.A.v);
      field<BF_B>(a.Bm, j, st.B.v);
    }
    if constexpr (WQ) field<BF_Q, LAST>(a.Q, j, st.Q.v);
    if constexpr (REST) {
      field<BF_R, LAST>(a.R, j, st.R.v);
      field<BF_M, LAST>(a.M, j, st.M.v);
      tload_pol<NU, L, LAST>(a.r, traj, j, l, cmax, st.r.v);
    }
  }
  NOC_DEV void stage(int s, int j, double reg, StageData<NX, NU>& st) const { stage_part<0>(s, j, reg, st); }
  NOC_DEV void stage_last(int s, int j, double reg, StageData<NX, NU>& st) const {
    stage_part<0, true>(s, j, reg, st);
  }
  NOC_DEV void ab(int s, int j, Mat<NX, NX>& A, Mat<NX, NU>& Bm, Vec<NX>& c) const {
    (void)s;
    field<BF_A, true>(a.A, j, A.v);  // phase 4: the last read of A, B (non-temporal)
    field<BF_B, true>(a.Bm, j, Bm.v);
    set_zero(c);
  }
  NOC_DEV void cvec(int, int, Vec<NX>& c) const { set_zero(c); }
};

}  // namespace

#ifdef NOC_PERSIST_PROFILE
#define NOC_PHASE(i) do { const long long t_ = clock64(); if (b == 0 && lead) g_phase_cycles[i] += t_ - t_prev; t_prev = t_; } while (0)
// a sub-phase ending now, started at t0 (does not move t_prev)
#define NOC_SUB(i, t0) do { if (b == 0 && lead) g_phase_cycles[i] += clock64() - (t0); } while (0)
#define NOC_T0(v) const long long v = clock64()
#else
#define NOC_PHASE(i) do { } while (0)
#define NOC_SUB(i, t0) do { } while (0)
#define NOC_T0(v) do { } while (0)
#endif

// WPS: waves per SIMD the register budget is sized for.  2 = 256 registers per lane; 1 = 512, the
// upper half AGPRs, which the compiler uses as spill space instead of scratch (cart-pole: 460 B
// of scratch per lane at WPS = 2, none at WPS = 1), and which pays for the stage pairs below.
// RESUME: continue from the workspace state (NOC_WS_RESUME; its own instance, so the plain solve's
// register allocation does not carry the resume bookkeeping).
// STRUCT: the structure-aware blocks (block_struct.h; NOC_PERSIST_STRUCT=0 selects the dense
// instance, which computes the same doubles).
// SPEC: waves per trajectory, each solving one candidate of the regularisation's failure chain
// (speculative retries, below); 1 = the plain solver.  SPEC > 1 needs XLDS (every wave keeps its
// own copy of x, u).
template <int KIND, int NX, int NU, int WPS, bool RESUME, bool XLDS, bool STRUCT, int SPEC = 1>
__global__ __launch_bounds__(64 * SPEC, WPS) void ipm_solve_kernel(noc_family prm, noc_ipm_ws w, int mode,
                                                                int terminal, double bp0,
                                                                int max_solves) {
  static_assert(SPEC == 1 || XLDS, "speculative waves keep x, u in LDS");
  // one wave (= one 64-thread workgroup) per trajectory -- SPEC waves with SPEC > 1; w.order: the
  // launch order (a permutation)
  const int b = w.order ? w.order[blockIdx.x] : (int)blockIdx.x;
  const int l = SPEC > 1 ? (int)(threadIdx.x & 63) : (int)threadIdx.x;  // lane = chunk owner
  const int wv = SPEC > 1 ? (int)(threadIdx.x >> 6) : 0;                 // candidate of this wave
  const bool lead = (l == 0) && (wv == 0);  // writes the trajectory's results
  (void)lead;
  if (b < 0 || b >= w.Bt) return;  // an out-of-range order entry solves nothing (never faults)
  constexpr int KD = kd_width<NX, NU>();
  Fam<KIND, NX, NU> f(prm);
  using BS = BlockStruct<KIND, NX, NU, STRUCT>;
  constexpr int VA = BS::template nv<BF_A>(), VB = BS::template nv<BF_B>();
  constexpr int VQ = BS::template nv<BF_Q>(), VR = BS::template nv<BF_R>(), VM = BS::template nv<BF_M>();
  const int N = w.N;
  const Chunks ch(N, PL);
  const int start = ch.start(l), len = ch.len(l), cmax = ch.cmax;
  const bool last = (l == PL - 1);
  // Stage pairs: two stages per pass through the per-stage loops (linearise, costate + blocks,
  // trial), both loaded before either is computed, so their independent transcendental chains
  // (sincos, divisions, log) interleave.  Needs the 1-wave-per-SIMD register budget; the trip
  // count follows the wave-uniform chunk bound cmax (lanes past their own chunk compute a clamped
  // duplicate stage and discard it).
  const bool pair = (WPS == 1) && cmax >= 2;
  auto clampk = [&](int k) { return k < N - 1 ? k : N - 1; };
  double* const Xg = w.x + (size_t)b * (N + 1) * NX;
  double* const Ug = w.u + (size_t)b * N * NU;
  extern __shared__ __attribute__((aligned(16))) double noc_smem[];
  double* const X = XLDS ? noc_smem + xlds_off<NX, NU>(N, SPEC, wv) : Xg;
  double* const U = XLDS ? noc_smem + xlds_off<NX, NU>(N, SPEC, wv) + (N + 1) * NX : Ug;
  if constexpr (XLDS) {  // the workspace's x (a resume point's states) and u into LDS
    for (int i = l; i < (N + 1) * NX; i += 64) X[i] = Xg[i];
    for (int i = l; i < N * NU; i += 64) U[i] = Ug[i];
    wave_fence();
  }
  const double* slot = lds_slots<NX, NU, PL>(N);

  KKTArgs a{};
  a.N = N;
  a.B = w.Bt;
  a.mode = MODE_FULL;
  a.A = w.A; a.Bm = w.B; a.Q = w.Q; a.R = w.R; a.M = w.M; a.r = w.r; a.P = w.P; a.reg = w.reg;
  a.pred = w.pred; a.feasible = w.feasible;
  a.tiled = 1;
  a.lds_out = 1;  // dx, du stay in LDS (a.dx = a.du = NULL): the trial reads them there
  SpecIO* const io = SPEC > 1 ? spec_io<NX, NU>(N, SPEC, wv) : nullptr;
  if constexpr (SPEC > 1) {  // this wave's candidate: reg, pred, feasible in its LDS record
    a.reg = &io->reg;
    a.pred = &io->pred;
    a.feasible = &io->feasible;
  }

  double bp = bp0, rp = 1.0, rinc = 2.0, cost = 0.0, hu = 1.0, gnorm = 0.0;
  int it = 0, inner = 0, total_it = 0, solves = 0;
  bool capped = false;
  int phase = NOC_PHASE_DONE;     // the resume point a capped launch leaves in the workspace
  int entry = NOC_PHASE_ROLLOUT;  // RESUME: where this launch starts
  if constexpr (RESUME) {
    bp = w.bp[b]; rp = w.rp[b]; rinc = w.rinc[b]; cost = w.cost[b]; hu = w.hu[b];
    gnorm = w.gnorm[b]; it = w.it[b]; inner = w.inner[b]; total_it = w.total_it[b];
    solves = w.kkt_solves[b]; entry = resume_phase(w.phase[b]);
    if (entry == NOC_PHASE_DONE) return;  // uniform over the wave
  } else {
    if (lead && w.repeats) w.repeats[b] = 0;
  }

#ifdef NOC_PERSIST_PROFILE
  long long t_prev = clock64();
  if (lead && b < kTrajStamps) g_traj_times[b][0] = (long long)__builtin_amdgcn_s_memrealtime();
#endif
  // lc_fresh: the workspace's stage costs (w.lc) already belong to the current (x, u) -- the last
  // trial wrote them, and it was taken -- so the next linearisation skips f.stage_cost (the
  // trial evaluated the same function on the same doubles: x + dx is the update's own sum).  False
  // at every launch start (a resume may follow the per-phase driver, whose trial does not write
  // w.lc) and after every rollout (new barrier parameter).
  bool lc_fresh = false;
  for (;;) {  // ---------------- barrier stages (P:228-254) ----------------
    // rollout x_{k+1} = f(x_k, u_k) (noc/utils.py:57-63, P:133): every lane runs the recurrence
    // redundantly with u_k broadcast by readlane; lane t stores the states of block step t
    wave_fence();  // u was last written chunk-wise by the trials
    if (!RESUME || entry == NOC_PHASE_ROLLOUT) {
      double x[NX];
      NOC_UNROLL for (int i = 0; i < NX; ++i) x[i] = w.x0[(size_t)b * NX + i];
      if (l < NX) X[l] = x[l];
      for (int base = 0; base < N; base += 64) {
        const int k = base + l;
        double uk[NU];
        NOC_UNROLL for (int j = 0; j < NU; ++j) uk[j] = (k < N) ? U[(size_t)k * NU + j] : 0.0;
        double mine[NX];
        NOC_UNROLL for (int i = 0; i < NX; ++i) mine[i] = 0.0;
        const int cnt = (N - base < 64) ? (N - base) : 64;
        for (int t = 0; t < cnt; ++t) {
          double ut[NU], xn[NX];
          NOC_UNROLL for (int j = 0; j < NU; ++j) ut[j] = readlane_d(uk[j], t);
          f.step(x, ut, xn);
          NOC_UNROLL for (int i = 0; i < NX; ++i) {
            x[i] = xn[i];
            mine[i] = (l == t) ? xn[i] : mine[i];
          }
        }
        if (k < N) NOC_UNROLL for (int i = 0; i < NX; ++i) X[(size_t)(k + 1) * NX + i] = mine[i];
      }
    }
    wave_fence();  // states of every stage visible to their chunk owners
    NOC_PHASE(0);
    lc_fresh = false;
    // A SOLVE resume (a retry on the current point) recomputes the blocks from the workspace's
    // states -- the same doubles the capped launch had; the workspace blocks may be another
    // driver's layout (dense / compact) -- and keeps the solver state it left (cost, |Hu|,
    // ||cu||, the retry counter), like the wide kernel (ipm_wide.hip)
    bool relinearize = true;
    bool keep_state = RESUME && entry == NOC_PHASE_SOLVE;
    if constexpr (RESUME) entry = NOC_PHASE_ROLLOUT;
    bool stage_done = false;
    while (!stage_done) {  // ---------------- Newton iterations (P:127-225) ----------------
      const bool relinearized = relinearize;  // uniform over the workgroup
      if (relinearize) {
        // linearise the own chunk (P:13-28): A = fx, B = fu, cx, cu, stage cost
        struct LinOut {
          double fx[NX * NX], fu[NX * NU], cx[NX], cu[NU], lc;
        };
        auto lin_compute = [&](const double* x, const double* u, LinOut& o) {
          f.jac(x, u, o.fx, o.fu);
          BS::template fold_consts<BF_A>(prm, o.fx);  // structural entries as literals / parameters
          BS::template fold_consts<BF_B>(prm, o.fu);
          f.stage_grad(x, u, bp, o.cx, o.cu);
          if (!lc_fresh) o.lc = f.stage_cost(x, u, bp);  // uniform over the wave
        };
        auto lin_store = [&](int j, const LinOut& o) {  // compact A, B: variable entries only
          double va[VA > 0 ? VA : 1], vb[VB > 0 ? VB : 1];
          BS::template compress<BF_A>(o.fx, va);
          BS::template compress<BF_B>(o.fu, vb);
          if constexpr (VA > 0) tstore<VA, PL>(w.A, b, j, l, cmax, va);
          if constexpr (VB > 0) tstore<VB, PL>(w.B, b, j, l, cmax, vb);
          if (!lc_fresh) tstore<1, PL>(w.lc, b, j, l, cmax, &o.lc);
        };
        auto load_xu = [&](int k, double* x, double* u) {
          gload<NX>(X + (size_t)k * NX, x);
          NOC_UNROLL for (int i = 0; i < NU; ++i) u[i] = U[(size_t)k * NU + i];
        };
        // The costates are a reverse affine scan (C:34-54) fused with the LQ blocks (P:31-42).
        // Its in-chunk fold (G, g) <- (A' G, cx + A' g) runs inside the linearisation, which
        // walks the chunk backwards for it, on the A, cx it has just computed -- the same
        // operations in the same order as a separate pass reading them back from the workspace,
        // without that pass's loads (the solve moves ~6.5 TB/s at c3).
        Mat<NX, NX> G;
        Vec<NX> g;
        set_identity(G);
        set_zero(g);
        auto fold = [&](const LinOut& o, bool valid) {
          Mat<NX, NX> Gn;
          Vec<NX> gn;
          NOC_UNROLL for (int i = 0; i < NX; ++i) {
            double t = o.cx[i];
            NOC_UNROLL for (int m = 0; m < NX; ++m) if (BS::nzA(m, i)) t += o.fx[m * NX + i] * g[m];
            gn[i] = t;
            NOC_UNROLL for (int jj = 0; jj < NX; ++jj) {
              double u = 0.0;
              NOC_UNROLL for (int m = 0; m < NX; ++m) if (BS::nzA(m, i)) u += o.fx[m * NX + i] * G(m, jj);
              Gn(i, jj) = u;
            }
          }
          NOC_UNROLL for (int i = 0; i < NX * NX; ++i) G.v[i] = valid ? Gn.v[i] : G.v[i];
          NOC_UNROLL for (int i = 0; i < NX; ++i) g.v[i] = valid ? gn.v[i] : g.v[i];
        };
        if (pair) {  // descending pairs over the wave-uniform chunk bound: loads, then both
                     // computations, then the stores and the fold (one basic block of work)
          for (int j = cmax - 1; j >= 0; j -= 2) {
            double x0[NX], u0[NU], x1[NX], u1[NU];
            load_xu(clampk(start + j), x0, u0);
            load_xu(clampk(start + (j - 1 >= 0 ? j - 1 : j)), x1, u1);
            const bool v0 = j < len, v1 = j - 1 >= 0 && j - 1 < len;
            LinOut o0, o1;
            lin_compute(x0, u0, o0);
            lin_compute(x1, u1, o1);
            if (v0) lin_store(j, o0);
            if (v1) lin_store(j - 1, o1);
            fold(o0, v0);
            fold(o1, v1);
          }
        } else {
          for (int j = len - 1; j >= 0; --j) {
            double x[NX], u[NU];
            load_xu(start + j, x, u);
            LinOut o;
            lin_compute(x, u, o);
            lin_store(j, o);
            fold(o, true);
          }
        }
        NOC_PHASE(1);
        const double* xN = X + (size_t)N * NX;
        double lamN[NX];
        NOC_T0(t_cs);
        f.final_grad(xN, lamN);  // grad(final_cost) (C:35)
        if (last) {
          NOC_UNROLL for (int i = 0; i < NX; ++i) {
            double t = g[i];
            NOC_UNROLL for (int m = 0; m < NX; ++m) t += G(i, m) * lamN[m];
            g[i] = t;
          }
          set_zero(G);
        }
#pragma unroll 1
        for (int d = 1; d < PL; d <<= 1) {
          Mat<NX, NX> G2;
          Vec<NX> g2;
          shfl_down_arr<NX * NX>(G.v, G2.v, d, PL);
          shfl_down_arr<NX>(g.v, g2.v, d, PL);
          Mat<NX, NX> Gn;
          NOC_UNROLL for (int i = 0; i < NX; ++i) {
            double t = g[i];
            NOC_UNROLL for (int m = 0; m < NX; ++m) t += G(i, m) * g2[m];
            g[i] = t;
            NOC_UNROLL for (int jj = 0; jj < NX; ++jj) {
              double u = 0.0;
              NOC_UNROLL for (int m = 0; m < NX; ++m) u += G(i, m) * G2(m, jj);
              Gn(i, jj) = u;
            }
          }
          G = Gn;
        }
        // The costates stay in registers: the solve does not store lambda to the workspace (a
        // strided 8 * nx bytes per stage and lane, c3 ipm_solve -2.7 %, profiles/r05/lam_store/)
        double lam[NX];
        shfl_down_arr<NX>(g.v, lam, 1, PL);
        if (last) NOC_UNROLL for (int i = 0; i < NX; ++i) lam[i] = lamN[i];
        NOC_SUB(7, t_cs);
        double csum = 0.0, hmax = 0.0, g2s = 0.0;
        // One stage of the costate sweep fused with its LQ blocks.  `valid` = false computes on a
        // clamped duplicate stage and leaves lambda, the sums and memory untouched (selects, not
        // branches, so a pair of stages stays one basic block).
        struct StageIn {
          double A[NX * NX], Bm[NX * NU], cx[NX], cu[NU], lc, x[NX], u[NU];
        };
        auto load_in = [&](int j, StageIn& in) {
          // 0 <= j < cmax: every lane's tiled slots exist up to cmax; for a slot past the lane's
          // own chunk the data are a discarded duplicate (x, u clamped into the horizon)
          double va[VA > 0 ? VA : 1], vb[VB > 0 ? VB : 1];
          if constexpr (VA > 0) tload<VA, PL>(w.A, b, j, l, cmax, va);
          if constexpr (VB > 0) tload<VB, PL>(w.B, b, j, l, cmax, vb);
          BS::template expand<BF_A>(prm, va, in.A);
          BS::template expand<BF_B>(prm, vb, in.Bm);
          tload<1, PL>(w.lc, b, j, l, cmax, &in.lc);
          load_xu(clampk(start + j), in.x, in.u);
          // cx, cu re-evaluated (the linearisation's values bit for bit) instead of stored and read
          // back: a workspace round trip of nx + nu doubles per stage against one stage_grad
          f.stage_grad(in.x, in.u, bp, in.cx, in.cu);
        };
        // LQ blocks at lambda_{k+1} (P:35-37): Q = cxx + l.fxx, R = cuu + l.fuu, M = cxu + l.fxu;
        // ru_k = cu_k + fu_k' lambda_{k+1} (P:34); then lambda_k = cx_k + fx_k' lambda_{k+1}
        struct StageOut {
          Sym<NX> Qs;
          Sym<NU> Rs;
          double M[NX * NU], rr[NU], lam[NX];
        };
        auto cost_compute = [&](const StageIn& in, bool valid, StageOut& o) {
          double Q[NX * NX], R[NU * NU];
          f.stage_hess(in.x, in.u, bp, Q, R, o.M);
          f.add_hess_l(in.x, in.u, lam, Q, R, o.M);
          BS::template fold_consts<BF_M>(prm, o.M);
          NOC_UNROLL for (int i = 0; i < NX; ++i)
            NOC_UNROLL for (int jj = i; jj < NX; ++jj) o.Qs(i, jj) = (i == jj) ? Q[i * NX + i] : 0.5 * (Q[i * NX + jj] + Q[jj * NX + i]);
          NOC_UNROLL for (int i = 0; i < NU; ++i)
            NOC_UNROLL for (int jj = i; jj < NU; ++jj) o.Rs(i, jj) = (i == jj) ? R[i * NU + i] : 0.5 * (R[i * NU + jj] + R[jj * NU + i]);
          BS::template fold_consts<BF_Q>(prm, o.Qs.v);
          BS::template fold_consts<BF_R>(prm, o.Rs.v);
          NOC_UNROLL for (int jj = 0; jj < NU; ++jj) {
            double r = in.cu[jj];
            NOC_UNROLL for (int i = 0; i < NX; ++i) if (BS::nzB(i, jj)) r += in.Bm[i * NU + jj] * lam[i];
            o.rr[jj] = r;
            hmax = valid ? nan_max(hmax, fabs(r)) : hmax;
            g2s = valid ? g2s + in.cu[jj] * in.cu[jj] : g2s;
          }
          NOC_UNROLL for (int i = 0; i < NX; ++i) {
            double t = in.cx[i];
            NOC_UNROLL for (int m = 0; m < NX; ++m) if (BS::nzA(m, i)) t += in.A[m * NX + i] * lam[m];
            o.lam[i] = t;
          }
          csum = valid ? csum + in.lc : csum;
          NOC_UNROLL for (int i = 0; i < NX; ++i) lam[i] = valid ? o.lam[i] : lam[i];
        };
        auto cost_store = [&](int j, const StageIn& in, const StageOut& o) {
          const int k = start + j;
          double vq[VQ > 0 ? VQ : 1], vr[VR > 0 ? VR : 1], vm[VM > 0 ? VM : 1];
          BS::template compress<BF_Q>(o.Qs.v, vq);
          BS::template compress<BF_R>(o.Rs.v, vr);
          BS::template compress<BF_M>(o.M, vm);
          if constexpr (VQ > 0) tstore<VQ, PL>(w.Q, b, j, l, cmax, vq);
          if constexpr (VR > 0) tstore<VR, PL>(w.R, b, j, l, cmax, vr);
          if constexpr (VM > 0) tstore<VM, PL>(w.M, b, j, l, cmax, vm);
          if (terminal == NOC_TERMINAL_STAGE0 && k == 0) {  // XT = Q[0] (P:73), full matrix
            double Q[NX * NX];
            NOC_UNROLL for (int i = 0; i < NX; ++i) NOC_UNROLL for (int jj = 0; jj < NX; ++jj) Q[i * NX + jj] = o.Qs(i, jj);
            gstore<NX * NX>(w.P + (size_t)b * NX * NX, Q);
          }
          tstore<NU, PL>(w.r, b, j, l, cmax, o.rr);
        };
        if (pair) {  // descending pairs over the wave-uniform chunk bound; short lanes skip slots
          for (int j = cmax - 1; j >= 0; j -= 2) {
            StageIn in0, in1;
            load_in(j, in0);
            load_in(j - 1 >= 0 ? j - 1 : j, in1);
            const bool v0 = j < len, v1 = j - 1 >= 0 && j - 1 < len;
            StageOut o0, o1;
            cost_compute(in0, v0, o0);
            cost_compute(in1, v1, o1);
            if (v0) cost_store(j, in0, o0);
            if (v1) cost_store(j - 1, in1, o1);
          }
        } else {
          for (int j = len - 1; j >= 0; --j) {
            StageIn in;
            load_in(j, in);
            StageOut o;
            cost_compute(in, true, o);
            cost_store(j, in, o);
          }
        }
        // lambda at the chunk start := the scan's value g (not this lane's sweep): it is exactly the
        // boundary costate the previous lane used, so every consumer of lambda_k sees one value
        {  // the __shfl_xor butterflies with VALU partners (bit-identical, small_linalg.h)
          const int ln = (int)__lane_id();
          auto add = [](double x, double y) { return x + y; };
          csum = segment_allreduce<PL>(csum, ln, add);
          g2s = segment_allreduce<PL>(g2s, ln, add);
          hmax = segment_allreduce<PL>(hmax, ln, [](double x, double y) { return nan_max(x, y); });
        }
        if (terminal == NOC_TERMINAL_FINAL_COST && last) {  // hessian(final_cost) (S:66)
          double P[NX * NX];
          f.final_hess(xN, P);
          gstore<NX * NX>(w.P + (size_t)b * NX * NX, P);
        }
        if (!keep_state) {
          // total_cost(x, u, bp) (P:142); x_N is the last lane's own (trial) store
          cost = readlane_d(csum + f.final_cost(xN), PL - 1);
          hu = hmax;                                      // max |Hu| (P:158)
          gnorm = sqrt(g2s);                              // ||cu||_F (P:116)
          inner = 0;
        }
        keep_state = false;
        // regularisation: par R += rp*||cu||*I (P:116-118); seq Quu += mu*I (S:51)
        relinearize = false;
      }
      // The candidates of this solve: candidate k is the regularisation the solver reaches after
      // k rejected trials at this point (P:167-173 / S:139-144).  SPEC = 1: only k = 0, stored per
      // trajectory as before; SPEC > 1: wave k solves candidate k (its LDS record).
      double c_reg[SPEC];
      {
        double r = rp, ri = rinc;
        NOC_UNROLL for (int k = 0; k < SPEC; ++k) {
          c_reg[k] = (mode == NOC_MODE_PAR) ? r * gnorm : r;
          r = r * ri;
          ri = 2.0 * ri;
          if (mode == NOC_MODE_PAR) r = fmin(fmax(r, 1e-16), 1e16);
        }
      }
      if constexpr (SPEC == 1) {
        w.reg[b] = c_reg[0];  // every lane stores the same value and reads its own store back
      } else {
        double rw = c_reg[0];
        NOC_UNROLL for (int k = 1; k < SPEC; ++k) rw = (wv == k) ? c_reg[k] : rw;
        io->reg = rw;
      }
      NOC_PHASE(2);
      wave_fence();  // the terminal Hessian (stage-0 lane) and the blocks before the scan
      // SPEC > 1: every wave has written the blocks (the same doubles) and read w.lc before any
      // wave's trial overwrites w.lc (a retry reads neither: no barrier)
      if constexpr (SPEC > 1) {
        if (relinearized) __syncthreads();
      }
      {  // park the state (every lane stores the same values)
        IpmState* st = state_slot<NX, NU>(N, SPEC, wv);
        st->bp = bp; st->rp = rp; st->rinc = rinc; st->cost = cost; st->hu = hu; st->gnorm = gnorm;
        st->it = it; st->inner = inner; st->total_it = total_it; st->solves = solves;
      }
      // ---------------- KKT solve (par_Newton, P:107-124) ----------------
      // HANDOFF on (phase 3 hands the chunk's first A, B to phase 4 in registers): the two-wave
      // cart-pole instance's scratch 524 -> 560 B/lane, but the solve is bound by its workspace
      // traffic -- c3 ipm_solve -2.4 %, c2 -1 %, bit-identical (profiles/r05/handoff_persist/)
      {
        const CompactSrc<BS, NX, NU, PL> src{a, prm, b, l, cmax, (size_t)b * N};
        kkt_scan_wave_src<NX, NU, PL, false, true, CompactSrc<BS, NX, NU, PL>, 0, true, false, false, false,
                          (SPEC > 1)>(a, b, l, src);
      }
      wave_fence();  // pred / feasible written by lane 0
      {
        const IpmState* st = state_slot<NX, NU>(N, SPEC, wv);
        bp = st->bp; rp = st->rp; rinc = st->rinc; cost = st->cost; hu = st->hu; gnorm = st->gnorm;
        it = st->it; inner = st->inner; total_it = st->total_it; solves = st->solves;
      }
      NOC_PHASE(3);
      // ---------------- trial point (P:156-175 / S:121-161) ----------------
      // (SPEC > 1: wave 0's trial costs go to w.lc -- the next linearisation's if its candidate is
      // taken; the other waves' are recomputed there, the same doubles)
      NOC_T0(t_tr);
      double tsum = 0.0;
      int ok = 1;
      const bool lc_out = SPEC == 1 || wv == 0;
      auto trial_load = [&](int k, double* xt, double* ut) {
        NOC_UNROLL for (int i = 0; i < NX; ++i) xt[i] = X[(size_t)k * NX + i] + slot[k * KD + i];
        NOC_UNROLL for (int jj = 0; jj < NU; ++jj) ut[jj] = U[(size_t)k * NU + jj] + slot[k * KD + NX + jj];
      };
      if (pair) {  // both stages loaded, then both costs; summed in stage order like trial_kernel
        for (int j = 0; j < cmax; j += 2) {
          double xt0[NX], ut0[NU], xt1[NX], ut1[NU];
          trial_load(clampk(start + j), xt0, ut0);
          trial_load(clampk(start + j + 1), xt1, ut1);
          const double c0 = f.stage_cost(xt0, ut0, bp);
          const double c1 = f.stage_cost(xt1, ut1, bp);
          const bool f0 = f.feasible(xt0, ut0), f1 = f.feasible(xt1, ut1);
          if (j < len) { ok &= f0 ? 1 : 0; tsum += c0; if (lc_out) tstore<1, PL>(w.lc, b, j, l, cmax, &c0); }
          if (j + 1 < len) { ok &= f1 ? 1 : 0; tsum += c1; if (lc_out) tstore<1, PL>(w.lc, b, j + 1, l, cmax, &c1); }
        }
      } else {
        for (int j = 0; j < len; ++j) {
          double xt[NX], ut[NU];
          trial_load(start + j, xt, ut);
          ok &= f.feasible(xt, ut) ? 1 : 0;
          const double c = f.stage_cost(xt, ut, bp);
          tsum += c;
          if (lc_out) tstore<1, PL>(w.lc, b, j, l, cmax, &c);  // the next linearisation's, if taken
        }
      }
      if (last) {
        double xt[NX];
        NOC_UNROLL for (int i = 0; i < NX; ++i) xt[i] = X[(size_t)N * NX + i] + slot[N * KD + i];
        tsum += f.final_cost(xt);
      }
      tsum = wave_sum(tsum);
      const bool traj_ok = __all(ok);
      NOC_SUB(6, t_tr);
      // the candidates' outcomes: new cost (P:159-163, S:126-129), pred, backward feasibility
      double c_new[SPEC], c_pred[SPEC];
      bool c_bwd[SPEC];
      if constexpr (SPEC == 1) {
        c_new[0] = traj_ok ? tsum : INFINITY;
        c_pred[0] = w.pred[b];
        c_bwd[0] = w.feasible[b] != 0;
      } else {
        if (l == 0) io->new_cost = traj_ok ? tsum : INFINITY;
        __syncthreads();  // every candidate's outcome in LDS
        const SpecIO* io0 = spec_io<NX, NU>(N, SPEC, 0);
        NOC_UNROLL for (int k = 0; k < SPEC; ++k) {
          c_new[k] = io0[k].new_cost;
          c_pred[k] = io0[k].pred;
          c_bwd[k] = io0[k].feasible != 0;
        }
      }
      // The accept tests in solve order.  Candidate k > 0 counts only if the solver reaches it:
      // every earlier one rejected without ending the iteration, no stop, no cap, and its
      // regularisation the one the sequential solver would use next (bit for bit) -- so the
      // decisions, counters and iterates are the sequential solver's.
      int winner = -1;
      bool stop = false;
      NOC_UNROLL for (int k = 0; k < SPEC; ++k) {
        if (k > 0) {
          const double reg_next = (mode == NOC_MODE_PAR) ? rp * gnorm : rp;
          if (stage_done || relinearize || reg_next != c_reg[k]) break;
        }
        const double new_cost = c_new[k];
        const double pred = c_pred[k];
        const bool bwd_ok = c_bwd[k];
        const double gain = (new_cost - cost) / pred;             // P:164-165
        const bool success = (gain > 0.0) && bwd_ok;              // P:166 / S:137
#ifdef NOC_DECISION_TRACE
        if (lead) NOC_TRACE_DECISION(g_dtrace, b, solves, bp, it, inner, cost, new_cost, pred, gain,
                                     success, rp, rinc, hu, bwd_ok);
#endif
        const double shrink = rp_shrink(gain);  // P:169 / S:141 (noc_internal.h)
        const double rp_used = rp;
        rp = success ? rp * shrink : rp * rinc;                   // P:167-171 / S:139-143
        rinc = success ? 2.0 : 2.0 * rinc;                        // P:172 / S:144
        bool take, end_iter;
        inner += 1;
        if (mode == NOC_MODE_PAR) {
          rp = fmin(fmax(rp, 1e-16), 1e16);                       // P:173
          // identical retries at the rp clip: accounted, not recomputed (noc_internal.h)
          const int rep = par_retry_repeats(w, success, rp_used, rp, inner, max_solves - solves - 1);
          if (rep > 0) {
            inner += rep;
            solves += rep;
            rinc = ldexp(rinc, rep);  // r_inc doubles per retry (P:172)
            if (lead && w.repeats) w.repeats[b] += rep;
          }
          end_iter = success || inner > 500;                      // P:177-182
          take = end_iter;                                        // last trial kept (P:175, P:184)
          stop = end_iter && (hu < 1e-4 || it + 1 > 1000);        // P:199-202
        } else {
          take = success;                                         // S:145-146
          end_iter = true;
          stop = (hu < 1e-4) && bwd_ok;                           // S:157-161
        }
        if (take) winner = k;
#ifdef NOC_PERSIST_PROFILE
        if (b == 0 && lead) g_phase_cycles[5] += 1;
#endif
        solves += 1;
        it += end_iter ? 1 : 0;
        if (stop) {                                               // barrier stage finished
          total_it += it;                                         // P:239 / S:187
          bp = bp / 5.0;                                          // P:238 / S:186
          it = 0;
          rp = 1.0;                                               // P:134 / S:110
          rinc = 2.0;                                             // P:135 / S:111
          stage_done = true;
        } else if (mode == NOC_MODE_PAR) {
          relinearize = end_iter;
        } else {
          relinearize = success;  // a rejected seq step only changes the regularisation
        }
        if (solves >= max_solves) {  // capped: record where a later launch continues
          capped = true;
          phase = stage_done ? NOC_PHASE_ROLLOUT : (relinearize ? NOC_PHASE_LINEARIZE : NOC_PHASE_SOLVE);
          if (stage_done && (!(bp > 1e-4) || (w.flags & NOC_WS_ONE_STAGE))) phase = NOC_PHASE_DONE;
          break;
        }
      }
      if (winner >= 0) {  // x <- x + dx, u <- u + du on the own chunk (its later readers are this lane)
        const double* ws = slot + (winner - wv) * slot_doubles<NX, NU>(N);  // the winner's slots
        for (int j = 0; j < len; ++j) {
          const int k = start + j;
          NOC_UNROLL for (int i = 0; i < NX; ++i) X[(size_t)k * NX + i] += ws[k * KD + i];
          NOC_UNROLL for (int jj = 0; jj < NU; ++jj) U[(size_t)k * NU + jj] += ws[k * KD + NX + jj];
        }
        if (last) NOC_UNROLL for (int i = 0; i < NX; ++i) X[(size_t)N * NX + i] += ws[N * KD + i];
      }
      lc_fresh = winner == 0;  // uniform; candidate 0's trial stored this point's stage costs in w.lc
      __syncthreads();  // the next KKT solve overwrites the LDS slots read above
      NOC_PHASE(4);
      if (capped) break;
    }
    if (capped || !(bp > 1e-4)) break;                          // P:243-245
    if (w.flags & NOC_WS_ONE_STAGE) break;                      // newton_oc: one stage
  }
  if constexpr (XLDS) {  // states and controls back to the workspace (every copy is the same)
    wave_fence();
    if (wv == 0) {
      for (int i = l; i < (N + 1) * NX; i += 64) Xg[i] = X[i];
      for (int i = l; i < N * NU; i += 64) Ug[i] = U[i];
    }
  }
  if (lead) {
    w.bp[b] = bp;
    w.rp[b] = rp;
    w.rinc[b] = rinc;
    w.cost[b] = cost;
    w.hu[b] = hu;
    w.gnorm[b] = gnorm;
    w.it[b] = it;
    w.inner[b] = inner;
    w.total_it[b] = total_it;
    w.kkt_solves[b] = solves;
    w.kkt_active[b] = 0;
    w.phase[b] = phase;
#ifdef NOC_PERSIST_PROFILE
    if (b < kTrajStamps) g_traj_times[b][1] = (long long)__builtin_amdgcn_s_memrealtime();
#endif
  }
}

// LDS of one persistent workgroup: the trajectory's KKT slots + the parked state.  Up to 64 KB
// (long horizons at small batch, e.g. the reference's N = 1000 timing runs: 2 workgroups per CU).
static size_t solve_lds_bytes(int nx, int nu, int N) {
  const size_t slots = (size_t)(((long long)N * nu * (nx + 1) + nx + 1) & ~1LL) * sizeof(double);
  const size_t bytes = slots + sizeof(IpmState) + 16;
  return bytes <= 65536 ? bytes : 0;
}

// SIMDs of the current device (4 per CU); 0 if the query fails
static int device_simds() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  return 4 * cus;
}

// Families whose kernel spills at 2 waves per SIMD (cart-pole) get a second instance at 1 wave per
// SIMD (512 registers per lane: no scratch, stage pairs), used when the batch fits one wave per
// SIMD anyway (B <= 4 x CUs: the reference's B = 1 runs, c2-sized batches); larger batches keep 2
// waves per SIMD for latency hiding.  The others stay at 2 waves (their 1-wave instance measured
// 5-7 % slower at B = 1).  NOC_PERSIST_WAVES=1|2 overrides the choice (timing experiments).
template <int KIND>
constexpr bool one_wave_instance() { return KIND == NOC_FAMILY_CARTPOLE; }

// grid: workgroups = the entries of w.order this launch solves (w.Bt without an order)
template <int KIND, int NX, int NU, int WPS, bool RESUME, bool XLDS>
static hipError_t launch_solve(const noc_family& p, const noc_ipm_ws& w, int mode, int terminal,
                               double bp0, int max_solves, size_t lds, hipStream_t s, int grid) {
  // the structure-aware blocks unless NOC_PERSIST_STRUCT=0 (per launch: tests switch it)
  const char* senv = getenv("NOC_PERSIST_STRUCT");
  if (senv && atoi(senv) == 0)
    hipLaunchKernelGGL((ipm_solve_kernel<KIND, NX, NU, WPS, RESUME, XLDS, false>), dim3(grid), dim3(64),
                       lds, s, p, w, mode, terminal, bp0, max_solves);
  else
    hipLaunchKernelGGL((ipm_solve_kernel<KIND, NX, NU, WPS, RESUME, XLDS, true>), dim3(grid), dim3(64),
                       lds, s, p, w, mode, terminal, bp0, max_solves);
  return hipGetLastError();
}

// Speculative retries (SPEC waves per trajectory, the one-wave-per-SIMD register budget): when
// the batch leaves SIMDs idle, a trajectory's workgroup runs SPEC waves on SPEC SIMDs, wave k
// solving the KKT system and the trial of the k-th candidate of the regularisation's failure chain
// (rp, rp r_inc, rp r_inc 2 r_inc, ...; P:167-173) at the same point; the accept tests are then
// replayed in solve order (ipm_solve_kernel), so counters and iterates are the one-wave solver's
// bit for bit.  A rejected trial no longer costs a KKT solve on the trajectory's serial chain:
// the heaviest of 512 cart-poles, 492 computed solves, takes 345 rounds at two candidates, 266 at
// four (tools/spec_estimate.py).  Needs x, u in LDS per wave.
// NOC_PERSIST_SPEC=1|2|4 overrides the choice.
static size_t spec_lds_rt(int nx, int nu, int N, int spec) {  // = xlds_off(N, spec, 0) + spec x, u
  const long long slots = ((long long)N * nu * (nx + 1) + nx + 1) & ~1LL;
  const long long xu = ((long long)(N + 1) * nx + (long long)N * nu + 1) & ~1LL;
  return (size_t)(spec * (slots + state_doubles() + xu) + specio_doubles(spec)) * sizeof(double);
}
template <int KIND, int NX, int NU>
static size_t spec_lds_bytes(int N, int spec) {
  return (size_t)(xlds_off<NX, NU>(N, spec, 0) + spec * xlds_doubles<NX, NU>(N)) * sizeof(double);
}
// Candidates per trajectory for this launch: 4 when four waves per trajectory still leave a SIMD
// each (B <= #SIMDs / 4), else 2 (B <= #SIMDs / 2), else 1; 1 for an ordered launch (its grid is
// the whole batch, most of it done), and when x, u of every wave do not fit 40 KB of LDS per wave.
// A resume may run them (the tail of a large batch, gathered: BatchedIPM.solve_persistent).  The
// families with a one-wave instance only (cart-pole).  NOC_PERSIST_SPEC=1|2|4 forces it.
static int spec_auto(const noc_family& p, const noc_ipm_ws& w, int simds, bool launch_state) {
  if (p.kind != NOC_FAMILY_CARTPOLE) return 1;
  if (launch_state && w.order) return 1;
  const char* senv = getenv("NOC_PERSIST_STRUCT");
  if (senv && atoi(senv) == 0) return 1;
  const char* env = getenv("NOC_PERSIST_SPEC");  // per launch (A/B sweeps in one process)
  int want;
  if (env) {
    want = atoi(env);
  } else if (simds <= 0) {
    want = 1;
  } else {
    want = (long long)w.Bt * 4 <= simds ? 4 : ((long long)w.Bt * 2 <= simds ? 2 : 1);
  }
  if (want != 2 && want != 4) return 1;
  return spec_lds_rt(p.nx, p.nu, w.N, want) <= (size_t)want * 40960u ? want : 1;
}
// grid: workgroups = the entries of w.order this launch solves (w.Bt without an order)
template <int KIND, int NX, int NU, int SPEC>
static hipError_t launch_spec(const noc_family& p, const noc_ipm_ws& w, int mode, int terminal,
                              double bp0, int max_solves, hipStream_t s, int grid = -1) {
  if (grid < 0) grid = w.Bt;
  const size_t lds = spec_lds_bytes<KIND, NX, NU>(w.N, SPEC);
  if (w.flags & NOC_WS_RESUME)
    hipLaunchKernelGGL((ipm_solve_kernel<KIND, NX, NU, 1, true, true, true, SPEC>), dim3(grid), dim3(64 * SPEC),
                       lds, s, p, w, mode, terminal, bp0, max_solves);
  else
    hipLaunchKernelGGL((ipm_solve_kernel<KIND, NX, NU, 1, false, true, true, SPEC>), dim3(grid), dim3(64 * SPEC),
                       lds, s, p, w, mode, terminal, bp0, max_solves);
  return hipGetLastError();
}

template <int KIND, int NX, int NU, int WPS>
static hipError_t solve_w(const noc_family& p, const noc_ipm_ws& w, int mode, int terminal,
                          double bp0, int max_solves, size_t lds, hipStream_t s, int grid = -1) {
  if (grid < 0) grid = w.Bt;
  // x, u in LDS (XLDS) when that keeps the residency the register budget allows: 8 waves per CU
  // at 2 waves per SIMD (<= 20 KB per wave), 4 at one wave per SIMD (<= 40 KB); longer horizons
  // keep them in the workspace.  NOC_PERSIST_XLDS=0 forces the workspace (A/B).
  const char* xenv = getenv("NOC_PERSIST_XLDS");  // per launch (tests switch it)
  const size_t xl = lds + (size_t)(((w.N + 1) * NX + w.N * NU + 1) & ~1) * sizeof(double);
  const bool xlds = !(xenv && atoi(xenv) == 0) && xl <= (WPS == 1 ? 40960u : 20480u);
  const bool res = (w.flags & NOC_WS_RESUME) != 0;
  if (xlds)
    return res ? launch_solve<KIND, NX, NU, WPS, true, true>(p, w, mode, terminal, bp0, max_solves, xl, s, grid)
               : launch_solve<KIND, NX, NU, WPS, false, true>(p, w, mode, terminal, bp0, max_solves, xl, s, grid);
  return res ? launch_solve<KIND, NX, NU, WPS, true, false>(p, w, mode, terminal, bp0, max_solves, lds, s, grid)
             : launch_solve<KIND, NX, NU, WPS, false, false>(p, w, mode, terminal, bp0, max_solves, lds, s, grid);
}

// Heavy-first split of an ordered launch larger than one wave per SIMD (cart-pole): the first
// `heavy` entries of w.order -- the costliest trajectories (the probe-ordered resume,
// BatchedIPM.solve_persistent) -- run on the one-wave instance, a SIMD of their own, concurrently
// with the rest on the two-wave instance (second stream, event fork / join).  Every trajectory's
// result is the same on either instance (tested).  NOC_PERSIST_HEAVY=<n> sets the count.
// By default (cart-pole, N <= 320, #SIMDs < B <= 2 #SIMDs: the c3 slice of 2 GPUs) the costliest
// #SIMDs / 8 trajectories of the probe order run two speculative candidates each beside the rest
// on the two-wave instance: 2048 cart-poles 17.9 -> 16.3-16.8 ms (probe order alone;
// profiles/r06/t/).  At one wave per SIMD (1024) the split made the light end of the order wait
// for SIMDs: 11.4-11.6 ms on one batch but 16.2-18.5 ms on the c3 slices (profiles/r06/final_c4/),
// so not there; at c3 (4096) it measured slower (profiles/r06/q/).  NOC_PERSIST_HEAVY=<n> sets
// the count, NOC_PERSIST_HEAVY_SPEC=0|2 the candidates (0 turns the default split off).
static int heavy_count(const noc_ipm_ws& w, int simds, bool* spec2) {
  const char* env = getenv("NOC_PERSIST_HEAVY");  // per launch (A/B sweeps in one process)
  const char* hs = getenv("NOC_PERSIST_HEAVY_SPEC");
  *spec2 = false;
  if (!w.order || simds <= 0) return 0;
  int h;
  bool sp;
  if (env) {
    h = atoi(env);
    sp = hs && atoi(hs) == 2;
    if (w.Bt <= (sp ? simds / 2 : simds)) return 0;
  } else {
    if ((hs && atoi(hs) == 0) || w.N > 320 || w.Bt <= simds || w.Bt > 2 * simds) return 0;
    h = simds / 8;
    sp = true;
  }
  if (h < 0) h = 0;
  if (h > simds / 2) h = simds / 2;
  *spec2 = sp;
  return h < w.Bt ? h : 0;
}

template <int KIND, int NX, int NU, int REST_WPS = 2>
static hipError_t solve_split(const noc_family& p, const noc_ipm_ws& w, int mode, int terminal,
                              double bp0, int max_solves, size_t lds, hipStream_t s, int heavy,
                              bool spec2) {
  thread_local hipStream_t s2 = nullptr;
  thread_local hipEvent_t fork = nullptr, join = nullptr;
  if (!s2) {
    if (hipStreamCreateWithFlags(&s2, hipStreamNonBlocking) != hipSuccess) return hipErrorUnknown;
    if (hipEventCreateWithFlags(&fork, hipEventDisableTiming) != hipSuccess) return hipErrorUnknown;
    if (hipEventCreateWithFlags(&join, hipEventDisableTiming) != hipSuccess) return hipErrorUnknown;
  }
  hipError_t e;
  if ((e = hipEventRecord(fork, s)) != hipSuccess) return e;
  if ((e = hipStreamWaitEvent(s2, fork, 0)) != hipSuccess) return e;
  // the heavy launch first, so its workgroups are placed before the two-wave ones fill the SIMDs;
  // spec2: the heavy trajectories with two speculative candidates each
  if (spec2 && spec_lds_bytes<KIND, NX, NU>(w.N, 2) <= 2 * 40960u)
    e = launch_spec<KIND, NX, NU, 2>(p, w, mode, terminal, bp0, max_solves, s, heavy);
  else
    e = solve_w<KIND, NX, NU, 1>(p, w, mode, terminal, bp0, max_solves, lds, s, heavy);
  if (e != hipSuccess) return e;
  noc_ipm_ws rest = w;
  rest.order = w.order + heavy;
  if ((e = solve_w<KIND, NX, NU, REST_WPS>(p, rest, mode, terminal, bp0, max_solves, lds, s2, w.Bt - heavy)) !=
      hipSuccess)
    return e;
  if ((e = hipEventRecord(join, s2)) != hipSuccess) return e;
  return hipStreamWaitEvent(s, join, 0);
}

template <int KIND, int NX, int NU>
static hipError_t solve_t(const noc_family& p, const noc_ipm_ws& w, int mode, int terminal,
                          double bp0, int max_solves, hipStream_t s) {
  const size_t lds = solve_lds_bytes(NX, NU, w.N);
  if (lds == 0) return hipErrorInvalidValue;  // step does not fit in LDS: use the launch driver
  if constexpr (one_wave_instance<KIND>()) {
    static const int simds = device_simds();
    static const char* env = getenv("NOC_PERSIST_WAVES");
    const bool one = env ? atoi(env) == 1 : (simds > 0 && w.Bt <= simds);
    if (one) {
      bool sp1 = false;
      const int heavy1 = env ? 0 : heavy_count(w, simds, &sp1);
      if (heavy1 > 0)
        return solve_split<KIND, NX, NU, 1>(p, w, mode, terminal, bp0, max_solves, lds, s, heavy1, sp1);
      const int spec = spec_auto(p, w, simds, true);
      if (spec == 2) return launch_spec<KIND, NX, NU, 2>(p, w, mode, terminal, bp0, max_solves, s);
      if (spec == 4) return launch_spec<KIND, NX, NU, 4>(p, w, mode, terminal, bp0, max_solves, s);
      return solve_w<KIND, NX, NU, 1>(p, w, mode, terminal, bp0, max_solves, lds, s);
    }
    bool sp = false;
    const int heavy = env ? 0 : heavy_count(w, simds, &sp);
    if (heavy > 0) return solve_split<KIND, NX, NU>(p, w, mode, terminal, bp0, max_solves, lds, s, heavy, sp);
  }
  return solve_w<KIND, NX, NU, 2>(p, w, mode, terminal, bp0, max_solves, lds, s);
}

int debug_phase_cycles(long long* out, int n, int reset) {
  long long host[8], sub[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_phase_cycles), sizeof(host)) != hipSuccess) return -1;
#ifdef NOC_PERSIST_PROFILE  // the one-wave kernel's KKT sub-phases (kkt_scan_impl.h: NOC_STAMP)
  if (hipMemcpyFromSymbol(sub, HIP_SYMBOL(g_scan_sub), sizeof(sub)) != hipSuccess) return -1;
#endif
  long long wide[16];
  if (debug_wide_cycles(wide, 16, reset) != 0) return -1;  // the wide kernel's (ipm_wide.hip)
  for (int i = 0; i < n && i < 16; ++i) out[i] = (i < 8 ? host[i] : sub[i - 8]) + wide[i];
  if (reset) {
    const long long zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase_cycles), zero, sizeof(zero)) != hipSuccess) return -1;
#ifdef NOC_PERSIST_PROFILE
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_scan_sub), zero, sizeof(zero)) != hipSuccess) return -1;
#endif
  }
  return 0;
}

// decision-trace buffer of both persistent kernels; 1 if this build records (NOC_DECISION_TRACE),
// 0 if it has no trace code, -1 on a HIP error
int debug_set_decision_trace(double* buf, int cap, int ntraj) {
  const DecisionTrace t{buf, cap, ntraj};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_dtrace), &t, sizeof(t)) != hipSuccess) return -1;
  if (wide_set_decision_trace(t) != 0) return -1;
#ifdef NOC_DECISION_TRACE
  return 1;
#else
  return 0;
#endif
}

int debug_traj_times(long long* out, int n) {
  if (n > kTrajStamps) n = kTrajStamps;
  if (n <= 0) return 0;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_traj_times), (size_t)n * 2 * sizeof(long long)) ==
                 hipSuccess ? 0 : -1;
}

// persistent instances exist for the families with nx <= 4 (an nx = 8 scan element does not fit a
// wave's registers next to the solver state: those run the launch-per-phase driver)
template <int NX>
constexpr bool persistent_instance() { return NX <= 4; }

bool ipm_solve_supported(const noc_family& p, int N, int lanes) {
  if (lanes != PL || !family_supported(p)) return false;
  bool inst = false;
#define NOC_FAMILY(K, X, U) \
  if (p.kind == K && p.nx == X && p.nu == U) inst = persistent_instance<X>();
#include NOC_FAMILIES_DEF
#undef NOC_FAMILY
  return inst && solve_lds_bytes(p.nx, p.nu, N) > 0;
}

template <int K, int X, int U>
static hipError_t solve_family(const noc_family& p, const noc_ipm_ws& w, int mode, int terminal,
                               double bp0, int max_solves, hipStream_t s) {
  if constexpr (persistent_instance<X>()) return solve_t<K, X, U>(p, w, mode, terminal, bp0, max_solves, s);
  else return hipErrorInvalidValue;
}

// The wide kernel (ipm_wide.hip: 4 waves and the LDS of one CU per trajectory) when the batch
// leaves CUs idle anyway (B <= #CUs: the reference's B = 1 runs) and the horizon gives the
// one-wave kernel more than two stages per lane: at N <= 128 the one-wave solve is faster (its
// KKT scan needs no cross-wave join), beyond it the wide one (B = 1, per KKT solve: pendulum
// N=200 16.5 vs 20.4 us, N=800 32 vs 57 us; cart-pole N=128 31.6 vs 25.7 us, N=200 33.0 vs
// 35.2 us -- profiles/r02/wide/crossover.jsonl).  NOC_PERSIST_WIDE=0|1 overrides.
// (Re-packing the last <= #CUs trajectories of a large batch onto it was measured and dropped:
// those are Newton retries, KKT-bound, and the wide KKT solve is no faster -- DESIGN.md §3.7.)
// Where the speculative candidates apply (cart-pole, B <= #SIMDs / 2) and the horizon gives the
// one-wave kernel at most five stages per lane (N <= 320), they beat the wide kernel: cart-pole
// B = 1 N = 200 / 300 5.19 / 5.92 ms against 5.88 / 6.32 ms, N = 200 B = 64 / 256 7.54 / 8.30 ms
// against 9.53 / 10.28 ms; at N = 400 the wide kernel is ahead (6.57 vs 7.02 ms;
// profiles/r06/n/).  The choice ignores resume and order, so a capped solve resumes on the kernel
// family (one-wave) it started on.
static bool use_wide(const noc_family& p, const noc_ipm_ws& w) {
  const char* env = getenv("NOC_PERSIST_WIDE");
  if (env && atoi(env) == 0) return false;
  if (!ipm_wide_supported(p, w.N)) return false;
  if (env && atoi(env) == 1) return true;
  static const int simds = device_simds();
  const int cus = simds / 4;
  if (w.N <= 320 && spec_auto(p, w, simds, false) > 1) return false;
  return cus > 0 && w.Bt <= cus && w.N > 128;
}

hipError_t ipm_solve(const noc_family& p, const noc_ipm_ws& w, int mode, int terminal, double bp0,
                     int max_solves, hipStream_t s) {
  if (use_wide(p, w)) {
    static const int cus = device_simds() / 4;
    return ipm_solve_wide(p, w, mode, terminal, bp0, max_solves, nullptr, nullptr, w.Bt,
                          wide_waves(p, w, cus), s);
  }
#define NOC_FAMILY(K, X, U)                                                              \
  if (p.kind == K && p.nx == X && p.nu == U)                                             \
    return solve_family<K, X, U>(p, w, mode, terminal, bp0, max_solves, s);
#include NOC_FAMILIES_DEF
#undef NOC_FAMILY
  return hipErrorInvalidValue;
}

}  // namespace noc
