// Wide persistent interior-point solver: the whole barrier schedule of ONE trajectory per
// W-wave workgroup (W = 4: 256 lanes), the trajectory's LQ blocks, states, controls and step held
// in LDS for the whole solve (fp64, gfx950).
//
// Same reference control flow as ipm_persistent.hip (par_interior_point_optimal_control /
// newton_oc, noc/par_interior_point_newton.py:127-254; seq S:108-202), for the regime where the
// batch does not fill the chip -- the reference's own B = 1 timing runs and the stragglers of a
// large batch -- where a trajectory's latency is the wall time:
//   * the stage-parallel work (linearise P:13-28, the costate sweep C:34-54 fused with the LQ
//     blocks P:31-42, the trial point P:156-175) is spread over 64 W lanes: one stage per lane up
//     to N = 64 W instead of N / 64;
//   * the KKT scan (par_Newton, P:107-124) keeps the in-wave reverse Sklansky scan of the 64-lane
//     scan (kkt_scan_impl.h: chunk element by Riccati-form prepend, combine_sklansky) and joins the
//     W waves through LDS with value-only applications of the later waves' aggregates, so the
//     dependent chain stays at six combine levels while each lane's chunk shrinks to one stage;
//     the forward affine scan is joined the same way;
//   * nothing goes through HBM between the phases (linearise -> costates -> LQ
//     blocks -> KKT solve -> trial in one launch, blocks resident in LDS).
// Layouts in LDS are field-major ([element][stage]) so that lanes holding consecutive stages
// touch consecutive words.  One workgroup per CU (the LDS image is up to ~150 KB).
#include <hip/hip_runtime.h>
#include <cstdlib>

#include "../../include/noc_hip.h"
#include "block_struct.h"
#include "ipm_family.h"
#include "kkt_scan_impl.h"
#include "noc_internal.h"

namespace noc {

// Per-phase cycle counters of workgroup 0 (timing-only, -DNOC_PERSIST_PROFILE builds; summed into
// noc_debug_phase_cycles with the one-wave kernel's): rollout, linearise, costate + blocks, KKT
// scan, trial, number of Newton iterations.
__device__ long long g_wide_cycles[16];
// decision trace (-DNOC_DECISION_TRACE builds only; noc_internal.h)
__device__ DecisionTrace g_wide_dtrace;
#ifdef NOC_PERSIST_PROFILE
#define NOC_WPHASE(i) do { const long long t_ = clock64(); if (b == 0 && t == 0) g_wide_cycles[i] += t_ - t_prev; t_prev = t_; } while (0)
// sub-phases of the KKT solve (slots 8..15), timed by wave 0 lane 0 without moving t_prev
#define NOC_WSUB(i) do { const long long t_ = clock64(); if (b == 0 && t == 0) g_wide_cycles[8 + (i)] += t_ - t_sub; t_sub = t_; } while (0)
#else
#define NOC_WPHASE(i) do { } while (0)
#define NOC_WSUB(i) do { } while (0)
#endif

namespace {

constexpr int kWideWaves = 4;

// LDS image of one trajectory (offsets in doubles).  A, B, Q, R, M hold only the variable entries
// of the blocks (BS = BlockStruct: block_struct.h; the constants are rebuilt where they are read),
// which cuts cart-pole N = 200 from 84.5 to 47 KB -- two workgroups per CU for the two-wave
// instance.
template <int NX, int NU, class BS>
struct WideLds {
  static constexpr int KD = NU * (NX + 1);
  int x, u, A, B, Q, R, M, r, cx, cu, lc, kd, agg, red, P, total;
  __host__ __device__ WideLds(int N, int W) {
    int o = 0;
    x = o; o += (N + 1) * NX;
    u = o; o += N * NU;
    A = o; o += BS::template nv<BF_A>() * N;
    B = o; o += BS::template nv<BF_B>() * N;
    Q = o; o += BS::template nv<BF_Q>() * N;
    R = o; o += BS::template nv<BF_R>() * N;
    M = o; o += BS::template nv<BF_M>() * N;
    r = o; o += NU * N;
    cx = o; o += NX * N;
    cu = o; o += NU * N;
    lc = o; o += N;
    kd = o; o += KD * (N + 1);  // K, d per stage; then dx [i][0..N], du [NX + j][0..N-1]
    agg = o; o += W * 64;       // per-wave aggregates (scan elements / affine maps)
    red = o; o += W * 8;        // per-wave partial reductions
    P = o; o += NX * NX;        // terminal Hessian
    total = o;
  }
};

template <int E>
NOC_DEV void fget(const double* base, int N, int s, double* v) {
  NOC_UNROLL for (int e = 0; e < E; ++e) v[e] = base[(size_t)e * N + s];
}
template <int E>
NOC_DEV void fput(double* base, int N, int s, const double* v) {
  NOC_UNROLL for (int e = 0; e < E; ++e) base[(size_t)e * N + s] = v[e];
}
// a block field through its compact record: the variable entries stored, the constants rebuilt
template <class BS, int F>
NOC_DEV void bput(double* base, int N, int s, const double* full) {
  constexpr int EV = BS::template nv<F>();
  double v[EV > 0 ? EV : 1];
  BS::template compress<F>(full, v);
  fput<EV>(base, N, s, v);
}
template <class BS, int F>
NOC_DEV void bget(const noc_family& p, const double* base, int N, int s, double* full) {
  constexpr int EV = BS::template nv<F>();
  double v[EV > 0 ? EV : 1];
  fget<EV>(base, N, s, v);
  BS::template expand<F>(p, v, full);
}

template <int NX>
NOC_DEV void elem_put(double* p, const Elem<NX>& e) {
  int o = 0;
  NOC_UNROLL for (int i = 0; i < NX * NX; ++i) p[o++] = e.A.v[i];
  NOC_UNROLL for (int i = 0; i < NX; ++i) p[o++] = e.b.v[i];
  NOC_UNROLL for (int i = 0; i < Sym<NX>::SZ; ++i) p[o++] = e.C.v[i];
  NOC_UNROLL for (int i = 0; i < NX; ++i) p[o++] = e.nu.v[i];
  NOC_UNROLL for (int i = 0; i < Sym<NX>::SZ; ++i) p[o++] = e.J.v[i];
}
template <int NX>
NOC_DEV void elem_get(const double* p, Elem<NX>& e) {
  int o = 0;
  NOC_UNROLL for (int i = 0; i < NX * NX; ++i) e.A.v[i] = p[o++];
  NOC_UNROLL for (int i = 0; i < NX; ++i) e.b.v[i] = p[o++];
  NOC_UNROLL for (int i = 0; i < Sym<NX>::SZ; ++i) e.C.v[i] = p[o++];
  NOC_UNROLL for (int i = 0; i < NX; ++i) e.nu.v[i] = p[o++];
  NOC_UNROLL for (int i = 0; i < Sym<NX>::SZ; ++i) e.J.v[i] = p[o++];
}

}  // namespace

// W waves per trajectory (blockDim = 64 W), one workgroup per trajectory at a time: workgroup g
// solves trajectories idx[g], idx[g + grid], ... of the *count listed (idx == NULL: 0..Bt-1).
template <int KIND, int NX, int NU, int W>
__global__ __launch_bounds__(64 * W, 1) void ipm_wide_kernel(noc_family prm, noc_ipm_ws w, int mode,
                                                             int terminal, double bp0,
                                                             int max_solves, const int* idx,
                                                             const int* count) {
  constexpr int T = 64 * W;
  constexpr int KD = NU * (NX + 1);
  using BS = BlockStruct<KIND, NX, NU, true>;
  constexpr int ESZ = NX * NX + 2 * NX + 2 * Sym<NX>::SZ;  // scan element in doubles
  static_assert(ESZ <= 64 && NX * NX + NX <= 64, "aggregate slot");
  extern __shared__ __attribute__((aligned(16))) double noc_smem[];
  // one wave per SIMD: the W waves of the workgroup on W different SIMDs.  With fewer registers
  // (pendulum: 189 VGPRs, two waves could share a SIMD) the dispatcher may stack the workgroup's
  // waves on fewer SIMDs than the CU has, and their VALU-bound scans then take turns; claiming the
  // whole register file rules that out (the workgroup holds the CU's LDS anyway)
  asm volatile("" ::: "a255");
  const int t = threadIdx.x, wv = t >> 6, l = t & 63;
  const int n_traj = count ? *count : w.Bt;
  for (int jb = blockIdx.x; jb < n_traj; jb += gridDim.x) {  // uniform over the workgroup
  const int b = idx ? idx[jb] : jb;
  Fam<KIND, NX, NU> f(prm);
  const int N = w.N;
  const WideLds<NX, NU, BS> L(N, W);
  double* sx = noc_smem + L.x;
  double* su = noc_smem + L.u;
  double* sA = noc_smem + L.A;
  double* sB = noc_smem + L.B;
  double* sQ = noc_smem + L.Q;
  double* sR = noc_smem + L.R;
  double* sM = noc_smem + L.M;
  double* sr = noc_smem + L.r;
  double* scx = noc_smem + L.cx;
  double* scu = noc_smem + L.cu;
  double* slc = noc_smem + L.lc;
  double* skd = noc_smem + L.kd;
  double* sagg = noc_smem + L.agg;
  double* sred = noc_smem + L.red;
  double* sP = noc_smem + L.P;
  const Chunks ch(N, T);
  const int start = ch.start(t), len = ch.len(t);
  const bool last = (t == T - 1);
  double* Xg = w.x + (size_t)b * (N + 1) * NX;
  double* Ug = w.u + (size_t)b * N * NU;
  // dx, du live in the K/d region once the forward pass has consumed the gains
  auto dxs = [&](int i, int s) -> double& { return skd[(size_t)i * (N + 1) + s]; };
  auto dus = [&](int j, int s) -> double& { return skd[(size_t)(NX + j) * (N + 1) + s]; };
  auto kds = [&](int i, int s) -> double& { return skd[(size_t)i * (N + 1) + s]; };

  // workgroup reductions of up to 4 doubles (sum / nan-propagating max), every thread gets the
  // result, combined in wave order (deterministic)
  auto wg_reduce = [&](double* v, int n, const bool* is_max) {
    NOC_UNROLL for (int k = 0; k < 4; ++k) {
      if (k < n) {
        // VALU butterfly (small_linalg.h), bit-identical to the __shfl_xor loop
        const double r = v[k];
        v[k] = is_max[k] ? segment_allreduce<64>(r, l, [](double x, double y) { return nan_max(x, y); })
                         : segment_allreduce<64>(r, l, [](double x, double y) { return x + y; });
      }
    }
    __syncthreads();
    if (l == 0) NOC_UNROLL for (int k = 0; k < 4; ++k) if (k < n) sred[wv * 8 + k] = v[k];
    __syncthreads();
    NOC_UNROLL for (int k = 0; k < 4; ++k) {
      if (k < n) {
        double a = sred[k];
        for (int q = 1; q < W; ++q) a = is_max[k] ? nan_max(a, sred[q * 8 + k]) : a + sred[q * 8 + k];
        v[k] = a;
      }
    }
  };

  // controls in
  for (int i = t; i < N * NU; i += T) su[(i % NU) * N + i / NU] = Ug[i];
  __syncthreads();

  double bp = bp0, rp = 1.0, rinc = 2.0, cost = 0.0, hu = 1.0, gnorm = 0.0;
  int it = 0, inner = 0, total_it = 0, solves = 0;
  int phase = NOC_PHASE_ROLLOUT;  // where this launch starts (NOC_WS_RESUME) / stopped
  if (w.flags & NOC_WS_RESUME) {
    bp = w.bp[b]; rp = w.rp[b]; rinc = w.rinc[b]; cost = w.cost[b]; hu = w.hu[b];
    gnorm = w.gnorm[b]; it = w.it[b]; inner = w.inner[b]; total_it = w.total_it[b];
    solves = w.kkt_solves[b]; phase = resume_phase(w.phase[b]);
  } else if (t == 0 && w.repeats) {
    w.repeats[b] = 0;
  }
  if (phase == NOC_PHASE_DONE) continue;  // uniform; no LDS written yet
  // resuming inside a barrier stage: the states are the workspace's (the blocks are recomputed
  // from them -- the same values -- but a SOLVE resume keeps its retry counter)
  bool keep_inner = phase == NOC_PHASE_SOLVE;
  if (phase != NOC_PHASE_ROLLOUT)
    for (int i = t; i < (N + 1) * NX; i += T) sx[i] = Xg[i];
  __syncthreads();
#ifdef NOC_PERSIST_PROFILE
  long long t_prev = clock64();
#endif

  for (;;) {  // ---------------- barrier stages (P:228-254) ----------------
    // rollout (U:57-63, P:133): wave 0 runs the recurrence, lane (k mod 64) keeps stage k
    if (phase == NOC_PHASE_ROLLOUT && wv == 0) {
      double x[NX];
      NOC_UNROLL for (int i = 0; i < NX; ++i) x[i] = w.x0[(size_t)b * NX + i];
      if (l < NX) sx[l] = x[l];
      for (int k = 0; k < N; ++k) {
        double uk[NU], xn[NX];
        NOC_UNROLL for (int j = 0; j < NU; ++j) uk[j] = su[(size_t)j * N + k];
        f.step(x, uk, xn);
        NOC_UNROLL for (int i = 0; i < NX; ++i) x[i] = xn[i];
        if (l == (k & 63)) NOC_UNROLL for (int i = 0; i < NX; ++i) sx[(size_t)(k + 1) * NX + i] = xn[i];
      }
    }
    __syncthreads();
    NOC_WPHASE(0);
    bool relinearize = true, stage_done = false;
    while (!stage_done) {  // ---------------- Newton iterations (P:127-225) ----------------
      if (relinearize) {
        // linearise the own stages (P:13-28)
        for (int s = start; s < start + len; ++s) {
          double x[NX], u[NU], fx[NX * NX], fu[NX * NU], cx[NX], cu[NU];
          NOC_UNROLL for (int i = 0; i < NX; ++i) x[i] = sx[(size_t)s * NX + i];
          NOC_UNROLL for (int j = 0; j < NU; ++j) u[j] = su[(size_t)j * N + s];
          f.jac(x, u, fx, fu);
          BS::template fold_consts<BF_A>(prm, fx);
          BS::template fold_consts<BF_B>(prm, fu);
          f.stage_grad(x, u, bp, cx, cu);
          bput<BS, BF_A>(sA, N, s, fx);
          bput<BS, BF_B>(sB, N, s, fu);
          fput<NX>(scx, N, s, cx);
          fput<NU>(scu, N, s, cu);
          slc[s] = f.stage_cost(x, u, bp);
        }
        NOC_WPHASE(1);
        // costates (C:34-54): chunk map lambda_start = G lambda_end + g, in-wave reverse scan,
        // the waves joined through LDS, then the sweep fused with the LQ blocks (P:31-42)
        const double* xN = sx + (size_t)N * NX;
        double lamN[NX];
        f.final_grad(xN, lamN);  // grad(final_cost) (C:35)
        Mat<NX, NX> G;
        Vec<NX> g;
        set_identity(G);
        set_zero(g);
        for (int s = start + len - 1; s >= start; --s) {
          double A[NX * NX], cx[NX];
          bget<BS, BF_A>(prm, sA, N, s, A);
          fget<NX>(scx, N, s, cx);
          Mat<NX, NX> Gn;
          Vec<NX> gn;
          NOC_UNROLL for (int i = 0; i < NX; ++i) {
            double a = cx[i];
            NOC_UNROLL for (int m = 0; m < NX; ++m) if (BS::nzA(m, i)) a += A[m * NX + i] * g[m];
            gn[i] = a;
            NOC_UNROLL for (int j = 0; j < NX; ++j) {
              double c = 0.0;
              NOC_UNROLL for (int m = 0; m < NX; ++m) if (BS::nzA(m, i)) c += A[m * NX + i] * G(m, j);
              Gn(i, j) = c;
            }
          }
          G = Gn;
          g = gn;
        }
        if (last) {
          NOC_UNROLL for (int i = 0; i < NX; ++i) {
            double a = g[i];
            NOC_UNROLL for (int m = 0; m < NX; ++m) a += G(i, m) * lamN[m];
            g[i] = a;
          }
          set_zero(G);
        }
#pragma unroll 1
        for (int d = 1; d < 64; d <<= 1) {
          Mat<NX, NX> G2;
          Vec<NX> g2;
          shfl_down_arr<NX * NX>(G.v, G2.v, d, 64);
          shfl_down_arr<NX>(g.v, g2.v, d, 64);
          if (l + d >= 64) {  // no partner in this wave: compose with the identity map
            set_identity(G2);
            set_zero(g2);
          }
          Mat<NX, NX> Gn;
          NOC_UNROLL for (int i = 0; i < NX; ++i) {
            double a = g[i];
            NOC_UNROLL for (int m = 0; m < NX; ++m) a += G(i, m) * g2[m];
            g[i] = a;
            NOC_UNROLL for (int j = 0; j < NX; ++j) {
              double c = 0.0;
              NOC_UNROLL for (int m = 0; m < NX; ++m) c += G(i, m) * G2(m, j);
              Gn(i, j) = c;
            }
          }
          G = Gn;
        }
        // wave aggregates (lane 0: the map over the whole wave) -> LDS
        if (l == 0) {
          NOC_UNROLL for (int i = 0; i < NX * NX; ++i) sagg[wv * 64 + i] = G.v[i];
          NOC_UNROLL for (int i = 0; i < NX; ++i) sagg[wv * 64 + NX * NX + i] = g[i];
        }
        __syncthreads();
        // costate at the end of this wave's span: the last wave's map is constant, earlier ones
        // compose the later waves' maps
        double lw[NX];
        NOC_UNROLL for (int i = 0; i < NX; ++i) lw[i] = (wv == W - 1) ? lamN[i] : sagg[(W - 1) * 64 + NX * NX + i];
        for (int q = W - 2; q > wv; --q) {
          double ln[NX];
          NOC_UNROLL for (int i = 0; i < NX; ++i) {
            double a = sagg[q * 64 + NX * NX + i];
            NOC_UNROLL for (int m = 0; m < NX; ++m) a += sagg[q * 64 + i * NX + m] * lw[m];
            ln[i] = a;
          }
          NOC_UNROLL for (int i = 0; i < NX; ++i) lw[i] = ln[i];
        }
        // this lane's chunk-end costate: lane l+1's in-wave map applied to lw (lane 63: lw)
        Mat<NX, NX> Gd;
        Vec<NX> gd;
        wave_shift_down1<NX * NX>(G.v, Gd.v);  // DPP; lane 63 uses lw below
        wave_shift_down1<NX>(g.v, gd.v);
        double lam[NX];
        NOC_UNROLL for (int i = 0; i < NX; ++i) {
          double a = gd[i];
          NOC_UNROLL for (int m = 0; m < NX; ++m) a += Gd(i, m) * lw[m];
          lam[i] = (l == 63) ? lw[i] : a;
        }
        double red[4] = {0.0, 0.0, 0.0, 0.0};  // cost, max|Hu|, ||cu||^2
        for (int s = start + len - 1; s >= start; --s) {
          double x[NX], u[NU], A[NX * NX], Bm[NX * NU], cx[NX], cu[NU];
          NOC_UNROLL for (int i = 0; i < NX; ++i) x[i] = sx[(size_t)s * NX + i];
          NOC_UNROLL for (int j = 0; j < NU; ++j) u[j] = su[(size_t)j * N + s];
          bget<BS, BF_A>(prm, sA, N, s, A);
          bget<BS, BF_B>(prm, sB, N, s, Bm);
          fget<NX>(scx, N, s, cx);
          fget<NU>(scu, N, s, cu);
          // Q = cxx + l.fxx, R = cuu + l.fuu, M = cxu + l.fxu at l = lambda_{s+1} (P:35-37)
          double Qf[NX * NX], Rf[NU * NU], M[NX * NU], rr[NU];
          f.stage_hess(x, u, bp, Qf, Rf, M);
          f.add_hess_l(x, u, lam, Qf, Rf, M);
          BS::template fold_consts<BF_M>(prm, M);
          Sym<NX> Qs;
          Sym<NU> Rs;
          NOC_UNROLL for (int i = 0; i < NX; ++i)
            NOC_UNROLL for (int j = i; j < NX; ++j) Qs(i, j) = (i == j) ? Qf[i * NX + i] : 0.5 * (Qf[i * NX + j] + Qf[j * NX + i]);
          NOC_UNROLL for (int i = 0; i < NU; ++i)
            NOC_UNROLL for (int j = i; j < NU; ++j) Rs(i, j) = (i == j) ? Rf[i * NU + i] : 0.5 * (Rf[i * NU + j] + Rf[j * NU + i]);
          BS::template fold_consts<BF_Q>(prm, Qs.v);
          BS::template fold_consts<BF_R>(prm, Rs.v);
          NOC_UNROLL for (int j = 0; j < NU; ++j) {  // ru = cu + fu' lambda_{s+1} (P:34)
            double a = cu[j];
            NOC_UNROLL for (int i = 0; i < NX; ++i) if (BS::nzB(i, j)) a += Bm[i * NU + j] * lam[i];
            rr[j] = a;
            red[1] = nan_max(red[1], fabs(a));
            red[2] += cu[j] * cu[j];
          }
          bput<BS, BF_Q>(sQ, N, s, Qs.v);
          bput<BS, BF_R>(sR, N, s, Rs.v);
          bput<BS, BF_M>(sM, N, s, M);
          fput<NU>(sr, N, s, rr);
          if (terminal == NOC_TERMINAL_STAGE0 && s == 0)  // XT = Q[0] (P:73)
            NOC_UNROLL for (int i = 0; i < NX; ++i) NOC_UNROLL for (int j = 0; j < NX; ++j) sP[i * NX + j] = Qs(i, j);
          double ln[NX];  // lambda_s = cx_s + fx_s' lambda_{s+1}
          NOC_UNROLL for (int i = 0; i < NX; ++i) {
            double a = cx[i];
            NOC_UNROLL for (int m = 0; m < NX; ++m) if (BS::nzA(m, i)) a += A[m * NX + i] * lam[m];
            ln[i] = a;
          }
          NOC_UNROLL for (int i = 0; i < NX; ++i) lam[i] = ln[i];
          red[0] += slc[s];
        }
        if (terminal == NOC_TERMINAL_FINAL_COST && last) f.final_hess(xN, sP);  // S:66
        const bool is_max[4] = {false, true, false, false};
        wg_reduce(red, 3, is_max);
        cost = red[0] + f.final_cost(xN);  // total_cost(x, u, bp) (P:142)
        hu = red[1];                       // max |Hu| (P:158)
        gnorm = sqrt(red[2]);              // ||cu||_F (P:116)
        if (!keep_inner) inner = 0;
        keep_inner = false;
        relinearize = false;
      }
      const double reg = (mode == NOC_MODE_PAR) ? rp * gnorm : rp;  // P:116-118 / S:51
      __syncthreads();  // blocks and the terminal Hessian complete before the scan reads them
      NOC_WPHASE(2);
#ifdef NOC_PERSIST_PROFILE
      long long t_sub = clock64();
#endif

      // ---------------- KKT solve (par_Newton, P:107-124) ----------------
      // phase 1: this lane's chunk element (Riccati-form prepend, kkt_scan_impl.h)
      auto stage_from_lds = [&](int s, StageData<NX, NU>& st) {
        bget<BS, BF_A>(prm, sA, N, s, st.A.v);
        bget<BS, BF_B>(prm, sB, N, s, st.B.v);
        bget<BS, BF_Q>(prm, sQ, N, s, st.Q.v);
        bget<BS, BF_R>(prm, sR, N, s, st.R.v);
        bget<BS, BF_M>(prm, sM, N, s, st.M.v);
        fget<NU>(sr, N, s, st.r.v);
      };
      Sym<NX> Pt;
      NOC_UNROLL for (int i = 0; i < NX; ++i) NOC_UNROLL for (int j = i; j < NX; ++j) Pt(i, j) = (i == j) ? sP[i * NX + i] : 0.5 * (sP[i * NX + j] + sP[j * NX + i]);
      Elem<NX> e;
      set_zero(e.b);
      set_zero(e.C);
      set_zero(e.nu);
      if (last) { set_zero(e.A); e.J = Pt; } else { set_identity(e.A); set_zero(e.J); }
      for (int s = start + len - 1; s >= start; --s) {
        StageData<NX, NU> st;
        stage_from_lds(s, st);
        prepend<NX, NU, false, BS>(e, st, reg);
      }
      NOC_WSUB(0);
      // phase 2: in-wave reverse Sklansky scan (the last wave's elements end at the terminal
      // cost, so its last level is value-only), then the waves joined through LDS.  The upper
      // half of every level keeps its element, so a wave whose last lane does not end at the
      // terminal cost needs no padding.
      combine_sklansky<NX, false, 0>(e);
      combine_sklansky<NX, false, 1>(e);
      combine_sklansky<NX, false, 2>(e);
      combine_sklansky<NX, false, 3>(e);
      combine_sklansky<NX, false, 4>(e);
      if (wv == W - 1) combine_sklansky<NX, true, 5>(e);  // wave-uniform branch
      else combine_sklansky<NX, false, 5>(e);
      NOC_WSUB(1);
      __syncthreads();  // the aggregate slots were last read by the costate phase
      if (l == 0) elem_put<NX>(sagg + wv * 64, e);
      __syncthreads();
      // value at the start of the next wave's span: later aggregates applied from the end
      Sym<NX> Jw;
      Vec<NX> nw;
      set_zero(Jw);
      set_zero(nw);
      if (wv < W - 1) {
        Elem<NX> ag;
        elem_get<NX>(sagg + (W - 1) * 64, ag);  // value-only (ends at the terminal cost)
        Jw = ag.J;
        nw = ag.nu;
        for (int q = W - 2; q > wv; --q) {
          elem_get<NX>(sagg + q * 64, ag);
          apply_value<NX>(ag, Jw, nw);
          Jw = ag.J;
          nw = ag.nu;
        }
        apply_value<NX>(e, Jw, nw);  // this lane's true value at its chunk start
      }
      NOC_WSUB(2);
      // phase 3: in-chunk Riccati from the true value at the chunk end (lane l+1's start value;
      // lane 63: the next wave's; the horizon's last lane: the terminal cost)
      Sym<NX> S;
      Vec<NX> v;
      wave_shift_down1<Sym<NX>::SZ>(e.J.v, S.v);  // DPP; lane 63: the next wave's value below
      wave_shift_down1<NX>(e.nu.v, v.v);
      if (l == 63) { S = Jw; v = nw; }
      if (last) { S = Pt; set_zero(v); }
      Mat<NX, NX> Phi;
      Vec<NX> phi;
      set_identity(Phi);
      set_zero(phi);
      double kred[4] = {0.0, 1.0, 0.0, 0.0};  // pred, feasible (as a min), unused
      for (int s = start + len - 1; s >= start; --s) {
        StageData<NX, NU> st;
        stage_from_lds(s, st);
        Mat<NX, NX> SA;
        Mat<NX, NU> SB;
        NOC_UNROLL for (int i = 0; i < NX; ++i) {
          NOC_UNROLL for (int j = 0; j < NX; ++j) {
            double a = 0.0;
            NOC_UNROLL for (int k = 0; k < NX; ++k) if (BS::nzA(k, j)) a += S(i, k) * st.A(k, j);
            SA(i, j) = a;
          }
          NOC_UNROLL for (int j = 0; j < NU; ++j) {
            double a = 0.0;
            NOC_UNROLL for (int k = 0; k < NX; ++k) if (BS::nzB(k, j)) a += S(i, k) * st.B(k, j);
            SB(i, j) = a;
          }
        }
        Sym<NU> Quu;
        NOC_UNROLL for (int i = 0; i < NU; ++i)
          NOC_UNROLL for (int j = i; j < NU; ++j) {
            double a = (i == j) ? st.R(i, j) + reg : st.R(i, j);
            NOC_UNROLL for (int k = 0; k < NX; ++k) if (BS::nzB(k, i)) a += st.B(k, i) * SB(k, j);
            Quu(i, j) = a;
          }
        double Y[NU][NX + 1];
        Mat<NU, NX> Qux;
        Vec<NU> Qu;
        NOC_UNROLL for (int i = 0; i < NU; ++i) {
          NOC_UNROLL for (int j = 0; j < NX; ++j) {
            double a = st.M(j, i);
            NOC_UNROLL for (int k = 0; k < NX; ++k) if (BS::nzA(k, j)) a += SB(k, i) * st.A(k, j);
            Qux(i, j) = a;
            Y[i][j] = a;
          }
          double a = st.r[i];
          NOC_UNROLL for (int k = 0; k < NX; ++k) if (BS::nzB(k, i)) a += st.B(k, i) * v[k];
          Qu[i] = a;
          Y[i][NX] = a;
        }
        kred[1] = ldl_solve<NU, NX + 1>(Quu, Y) ? kred[1] : 0.0;  // Quu > 0 (S:52-53)
        double Kk[NU * (NX + 1)];
        NOC_UNROLL for (int i = 0; i < NU; ++i) {
          NOC_UNROLL for (int j = 0; j < NX; ++j) Kk[i * NX + j] = -Y[i][j];
          Kk[NU * NX + i] = -Y[i][NX];
        }
        NOC_UNROLL for (int i = 0; i < KD; ++i) kds(i, s) = Kk[i];
        NOC_UNROLL for (int i = 0; i < NU; ++i) {  // dV = k'Qu + 1/2 k'Quu k (S:63)
          const double ki = Kk[NU * NX + i];
          double qk = 0.0;
          NOC_UNROLL for (int j = 0; j < NU; ++j) qk += Quu(i, j) * Kk[NU * NX + j];
          kred[0] += ki * Qu[i] + 0.5 * ki * qk;
        }
        Sym<NX> Sn;  // S <- Q + A'SA + Qux'K ; v <- A'v + Qux'k
        NOC_UNROLL for (int i = 0; i < NX; ++i)
          NOC_UNROLL for (int j = i; j < NX; ++j) {
            double a = st.Q(i, j);
            NOC_UNROLL for (int k = 0; k < NX; ++k) if (BS::nzA(k, i)) a += st.A(k, i) * SA(k, j);
            NOC_UNROLL for (int q = 0; q < NU; ++q) a += Qux(q, i) * Kk[q * NX + j];
            Sn(i, j) = a;
          }
        Vec<NX> vn;
        NOC_UNROLL for (int i = 0; i < NX; ++i) {
          double a = 0.0;
          NOC_UNROLL for (int k = 0; k < NX; ++k) if (BS::nzA(k, i)) a += st.A(k, i) * v[k];
          NOC_UNROLL for (int q = 0; q < NU; ++q) a += Qux(q, i) * Kk[NU * NX + q];
          vn[i] = a;
        }
        S = Sn;
        v = vn;
        // closed loop of this stage: Phi <- Phi (A + B K), phi <- phi + Phi B k
        Mat<NX, NX> F;
        Vec<NX> fv;
        NOC_UNROLL for (int i = 0; i < NX; ++i) {
          NOC_UNROLL for (int j = 0; j < NX; ++j) {
            double a = st.A(i, j);
            NOC_UNROLL for (int q = 0; q < NU; ++q) if (BS::nzB(i, q)) a += st.B(i, q) * Kk[q * NX + j];
            F(i, j) = a;
          }
          double a = 0.0;
          NOC_UNROLL for (int q = 0; q < NU; ++q) if (BS::nzB(i, q)) a += st.B(i, q) * Kk[NU * NX + q];
          fv[i] = a;
        }
        Mat<NX, NX> Pn;
        NOC_UNROLL for (int i = 0; i < NX; ++i) {
          double a = phi[i];
          NOC_UNROLL for (int k = 0; k < NX; ++k) a += Phi(i, k) * fv[k];
          phi[i] = a;
          NOC_UNROLL for (int j = 0; j < NX; ++j) {
            double c = 0.0;
            NOC_UNROLL for (int k = 0; k < NX; ++k) c += Phi(i, k) * F(k, j);
            Pn(i, j) = c;
          }
        }
        Phi = Pn;
      }
      {
        const bool is_max[4] = {false, false, false, false};
        double kr[4] = {kred[0], 0.0, 0.0, 0.0};
        NOC_WSUB(3);
        wg_reduce(kr, 1, is_max);
        kred[0] = kr[0];
        kred[1] = __syncthreads_and(kred[1] != 0.0) ? 1.0 : 0.0;
      }
      NOC_WSUB(4);
      const double pred = kred[0];
      const bool bwd_ok = kred[1] != 0.0;
      // phase 4: forward affine scan from dx_0 = 0 (P:121-123); thread 0's map is constant
      if (t == 0) set_zero(Phi);
      // in-wave inclusive prefix of the chunk maps: Sklansky with VALU partners (small_linalg.h)
      affine_prefix_sklansky<NX, 64>(Phi, phi);
      __syncthreads();  // aggregate slots (read by the backward join above)
      if (l == 63) {
        NOC_UNROLL for (int i = 0; i < NX * NX; ++i) sagg[wv * 64 + i] = Phi.v[i];
        NOC_UNROLL for (int i = 0; i < NX; ++i) sagg[wv * 64 + NX * NX + i] = phi[i];
      }
      __syncthreads();
      double xw[NX];  // state at the start of this wave's span
      NOC_UNROLL for (int i = 0; i < NX; ++i) xw[i] = (wv == 0) ? 0.0 : sagg[NX * NX + i];
      for (int q = 1; q < wv; ++q) {
        double xn[NX];
        NOC_UNROLL for (int i = 0; i < NX; ++i) {
          double a = sagg[q * 64 + NX * NX + i];
          NOC_UNROLL for (int k = 0; k < NX; ++k) a += sagg[q * 64 + i * NX + k] * xw[k];
          xn[i] = a;
        }
        NOC_UNROLL for (int i = 0; i < NX; ++i) xw[i] = xn[i];
      }
      Vec<NX> x;  // this chunk's start state: lane l-1's inclusive prefix applied to xw
      {
        Mat<NX, NX> oP;
        Vec<NX> op;
        wave_shift_up1<NX * NX>(Phi.v, oP.v);  // DPP; lane 0 uses xw
        wave_shift_up1<NX>(phi.v, op.v);
        NOC_UNROLL for (int i = 0; i < NX; ++i) {
          double a = op[i];
          NOC_UNROLL for (int k = 0; k < NX; ++k) a += oP(i, k) * xw[k];
          x[i] = (l == 0) ? xw[i] : a;
        }
      }
      NOC_WSUB(5);
      // propagate the chunk: u = K x + d, x+ = A x + B u (the gains are read, then the same LDS
      // words are overwritten by dx, du -- each stage's K, d only by its own lane)
      for (int s = start; s < start + len; ++s) {
        double Kk[KD], A[NX * NX], Bm[NX * NU];
        NOC_UNROLL for (int i = 0; i < KD; ++i) Kk[i] = kds(i, s);
        bget<BS, BF_A>(prm, sA, N, s, A);
        bget<BS, BF_B>(prm, sB, N, s, Bm);
        double u[NU];
        NOC_UNROLL for (int i = 0; i < NU; ++i) {
          double a = Kk[NU * NX + i];
          NOC_UNROLL for (int k = 0; k < NX; ++k) a += Kk[i * NX + k] * x[k];
          u[i] = a;
        }
        double xn[NX];
        NOC_UNROLL for (int i = 0; i < NX; ++i) {
          double a = 0.0;
          NOC_UNROLL for (int k = 0; k < NX; ++k) if (BS::nzA(i, k)) a += A[i * NX + k] * x[k];
          NOC_UNROLL for (int j = 0; j < NU; ++j) if (BS::nzB(i, j)) a += Bm[i * NU + j] * u[j];
          xn[i] = a;
        }
        // the K/d region is [KD][N+1] and dx / du reuse rows 0..NX-1 / NX..NX+NU-1 of it: the
        // gains of stage s are consumed above before these stores
        NOC_UNROLL for (int i = 0; i < NX; ++i) dxs(i, s) = x[i];
        NOC_UNROLL for (int j = 0; j < NU; ++j) dus(j, s) = u[j];
        NOC_UNROLL for (int i = 0; i < NX; ++i) x[i] = xn[i];
      }
      if (last) NOC_UNROLL for (int i = 0; i < NX; ++i) dxs(i, N) = x[i];
      __syncthreads();
      NOC_WSUB(6);
      NOC_WPHASE(3);

      // ---------------- trial point (P:156-175 / S:121-161) ----------------
      double tr[4] = {0.0, 0.0, 0.0, 0.0};
      int ok = 1;
      for (int s = start; s < start + len; ++s) {
        double xt[NX], ut[NU];
        NOC_UNROLL for (int i = 0; i < NX; ++i) xt[i] = sx[(size_t)s * NX + i] + dxs(i, s);
        NOC_UNROLL for (int j = 0; j < NU; ++j) ut[j] = su[(size_t)j * N + s] + dus(j, s);
        ok &= f.feasible(xt, ut) ? 1 : 0;
        tr[0] += f.stage_cost(xt, ut, bp);
      }
      if (last) {
        double xt[NX];
        NOC_UNROLL for (int i = 0; i < NX; ++i) xt[i] = sx[(size_t)N * NX + i] + dxs(i, N);
        tr[0] += f.final_cost(xt);
      }
      {
        const bool is_max[4] = {false, false, false, false};
        wg_reduce(tr, 1, is_max);
      }
      const bool traj_ok = __syncthreads_and(ok != 0);
      const double new_cost = traj_ok ? tr[0] : INFINITY;       // P:159-163, S:126-129
      const double gain = (new_cost - cost) / pred;             // P:164-165
      const bool success = (gain > 0.0) && bwd_ok;              // P:166 / S:137
#ifdef NOC_DECISION_TRACE
      if (t == 0) NOC_TRACE_DECISION(g_wide_dtrace, b, solves, bp, it, inner, cost, new_cost, pred,
                                     gain, success, rp, rinc, hu, bwd_ok);
#endif
      const double shrink = rp_shrink(gain);  // P:169 / S:141 (noc_internal.h)
      const double rp_used = rp;
      rp = success ? rp * shrink : rp * rinc;                   // P:167-171 / S:139-143
      rinc = success ? 2.0 : 2.0 * rinc;                        // P:172 / S:144
      bool take, end_iter, stop;
      inner += 1;
      if (mode == NOC_MODE_PAR) {
        rp = fmin(fmax(rp, 1e-16), 1e16);                       // P:173
        // identical retries at the rp clip: accounted, not recomputed (noc_internal.h)
        const int rep = par_retry_repeats(w, success, rp_used, rp, inner, max_solves - solves - 1);
        if (rep > 0) {
          inner += rep;
          solves += rep;
          rinc = ldexp(rinc, rep);  // r_inc doubles per retry (P:172)
          if (t == 0 && w.repeats) w.repeats[b] += rep;
        }
        end_iter = success || inner > 500;                      // P:177-182
        take = end_iter;                                        // last trial kept (P:175, P:184)
        stop = end_iter && (hu < 1e-4 || it + 1 > 1000);        // P:199-202
      } else {
        take = success;                                         // S:145-146
        end_iter = true;
        stop = (hu < 1e-4) && bwd_ok;                           // S:157-161
      }
      if (take) {  // x <- x + dx, u <- u + du
        for (int s = start; s < start + len; ++s) {
          NOC_UNROLL for (int i = 0; i < NX; ++i) sx[(size_t)s * NX + i] += dxs(i, s);
          NOC_UNROLL for (int j = 0; j < NU; ++j) su[(size_t)j * N + s] += dus(j, s);
        }
        if (last) NOC_UNROLL for (int i = 0; i < NX; ++i) sx[(size_t)N * NX + i] += dxs(i, N);
      }
      __syncthreads();
      NOC_WPHASE(4);
#ifdef NOC_PERSIST_PROFILE
      if (b == 0 && t == 0) g_wide_cycles[5] += 1;
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
      // where a later launch would continue (the resume point)
      phase = stage_done ? NOC_PHASE_ROLLOUT : (relinearize ? NOC_PHASE_LINEARIZE : NOC_PHASE_SOLVE);
      if (stage_done && (!(bp > 1e-4) || (w.flags & NOC_WS_ONE_STAGE))) phase = NOC_PHASE_DONE;
      if (phase == NOC_PHASE_DONE || solves >= max_solves) break;
    }
    if (phase != NOC_PHASE_ROLLOUT || solves >= max_solves) break;  // P:243-245 / capped
  }
  // results out: states, controls, the solver state
  for (int i = t; i < (N + 1) * NX; i += T) Xg[i] = sx[i];
  for (int i = t; i < N * NU; i += T) Ug[i] = su[(i % NU) * N + i / NU];
  if (t == 0) {
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
  }
  __syncthreads();  // the next trajectory's controls overwrite the LDS read above
  }
}

int wide_set_decision_trace(const DecisionTrace& t) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_wide_dtrace), &t, sizeof(t)) == hipSuccess ? 0 : -1;
}

int debug_wide_cycles(long long* out, int n, int reset) {
  long long host[16];
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wide_cycles), sizeof(host)) != hipSuccess) return -1;
  for (int i = 0; i < n && i < 16; ++i) out[i] = host[i];
  if (reset) {
    const long long zero[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_wide_cycles), zero, sizeof(zero)) != hipSuccess) return -1;
  }
  return 0;
}

// LDS bytes of one W-wave workgroup of family p, 0 if the trajectory does not fit in a CU
template <int K, int X, int U>
static size_t wide_lds_t(int N, int W) {
  const size_t bytes = (size_t)WideLds<X, U, BlockStruct<K, X, U, true>>(N, W).total * sizeof(double);
  return bytes <= 160 * 1024 - 1024 ? bytes : 0;
}
size_t wide_lds_bytes(const noc_family& p, int N, int W) {
#define NOC_FAMILY(K, X, U) \
  if (p.kind == K && p.nx == X && p.nu == U) return wide_lds_t<K, X, U>(N, W);
#include NOC_FAMILIES_DEF
#undef NOC_FAMILY
  return 0;
}

// Waves per trajectory: 4 when the batch leaves CUs idle (B <= #CUs: one workgroup per CU), 2
// when two two-wave workgroups fit a CU (512 registers per lane: one wave per SIMD) -- B up to
// 2 x #CUs, the 8-GPU slice of c3.  NOC_WIDE_WAVES=2|4 forces one (per launch).
int wide_waves(const noc_family& p, const noc_ipm_ws& w, int cus) {
  const char* env = getenv("NOC_WIDE_WAVES");
  if (env && (atoi(env) == 2 || atoi(env) == 4)) return atoi(env);
  if (cus > 0 && w.Bt <= cus) return 4;
  const size_t two = wide_lds_bytes(p, w.N, 2);
  return (two > 0 && two <= 80 * 1024 - 512) ? 2 : 4;
}

template <int K, int X, int U>
static hipError_t wide_family(const noc_family& p, const noc_ipm_ws& w, int mode, int terminal,
                              double bp0, int max_solves, const int* idx, const int* count,
                              int grid, int W, hipStream_t s) {
  if constexpr (X <= 4) {
    const size_t lds = wide_lds_t<K, X, U>(w.N, W);
    if (lds == 0 || grid <= 0) return hipErrorInvalidValue;
    if (W == 2)
      hipLaunchKernelGGL((ipm_wide_kernel<K, X, U, 2>), dim3(grid), dim3(128), lds, s, p, w, mode,
                         terminal, bp0, max_solves, idx, count);
    else
      hipLaunchKernelGGL((ipm_wide_kernel<K, X, U, kWideWaves>), dim3(grid), dim3(64 * kWideWaves),
                         lds, s, p, w, mode, terminal, bp0, max_solves, idx, count);
    return hipGetLastError();
  } else {
    return hipErrorInvalidValue;
  }
}

bool ipm_wide_supported(const noc_family& p, int N) {
  return family_supported(p) && p.nx <= 4 && wide_lds_bytes(p, N, kWideWaves) > 0;
}

hipError_t ipm_solve_wide(const noc_family& p, const noc_ipm_ws& w, int mode, int terminal,
                          double bp0, int max_solves, const int* idx, const int* count, int grid,
                          int W, hipStream_t s) {
#define NOC_FAMILY(K, X, U)                                                              \
  if (p.kind == K && p.nx == X && p.nu == U)                                             \
    return wide_family<K, X, U>(p, w, mode, terminal, bp0, max_solves, idx, count, grid, W, s);
#include NOC_FAMILIES_DEF
#undef NOC_FAMILY
  return hipErrorInvalidValue;
}

}  // namespace noc
