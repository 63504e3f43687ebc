// Interior-point Newton loop kernels for the registered problem families (fp64, gfx950).
//
// One host iteration of the batched driver (noc/par_interior_point_newton.py of this package)
// launches, each masked by the per-trajectory phase so every trajectory follows its own
// reference control flow (vmap semantics of the reference's nested while_loops):
//   rollout   (phase ROLLOUT)   noc/utils.py:57-63, at the start of each barrier stage (P:133)
//   linearize (phase LINEARIZE) derivatives of P:13-28 at (x_k, u_k): A=fx, B=fu, cx, cu, l_k
//   costate   (phase LINEARIZE) lambda scan C:43-54 + ru = cu + fu' lambda (P:34), total cost
//                               (P:142), |Hu|inf (P:158), ||cu||_F (P:116), terminal Hessian
//   assemble  (phase LINEARIZE) Q, R, M of compute_lqr_params (P:31-42)
//   [kkt_scan (phase SOLVE)     par_Newton's solve, P:119-123]
//   trial     (phase SOLVE)     trial point, feasibility, gain ratio, rp / r_inc update, accept,
//                               Newton stop test, barrier schedule (P:156-254; seq mode S:121-202)
#include <hip/hip_runtime.h>

#include <cmath>

#include "../../include/noc_hip.h"
#include "ipm_family.h"
#include "noc_internal.h"
#include "small_linalg.h"

namespace noc {

// Rollout x_{k+1} = f(x_k, u_k) (noc/utils.py:57-63), one wave64 per trajectory.  The recurrence
// is inherently sequential; every lane evaluates it redundantly (free in SIMD) with u_k broadcast
// from registers (v_readlane), so the dependent chain never waits on memory: controls are read and
// states written 64 stages at a time, coalesced.
// take_pending: also roll out trajectories the last trial marked ROLLOUT_PENDING (the
// single-stream loop, where nothing else runs concurrently).  The two-stream loop passes 0: its
// rollout runs beside the main stream's trial kernel, which may mark a trajectory (after writing
// its new u) at any moment; only the main stream's promote, ordered after that trial, turns the
// mark into ROLLOUT, so this kernel sees exactly the trajectories marked before it was launched.
template <int KIND, int NX, int NU>
__global__ __launch_bounds__(256) void rollout_kernel(noc_family prm, noc_ipm_ws w, int take_pending) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= w.Bt) return;
  const int ph = w.phase[b];
  if (!(ph == NOC_PHASE_ROLLOUT || (take_pending && ph == NOC_PHASE_ROLLOUT_PENDING))) return;  // uniform per wave
  Fam<KIND, NX, NU> f(prm);
  const int N = w.N;
  double x[NX];
  NOC_UNROLL for (int i = 0; i < NX; ++i) x[i] = w.x0[(size_t)b * NX + i];
  double* X = w.x + (size_t)b * (N + 1) * NX;
  const double* U = w.u + (size_t)b * N * NU;
  if (lane < NX) X[lane] = x[lane];
  for (int base = 0; base < N; base += 64) {
    const int k = base + lane;
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
        mine[i] = (lane == t) ? xn[i] : mine[i];
      }
    }
    if (k < N) NOC_UNROLL for (int i = 0; i < NX; ++i) X[(size_t)(k + 1) * NX + i] = mine[i];
  }
  if (lane == 0) w.phase[b] = NOC_PHASE_ROLLED;
}

// ROLLED -> LINEARIZE; ROLLOUT_PENDING -> ROLLOUT (the next step's rollout picks it up)
__global__ __launch_bounds__(256) void promote_kernel(noc_ipm_ws w) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= w.Bt) return;
  const int ph = w.phase[b];
  if (ph == NOC_PHASE_ROLLED) w.phase[b] = NOC_PHASE_LINEARIZE;
  else if (ph == NOC_PHASE_ROLLOUT_PENDING) w.phase[b] = NOC_PHASE_ROLLOUT;
}

// thread per (trajectory, chunk slot, lane) in tiled order: the A/B stores are coalesced
template <int KIND, int NX, int NU>
__global__ __launch_bounds__(256) void linearize_kernel(noc_family prm, noc_ipm_ws w) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int N = w.N, L = w.lanes;
  const Chunks ch(N, L);
  if (t >= (long long)w.Bt * ch.cmax * L) return;
  const int b = (int)(t / ((long long)ch.cmax * L));
  const int rem = (int)(t % ((long long)ch.cmax * L));
  const int j = rem / L, l = rem % L;
  if (j >= ch.len(l) || w.phase[b] != NOC_PHASE_LINEARIZE) return;
  const int k = ch.start(l) + j;
  const size_t tn = (size_t)b * N + k;
  Fam<KIND, NX, NU> f(prm);
  const double bp = w.bp[b];
  double x[NX], u[NU];
  gload<NX>(w.x + ((size_t)b * (N + 1) + k) * NX, x);
  NOC_UNROLL for (int i = 0; i < NU; ++i) u[i] = w.u[tn * NU + i];
  double fx[NX * NX], fu[NX * NU], cx[NX], cu[NU];  // all stored tiled
  f.jac(x, u, fx, fu);
  f.stage_grad(x, u, bp, cx, cu);
  tstore_rt<NX * NX>(w.A, L, ch.cmax, b, j, l, fx);
  tstore_rt<NX * NU>(w.B, L, ch.cmax, b, j, l, fu);
  tstore_rt<NX>(w.cx, L, ch.cmax, b, j, l, cx);
  tstore_rt<NU>(w.cu, L, ch.cmax, b, j, l, cu);
  const double lc = f.stage_cost(x, u, bp);
  tstore_rt<1>(w.lc, L, ch.cmax, b, j, l, &lc);
}

// Costates as a reverse affine scan over the horizon (the par_costates pattern, C:34-40),
// one L-lane segment per trajectory with the KKT scan's chunk geometry (tiled A, B, cx, cu, lc):
//   lambda_k = cx_k + A_k' lambda_{k+1},  lambda_N = grad final_cost (C:44-52)
// plus, per trajectory: ru_k = cu_k + B_k' lambda_{k+1} (P:34, tiled), total cost (P:142),
// max|ru| (P:158), ||cu||_F (P:116), the regularisation fed to the KKT solve and the terminal
// Hessian hessian(final_cost) (S:66).
template <int KIND, int NX, int NU, int L>
__global__ __launch_bounds__(64) void costate_scan_kernel(noc_family prm, noc_ipm_ws w, int mode) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = tid / L, l = tid % L;
  if (b >= w.Bt || w.phase[b] != NOC_PHASE_LINEARIZE) return;  // uniform per segment
  Fam<KIND, NX, NU> f(prm);
  const int N = w.N;
  const Chunks ch(N, L);
  const int start = ch.start(l), len = ch.len(l);
  const bool last = (l == L - 1);
  const double* xN = w.x + ((size_t)b * (N + 1) + N) * NX;
  double lamN[NX];
  f.final_grad(xN, lamN);  // grad(final_cost) (C:35)
  // phases 1-2 (L > 1): chunk maps and their scan; L = 1 (grouped layout, one lane per
  // trajectory) sweeps the whole horizon from lambda_N directly
  Mat<NX, NX> G;
  Vec<NX> g;
  set_zero(g);
  if constexpr (L > 1) {
    // phase 1: chunk map lambda_start = G lambda_end + g
    set_identity(G);
    for (int k = start + len - 1; k >= start; --k) {
      double A[NX * NX], cx[NX];
      tload_rt<NX * NX>(w.A, L, ch.cmax, b, k - start, l, A);
      tload_rt<NX>(w.cx, L, ch.cmax, b, k - start, l, cx);
      Mat<NX, NX> Gn;
      Vec<NX> gn;
      NOC_UNROLL for (int i = 0; i < NX; ++i) {
        double t = cx[i];
        NOC_UNROLL for (int m = 0; m < NX; ++m) t += A[m * NX + i] * g[m];
        gn[i] = t;
        NOC_UNROLL for (int j = 0; j < NX; ++j) {
          double u = 0.0;
          NOC_UNROLL for (int m = 0; m < NX; ++m) u += A[m * NX + i] * G(m, j);
          Gn(i, j) = u;
        }
      }
      G = Gn;
      g = gn;
    }
    if (last) {  // the last chunk ends at the terminal costate: its map becomes constant
      NOC_UNROLL for (int i = 0; i < NX; ++i) {
        double t = g[i];
        NOC_UNROLL for (int m = 0; m < NX; ++m) t += G(i, m) * lamN[m];
        g[i] = t;
      }
      set_zero(G);
    }
    // phase 2: reverse Hillis-Steele; lanes without a partner get their own (already constant) map
  #pragma unroll 1
    for (int d = 1; d < L; d <<= 1) {
      Mat<NX, NX> G2;
      Vec<NX> g2;
      shfl_down_arr<NX * NX>(G.v, G2.v, d, L);
      shfl_down_arr<NX>(g.v, g2.v, d, L);
      Mat<NX, NX> Gn;
      NOC_UNROLL for (int i = 0; i < NX; ++i) {
        double t = g[i];
        NOC_UNROLL for (int m = 0; m < NX; ++m) t += G(i, m) * g2[m];
        g[i] = t;
        NOC_UNROLL for (int j = 0; j < NX; ++j) {
          double u = 0.0;
          NOC_UNROLL for (int m = 0; m < NX; ++m) u += G(i, m) * G2(m, j);
          Gn(i, j) = u;
        }
      }
      G = Gn;
    }
  }
  // phase 3: sweep the chunk from its true end costate
  double lam[NX];
  if constexpr (L > 1) shfl_down_arr<NX>(g.v, lam, 1, L);
  if (last) NOC_UNROLL for (int i = 0; i < NX; ++i) lam[i] = lamN[i];
  double* LAM = w.lam + (size_t)b * (N + 1) * NX;
  if (last) gstore<NX>(LAM + (size_t)N * NX, lamN);
  double cost = 0.0, hu = 0.0, g2s = 0.0;
  for (int k = start + len - 1; k >= start; --k) {
    double A[NX * NX], Bm[NX * NU], cx[NX], cu[NU], lc, rr[NU];
    tload_rt<NX * NX>(w.A, L, ch.cmax, b, k - start, l, A);
    tload_rt<NX * NU>(w.B, L, ch.cmax, b, k - start, l, Bm);
    tload_rt<NX>(w.cx, L, ch.cmax, b, k - start, l, cx);
    tload_rt<NU>(w.cu, L, ch.cmax, b, k - start, l, cu);
    tload_rt<1>(w.lc, L, ch.cmax, b, k - start, l, &lc);
    NOC_UNROLL for (int jj = 0; jj < NU; ++jj) {  // ru_k = cu_k + fu_k' lambda_{k+1}  (P:34)
      double r = cu[jj];
      NOC_UNROLL for (int i = 0; i < NX; ++i) r += Bm[i * NU + jj] * lam[i];
      rr[jj] = r;
      hu = nan_max(hu, fabs(r));
      g2s += cu[jj] * cu[jj];
    }
    tstore_rt<NU>(w.r, L, ch.cmax, b, k - start, l, rr);
    double ln[NX];
    NOC_UNROLL for (int i = 0; i < NX; ++i) {
      double t = cx[i];
      NOC_UNROLL for (int m = 0; m < NX; ++m) t += A[m * NX + i] * lam[m];
      ln[i] = t;
    }
    NOC_UNROLL for (int i = 0; i < NX; ++i) lam[i] = ln[i];
    gstore<NX>(LAM + (size_t)k * NX, lam);
    cost += lc;
  }
  // lambda at the chunk start := the scan's value g (not this lane's sweep): it is exactly the
  // boundary costate the previous lane used, so every consumer of lambda_k sees one value
  if (L > 1 && len > 0) gstore<NX>(LAM + (size_t)start * NX, g.v);
  NOC_UNROLL for (int off = L / 2; off > 0; off >>= 1) {
    cost += __shfl_xor(cost, off, L);
    g2s += __shfl_xor(g2s, off, L);
    hu = nan_max(hu, __shfl_xor(hu, off, L));
  }
  if (l != 0) return;
  double P[NX * NX];
  f.final_hess(xN, P);  // hessian(final_cost) (S:66)
  gstore<NX * NX>(w.P + (size_t)b * NX * NX, P);
  w.cost[b] = cost + f.final_cost(xN);   // total_cost(x, u, bp) (P:142)
  w.hu[b] = hu;                          // max |Hu| (P:158)
  const double gn = sqrt(g2s);           // ||cu||_F (P:116)
  w.gnorm[b] = gn;
  // regularisation fed to the KKT solve: par R += rp*||cu||*I (P:116-118); seq Quu += mu*I (S:51)
  w.reg[b] = (mode == NOC_MODE_PAR) ? w.rp[b] * gn : w.rp[b];
  w.inner[b] = 0;
}

template <int KIND, int NX, int NU>
static void launch_costate(const noc_family& p, const noc_ipm_ws& w, int mode, hipStream_t s) {
  const int L = w.lanes;
  const unsigned grid = (unsigned)(((long long)w.Bt * L + 63) / 64);
  switch (L) {
    case 64: hipLaunchKernelGGL((costate_scan_kernel<KIND, NX, NU, 64>), dim3(grid), dim3(64), 0, s, p, w, mode); break;
    case 32: hipLaunchKernelGGL((costate_scan_kernel<KIND, NX, NU, 32>), dim3(grid), dim3(64), 0, s, p, w, mode); break;
    case 16: hipLaunchKernelGGL((costate_scan_kernel<KIND, NX, NU, 16>), dim3(grid), dim3(64), 0, s, p, w, mode); break;
    case 8: hipLaunchKernelGGL((costate_scan_kernel<KIND, NX, NU, 8>), dim3(grid), dim3(64), 0, s, p, w, mode); break;
    default: hipLaunchKernelGGL((costate_scan_kernel<KIND, NX, NU, 1>), dim3(grid), dim3(64), 0, s, p, w, mode); break;
  }
}

template <int KIND, int NX, int NU>
__global__ __launch_bounds__(256) void assemble_kernel(noc_family prm, noc_ipm_ws w, int terminal) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int N = w.N, L = w.lanes;
  const Chunks ch(N, L);
  if (t >= (long long)w.Bt * ch.cmax * L) return;
  const int b = (int)(t / ((long long)ch.cmax * L));
  const int rem = (int)(t % ((long long)ch.cmax * L));
  const int j = rem / L, l = rem % L;
  if (j >= ch.len(l) || w.phase[b] != NOC_PHASE_LINEARIZE) return;
  const int k = ch.start(l) + j;
  const size_t tn = (size_t)b * N + k;
  Fam<KIND, NX, NU> f(prm);
  const double bp = w.bp[b];
  double x[NX], u[NU], lam[NX];
  gload<NX>(w.x + ((size_t)b * (N + 1) + k) * NX, x);
  NOC_UNROLL for (int i = 0; i < NU; ++i) u[i] = w.u[tn * NU + i];
  gload<NX>(w.lam + ((size_t)b * (N + 1) + k + 1) * NX, lam);
  // Q = cxx + l.fxx ; R = cuu + l.fuu ; M = cxu + l.fxu  (P:35-37), l = lambda_{k+1}
  double Q[NX * NX], R[NU * NU], M[NX * NU];
  f.stage_hess(x, u, bp, Q, R, M);
  f.add_hess_l(x, u, lam, Q, R, M);
  Sym<NX> Qs;
  Sym<NU> Rs;
  NOC_UNROLL for (int i = 0; i < NX; ++i)
    NOC_UNROLL for (int jj = i; jj < NX; ++jj) Qs(i, jj) = (i == jj) ? Q[i * NX + i] : 0.5 * (Q[i * NX + jj] + Q[jj * NX + i]);
  NOC_UNROLL for (int i = 0; i < NU; ++i)
    NOC_UNROLL for (int jj = i; jj < NU; ++jj) Rs(i, jj) = (i == jj) ? R[i * NU + i] : 0.5 * (R[i * NU + jj] + R[jj * NU + i]);
  tstore_rt<Sym<NX>::SZ>(w.Q, L, ch.cmax, b, j, l, Qs.v);
  tstore_rt<Sym<NU>::SZ>(w.R, L, ch.cmax, b, j, l, Rs.v);
  tstore_rt<NX * NU>(w.M, L, ch.cmax, b, j, l, M);
  if (terminal == NOC_TERMINAL_STAGE0 && k == 0) gstore<NX * NX>(w.P + (size_t)b * NX * NX, Q);  // P:73
}

__global__ __launch_bounds__(256) void mark_solve_kernel(noc_ipm_ws w) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= w.Bt) return;
  const int ph = w.phase[b];
  if (ph == NOC_PHASE_LINEARIZE) w.phase[b] = NOC_PHASE_SOLVE;
  w.kkt_active[b] = (ph == NOC_PHASE_LINEARIZE || ph == NOC_PHASE_SOLVE) ? 1 : 0;
}

// ------------------------------------------------------------------------------------------------
// trial point + Newton / barrier logic: one wave64 per trajectory (4 per 256-thread block)

template <int KIND, int NX, int NU>
__global__ __launch_bounds__(256) void trial_kernel(noc_family prm, noc_ipm_ws w, int mode) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= w.Bt || w.phase[b] != NOC_PHASE_SOLVE) return;  // uniform per wave
  Fam<KIND, NX, NU> f(prm);
  const int N = w.N;
  const double bp = w.bp[b];
  const double* X = w.x + (size_t)b * (N + 1) * NX;
  const double* DX = w.dx + (size_t)b * (N + 1) * NX;
  const double* U = w.u + (size_t)b * N * NU;
  const double* DU = w.du + (size_t)b * N * NU;
  // lane l sums the stages of horizon chunk l (the 64-lane chunk geometry) and the last lane adds
  // the final cost: the same summation order as the persistent solver (ipm_persistent.hip), so
  // both drivers take identical accept / reject decisions
  double csum = 0.0;
  int ok = 1;
  const Chunks ch(N, 64);
  for (int k = ch.start(lane); k < ch.start(lane) + ch.len(lane); ++k) {
    double xt[NX], ut[NU];
    NOC_UNROLL for (int i = 0; i < NX; ++i) xt[i] = X[(size_t)k * NX + i] + DX[(size_t)k * NX + i];
    NOC_UNROLL for (int j = 0; j < NU; ++j) ut[j] = U[(size_t)k * NU + j] + DU[(size_t)k * NU + j];
    ok &= f.feasible(xt, ut) ? 1 : 0;
    csum += f.stage_cost(xt, ut, bp);
  }
  if (lane == 63) {
    double xt[NX];
    NOC_UNROLL for (int i = 0; i < NX; ++i) xt[i] = X[(size_t)N * NX + i] + DX[(size_t)N * NX + i];
    csum += f.final_cost(xt);
  }
  csum = wave_sum(csum);
  const bool traj_ok = __all(ok);
  // new_cost = where(feasible, total_cost(trial), inf)   (P:159-163, S:126-129)
  const double new_cost = traj_ok ? csum : INFINITY;
  const double cost = w.cost[b];
  const double pred = w.pred[b];
  const bool bwd_ok = w.feasible[b] != 0;
  const double gain = (new_cost - cost) / pred;           // P:164-165
  const bool success = (gain > 0.0) && bwd_ok;            // P:166 / S:137
  double rp = w.rp[b], rinc = w.rinc[b];
  const double rp_used = rp;
  const double shrink = rp_shrink(gain);  // P:169 / S:141 (noc_internal.h)
  rp = success ? rp * shrink : rp * rinc;                 // P:167-171 / S:139-143
  rinc = success ? 2.0 : 2.0 * rinc;                      // P:172 / S:144
  bool take, end_iter, stop;
  int inner = w.inner[b] + 1, rep = 0;
  if (mode == NOC_MODE_PAR) {
    rp = fmin(fmax(rp, 1e-16), 1e16);                     // P:173
    // identical retries at the rp clip: accounted, not recomputed (noc_internal.h)
    rep = par_retry_repeats(w, success, rp_used, rp, inner, 501);
    inner += rep;
    rinc = ldexp(rinc, rep);                              // r_inc doubles per retry (P:172)
    end_iter = success || inner > 500;                    // P:177-182
    take = end_iter;                                      // the last trial is kept (P:175, P:184)
    stop = end_iter && (w.hu[b] < 1e-4 || w.it[b] + 1 > 1000);  // P:199-202
  } else {
    take = success;                                       // S:145-146
    end_iter = true;
    stop = (w.hu[b] < 1e-4) && bwd_ok;                    // S:157-161
  }
  if (take) {  // x <- x + dx, u <- u + du
    double* Xw = w.x + (size_t)b * (N + 1) * NX;
    double* Uw = w.u + (size_t)b * N * NU;
    for (int k = lane; k <= N; k += 64) {
      NOC_UNROLL for (int i = 0; i < NX; ++i) Xw[(size_t)k * NX + i] += DX[(size_t)k * NX + i];
      if (k < N) NOC_UNROLL for (int j = 0; j < NU; ++j) Uw[(size_t)k * NU + j] += DU[(size_t)k * NU + j];
    }
  }
  if (lane != 0) return;
  w.kkt_solves[b] += 1 + rep;
  if (w.repeats) w.repeats[b] += rep;
  w.inner[b] = inner;
  int it = w.it[b] + (end_iter ? 1 : 0);
  int phase;
  if (stop) {                                             // barrier stage finished
    w.total_it[b] += it;                                  // P:239 / S:187
    const double nbp = bp / 5.0;                          // P:238 / S:186
    w.bp[b] = nbp;
    it = 0;
    rp = 1.0;                                             // P:134 / S:110
    rinc = 2.0;                                           // P:135 / S:111
    // P:243-245; the rollout of the new stage happens in the next step (ROLLOUT_PENDING, see
    // rollout_kernel)
    // (NOC_WS_ONE_STAGE: newton_oc runs a single barrier stage)
    phase = (nbp > 1e-4 && !(w.flags & NOC_WS_ONE_STAGE)) ? NOC_PHASE_ROLLOUT_PENDING : NOC_PHASE_DONE;
  } else if (mode == NOC_MODE_PAR) {
    phase = end_iter ? NOC_PHASE_LINEARIZE : NOC_PHASE_SOLVE;
  } else {
    // seq: the next iteration linearises at x (+step if taken); a rejected step leaves x, u
    // unchanged, so only the regularisation changes (same blocks, cheaper: skip relinearising)
    phase = success ? NOC_PHASE_LINEARIZE : NOC_PHASE_SOLVE;
  }
  w.it[b] = it;
  w.rp[b] = rp;
  w.rinc[b] = rinc;
  if (phase == NOC_PHASE_SOLVE) w.reg[b] = (mode == NOC_MODE_PAR) ? rp * w.gnorm[b] : rp;
  w.phase[b] = phase;
}

__global__ __launch_bounds__(256) void init_kernel(noc_ipm_ws w, double bp0) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= w.Bt) return;
  w.phase[b] = NOC_PHASE_ROLLOUT;
  w.kkt_active[b] = 1;
  w.it[b] = 0;
  w.inner[b] = 0;
  w.total_it[b] = 0;
  w.kkt_solves[b] = 0;
  if (w.repeats) w.repeats[b] = 0;
  w.bp[b] = bp0;
  w.rp[b] = 1.0;
  w.rinc[b] = 2.0;
  w.hu[b] = 1.0;
}

// ------------------------------------------------------------------------------------------------
template <int KIND, int NX, int NU>
static hipError_t rollout_t(const noc_family& p, const noc_ipm_ws& w, hipStream_t s,
                           int take_pending) {
  hipLaunchKernelGGL((rollout_kernel<KIND, NX, NU>), dim3((w.Bt + 3) / 4), dim3(256), 0, s, p, w,
                     take_pending);
  return hipGetLastError();
}

// linearise + costates + LQ blocks for phase-LINEARIZE trajectories, then LINEARIZE -> SOLVE
template <int KIND, int NX, int NU>
static hipError_t prepare_main_t(const noc_family& p, const noc_ipm_ws& w, int mode, int terminal,
                                 hipStream_t s) {
  const int bt_grid = (w.Bt + 255) / 256;
  const long long cmax = (w.N + w.lanes - 1) / w.lanes;
  const unsigned st_grid = (unsigned)(((long long)w.Bt * cmax * w.lanes + 255) / 256);
  hipLaunchKernelGGL((linearize_kernel<KIND, NX, NU>), dim3(st_grid), dim3(256), 0, s, p, w);
  launch_costate<KIND, NX, NU>(p, w, mode, s);
  hipLaunchKernelGGL((assemble_kernel<KIND, NX, NU>), dim3(st_grid), dim3(256), 0, s, p, w, terminal);
  hipLaunchKernelGGL(mark_solve_kernel, dim3(bt_grid), dim3(256), 0, s, w);
  return hipGetLastError();
}

template <int KIND, int NX, int NU>
static hipError_t prepare_t(const noc_family& p, const noc_ipm_ws& w, int mode, int terminal,
                            hipStream_t s) {
  hipError_t e = rollout_t<KIND, NX, NU>(p, w, s, 1);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(promote_kernel, dim3((w.Bt + 255) / 256), dim3(256), 0, s, w);
  return prepare_main_t<KIND, NX, NU>(p, w, mode, terminal, s);
}

template <int KIND, int NX, int NU>
static hipError_t trial_t(const noc_family& p, const noc_ipm_ws& w, int mode, hipStream_t s) {
  const unsigned grid = (unsigned)((w.Bt + 3) / 4);
  hipLaunchKernelGGL((trial_kernel<KIND, NX, NU>), dim3(grid), dim3(256), 0, s, p, w, mode);
  return hipGetLastError();
}

// family dispatch: one instantiation per NOC_FAMILY line of families.def
hipError_t ipm_prepare(const noc_family& p, const noc_ipm_ws& w, int mode, int terminal,
                       hipStream_t s) {
#define NOC_FAMILY(K, X, U) \
  if (p.kind == K && p.nx == X && p.nu == U) return prepare_t<K, X, U>(p, w, mode, terminal, s);
#include NOC_FAMILIES_DEF
#undef NOC_FAMILY
  return hipErrorInvalidValue;
}

hipError_t ipm_rollout(const noc_family& p, const noc_ipm_ws& w, hipStream_t s) {
#define NOC_FAMILY(K, X, U) \
  if (p.kind == K && p.nx == X && p.nu == U) return rollout_t<K, X, U>(p, w, s, 0);
#include NOC_FAMILIES_DEF
#undef NOC_FAMILY
  return hipErrorInvalidValue;
}

hipError_t ipm_prepare_main(const noc_family& p, const noc_ipm_ws& w, int mode, int terminal,
                            hipStream_t s) {
#define NOC_FAMILY(K, X, U) \
  if (p.kind == K && p.nx == X && p.nu == U) return prepare_main_t<K, X, U>(p, w, mode, terminal, s);
#include NOC_FAMILIES_DEF
#undef NOC_FAMILY
  return hipErrorInvalidValue;
}

hipError_t ipm_promote(const noc_ipm_ws& w, hipStream_t s) {
  hipLaunchKernelGGL(promote_kernel, dim3((w.Bt + 255) / 256), dim3(256), 0, s, w);
  return hipGetLastError();
}

hipError_t ipm_trial(const noc_family& p, const noc_ipm_ws& w, int mode, hipStream_t s) {
#define NOC_FAMILY(K, X, U) \
  if (p.kind == K && p.nx == X && p.nu == U) return trial_t<K, X, U>(p, w, mode, s);
#include NOC_FAMILIES_DEF
#undef NOC_FAMILY
  return hipErrorInvalidValue;
}

hipError_t ipm_init(const noc_ipm_ws& w, double bp0, hipStream_t s) {
  hipLaunchKernelGGL(init_kernel, dim3((w.Bt + 255) / 256), dim3(256), 0, s, w, bp0);
  return hipGetLastError();
}

bool family_supported(const noc_family& p) {
#define NOC_FAMILY(K, X, U) \
  if (p.kind == K && p.nx == X && p.nu == U) return true;
#include NOC_FAMILIES_DEF
#undef NOC_FAMILY
  return false;
}

}  // namespace noc
