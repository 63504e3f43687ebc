// Batched parallel-in-time KKT solve of the interior-point Newton step (fp64, gfx950).
//
// Replaces paroc.par_bwd_pass + paroc.par_fwd_pass as called by par_Newton
// (noc/par_interior_point_newton.py:119-123) and examples/linear_mpc_parallel.py:68-69.
// Mathematically it is the stage-structured KKT solve of seq_interior_point_newton.bwd_pass /
// fwd_pass (noc/seq_interior_point_newton.py:42-90), computed as an associative scan along the
// horizon (Saerkkae & Garcia-Fernandez temporal-parallel LQ, the algorithm behind paroc).
//
// Mapping (one trajectory per L-lane segment of a wave64; L = 64 is one trajectory per wave):
//   * lane l of the segment owns the contiguous chunk of stages [start_l, start_l + len_l);
//   * phase 1  in-chunk element   : the lane folds its stages right-to-left into one scan element
//                                  (A, b, C, nu, J) with the Riccati-form "prepend" (no R^-1);
//                                  the segment's last lane starts from the terminal cost.
//   * phase 2  cross-lane scan    : reverse Sklansky tree over the L lanes, DPP / readlane partners;
//                                  afterwards lane l holds the value function at start_l.
//   * phase 3  in-chunk Riccati   : from the true boundary value (lane l+1's result) the lane runs
//                                  the sequential Riccati over its chunk -> gains K, d, value S, v,
//                                  pred (sum dV), feasibility (LDL' pivots > 0), and composes its
//                                  chunk's closed-loop affine map.
//   * phase 4  forward scan       : inclusive forward scan of the affine maps (noc/costates.py:6-12
//                                  combine pattern) gives each lane its start state; the lane then
//                                  propagates dx, du through its chunk.
// Conventions: include/noc_hip.h.
#pragma once
#include <hip/hip_runtime.h>

#include "small_linalg.h"
#include "noc_internal.h"

// The scan is compiled with cross-statement FMA contraction (the library default is
// -ffp-contract=on, which keeps the interior-point drivers' arithmetic independent of inlining
// context); every kernel that inlines this scan sees the same pragma, so the standalone and the
// persistent KKT solves still round identically.
#pragma clang fp contract(fast)

#ifndef NOC_KKT_WAVES_PER_SIMD
#define NOC_KKT_WAVES_PER_SIMD 2
#endif


namespace noc {

// Diagnostic build only (-DNOC_SCAN_STAMPS, `make stamps-lib`): lane 0 of every wave of the
// standalone scan kernel records s_memrealtime (100 MHz) and s_memtime (shader clock) at the phase
// boundaries into a device table read back by noc_debug_scan_stamps (tools/scan_stamps.py).  The
// stamps go to their own buffer only; no output is computed from them.
#ifdef NOC_SCAN_STAMPS
constexpr int kStampWaves = 65536, kStampSlots = 8;
__device__ long long g_scan_stamps[kStampWaves][kStampSlots][2];
#define NOC_STAMP(i)                                                                         \
  do {                                                                                       \
    const unsigned wv_ = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;                      \
    if ((threadIdx.x & 63) == 0 && wv_ < kStampWaves) {                                      \
      g_scan_stamps[wv_][i][0] = (long long)__builtin_amdgcn_s_memrealtime();                \
      g_scan_stamps[wv_][i][1] = (long long)__builtin_amdgcn_s_memtime();                    \
    }                                                                                        \
  } while (0)
#define NOC_STAMP_DECL do { } while (0)
#elif defined(NOC_PERSIST_PROFILE)
// The persistent solvers' profile build (prof_ipm_persistent.o): cycles between the scan's phase
// boundaries for trajectory 0, lane 0, summed over its solves (noc_debug_phase_cycles slots 9-14:
// in-chunk elements, cross-lane scan, in-chunk Riccati, forward scan, propagation, copy-out)
static __device__ long long g_scan_sub[8];
#define NOC_STAMP_DECL long long stamp_prev_ = 0
#define NOC_STAMP(i)                                                                         \
  do {                                                                                       \
    const long long t_ = clock64();                                                          \
    if ((i) > 0 && traj == 0 && l == 0) g_scan_sub[i] += t_ - stamp_prev_;                   \
    stamp_prev_ = t_;                                                                        \
  } while (0)
#else
#define NOC_STAMP(i) do { } while (0)
#define NOC_STAMP_DECL do { } while (0)
#endif

// Which entries of a stage's A, B may be nonzero: the generic scan takes every one; the persistent
// solver's structure-aware blocks (block_struct.h: BlockStruct) skip the products with structural
// zeros.  nzA / nzB are called with unrolled (compile-time) indices.
template <int NX, int NU>
struct DenseBlocks {
  static constexpr bool nzA(int, int) { return true; }
  static constexpr bool nzB(int, int) { return true; }
};

template <int NX, int NU>
struct StageData {
  Mat<NX, NX> A;
  Mat<NX, NU> B;
  Sym<NX> Q;
  Sym<NU> R;
  Mat<NX, NU> M;
  Vec<NU> r;
  Vec<NX> q;
  Vec<NX> c;
};

typedef __attribute__((address_space(3))) double lds_double;
typedef __attribute__((address_space(3))) noc_dbl2 lds_dbl2;

template <int NX>
struct Elem {
  Mat<NX, NX> A;
  Vec<NX> b;
  Sym<NX> C;
  Vec<NX> nu;
  Sym<NX> J;
};

// tiled load with the cache policy of a last use (LAST: non-temporal) or the default one
template <int E, int L, bool LAST>
NOC_DEV void tload_pol(const double* __restrict__ base, int traj, int j, int l, int cmax, double* dst) {
  if constexpr (LAST) tload_last<E, L>(base, traj, j, l, cmax, dst);
  else tload<E, L>(base, traj, j, l, cmax, dst);
}

// PART: 0 = the whole stage, 1 = everything but Q, 2 = Q only (phase 3 prefetches part 1 of the
// next stage and loads Q, which the Riccati step uses last, at the top of the current one),
// 3 = everything but A, B (the scan instances that keep A, B on chip: kkt_scan_wave_src, AB).
// LAST (phase 3, tiled): the solve's last read of Q, R, M, r, q -- non-temporal, so the lines
// they bring in do not displace blocks still to be re-read (other waves' chunks, this wave's A,
// B, c for phase 4) from the memory-side cache; A, B, c keep the default policy
template <int NX, int NU, int L, bool AFF, bool TILED, int PART = 0, bool LAST = false>
NOC_DEV void load_stage(const KKTArgs& a, int traj, size_t si, int j, int l, int cmax, double reg,
                        StageData<NX, NU>& st) {
  constexpr bool REST = PART != 2, WQ = PART != 1, WAB = REST && PART != 3;
  if constexpr (TILED) {
    if constexpr (WAB) {
      tload<NX * NX, L>(a.A, traj, j, l, cmax, st.A.v);
      tload<NX * NU, L>(a.Bm, traj, j, l, cmax, st.B.v);
    }
    if constexpr (WQ) tload_pol<Sym<NX>::SZ, L, LAST>(a.Q, traj, j, l, cmax, st.Q.v);
    if constexpr (REST) {
      tload_pol<Sym<NU>::SZ, L, LAST>(a.R, traj, j, l, cmax, st.R.v);
      tload_pol<NX * NU, L, LAST>(a.M, traj, j, l, cmax, st.M.v);
      tload_pol<NU, L, LAST>(a.r, traj, j, l, cmax, st.r.v);
      if constexpr (AFF) {
        if (a.q) tload_pol<NX, L, LAST>(a.q, traj, j, l, cmax, st.q.v); else set_zero(st.q);
        if (a.c) tload<NX, L>(a.c, traj, j, l, cmax, st.c.v); else set_zero(st.c);
      }
    }
  } else {
    if constexpr (WAB) {
      gload<NX * NX>(a.A + si * (NX * NX), st.A.v);
      gload<NX * NU>(a.Bm + si * (NX * NU), st.B.v);
    }
    if constexpr (WQ) gload_sym<NX, true>(a.Q + si * (NX * NX), st.Q);
    if constexpr (REST) {
      gload_sym<NU, true>(a.R + si * (NU * NU), st.R);
      gload<NX * NU>(a.M + si * (NX * NU), st.M.v);
      gload<NU>(a.r + si * NU, st.r.v);
      if constexpr (AFF) {
        if (a.q) gload<NX>(a.q + si * NX, st.q.v); else set_zero(st.q);
        if (a.c) gload<NX>(a.c + si * NX, st.c.v); else set_zero(st.c);
      }
    }
  }
  // reg is NOT added here: R + reg*I is formed where R is first used (prepend / riccati_stage),
  // so no arithmetic waits on the R load right after it is issued and a stage's loads can be
  // prefetched a stage ahead (phase 3)
  (void)reg;
}

// A, B (and c) of one stage for the forward pass / map composition
template <int NX, int NU, int L, bool AFF, bool TILED>
NOC_DEV void load_AB(const KKTArgs& a, int traj, size_t si, int j, int l, int cmax,
                     Mat<NX, NX>& A, Mat<NX, NU>& Bm, Vec<NX>& c) {
  set_zero(c);
  if constexpr (TILED) {
    // A, B are read for the last time here (phase 4 / the forward-mode map): non-temporal
    tload_last<NX * NX, L>(a.A, traj, j, l, cmax, A.v);
    tload_last<NX * NU, L>(a.Bm, traj, j, l, cmax, Bm.v);
    if constexpr (AFF) { if (a.c) tload<NX, L>(a.c, traj, j, l, cmax, c.v); }
  } else {
    gload<NX * NX>(a.A + si * (NX * NX), A.v);
    gload<NX * NU>(a.Bm + si * (NX * NU), Bm.v);
    if constexpr (AFF) { if (a.c) gload<NX>(a.c + si * NX, c.v); }
  }
}

// gains K (NU x NX) followed by d (NU), packed as Kk[NU*(NX+1)]
template <int NX, int NU, int L, bool TILED>
NOC_DEV void store_Kd(const KKTArgs& a, int traj, size_t si, int j, int l, int cmax, const double* Kk) {
  if constexpr (TILED) {
    tstore<NU * NX, L>(a.K, traj, j, l, cmax, Kk);
    tstore<NU, L>(a.d, traj, j, l, cmax, Kk + NU * NX);
  } else {
    gstore<NU * NX>(a.K + si * (NU * NX), Kk);
    gstore<NU>(a.d + si * NU, Kk + NU * NX);
  }
}
template <int NX, int NU, int L, bool TILED>
NOC_DEV void load_Kd(const KKTArgs& a, int traj, size_t si, int j, int l, int cmax, double* Kk) {
  if constexpr (TILED) {
    tload<NU * NX, L>(a.K, traj, j, l, cmax, Kk);
    tload<NU, L>(a.d, traj, j, l, cmax, Kk + NU * NX);
  } else {
    gload<NU * NX>(a.K + si * (NU * NX), Kk);
    gload<NU>(a.d + si * NU, Kk + NU * NX);
  }
}

// e <- stage (x) e   (Riccati-form prepend of one stage to the chunk element)
template <int NX, int NU, bool AFF, class ST = DenseBlocks<NX, NU>>
NOC_DEV void prepend(Elem<NX>& e, const StageData<NX, NU>& st, double reg) {
  Mat<NX, NX> JA;
  Mat<NX, NU> JB;
  NOC_UNROLL for (int i = 0; i < NX; ++i) {
    NOC_UNROLL for (int j = 0; j < NX; ++j) {
      double s = 0.0;
      NOC_UNROLL for (int k = 0; k < NX; ++k) if (ST::nzA(k, j)) s += e.J(i, k) * st.A(k, j);
      JA(i, j) = s;
    }
    NOC_UNROLL for (int j = 0; j < NU; ++j) {
      double s = 0.0;
      NOC_UNROLL for (int k = 0; k < NX; ++k) if (ST::nzB(k, j)) s += e.J(i, k) * st.B(k, j);
      JB(i, j) = s;
    }
  }
  Vec<NX> g;
  NOC_UNROLL for (int i = 0; i < NX; ++i) {
    double s = e.nu[i];
    if constexpr (AFF) { NOC_UNROLL for (int k = 0; k < NX; ++k) s += e.J(i, k) * st.c[k]; }
    g[i] = s;
  }
  Sym<NU> W;
  NOC_UNROLL for (int i = 0; i < NU; ++i)
    NOC_UNROLL for (int j = i; j < NU; ++j) {
      double s = (i == j) ? st.R(i, j) + reg : st.R(i, j);  // R + reg I (P:116-118)
      NOC_UNROLL for (int k = 0; k < NX; ++k) if (ST::nzB(k, i)) s += st.B(k, i) * JB(k, j);
      W(i, j) = s;
    }
  // AB = e.A * B
  Mat<NX, NU> AB;
  NOC_UNROLL for (int i = 0; i < NX; ++i)
    NOC_UNROLL for (int j = 0; j < NU; ++j) {
      double s = 0.0;
      NOC_UNROLL for (int k = 0; k < NX; ++k) if (ST::nzB(k, j)) s += e.A(i, k) * st.B(k, j);
      AB(i, j) = s;
    }
  // Y = [Qux | Qu | AB']  (NU x (2NX+1))
  constexpr int NR = 2 * NX + 1;
  double Y[NU][NR];
  Mat<NU, NX> Qux;
  NOC_UNROLL for (int i = 0; i < NU; ++i) {
    NOC_UNROLL for (int j = 0; j < NX; ++j) {
      double s = st.M(j, i);
      NOC_UNROLL for (int k = 0; k < NX; ++k) if (ST::nzA(k, j)) s += JB(k, i) * st.A(k, j);
      Qux(i, j) = s;
      Y[i][j] = s;
    }
    double s = st.r[i];
    NOC_UNROLL for (int k = 0; k < NX; ++k) if (ST::nzB(k, i)) s += st.B(k, i) * g[k];
    Y[i][NX] = s;
    NOC_UNROLL for (int t = 0; t < NX; ++t) Y[i][NX + 1 + t] = AB(t, i);
  }
  (void)ldl_solve<NU, NR>(W, Y);  // Y <- W^-1 Y   (K = -Y[:, :NX], k = -Y[:, NX])
  // J <- Q + A' J A + Qux' K ;  nu <- q + A' g + Qux' k
  Sym<NX> Jn;
  NOC_UNROLL for (int i = 0; i < NX; ++i)
    NOC_UNROLL for (int j = i; j < NX; ++j) {
      double s = st.Q(i, j);
      NOC_UNROLL for (int k = 0; k < NX; ++k) if (ST::nzA(k, i)) s += st.A(k, i) * JA(k, j);
      NOC_UNROLL for (int t = 0; t < NU; ++t) s -= Qux(t, i) * Y[t][j];
      Jn(i, j) = s;
    }
  NOC_UNROLL for (int i = 0; i < NX; ++i) {
    double s = AFF ? st.q[i] : 0.0;
    NOC_UNROLL for (int k = 0; k < NX; ++k) if (ST::nzA(k, i)) s += st.A(k, i) * g[k];
    NOC_UNROLL for (int t = 0; t < NU; ++t) s -= Qux(t, i) * Y[t][NX];
    e.nu[i] = s;
  }
  e.J = Jn;
  // C <- C + AB W^-1 AB'
  NOC_UNROLL for (int i = 0; i < NX; ++i)
    NOC_UNROLL for (int j = i; j < NX; ++j) {
      double s = e.C(i, j);
      NOC_UNROLL for (int t = 0; t < NU; ++t) s += AB(i, t) * Y[t][NX + 1 + j];
      e.C(i, j) = s;
    }
  // F = A + B K, f = B k + c ;  b <- eA f + b ; A <- eA F
  Mat<NX, NX> F;
  Vec<NX> f;
  NOC_UNROLL for (int i = 0; i < NX; ++i) {
    NOC_UNROLL for (int j = 0; j < NX; ++j) {
      double s = st.A(i, j);
      NOC_UNROLL for (int t = 0; t < NU; ++t) if (ST::nzB(i, t)) s -= st.B(i, t) * Y[t][j];
      F(i, j) = s;
    }
    double s = AFF ? st.c[i] : 0.0;
    NOC_UNROLL for (int t = 0; t < NU; ++t) if (ST::nzB(i, t)) s -= st.B(i, t) * Y[t][NX];
    f[i] = s;
  }
  Mat<NX, NX> An;
  NOC_UNROLL for (int i = 0; i < NX; ++i) {
    double sb = e.b[i];
    NOC_UNROLL for (int k = 0; k < NX; ++k) sb += e.A(i, k) * f[k];
    e.b[i] = sb;
    NOC_UNROLL for (int j = 0; j < NX; ++j) {
      double s = 0.0;
      NOC_UNROLL for (int k = 0; k < NX; ++k) s += e.A(i, k) * F(k, j);
      An(i, j) = s;
    }
  }
  e.A = An;
}

// e1 <- e1 (x) e2 at level SK of the reverse Sklansky scan over a segment (e1 covers the earlier
// interval, e2 = the partner's element, the later one).  At level SK the lanes whose bit SK is
// clear combine with the FIRST lane of the upper half of their aligned 2^(SK+1)-lane block; the
// others keep e1 unchanged.  The partner's fields are fetched on the VALU (DPP / v_readlane,
// small_linalg.h: sklansky_rev_fetch) at the segment's full EXEC -- a DPP source lane must be
// active -- in two batches (J, nu first, then A, b, C) so that at most one half of e2 is live;
// the arithmetic then runs under EXEC = the combining lanes only, so the lanes that keep their
// element need neither an identity partner nor selects.
// VALUE_ONLY: every right operand is value-only (the last level: partner l + L/2 covers the end),
// so the result is value-only too and only J, nu are formed (T A1 is the only solve needed); A, b,
// C are zeroed in every lane.
// T = (I + C1 J2)^-1: nx = 2 in closed form (one division; det(I + C1 J2) >= 1 for C1, J2 >= 0);
// larger nx by threshold-checked Gaussian elimination without row exchanges, redone with partial
// pivoting by the whole segment (uniform branch, so the re-fetch is legal) if any lane's check
// fails.
template <int NX, bool VALUE_ONLY, int SK, bool MASKED = (NX <= 2)>
NOC_DEV void combine_sklansky(Elem<NX>& e1) {
  const int lane = (int)__lane_id();
  // MASKED: the arithmetic under EXEC = the combining lanes; else every lane computes, the others
  // with the exact identity element as partner (which leaves them unchanged, at one select per
  // fetched dword): at two waves per SIMD (256 registers) nx = 4 elements are too large to keep
  // old and new values apart across the branches without spilling.  The two-wave segments (512
  // registers) mask every nx: their phase 2 28.4 k -> 26.3 k cycles per wave (512-per-GPU shard);
  // the wide persistent solver, whose cart-pole instance already keeps 116 values in AGPRs, was
  // 1.5-2.5 % slower masked and keeps the selects (profiles/r03/two_wave/)
  const bool act = MASKED ? !(lane & (1 << SK)) : true;
  const bool comb = !(lane & (1 << SK));
  auto fetch = [&](double v, double idv) {
    const double p = sklansky_rev_fetch<SK>(v, lane);
    return MASKED ? p : (comb ? p : idv);
  };
  Sym<NX> J2;
  Vec<NX> nu2;
  auto fetch_value = [&]() {
    NOC_UNROLL for (int i = 0; i < Sym<NX>::SZ; ++i) J2.v[i] = fetch(e1.J.v[i], 0.0);
    NOC_UNROLL for (int i = 0; i < NX; ++i) nu2.v[i] = fetch(e1.nu.v[i], 0.0);
  };
  constexpr int NR = VALUE_ONLY ? NX : 2 * NX + 1;
  double X[NX][NX];
  double Y[NX][NR];
  auto build = [&]() {  // X = I + C1 J2,  Y = [A1 | b1 - C1 nu2 | C1]
    NOC_UNROLL for (int i = 0; i < NX; ++i) {
      NOC_UNROLL for (int j = 0; j < NX; ++j) {
        double s = (i == j) ? 1.0 : 0.0;
        NOC_UNROLL for (int k = 0; k < NX; ++k) s += e1.C(i, k) * J2(k, j);
        X[i][j] = s;
        Y[i][j] = e1.A(i, j);
        if constexpr (!VALUE_ONLY) Y[i][NX + 1 + j] = e1.C(i, j);
      }
      if constexpr (!VALUE_ONLY) {
        double s = e1.b[i];
        NOC_UNROLL for (int k = 0; k < NX; ++k) s -= e1.C(i, k) * nu2[k];
        Y[i][NX] = s;
      }
    }
  };
  fetch_value();
  //  J2A1 = J2 A1,  w = nu2 + J2 b1   (e1.A, e1.b are still the pre-combine values)
  Mat<NX, NX> J2A1;
  Vec<NX> w;
  bool ok = true;
  if (act) {
    build();
    NOC_UNROLL for (int i = 0; i < NX; ++i) {
      double sw = nu2[i];
      NOC_UNROLL for (int k = 0; k < NX; ++k) sw += J2(i, k) * e1.b[k];
      w[i] = sw;
      NOC_UNROLL for (int j = 0; j < NX; ++j) {
        double s = 0.0;
        NOC_UNROLL for (int k = 0; k < NX; ++k) s += J2(i, k) * e1.A(k, j);
        J2A1(i, j) = s;
      }
    }
    if constexpr (NX == 2) solve2_closed<NR>(X, Y);  // Y = [TA | Tb | TC]
    else ok = lu_np_solve<NX, NR>(X, Y);
  }
  if constexpr (NX != 2) {
    if (__any(!ok)) {  // uniform over the segment: J2 / nu2 re-fetched instead of kept live
      fetch_value();
      if (act) {
        build();
        lu_pp_solve<NX, NR>(X, Y);
      }
    }
  }
  if (act) {  // J = J1 + TA' J2 A1 ; nu = nu1 + TA' w
    NOC_UNROLL for (int i = 0; i < NX; ++i) {
      NOC_UNROLL for (int j = i; j < NX; ++j) {
        double s = e1.J(i, j);
        NOC_UNROLL for (int k = 0; k < NX; ++k) s += Y[k][i] * J2A1(k, j);
        e1.J(i, j) = s;
      }
      double s = e1.nu[i];
      NOC_UNROLL for (int k = 0; k < NX; ++k) s += Y[k][i] * w[k];
      e1.nu[i] = s;
    }
  }
  if constexpr (VALUE_ONLY) {
    set_zero(e1.A);
    set_zero(e1.b);
    set_zero(e1.C);
  } else {
    // second batch: the partner's A, b, C (no lane has modified them at this level)
    Mat<NX, NX> A2;
    Vec<NX> b2;
    Sym<NX> C2;
    NOC_UNROLL for (int i = 0; i < NX; ++i)
      NOC_UNROLL for (int j = 0; j < NX; ++j) A2(i, j) = fetch(e1.A(i, j), i == j ? 1.0 : 0.0);
    NOC_UNROLL for (int i = 0; i < NX; ++i) b2.v[i] = fetch(e1.b.v[i], 0.0);
    NOC_UNROLL for (int i = 0; i < Sym<NX>::SZ; ++i) C2.v[i] = fetch(e1.C.v[i], 0.0);
    if (act) {  // A = A2 TA ; b = A2 Tb + b2 ; C = A2 TC A2' + C2
      Mat<NX, NX> T2;  // A2 * TC
      NOC_UNROLL for (int i = 0; i < NX; ++i) {
        double sb = b2[i];
        NOC_UNROLL for (int k = 0; k < NX; ++k) sb += A2(i, k) * Y[k][NX];
        e1.b[i] = sb;
        NOC_UNROLL for (int j = 0; j < NX; ++j) {
          double sa = 0.0, st = 0.0;
          NOC_UNROLL for (int k = 0; k < NX; ++k) {
            sa += A2(i, k) * Y[k][j];
            st += A2(i, k) * Y[k][NX + 1 + j];
          }
          e1.A(i, j) = sa;
          T2(i, j) = st;
        }
      }
      NOC_UNROLL for (int i = 0; i < NX; ++i)
        NOC_UNROLL for (int j = i; j < NX; ++j) {
          double s = C2(i, j);
          NOC_UNROLL for (int k = 0; k < NX; ++k) s += T2(i, k) * A2(j, k);
          e1.C(i, j) = s;
        }
    }
  }
}

// Phase 2 as a reverse Sklansky scan over an L-lane segment: log2(L) levels, partners on the VALU;
// the last level's partner (lane L/2 of the segment) covers the terminal cost -> value-only.
template <int NX, int L, int K = 0, bool MASKED = (NX <= 2)>
NOC_DEV void rev_scan_sklansky(Elem<NX>& e) {
  NOC_ISA_MARK("rev", K);
  if constexpr ((2 << K) < L) {
    combine_sklansky<NX, false, K, MASKED>(e);
    rev_scan_sklansky<NX, L, K + 1, MASKED>(e);
  } else if constexpr ((2 << K) == L) {
    combine_sklansky<NX, true, K, MASKED>(e);
    NOC_ISA_MARK("rev", K + 1);
  }
}

// On-chip slot region of one trajectory (one per L-lane segment of the workgroup): N slots
// of KD = NU*(NX+1) doubles (K_s, d_s after phase 3, then x_s, u_s in phase 4) + x_N.
template <int NX, int NU>
__host__ __device__ constexpr int kd_width() { return NU * (NX + 1); }
template <int NX, int NU, int L>
NOC_DEV double* lds_slots(int N) {
  extern __shared__ __attribute__((aligned(16))) double noc_smem[];
  const int per_traj = (N * kd_width<NX, NU>() + NX + 1) & ~1;
  return noc_smem + (size_t)(threadIdx.x / L) * per_traj;
}
// Two-wave segments (L = 128, one trajectory per 128-thread block): the cross-wave hand-offs go
// through a small LDS region behind the slots (at 0 when the slots are not staged): the later
// wave's value at its start (J, nu), the state at its start, the later wave's pred / feasibility.
template <int NX>
__host__ __device__ constexpr int join_doubles() { return ((NX * (NX + 1)) / 2 + 2 * NX + 2 + 1) & ~1; }
template <int NX, int NU>
NOC_DEV double* lds_join(int N, bool slots_staged) {
  extern __shared__ __attribute__((aligned(16))) double noc_smem[];
  return noc_smem + (slots_staged ? ((N * kd_width<NX, NU>() + NX + 1) & ~1) : 0);
}

// A, B slots of the instances that own a SIMD (AB; a.ab_slots > 0): phase 1 parks each stage's A,
// B of chunk slots j < a.ab_slots in LDS, phases 3 and 4 read them back from there instead of
// re-reading them from the memory-side cache.  Behind the block's K, d slot regions (and the
// two-wave join region), one region per wave: [slot j][16-byte granule g][lane] -- every access a
// conflict-free ds_read / ds_write_b128 of the lane's own granule.
template <int NX, int NU>
__host__ __device__ constexpr int ab_granules() { return (NX * NX + NX * NU) / 2; }
template <int NX, int NU>
__host__ __device__ constexpr bool ab_supported() { return (NX * NX) % 2 == 0 && (NX * NU) % 2 == 0; }
template <int NX, int NU>
NOC_DEV lds_double* lds_ab(int lds_base, int ab_slots) {
  extern __shared__ __attribute__((aligned(16))) double noc_smem[];
  return (lds_double*)(noc_smem + lds_base + (size_t)(threadIdx.x / 64) * ab_slots * ab_granules<NX, NU>() * 128 +
                      2 * (threadIdx.x & 63));
}

template <int NX, int NU>
NOC_DEV void ab_store(lds_double* lab, int j, const Mat<NX, NX>& A, const Mat<NX, NU>& Bm) {
  lds_double* p = lab + j * ab_granules<NX, NU>() * 128;
  NOC_UNROLL for (int q = 0; q < NX * NX / 2; ++q) {
    noc_dbl2 v;
    v.x = A.v[2 * q];
    v.y = A.v[2 * q + 1];
    *reinterpret_cast<lds_dbl2*>(p + q * 128) = v;
  }
  NOC_UNROLL for (int q = 0; q < NX * NU / 2; ++q) {
    noc_dbl2 v;
    v.x = Bm.v[2 * q];
    v.y = Bm.v[2 * q + 1];
    *reinterpret_cast<lds_dbl2*>(p + (NX * NX / 2 + q) * 128) = v;
  }
}
template <int NX, int NU>
NOC_DEV void ab_load(const lds_double* lab, int j, Mat<NX, NX>& A, Mat<NX, NU>& Bm) {
  const lds_double* p = lab + j * ab_granules<NX, NU>() * 128;
  NOC_UNROLL for (int q = 0; q < NX * NX / 2; ++q) {
    const noc_dbl2 v = *reinterpret_cast<const lds_dbl2*>(p + q * 128);
    A.v[2 * q] = v.x;
    A.v[2 * q + 1] = v.y;
  }
  NOC_UNROLL for (int q = 0; q < NX * NU / 2; ++q) {
    const noc_dbl2 v = *reinterpret_cast<const lds_dbl2*>(p + (NX * NX / 2 + q) * 128);
    Bm.v[2 * q] = v.x;
    Bm.v[2 * q + 1] = v.y;
  }
}

// e1 <- e1 (x) (value-only e2 = (J2, nu2)): the true value function at e1's start given the value
// at its end (the VALUE_ONLY branch of combine_sklansky with the partner given explicitly; the
// cross-wave joins of the two-wave scan and of the wide persistent solver, ipm_wide.hip)
template <int NX>
NOC_DEV void apply_value(Elem<NX>& e1, const Sym<NX>& J2, const Vec<NX>& nu2) {
  double X[NX][NX], Y[NX][NX];
  auto build = [&]() {
    NOC_UNROLL for (int i = 0; i < NX; ++i)
      NOC_UNROLL for (int j = 0; j < NX; ++j) {
        double s = (i == j) ? 1.0 : 0.0;
        NOC_UNROLL for (int k = 0; k < NX; ++k) s += e1.C(i, k) * J2(k, j);
        X[i][j] = s;
        Y[i][j] = e1.A(i, j);
      }
  };
  build();
  Mat<NX, NX> J2A1;
  Vec<NX> w;
  NOC_UNROLL for (int i = 0; i < NX; ++i) {
    double sw = nu2[i];
    NOC_UNROLL for (int k = 0; k < NX; ++k) sw += J2(i, k) * e1.b[k];
    w[i] = sw;
    NOC_UNROLL for (int j = 0; j < NX; ++j) {
      double s = 0.0;
      NOC_UNROLL for (int k = 0; k < NX; ++k) s += J2(i, k) * e1.A(k, j);
      J2A1(i, j) = s;
    }
  }
  // nx = 2: closed form (det(I + C1 J2) >= 1), as combine_sklansky; else the threshold-checked
  // elimination with a per-lane fallback (no shuffles here, so no uniformity is needed)
  if constexpr (NX == 2) {
    solve2_closed<NX>(X, Y);
  } else if (!lu_np_solve<NX, NX>(X, Y)) {
    build();
    lu_pp_solve<NX, NX>(X, Y);
  }
  NOC_UNROLL for (int i = 0; i < NX; ++i) {
    NOC_UNROLL for (int j = i; j < NX; ++j) {
      double s = e1.J(i, j);
      NOC_UNROLL for (int k = 0; k < NX; ++k) s += Y[k][i] * J2A1(k, j);
      e1.J(i, j) = s;
    }
    double s = e1.nu[i];
    NOC_UNROLL for (int k = 0; k < NX; ++k) s += Y[k][i] * w[k];
    e1.nu[i] = s;
  }
  set_zero(e1.A);
  set_zero(e1.b);
  set_zero(e1.C);
}

// Where the scan gets a stage's LQ blocks: from the KKTArgs arrays (tiled or natural layout).
// The persistent solver passes a source that recomputes them from (x, u, lambda) instead.
template <int NX, int NU, int L, bool AFF, bool TILED>
struct ArgsSrc {
  using Struct = DenseBlocks<NX, NU>;
  const KKTArgs& a;
  int traj, l, cmax;
  size_t tN;
  NOC_DEV void stage(int s, int j, double reg, StageData<NX, NU>& st) const {
    load_stage<NX, NU, L, AFF, TILED>(a, traj, tN + s, j, l, cmax, reg, st);
  }
  template <int PART, bool LAST = false>
  NOC_DEV void stage_part(int s, int j, double reg, StageData<NX, NU>& st) const {
    load_stage<NX, NU, L, AFF, TILED, PART, LAST>(a, traj, tN + s, j, l, cmax, reg, st);
  }
  NOC_DEV void stage_last(int s, int j, double reg, StageData<NX, NU>& st) const {  // phase 3
    load_stage<NX, NU, L, AFF, TILED, 0, true>(a, traj, tN + s, j, l, cmax, reg, st);
  }
  NOC_DEV void ab(int s, int j, Mat<NX, NX>& A, Mat<NX, NU>& Bm, Vec<NX>& c) const {
    load_AB<NX, NU, L, AFF, TILED>(a, traj, tN + s, j, l, cmax, A, Bm, c);
  }
  NOC_DEV void cvec(int s, int j, Vec<NX>& c) const {  // the affine term alone (a.c set)
    if constexpr (TILED) tload<NX, L>(a.c, traj, j, l, cmax, c.v);
    else gload<NX>(a.c + (tN + s) * NX, c.v);
  }
};

// The whole KKT solve of trajectory `traj` by lane `l` of its L-lane segment (the kernel below;
// also called by the persistent interior-point solver, ipm_persistent.hip).  With lds_out set and
// dx = du = NULL the step stays in the LDS slots (x_s at slot s, u_s after it, x_N at slot N).
// CACHE > 0 (caller guarantees every chunk has <= CACHE stages): the lane's chunk is loaded into
// registers once, all loads issued up front, and phases 1, 3 and 4 read it from there -- one pass
// over the blocks and one exposed memory latency instead of three dependent load chains (small
// nx with one- or two-stage chunks, c2).
// HANDOFF: phase 3 hands the chunk's first stage (A, B) to phase 4 in registers (standalone
// scan: −1 stage of phase 4's re-reads); also inside the persistent solver since round 5, whose
// solve is bound by its workspace traffic (profiles/r05/handoff_persist/).
// BIG: the instance owns a SIMD (512 registers): the combines run masked (no identity partner).
// AB (default: the 512-register L = 32 / 64 instances, BIG, where one wave per SIMD leaves 40 KB of
// LDS per wave): A, B of chunk slots j < a.ab_slots stay in LDS from phase 1 to phases 3 and 4
// (lds_ab); a.ab_slots = 0 turns it off at run time.  Not in the two-wave segments (L = 128): their
// re-reads are L2 hits already, and the slots measured +2.5 % there (profiles/r05/ab_slots/).
// IO0: reg, pred and feasible are one slot each (a.reg[0], a.pred[0], a.feasible[0]) instead of
// per-trajectory arrays -- the persistent solver's speculative candidates (ipm_persistent.hip: SPEC)
// each solve the same blocks with their own regularisation and keep those three in LDS.
template <int NX, int NU, int L, bool AFF, bool TILED, class SRC, int CACHE = 0, bool HANDOFF = true,
          bool BIG = false, bool NT3 = false, bool AB = (BIG && ab_supported<NX, NU>()), bool IO0 = false>
NOC_DEV void kkt_scan_wave_src(const KKTArgs& a, const int traj, const int l, const SRC& src) {
  constexpr int KD = kd_width<NX, NU>();
  using ST = typename SRC::Struct;  // structural zeros of A, B (DenseBlocks: none)
  if (traj >= a.B) return;                     // uniform over the segment
  if (a.active && a.active[traj] == 0) return;  // uniform over the segment
  const int N = a.N;
  const int base = N / L, rem = N % L;
  const int len = base + (l < rem ? 1 : 0);
  const int start = l * base + (l < rem ? l : rem);
  const bool last = (l == L - 1);
  const int io = IO0 ? 0 : traj;
  const double reg = a.reg ? a.reg[io] : 0.0;
  const size_t tN = (size_t)traj * N;
  const int cmax = base + (rem ? 1 : 0);
  // LW lanes of one wave in the segment, W waves per segment (W = 2: L = 128, the horizon split
  // over the two waves of a 128-thread block; the wave-level scans run per wave and are joined
  // through LDS -- for batches too small to give every SIMD a wave at L = 64)
  constexpr int LW = L > 64 ? 64 : L;
  constexpr int W = L / LW;
  static_assert(W == 1 || W == 2, "segments of up to two waves");
  const int wv = l / LW, lw = l % LW;
  double* join = nullptr;
  if constexpr (W > 1) join = lds_join<NX, NU>(N, a.lds_out != 0);
  (void)wv;
  (void)lw;
  (void)join;
  lds_double* lab = nullptr;
  int abn = 0;  // chunk slots whose A, B are parked in LDS
  if constexpr (AB) {
    // (MODE_FWD has no phase 1 to park them; ablation bit 4 reads other trajectories' blocks;
    // ablation bit 6 turns the slots off -- results identical, tests/test_kkt_gpu.py)
    abn = (CACHE == 0 && a.mode != MODE_FWD && !(a.ablate & (16 | 64))) ? a.ab_slots : 0;
    if (abn > 0) lab = lds_ab<NX, NU>(a.lds_base, a.ab_slots);
  }
  NOC_STAMP_DECL;
  NOC_STAMP(0);
  StageData<NX, NU> cache[CACHE > 0 ? CACHE : 1];
  if constexpr (CACHE > 0) {
    if (a.mode != MODE_FWD) {
      NOC_UNROLL for (int jj = 0; jj < CACHE; ++jj)
        if (jj < len) src.stage(start + jj, jj, reg, cache[jj]);
    }
  }

  Mat<NX, NX> Phi;
  Vec<NX> phi;
  // A, B (and c) of the chunk's first stage: phase 3 reads them last, phase 4 first -- handed over
  // in registers instead of re-read (one stage of phase 4's A, B stream and its first exposed load)
  Mat<NX, NX> hA;
  Mat<NX, NU> hB;
  Vec<NX> hc;
  bool handed = false;
  // ablation bit 4 (timing only, results wrong): phases 3 and 4 re-read the blocks of trajectory
  // traj & 1 instead of their own -- an L2-resident working set, so the time they lose against
  // the full kernel is the cost of re-reading the blocks from beyond L2
  SRC src_re = src;
  if (a.ablate & 16) { src_re.traj = traj & 1; src_re.tN = (size_t)(traj & 1) * N; }
  if (a.mode != MODE_FWD) {
    // ---------------- phase 1: in-chunk element ----------------
    Elem<NX> e;
    set_zero(e.b);
    set_zero(e.C);
    if (last) {  // terminal cost (0, 0, 0, p, P)
      set_zero(e.A);
      set_zero(e.nu);
      gload_sym<NX, true>(a.P + (size_t)traj * NX * NX, e.J);
      if constexpr (AFF) { if (a.p) gload<NX>(a.p + (size_t)traj * NX, e.nu.v); }
    } else {
      set_identity(e.A);
      set_zero(e.nu);
      set_zero(e.J);
    }
    if constexpr (CACHE > 0) {
      NOC_UNROLL for (int jj = CACHE - 1; jj >= 0; --jj)
        if (jj < len) prepend<NX, NU, AFF, ST>(e, cache[jj], reg);
    } else {
      for (int s = start + len - 1; s >= start; --s) {
        StageData<NX, NU> st;
        src.stage(s, s - start, reg, st);
        if constexpr (AB) { if (s - start < abn) ab_store<NX, NU>(lab, s - start, st.A, st.B); }
        prepend<NX, NU, AFF, ST>(e, st, reg);
      }
    }
    NOC_STAMP(1); NOC_ISA_MARK("phase", 1);
    // ---------------- phase 2: reverse Sklansky scan across lanes ----------------
    if constexpr (W == 1) {
      if (!(a.ablate & 1)) rev_scan_sklansky<NX, L, 0, (NX <= 2 || BIG)>(e);
    } else {
      if (!(a.ablate & 1)) {
        // per wave; wave 1 ends at the terminal cost (value-only last level), wave 0 at wave 1's
        // start (full last level: its elements are joined below)
        combine_sklansky<NX, false, 0, true>(e);
        combine_sklansky<NX, false, 1, true>(e);
        combine_sklansky<NX, false, 2, true>(e);
        combine_sklansky<NX, false, 3, true>(e);
        combine_sklansky<NX, false, 4, true>(e);
        if (wv == W - 1) combine_sklansky<NX, true, 5, true>(e);  // wave-uniform branch
        else combine_sklansky<NX, false, 5, true>(e);
      }
      // join: wave 1's value at its start, applied to every lane of wave 0
      if (wv == 1 && lw == 0) {
        NOC_UNROLL for (int i = 0; i < Sym<NX>::SZ; ++i) join[i] = e.J.v[i];
        NOC_UNROLL for (int i = 0; i < NX; ++i) join[Sym<NX>::SZ + i] = e.nu.v[i];
      }
      __syncthreads();
      if (wv == 0) {
        Sym<NX> Jw;
        Vec<NX> nw;
        NOC_UNROLL for (int i = 0; i < Sym<NX>::SZ; ++i) Jw.v[i] = join[i];
        NOC_UNROLL for (int i = 0; i < NX; ++i) nw.v[i] = join[Sym<NX>::SZ + i];
        apply_value<NX>(e, Jw, nw);
      }
    }
    if (a.ablate & 4) {  // phase 1 (+2) only: keep the element alive, skip the rest
      if (a.pred) a.pred[io] = e.J(0, 0) + e.A(0, 0) + e.C(0, 0) + e.nu[0] + e.b[0];
      return;
    }
    NOC_STAMP(2); NOC_ISA_MARK("phase", 2);
    // ---------------- phase 3: in-chunk Riccati from the true boundary ----------------
    Sym<NX> S;
    Vec<NX> v;
    wave_shift_down1<Sym<NX>::SZ>(e.J.v, S.v);  // lane l+1's value; the segment's last lane:
    wave_shift_down1<NX>(e.nu.v, v.v);          // overwritten below (terminal / join)
    if constexpr (W > 1) {  // wave 0's last lane ends where wave 1 starts
      if (wv == 0 && lw == LW - 1) {
        NOC_UNROLL for (int i = 0; i < Sym<NX>::SZ; ++i) S.v[i] = join[i];
        NOC_UNROLL for (int i = 0; i < NX; ++i) v.v[i] = join[Sym<NX>::SZ + i];
      }
    }
    if (last) {  // boundary of the last chunk: the terminal cost itself (reloaded, not kept live)
      gload_sym<NX, true>(a.P + (size_t)traj * NX * NX, S);
      set_zero(v);
      if constexpr (AFF) { if (a.p) gload<NX>(a.p + (size_t)traj * NX, v.v); }
      if (a.S) gstore_sym<NX>(a.S + (tN + traj + N) * (NX * NX), S);
      if (a.v) gstore<NX>(a.v + (tN + traj + N) * NX, v.v);
    }
    set_identity(Phi);
    set_zero(phi);
    double pred = 0.0;
    int feas = 1;
    double* skd = lds_slots<NX, NU, L>(N);  // K, d stay on chip for phase 4 when staged
    // phase 3's re-read of a stage: the last use of Q, R, M, r, q -- non-temporal in the NT3
    // instances (the launcher's cache policy, kkt_nt3)
    auto stage3 = [&](int s, StageData<NX, NU>& st) {
      if constexpr (NT3) src_re.stage_last(s, s - start, reg, st);
      else src_re.stage(s, s - start, reg, st);
    };
    auto riccati_stage = [&](const int s, const StageData<NX, NU>& st) {
      Mat<NX, NX> SA;
      Mat<NX, NU> SB;
      NOC_UNROLL for (int i = 0; i < NX; ++i) {
        NOC_UNROLL for (int j = 0; j < NX; ++j) {
          double t = 0.0;
          NOC_UNROLL for (int k = 0; k < NX; ++k) if (ST::nzA(k, j)) t += S(i, k) * st.A(k, j);
          SA(i, j) = t;
        }
        NOC_UNROLL for (int j = 0; j < NU; ++j) {
          double t = 0.0;
          NOC_UNROLL for (int k = 0; k < NX; ++k) if (ST::nzB(k, j)) t += S(i, k) * st.B(k, j);
          SB(i, j) = t;
        }
      }
      Vec<NX> g;
      NOC_UNROLL for (int i = 0; i < NX; ++i) {
        double t = v[i];
        if constexpr (AFF) { NOC_UNROLL for (int k = 0; k < NX; ++k) t += S(i, k) * st.c[k]; }
        g[i] = t;
      }
      Sym<NU> Quu;
      NOC_UNROLL for (int i = 0; i < NU; ++i)
        NOC_UNROLL for (int j = i; j < NU; ++j) {
          double t = (i == j) ? st.R(i, j) + reg : st.R(i, j);  // R + reg I (P:116-118)
          NOC_UNROLL for (int k = 0; k < NX; ++k) if (ST::nzB(k, i)) t += st.B(k, i) * SB(k, j);
          Quu(i, j) = t;
        }
      constexpr int NR = NX + 1;
      double Y[NU][NR];
      Mat<NU, NX> Qux;
      Vec<NU> Qu;
      NOC_UNROLL for (int i = 0; i < NU; ++i) {
        NOC_UNROLL for (int j = 0; j < NX; ++j) {
          double t = st.M(j, i);
          NOC_UNROLL for (int k = 0; k < NX; ++k) if (ST::nzA(k, j)) t += SB(k, i) * st.A(k, j);
          Qux(i, j) = t;
          Y[i][j] = t;
        }
        double t = st.r[i];
        NOC_UNROLL for (int k = 0; k < NX; ++k) if (ST::nzB(k, i)) t += st.B(k, i) * g[k];
        Qu[i] = t;
        Y[i][NX] = t;
      }
      feas &= ldl_solve<NU, NR>(Quu, Y) ? 1 : 0;
      // K = -Y[:, :NX], k = -Y[:, NX]
      double Kk[NU * (NX + 1)];
      NOC_UNROLL for (int i = 0; i < NU; ++i) {
        NOC_UNROLL for (int j = 0; j < NX; ++j) Kk[i * NX + j] = -Y[i][j];
        Kk[NU * NX + i] = -Y[i][NX];
      }
      if (a.lds_out) {
        NOC_UNROLL for (int i = 0; i < NU * (NX + 1); ++i) skd[s * KD + i] = Kk[i];
      }
      if (a.K) store_Kd<NX, NU, L, TILED>(a, traj, tN + s, s - start, l, cmax, Kk);
      // dV = k'Qu + 1/2 k'Quu k   (noc/seq_interior_point_newton.py:63)
      NOC_UNROLL for (int i = 0; i < NU; ++i) {
        const double ki = Kk[NU * NX + i];
        double qk = 0.0;
        NOC_UNROLL for (int j = 0; j < NU; ++j) qk += Quu(i, j) * Kk[NU * NX + j];
        pred += ki * Qu[i] + 0.5 * ki * qk;
      }
      // S <- Q + A' S A + Qux' K ; v <- q + A' g + Qux' k
      Sym<NX> Sn;
      NOC_UNROLL for (int i = 0; i < NX; ++i)
        NOC_UNROLL for (int j = i; j < NX; ++j) {
          double t = st.Q(i, j);
          NOC_UNROLL for (int k = 0; k < NX; ++k) if (ST::nzA(k, i)) t += st.A(k, i) * SA(k, j);
          NOC_UNROLL for (int u = 0; u < NU; ++u) t += Qux(u, i) * Kk[u * NX + j];
          Sn(i, j) = t;
        }
      NOC_UNROLL for (int i = 0; i < NX; ++i) {
        double t = AFF ? st.q[i] : 0.0;
        NOC_UNROLL for (int k = 0; k < NX; ++k) if (ST::nzA(k, i)) t += st.A(k, i) * g[k];
        NOC_UNROLL for (int u = 0; u < NU; ++u) t += Qux(u, i) * Kk[NU * NX + u];
        v[i] = t;
      }
      S = Sn;
      if (a.S) gstore_sym<NX>(a.S + (tN + traj + s) * (NX * NX), S);
      if (a.v) gstore<NX>(a.v + (tN + traj + s) * NX, v.v);
      // closed-loop map of this stage: F = A + B K, f = B k + c ; phi += Phi f ; Phi <- Phi F
      Mat<NX, NX> F;
      Vec<NX> f;
      NOC_UNROLL for (int i = 0; i < NX; ++i) {
        NOC_UNROLL for (int j = 0; j < NX; ++j) {
          double t = st.A(i, j);
          NOC_UNROLL for (int u = 0; u < NU; ++u) if (ST::nzB(i, u)) t += st.B(i, u) * Kk[u * NX + j];
          F(i, j) = t;
        }
        double t = AFF ? st.c[i] : 0.0;
        NOC_UNROLL for (int u = 0; u < NU; ++u) if (ST::nzB(i, u)) t += st.B(i, u) * Kk[NU * NX + u];
        f[i] = t;
      }
      Mat<NX, NX> Pn;
      NOC_UNROLL for (int i = 0; i < NX; ++i) {
        double t = phi[i];
        NOC_UNROLL for (int k = 0; k < NX; ++k) t += Phi(i, k) * f[k];
        phi[i] = t;
        NOC_UNROLL for (int j = 0; j < NX; ++j) {
          double u = 0.0;
          NOC_UNROLL for (int k = 0; k < NX; ++k) u += Phi(i, k) * F(k, j);
          Pn(i, j) = u;
        }
      }
      Phi = Pn;
    };
    if constexpr (CACHE > 0) {
      NOC_UNROLL for (int jj = CACHE - 1; jj >= 0; --jj)
        if (jj < len) riccati_stage(start + jj, cache[jj]);
    } else {
      // not software pipelined: prefetching stage s-1 during stage s (registers) was measured
      // slower (phase 3 44k -> 60k cycles per wave at c3: the prefetch spills, and the phase runs
      // at the memory-side-cache rate, not at a per-stage latency, tools/scan_stamps.py)
      bool split = false;
      if constexpr (AB) split = abn > 0;
      if (split) {
        // AB: the chunk's slots j >= abn re-read whole, then j < abn with A, B from LDS -- two
        // branch-free loops; no hand-off (phase 4 reads slot 0's A, B from LDS as well)
        if constexpr (AB) {
          const int jl = len < abn ? len : abn;
          for (int s = start + len - 1; s >= start + jl; --s) {
            StageData<NX, NU> st;
            stage3(s, st);
            riccati_stage(s, st);
          }
          for (int s = start + jl - 1; s >= start; --s) {
            StageData<NX, NU> st;
            src_re.template stage_part<3, NT3>(s, s - start, reg, st);
            ab_load<NX, NU>(lab, s - start, st.A, st.B);
            riccati_stage(s, st);
          }
        }
      } else if constexpr (HANDOFF) {
        for (int s = start + len - 1; s > start; --s) {
          StageData<NX, NU> st;
          stage3(s, st);
          riccati_stage(s, st);
        }
        if (len > 0) {  // the chunk's first stage, peeled: its A, B (c) go on to phase 4
          StageData<NX, NU> st;
          stage3(start, st);
          riccati_stage(start, st);
          hA = st.A;
          hB = st.B;
          if constexpr (AFF) hc = st.c; else set_zero(hc);
          handed = a.mode == MODE_FULL && !(a.ablate & 32);
        }
      } else {
        for (int s = start + len - 1; s >= start; --s) {
          StageData<NX, NU> st;
          stage3(s, st);
          riccati_stage(s, st);
        }
      }
    }
    // segment reductions: pred = sum, feasible = and (VALU butterfly, small_linalg.h)
    segment_sum_and<LW>(pred, feas, (int)__lane_id());
    if constexpr (W > 1) {  // wave 0's sum + wave 1's sum
      constexpr int PO = Sym<NX>::SZ + 2 * NX;
      if (wv == 1 && lw == 0) {
        join[PO] = pred;
        join[PO + 1] = feas ? 1.0 : 0.0;
      }
      __syncthreads();
      if (l == 0) {
        pred += join[PO];
        feas &= join[PO + 1] != 0.0 ? 1 : 0;
      }
    }
    if (l == 0) {
      if (a.pred) a.pred[io] = pred;
      if (a.feasible) a.feasible[io] = feas;
    }
    NOC_STAMP(3); NOC_ISA_MARK("phase", 3);
    if (a.mode == MODE_BWD || (a.ablate & 2)) return;
  } else {
    // MODE_FWD: gains are inputs; compose the chunk's closed-loop map from A, B, K, d
    set_identity(Phi);
    set_zero(phi);
    for (int s = start + len - 1; s >= start; --s) {
      Mat<NX, NX> A;
      Mat<NX, NU> Bm;
      double Kk[NU * (NX + 1)];
      Vec<NX> cc;
      src.ab(s, s - start, A, Bm, cc);
      load_Kd<NX, NU, L, TILED>(a, traj, tN + s, s - start, l, cmax, Kk);
      Mat<NX, NX> F;
      Vec<NX> f;
      NOC_UNROLL for (int i = 0; i < NX; ++i) {
        NOC_UNROLL for (int j = 0; j < NX; ++j) {
          double t = A(i, j);
          NOC_UNROLL for (int u = 0; u < NU; ++u) if (ST::nzB(i, u)) t += Bm(i, u) * Kk[u * NX + j];
          F(i, j) = t;
        }
        double t = cc[i];
        NOC_UNROLL for (int u = 0; u < NU; ++u) if (ST::nzB(i, u)) t += Bm(i, u) * Kk[NU * NX + u];
        f[i] = t;
      }
      Mat<NX, NX> Pn;
      NOC_UNROLL for (int i = 0; i < NX; ++i) {
        double t = phi[i];
        NOC_UNROLL for (int k = 0; k < NX; ++k) t += Phi(i, k) * f[k];
        phi[i] = t;
        NOC_UNROLL for (int j = 0; j < NX; ++j) {
          double u = 0.0;
          NOC_UNROLL for (int k = 0; k < NX; ++k) u += Phi(i, k) * F(k, j);
          Pn(i, j) = u;
        }
      }
      Phi = Pn;
    }
  }

  // ---------------- phase 4: forward affine scan + chunk propagation ----------------
  Vec<NX> x0;
  set_zero(x0);
  if (a.x0) gload<NX>(a.x0 + (size_t)traj * NX, x0.v);
  if (l == 0) {
    NOC_UNROLL for (int i = 0; i < NX; ++i) {
      double t = phi[i];
      NOC_UNROLL for (int k = 0; k < NX; ++k) t += Phi(i, k) * x0[k];
      phi[i] = t;
    }
    set_zero(Phi);
  }
  affine_prefix_sklansky<NX, LW>(Phi, phi);  // partners on the VALU (small_linalg.h)
  Vec<NX> x;
  wave_shift_up1<NX>(phi.v, x.v);  // lane l-1's prefix; segment starts: x0 / the join below
  if (l == 0) x = x0;
  if constexpr (W > 1) {
    // wave 0's prefixes start from the constant map of lane 0, so its last one is the state at
    // wave 1's start; wave 1 applies its own (non-constant) prefixes to it
    constexpr int XO = Sym<NX>::SZ + NX;
    if (wv == 0 && lw == LW - 1) NOC_UNROLL for (int i = 0; i < NX; ++i) join[XO + i] = phi[i];
    Mat<NX, NX> oP;
    if (wv == 1) wave_shift_up1<NX * NX>(Phi.v, oP.v);  // wave-uniform branch; lane 0 unused
    __syncthreads();
    if (wv == 1) {
      Vec<NX> xw;
      NOC_UNROLL for (int i = 0; i < NX; ++i) xw[i] = join[XO + i];
      if (lw == 0) {
        x = xw;
      } else {
        NOC_UNROLL for (int i = 0; i < NX; ++i) {
          double t = x[i];
          NOC_UNROLL for (int k = 0; k < NX; ++k) t += oP(i, k) * xw[k];
          x[i] = t;
        }
      }
    }
  }
  NOC_STAMP(4); NOC_ISA_MARK("phase", 4);
  // dx/du rows go through LDS (slot s of the trajectory's region holds K_s, d_s from phase 3 and
  // is overwritten by x_s, u_s here) and leave as whole contiguous rows: per-lane direct stores
  // would touch one cache line per lane per store instruction.
  double* slot = lds_slots<NX, NU, L>(N);
  const bool via_lds = a.lds_out != 0;
  const bool kd_lds = via_lds && a.mode == MODE_FULL;
  Mat<NX, NX> nA;
  Mat<NX, NU> nB;
  double nK[NU * (NX + 1)];
  Vec<NX> nc;
  auto fetch = [&](int s) {
    src_re.ab(s, s - start, nA, nB, nc);
    if (kd_lds) {
      NOC_UNROLL for (int i = 0; i < NU * (NX + 1); ++i) nK[i] = slot[s * KD + i];
    } else {
      load_Kd<NX, NU, L, TILED>(a, traj, tN + s, s - start, l, cmax, nK);
    }
  };
  auto fwd_stage = [&](const int s, const Mat<NX, NX>& A, const Mat<NX, NU>& Bm, const Vec<NX>& cc,
                       const double* Kk) {
    Vec<NU> u;
    NOC_UNROLL for (int i = 0; i < NU; ++i) {
      double t = Kk[NU * NX + i];
      NOC_UNROLL for (int k = 0; k < NX; ++k) t += Kk[i * NX + k] * x[k];
      u[i] = t;
    }
    if (via_lds) {
      NOC_UNROLL for (int i = 0; i < NX; ++i) slot[s * KD + i] = x[i];
      NOC_UNROLL for (int i = 0; i < NU; ++i) slot[s * KD + NX + i] = u[i];
    } else {
      if (a.dx) gstore<NX>(a.dx + (tN + traj + s) * NX, x.v);
      if (a.du) gstore<NU>(a.du + (tN + s) * NU, u.v);
    }
    Vec<NX> xn;
    NOC_UNROLL for (int i = 0; i < NX; ++i) {
      double t = cc[i];
      NOC_UNROLL for (int k = 0; k < NX; ++k) if (ST::nzA(i, k)) t += A(i, k) * x[k];
      NOC_UNROLL for (int j = 0; j < NU; ++j) if (ST::nzB(i, j)) t += Bm(i, j) * u[j];
      xn[i] = t;
    }
    x = xn;
  };
  bool from_cache = false;
  if constexpr (CACHE > 0) from_cache = a.mode != MODE_FWD;
  if (from_cache) {
    if constexpr (CACHE > 0) {
      NOC_UNROLL for (int jj = 0; jj < CACHE; ++jj) {
        if (jj < len) {
          const int s = start + jj;
          double Kk[NU * (NX + 1)];
          if (kd_lds) {
            NOC_UNROLL for (int i = 0; i < NU * (NX + 1); ++i) Kk[i] = slot[s * KD + i];
          } else {
            load_Kd<NX, NU, L, TILED>(a, traj, tN + s, jj, l, cmax, Kk);
          }
          Vec<NX> cc;
          if constexpr (AFF) cc = cache[jj].c; else set_zero(cc);
          fwd_stage(s, cache[jj].A, cache[jj].B, cc, Kk);
        }
      }
    }
  } else {
    // AB: the chunk's first slots with A, B from LDS (no prefetch needed), then the rest as below
    int s0 = start;
    if constexpr (AB) {
      if (abn > 0) {
        const int jl = len < abn ? len : abn;
        for (int s = start; s < start + jl; ++s) {
          Mat<NX, NX> A;
          Mat<NX, NU> Bm;
          Vec<NX> cc;
          ab_load<NX, NU>(lab, s - start, A, Bm);
          set_zero(cc);
          if constexpr (AFF) { if (a.c) src_re.cvec(s, s - start, cc); }
          double Kk[NU * (NX + 1)];
          if (kd_lds) {
            NOC_UNROLL for (int i = 0; i < NU * (NX + 1); ++i) Kk[i] = slot[s * KD + i];
          } else {
            load_Kd<NX, NU, L, TILED>(a, traj, tN + s, s - start, l, cmax, Kk);
          }
          fwd_stage(s, A, Bm, cc, Kk);
        }
        s0 = start + jl;
      }
    }
    // one stage prefetched (a two-deep prefetch measured no faster: the propagation runs at the
    // rate the A, B re-reads stream at, not at the per-stage latency)
    if (s0 < start + len) {
      if (handed && s0 == start) {  // stage `start` from phase 3's registers; only its K, d from LDS
        nA = hA;
        nB = hB;
        nc = hc;
        if (kd_lds) {
          NOC_UNROLL for (int i = 0; i < NU * (NX + 1); ++i) nK[i] = slot[start * KD + i];
        } else {
          load_Kd<NX, NU, L, TILED>(a, traj, tN + start, 0, l, cmax, nK);
        }
      } else {
        fetch(s0);
      }
    }
    for (int s = s0; s < start + len; ++s) {
      const Mat<NX, NX> A = nA;
      const Mat<NX, NU> Bm = nB;
      const Vec<NX> cc = nc;
      double Kk[NU * (NX + 1)];
      NOC_UNROLL for (int i = 0; i < NU * (NX + 1); ++i) Kk[i] = nK[i];
      if (s + 1 < start + len) fetch(s + 1);  // prefetch the next stage
      fwd_stage(s, A, Bm, cc, Kk);
    }
  }
  NOC_STAMP(5); NOC_ISA_MARK("phase", 5);
  if (!via_lds) {
    if (last && a.dx) gstore<NX>(a.dx + (tN + traj + N) * NX, x.v);
    return;
  }
  if (last) NOC_UNROLL for (int i = 0; i < NX; ++i) slot[N * KD + i] = x[i];
  // orders the segment's LDS writes (one or two waves) before its reads.  With several
  // independent waves per workgroup (kkt_waves_per_block) every wave of the block reaches this one
  // barrier: the scan kernel sends waves without a trajectory to it too (kkt_scan_kernel).  (A
  // wave-scope fence instead -- no cross-wave wait -- measured 0.5-1.5 % slower at c3 and the
  // 512 shard, profiles/r04/fence_ab/.)
  __syncthreads();
  if (a.dx) {
    double* dst = a.dx + (tN + traj) * NX;
    if constexpr (NX % 2 == 0) {
      constexpr int H = NX / 2;
      double2* dst2 = reinterpret_cast<double2*>(dst);
      for (int i = l; i < (N + 1) * H; i += L) {
        const int s = i / H, e = 2 * (i - s * H);
        noc_dbl2 v;
        v.x = slot[s * KD + e];
        v.y = slot[s * KD + e + 1];
        __builtin_nontemporal_store(v, reinterpret_cast<noc_dbl2*>(dst2 + i));
      }
    } else {
      for (int i = l; i < (N + 1) * NX; i += L) {
        const int s = i / NX;
        dst[i] = slot[s * KD + (i - s * NX)];
      }
    }
  }
  if (a.du) {
    double* dst = a.du + tN * NU;
    for (int i = l; i < N * NU; i += L) {
      const int s = i / NU;
      dst[i] = slot[s * KD + NX + (i - s * NU)];
    }
  }
  NOC_STAMP(6);
}

template <int NX, int NU, int L, bool AFF, bool TILED, int CACHE = 0, bool HANDOFF = true,
          bool BIG = false, bool NT3 = false>
NOC_DEV void kkt_scan_wave(const KKTArgs& a, const int traj, const int l) {
  const int cmax = a.N / L + (a.N % L ? 1 : 0);
  const ArgsSrc<NX, NU, L, AFF, TILED> src{a, traj, l, cmax, (size_t)traj * a.N};
  kkt_scan_wave_src<NX, NU, L, AFF, TILED, ArgsSrc<NX, NU, L, AFF, TILED>, CACHE, HANDOFF, BIG, NT3>(a, traj,
                                                                                               l, src);
}

// BIG (L = 32, 64; nx = 3, 4): one wave per SIMD -- for batches whose waves all fit one per SIMD
// anyway (the 2048- and 1024-per-GPU shards): 512 registers (no spill) and masked combines, like
// the two-wave segments.
template <int NX, int NU, int L, bool AFF, bool TILED, int CACHE, bool BIG = false, bool NT3 = false>
__global__ __launch_bounds__(L > 64 ? L : 256, (L > 64 || BIG) ? 1 : NOC_KKT_WAVES_PER_SIMD) void kkt_scan_kernel(KKTArgs a) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  // Two-wave segments (L = 128) must put their two waves on DIFFERENT SIMDs: with <= 256
  // registers per wave the dispatcher placed both waves of a 128-thread block on one SIMD (their
  // combine levels then took turns on one VALU: phase 2 36.6 k vs 23.4 k cycles per wave,
  // profiles/r03/shards/stamps_s512_L128.txt).  Claiming the whole register file (the AGPR half
  // included: no wave of this kernel can share a SIMD) makes the two waves of a block land on two
  // SIMDs; the launch policy (kkt_pick_lanes) uses L = 128 only when every wave is then resident
  // at once (B * 2 <= #SIMDs).
  if constexpr (L > 64 || BIG) asm volatile("" ::: "a255");
  const int traj = tid / L;
  if constexpr (L <= 64) {
    // A wave with no trajectory to solve (past the batch, or masked off) still meets the one
    // workgroup barrier its block's other waves reach at the copy-out (lds_out, full / forward
    // mode, no early-exit ablation: the same condition as the main path's barrier), so every wave
    // of the block issues that barrier exactly once.  With L < 64 one wave holds several
    // segments, and only some may be dead: then the live segments' lanes issue the wave's one
    // barrier at the copy-out and the dead lanes just leave -- the barrier here is taken only by
    // a wave with no live segment at all (a wave-uniform branch, never lane-divergent).
    const bool dead = traj >= a.B || (a.active && a.active[traj] == 0);
    const bool wave_live = __any(!dead);  // voted at the wave's full EXEC, before any branch
    if (dead) {
      if (!wave_live && a.lds_out && a.mode != MODE_BWD && !(a.ablate & 6)) __syncthreads();
      return;
    }
  }
  kkt_scan_wave<NX, NU, L, AFF, TILED, CACHE, true, BIG, NT3 && TILED && CACHE == 0>(a, traj, tid % L);
}

// Register-cached chunk length for (NX, NU, L): only where a short chunk's blocks fit beside the
// scan element (nx = 2: 17 doubles per stage) and the lane count makes chunks short.
template <int NX, int NU, int L>
constexpr int kkt_cache_len() { return (NX <= 2 && L >= 32) ? 2 : 0; }


// ---------------------------------------------------------------------------------------------
// (not static: a shape whose instances take long to compile splits its lane counts over units,
// kkt_scan_8x4*.hip, by explicit instantiation)
template <int NX, int NU, int L, bool AFF>
hipError_t launch_kkt(const KKTArgs& a_in, hipStream_t stream) {
  KKTArgs a = a_in;
  const long long threads = (long long)a.B * L;
  constexpr int CC = kkt_cache_len<NX, NU, L>();
  const int cmax = a.N / L + (a.N % L ? 1 : 0);
  const bool cached = CC > 0 && cmax <= CC && !(a.ablate & 8);  // ablation bit 3: streamed chunks
  // the batch's waves fit one per SIMD: the 512-register instance (NOC_KKT_BIG=0 disables)
  const bool big = (L == 64 || L == 32) && NX >= 3 && NX <= 4 &&
                   (threads + 63) / 64 <= kkt_device_simds() && kkt_big_enabled();
  // L <= 64: wpb independent waves per workgroup (no LDS sharing; each its own slot region);
  // L = 128: one trajectory per two-wave workgroup (the waves join through LDS)
  const size_t slots1 = (a.mode == MODE_BWD || (!a.dx && !a.du)) ? 0 : kkt_lds_bytes_rt(NX, NU, a.N, L);
  int wpb = L > 64 ? 1 : kkt_waves_per_block((threads + 63) / 64, slots1);
  size_t lds = slots1 * wpb + (L > 64 ? join_doubles<NX>() * sizeof(double) : 0);
  a.lds_out = slots1 > 0 ? 1 : 0;
  a.ab_slots = 0;
  a.lds_base = 0;
  // The 512-register instances (BIG) have 40 KB of LDS per wave (160 KB per CU at one wave per
  // SIMD) against the slots' <= 20 KB: behind the slots they keep A, B of as many chunk slots as
  // fit (AB), one wave per workgroup
  if (big) {
    const size_t per_traj = (size_t)(((long long)a.N * kd_width<NX, NU>() + NX + 1) & ~1LL);
    const size_t segs = 64 / L;
    const size_t base = slots1 > 0 ? segs * per_traj : 0;
    const size_t waves = 1;
    const size_t budget = 40960 / sizeof(double);
    int ab = 0;
    if constexpr (ab_supported<NX, NU>()) {
      if (!cached && a.mode != MODE_FWD && kkt_ab_enabled()) {
        const size_t slot = (size_t)ab_granules<NX, NU>() * 128;
        const size_t fit = budget > base ? (budget - base) / (waves * slot) : 0;
        ab = (int)(fit < (size_t)cmax ? fit : (size_t)cmax);
      }
    }
    if (ab > 0) {
      a.ab_slots = ab;
      a.lds_base = (int)base;
      wpb = 1;
      lds = (base + waves * ab * (size_t)ab_granules<NX, NU>() * 128) * sizeof(double);
    }
  }
  const int block = L > 64 ? L : 64 * wpb;
  const unsigned grid = (unsigned)((threads + block - 1) / block);
  if (!a.lds_out && (!a.K || !a.d)) return hipErrorInvalidValue;  // K/d needed as workspace
  if (cached) {
    if (a.tiled)
      hipLaunchKernelGGL((kkt_scan_kernel<NX, NU, L, AFF, true, CC>), dim3(grid), dim3(block), lds, stream, a);
    else
      hipLaunchKernelGGL((kkt_scan_kernel<NX, NU, L, AFF, false, CC>), dim3(grid), dim3(block), lds, stream, a);
  } else if (big) {
    if constexpr ((L == 64 || L == 32) && NX >= 3 && NX <= 4) {
      if (a.tiled)
        hipLaunchKernelGGL((kkt_scan_kernel<NX, NU, L, AFF, true, 0, true>), dim3(grid), dim3(block), lds, stream, a);
      else
        hipLaunchKernelGGL((kkt_scan_kernel<NX, NU, L, AFF, false, 0, true>), dim3(grid), dim3(block), lds, stream, a);
    }
  } else if (!a.tiled) {
    hipLaunchKernelGGL((kkt_scan_kernel<NX, NU, L, AFF, false, 0>), dim3(grid), dim3(block), lds, stream, a);
  } else if constexpr (L > 64) {  // two-wave segments: non-temporal (kkt_nt3)
    hipLaunchKernelGGL((kkt_scan_kernel<NX, NU, L, AFF, true, 0, false, true>), dim3(grid), dim3(block), lds, stream, a);
  } else if constexpr (L == 32) {  // both policies, by the batch's size (kkt_nt3)
    if (kkt_nt3(a.B, a.N, NX, NU))
      hipLaunchKernelGGL((kkt_scan_kernel<NX, NU, L, AFF, true, 0, false, true>), dim3(grid), dim3(block), lds, stream,
                         a);
    else
      hipLaunchKernelGGL((kkt_scan_kernel<NX, NU, L, AFF, true, 0>), dim3(grid), dim3(block), lds, stream, a);
  } else {
    hipLaunchKernelGGL((kkt_scan_kernel<NX, NU, L, AFF, true, 0>), dim3(grid), dim3(block), lds, stream, a);
  }
  return hipGetLastError();
}

template <int NX, int NU, bool AFF>
static hipError_t dispatch_lanes(const KKTArgs& a, int lanes, hipStream_t stream) {
  switch (lanes) {
    case 128:  // two-wave segments: small nx only (nx = 8 batches use the group solve)
      if constexpr (NX <= 4) return launch_kkt<NX, NU, 128, AFF>(a, stream);
      else return hipErrorInvalidValue;
    case 64: return launch_kkt<NX, NU, 64, AFF>(a, stream);
    case 32: return launch_kkt<NX, NU, 32, AFF>(a, stream);
    case 16: return launch_kkt<NX, NU, 16, AFF>(a, stream);
    case 8: return launch_kkt<NX, NU, 8, AFF>(a, stream);
    default: return hipErrorInvalidValue;
  }
}

template <int NX, int NU>
static hipError_t dispatch_aff(const KKTArgs& a, int lanes, hipStream_t stream) {
  const bool aff = a.q || a.c || a.p;
  return aff ? dispatch_lanes<NX, NU, true>(a, lanes, stream)
             : dispatch_lanes<NX, NU, false>(a, lanes, stream);
}

}  // namespace noc

#pragma clang fp contract(on)
