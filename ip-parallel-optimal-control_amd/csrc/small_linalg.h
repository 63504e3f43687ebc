// Register-resident small dense linear algebra for the gfx950 KKT scan kernels (fp64).
//
// Every loop is fully unrolled over compile-time extents, so all matrix entries live in VGPRs
// (runtime-indexed register arrays would spill to scratch: cdna_hip_programming.md §5.4 rule 20).
// Symmetric matrices are stored packed (upper triangle, row-major) to cut VGPRs and shuffles.
#pragma once
#include <hip/hip_runtime.h>

namespace noc {

#define NOC_DEV __device__ __forceinline__
#define NOC_UNROLL _Pragma("unroll")

// ISA analysis builds only (-DNOC_ISA_MARKS, tools/isa_levels.py): an assembler comment at each
// level / phase boundary of the scans, so per-level instruction counts can be read off the .s file
#ifdef NOC_ISA_MARKS
#define NOC_ISA_MARK(tag, k) asm volatile("; NOC_MARK " tag " %0" ::"i"(k))
#else
#define NOC_ISA_MARK(tag, k) do { } while (0)
#endif

template <int R, int C>
struct Mat {
  double v[R * C];
  NOC_DEV double& operator()(int i, int j) { return v[i * C + j]; }
  NOC_DEV double operator()(int i, int j) const { return v[i * C + j]; }
};

template <int N>
struct Vec {
  double v[N];
  NOC_DEV double& operator[](int i) { return v[i]; }
  NOC_DEV double operator[](int i) const { return v[i]; }
};

template <int N>
struct Sym {
  static constexpr int SZ = N * (N + 1) / 2;
  double v[SZ];
  static __host__ __device__ constexpr int idx(int i, int j) {
    return i <= j ? i * N - (i * (i - 1)) / 2 + (j - i) : j * N - (j * (j - 1)) / 2 + (i - j);
  }
  NOC_DEV double& operator()(int i, int j) { return v[idx(i, j)]; }
  NOC_DEV double operator()(int i, int j) const { return v[idx(i, j)]; }
};

// ---------------------------------------------------------------------------------------------
// fills
template <int R, int C>
NOC_DEV void set_zero(Mat<R, C>& m) { NOC_UNROLL for (int i = 0; i < R * C; ++i) m.v[i] = 0.0; }
template <int N>
NOC_DEV void set_zero(Vec<N>& m) { NOC_UNROLL for (int i = 0; i < N; ++i) m.v[i] = 0.0; }
template <int N>
NOC_DEV void set_zero(Sym<N>& m) { NOC_UNROLL for (int i = 0; i < Sym<N>::SZ; ++i) m.v[i] = 0.0; }
template <int N>
NOC_DEV void set_identity(Mat<N, N>& m) {
  NOC_UNROLL for (int i = 0; i < N; ++i) NOC_UNROLL for (int j = 0; j < N; ++j) m(i, j) = (i == j) ? 1.0 : 0.0;
}

// ---------------------------------------------------------------------------------------------
// global loads (16-B vector loads when the element count is even; the host checks alignment)
template <int CNT>
NOC_DEV void gload(const double* __restrict__ src, double* dst) {
  if constexpr (CNT % 2 == 0) {
    const double2* s2 = reinterpret_cast<const double2*>(src);
    NOC_UNROLL for (int i = 0; i < CNT / 2; ++i) {
      double2 t = s2[i];
      dst[2 * i] = t.x;
      dst[2 * i + 1] = t.y;
    }
  } else {
    NOC_UNROLL for (int i = 0; i < CNT; ++i) dst[i] = src[i];
  }
}
template <int CNT>
NOC_DEV void gstore(double* __restrict__ dst, const double* src) {
  if constexpr (CNT % 2 == 0) {
    double2* d2 = reinterpret_cast<double2*>(dst);
    NOC_UNROLL for (int i = 0; i < CNT / 2; ++i) d2[i] = make_double2(src[2 * i], src[2 * i + 1]);
  } else {
    NOC_UNROLL for (int i = 0; i < CNT; ++i) dst[i] = src[i];
  }
}

// A value the compiler cannot see into: a product kept as its own rounded result.  The KKT scan
// units are built with -ffp-contract=fast, under which the backend may fuse ANY multiply into a
// following add, whatever the source's pragmas -- and it chooses per inlined copy.
NOC_DEV double opaque(double v) {
  asm volatile("" : "+v"(v));
  return v;
}

// load a full row-major N x N matrix and symmetrise it into packed storage.  OPAQUE: the
// off-diagonal 0.5 (a + b) passes through an empty asm, so it is rounded on its own.  A
// symmetrised Q(i, j) starts the KKT scan's Riccati sums S = Q + A'SA + ..., and two inlined
// copies of that step fused it differently -- fma(0.5, a + b, A * SA) in one, 0.5 (a + b) rounded
// then fma(A, SA, .) in the other (round 6 ISA: six v_fmac_f64 with 0.5 in the A, B-slot path's
// phase 3, six v_mul_f64 by 0.5 in the re-read path's), so the natural layout's results depended
// on which path the batch size selected (tests/test_kkt_gpu.py: test_ab_slots_equal_rereads).
// The scan loads with OPAQUE; the group solves do not (with it in their load of P, c4 measured
// 5.23 against 4.90 ms on one box, profiles/r06/m/).
template <int N, bool OPAQUE = false>
NOC_DEV void gload_sym(const double* __restrict__ src, Sym<N>& S) {
  double t[N * N];
  gload<N * N>(src, t);
  NOC_UNROLL for (int i = 0; i < N; ++i)
    NOC_UNROLL for (int j = i; j < N; ++j) {
      const double h = 0.5 * (t[i * N + j] + t[j * N + i]);
      S(i, j) = (i == j) ? t[i * N + i] : (OPAQUE ? opaque(h) : h);
    }
}
template <int N>
NOC_DEV void gstore_sym(double* __restrict__ dst, const Sym<N>& S) {
  double t[N * N];
  NOC_UNROLL for (int i = 0; i < N; ++i) NOC_UNROLL for (int j = 0; j < N; ++j) t[i * N + j] = S(i, j);
  gstore<N * N>(dst, t);
}

// ---------------------------------------------------------------------------------------------
// Tiled ("lane-interleaved") block layout, see include/noc_hip.h.  A field with E doubles per
// stage, trajectory segments of L lanes and cmax = ceil(N/L) chunk slots: stage s owned by lane l
// at chunk position j lives at
//   E even: (((traj*cmax + j)*(E/2) + e/2)*L + l)*2 + (e&1)     (16-byte granules)
//   E odd : ((traj*cmax + j)*E + e)*L + l                         (8-byte granules)
// so one wave-wide load of a granule is L*16 (L*8) contiguous bytes.
// lanes = 1 ("grouped" layout of the horizon-sequential group solve): records of GROUP_T
// trajectories, [traj / GROUP_T][stage][traj % GROUP_T][e] -- one wave's 8 trajectories of one
// stage are GROUP_T * E contiguous doubles per field (cmax == N when L == 1).
constexpr int GROUP_T = 8;
NOC_DEV size_t group_base(int E, int N, int traj, int s) {
  return (((size_t)(traj / GROUP_T) * N + s) * GROUP_T + (traj % GROUP_T)) * E;
}
template <int E, int L>
NOC_DEV size_t tile_base(int traj, int j, int l, int cmax) {
  if constexpr (L == 1) return group_base(E, cmax, traj, j);
  else if constexpr (E % 2 == 0) return (((size_t)traj * cmax + j) * (E / 2) * L + l) * 2;
  else return ((size_t)traj * cmax + j) * E * L + l;
}
template <int E, int L>
NOC_DEV void tload(const double* __restrict__ base, int traj, int j, int l, int cmax, double* dst) {
  const double* p = base + tile_base<E, L>(traj, j, l, cmax);
  if constexpr (E % 2 == 0) {
    NOC_UNROLL for (int q = 0; q < E / 2; ++q) {
      const double2 v = *reinterpret_cast<const double2*>(p + (size_t)q * 2 * L);
      dst[2 * q] = v.x;
      dst[2 * q + 1] = v.y;
    }
  } else {
    NOC_UNROLL for (int e = 0; e < E; ++e) dst[e] = p[(size_t)e * L];
  }
}
// the same for a last use of the data: non-temporal loads (streaming cache policy), so the
// blocks a later phase still re-reads keep the cache capacity
typedef double noc_dbl2 __attribute__((ext_vector_type(2)));
template <int E, int L>
NOC_DEV void tload_last(const double* __restrict__ base, int traj, int j, int l, int cmax, double* dst) {
  const double* p = base + tile_base<E, L>(traj, j, l, cmax);
  if constexpr (E % 2 == 0) {
    NOC_UNROLL for (int q = 0; q < E / 2; ++q) {
      const noc_dbl2 v = __builtin_nontemporal_load(reinterpret_cast<const noc_dbl2*>(p + (size_t)q * 2 * L));
      dst[2 * q] = v.x;
      dst[2 * q + 1] = v.y;
    }
  } else {
    NOC_UNROLL for (int e = 0; e < E; ++e) dst[e] = __builtin_nontemporal_load(p + (size_t)e * L);
  }
}
template <int E, int L>
NOC_DEV void tstore(double* __restrict__ base, int traj, int j, int l, int cmax, const double* src) {
  double* p = base + tile_base<E, L>(traj, j, l, cmax);
  if constexpr (E % 2 == 0) {
    NOC_UNROLL for (int q = 0; q < E / 2; ++q)
      *reinterpret_cast<double2*>(p + (size_t)q * 2 * L) = make_double2(src[2 * q], src[2 * q + 1]);
  } else {
    NOC_UNROLL for (int e = 0; e < E; ++e) p[(size_t)e * L] = src[e];
  }
}
// runtime-E variant (relayout / linearisation kernels)
NOC_DEV size_t tile_index(int E, int L, int cmax, int traj, int j, int l, int e) {
  if (L == 1) return group_base(E, cmax, traj, j) + e;
  if ((E & 1) == 0) return (((size_t)traj * cmax + j) * (E / 2) + (e >> 1)) * (2 * L) + 2 * l + (e & 1);
  return (((size_t)traj * cmax + j) * E + e) * L + l;
}
template <int E>
NOC_DEV void tload_rt(const double* __restrict__ base, int L, int cmax, int traj, int j, int l, double* dst) {
  const double* p = base + tile_index(E, L, cmax, traj, j, l, 0);
  if constexpr (E % 2 == 0) {
    NOC_UNROLL for (int q = 0; q < E / 2; ++q) {
      const double2 v = *reinterpret_cast<const double2*>(p + (size_t)q * 2 * L);
      dst[2 * q] = v.x;
      dst[2 * q + 1] = v.y;
    }
  } else {
    NOC_UNROLL for (int e = 0; e < E; ++e) dst[e] = p[(size_t)e * L];
  }
}
template <int E>
NOC_DEV void tstore_rt(double* __restrict__ base, int L, int cmax, int traj, int j, int l, const double* src) {
  double* p = base + tile_index(E, L, cmax, traj, j, l, 0);
  if constexpr (E % 2 == 0) {
    NOC_UNROLL for (int q = 0; q < E / 2; ++q)
      *reinterpret_cast<double2*>(p + (size_t)q * 2 * L) = make_double2(src[2 * q], src[2 * q + 1]);
  } else {
    NOC_UNROLL for (int e = 0; e < E; ++e) p[(size_t)e * L] = src[e];
  }
}
// chunk geometry of a horizon N split over L lanes (lanes < rem get one extra stage)
struct Chunks {
  int base, rem, cmax;
  NOC_DEV Chunks(int N, int L) : base(N / L), rem(N % L), cmax(N / L + (N % L ? 1 : 0)) {}
  NOC_DEV int start(int l) const { return l * base + (l < rem ? l : rem); }
  NOC_DEV int len(int l) const { return base + (l < rem ? 1 : 0); }
  NOC_DEV void owner(int s, int& l, int& j) const {  // stage -> (lane, chunk position)
    const int cut = rem * (base + 1);
    if (s < cut) { l = s / (base + 1); j = s - l * (base + 1); }
    else { l = rem + (s - cut) / base; j = (s - cut) - (l - rem) * base; }
  }
};

// ---------------------------------------------------------------------------------------------
// wave shuffles of whole register blocks (ds_bpermute under the hood, segment width W)
NOC_DEV double shfl_down_d(double x, int d, int w) { return __shfl_down(x, (unsigned)d, w); }
NOC_DEV double shfl_up_d(double x, int d, int w) { return __shfl_up(x, (unsigned)d, w); }

template <int CNT>
NOC_DEV void shfl_down_arr(const double* src, double* dst, int d, int w) {
  NOC_UNROLL for (int i = 0; i < CNT; ++i) dst[i] = shfl_down_d(src[i], d, w);
}
template <int CNT>
NOC_DEV void shfl_up_arr(const double* src, double* dst, int d, int w) {
  NOC_UNROLL for (int i = 0; i < CNT; ++i) dst[i] = shfl_up_d(src[i], d, w);
}

// By-one lane shifts across the whole wave on the VALU (DPP wave_shl:1 / wave_shr:1) instead of
// ds_bpermute: down, lane i <- lane i + 1; up, lane i <- lane i - 1; the wave's last (first) lane
// receives 0.  For any segment width L this equals __shfl_down / __shfl_up(v, 1, L) on every lane
// except each segment's last (first) lane -- which the KKT scan overwrites (terminal cost / x0 /
// the two-wave joins) -- and moves bits only.
template <int CNT>
NOC_DEV void wave_shift_down1(const double* src, double* dst) {
  NOC_UNROLL for (int i = 0; i < CNT; ++i) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(src[i]), 0x130, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(src[i]), 0x130, 0xF, 0xF, true);
    dst[i] = __hiloint2double(hi, lo);
  }
}
template <int CNT>
NOC_DEV void wave_shift_up1(const double* src, double* dst) {
  NOC_UNROLL for (int i = 0; i < CNT; ++i) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(src[i]), 0x138, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(src[i]), 0x138, 0xF, 0xF, true);
    dst[i] = __hiloint2double(hi, lo);
  }
}

// ---------------------------------------------------------------------------------------------
// Sklansky (tree) inclusive prefixes over an L-lane segment with partners fetched on the VALU
// instead of through the LDS pipe (sklansky_*_fetch below; the scans: sklansky_fwd_level here,
// kkt_scan_impl.h: combine_sklansky for the reverse scan of the KKT elements).
template <int CTRL, int BANK>
NOC_DEV double dpp_d(double old, double src) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(src), CTRL, 0xF, BANK, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(src), CTRL, 0xF, BANK, false);
  return __hiloint2double(hi, lo);
}
// DPP move with full row / bank masks (every lane is written, so no `old` operand: the compiler
// needs no copy of a source that stays live)
template <int CTRL>
NOC_DEV double dpp_full(double src) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(src), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(src), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
NOC_DEV double readlane_dbl(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}
// Level-4 partner of the Sklansky scans (h = 16) without the SGPR round trip of v_readlane: the
// xor-16 row of every lane by v_permlane16_swap (the pairing of segment_sum_and), then DPP
// row_newbcast:RL of that row.  UPPER: rows 1 and 3 receive lane RL of rows 0 and 2 (forward scan,
// RL = 15); else rows 0 and 2 receive lane RL of rows 1 and 3 (reverse scan, RL = 0).  The other
// rows receive values they must not use.  Moves only: bit-exact.
template <int RL, bool UPPER>
NOC_DEV double permrow_bcast(double v) {
  auto one = [](int x) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    const int p = UPPER ? (int)r[0] : (int)r[1];
    return __builtin_amdgcn_mov_dpp(p, 0x150 + RL, 0xF, 0xF, false);
  };
  return __hiloint2double(one(__double2hiint(v)), one(__double2loint(v)));
}
// Partner fetches of the Sklansky scans for the lanes that combine at level K (h = 2^K); the
// other lanes receive some other lane's value, which they must not use (they skip the level's
// arithmetic under EXEC).  Run at the segment's full EXEC: a DPP source lane must be active.
// Forward (prefix): the UPPER half of every aligned 2h-lane block reads the LAST lane of its lower
// half -- quad permutations (K = 0, 1), DPP row broadcasts (K = 2, 3), v_readlane (K = 4, 5: one
// source lane per half-wave).
template <int K>
NOC_DEV double sklansky_fwd_fetch(double v, int lane) {
  if constexpr (K == 0) {
    return dpp_full<0xA0>(v);                     // quad_perm [0, 0, 2, 2]
  } else if constexpr (K == 1) {
    return dpp_full<0x55>(v);                     // quad_perm [1, 1, 1, 1]
  } else if constexpr (K == 2) {
    return dpp_d<0x15B, 0x8>(dpp_full<0x153>(v), v);  // row_newbcast:3, lanes 12-15 from :11
  } else if constexpr (K == 3) {
    return dpp_full<0x157>(v);                    // row_newbcast:7
  } else if constexpr (K == 4) {
    return permrow_bcast<15, true>(v);            // lanes 16-31 <- 15, 48-63 <- 47
  } else {
    return readlane_dbl(v, 31);
  }
}
// Reverse (suffix): the LOWER half of every aligned 2h-lane block reads the FIRST lane of its
// upper half.
template <int K>
NOC_DEV double sklansky_rev_fetch(double v, int lane) {
  if constexpr (K == 0) {
    return dpp_full<0xF5>(v);                     // quad_perm [1, 1, 3, 3]
  } else if constexpr (K == 1) {
    return dpp_full<0xAA>(v);                     // quad_perm [2, 2, 2, 2]
  } else if constexpr (K == 2) {
    return dpp_d<0x15C, 0x4>(dpp_full<0x154>(v), v);  // row_newbcast:4, lanes 8-11 from :12
  } else if constexpr (K == 3) {
    return dpp_full<0x158>(v);                    // row_newbcast:8
  } else if constexpr (K == 4) {
    return permrow_bcast<0, false>(v);            // lanes 0-15 <- 16, 32-47 <- 48
  } else {
    return readlane_dbl(v, 32);
  }
}
// Butterfly all-reduce over an L-lane segment on the VALU, bit-identical to the __shfl_xor loop
// `for (off = L/2; off; off >>= 1) v = op(v, shfl_xor(v, off))`: the xor-32 / xor-16 partners
// by v_permlane32_swap / v_permlane16_swap, xor-8 by row_ror:8, xor-4 by row_ror:12 (lane i <-
// lane (i + 4) mod 16: the xor-4 partner for lanes 0-3 and 8-11 of a row, and its value for the
// others once every value is symmetric under xor-8), xor-2 / xor-1 by quad_perm.  Lane 0 of every
// segment -- the one whose result is used -- adds exactly the pairs of the shuffle loop.
template <int CTRL>
NOC_DEV int dpp_i(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }
template <int OFF>
NOC_DEV int xor_partner_i(int v, int lane) {
  if constexpr (OFF == 32) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (lane & 32) ? (int)r[0] : (int)r[1];
  } else if constexpr (OFF == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (lane & 16) ? (int)r[0] : (int)r[1];
  } else if constexpr (OFF == 8) {
    return dpp_i<0x128>(v);  // row_ror:8
  } else if constexpr (OFF == 4) {
    return dpp_i<0x12C>(v);  // row_ror:12: lane i <- lane (i + 4) mod 16
  } else if constexpr (OFF == 2) {
    return dpp_i<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  } else {
    return dpp_i<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  }
}
// The same butterfly for one double with any commutative op (sum, nan-propagating max): every
// lane of the segment ends with the value the __shfl_xor loop gives it -- bitwise, since each
// step adds the pair (v_l, v_{l^off}) and a + b == b + a -- without the LDS round trips of
// ds_bpermute (the interior-point solvers' wave reductions: trial cost, stage-cost sum, ||cu||,
// max |Hu|).
template <int L, class OP, int OFF = L / 2>
NOC_DEV double segment_allreduce(double v, int lane, OP op) {
  if constexpr (OFF >= 1) {
    const int lo = xor_partner_i<OFF>(__double2loint(v), lane);
    const int hi = xor_partner_i<OFF>(__double2hiint(v), lane);
    return segment_allreduce<L, OP, OFF / 2>(op(v, __hiloint2double(hi, lo)), lane, op);
  } else {
    return v;
  }
}
template <int L, int OFF = L / 2>
NOC_DEV void segment_sum_and(double& sum, int& all, int lane) {
  if constexpr (OFF >= 1) {
    const int lo = xor_partner_i<OFF>(__double2loint(sum), lane);
    const int hi = xor_partner_i<OFF>(__double2hiint(sum), lane);
    sum += __hiloint2double(hi, lo);
    all &= xor_partner_i<OFF>(all, lane);
    segment_sum_and<L, OFF / 2>(sum, all, lane);
  }
}

// Level K of the inclusive prefix of affine maps x -> Phi x + phi: the upper half of every aligned
// 2^(K+1)-lane block composes its map with the lower half's last prefix (under EXEC: the other
// lanes keep theirs exactly).
template <int K, int NX, int L>
NOC_DEV void sklansky_fwd_level(Mat<NX, NX>& Phi, Vec<NX>& phi, int lane) {
  if constexpr ((1 << K) < L) {
    // MASKED (small nx): the composition runs under EXEC = the combining lanes; larger nx compose
    // in every lane, the others with the identity map (fewer values live across a branch)
    constexpr bool MASKED = NX <= 2;
    const bool comb = (lane & (1 << K)) != 0;
    Mat<NX, NX> oP;
    Vec<NX> op;
    NOC_UNROLL for (int i = 0; i < NX; ++i) {
      NOC_UNROLL for (int j = 0; j < NX; ++j) {
        const double p = sklansky_fwd_fetch<K>(Phi(i, j), lane);
        oP(i, j) = (MASKED || comb) ? p : (i == j ? 1.0 : 0.0);
      }
      const double p = sklansky_fwd_fetch<K>(phi[i], lane);
      op[i] = (MASKED || comb) ? p : 0.0;
    }
    if (!MASKED || comb) {
      Mat<NX, NX> Pn;
      NOC_UNROLL for (int i = 0; i < NX; ++i) {
        double t = phi[i];
        NOC_UNROLL for (int k = 0; k < NX; ++k) t += Phi(i, k) * op[k];
        phi[i] = t;
        NOC_UNROLL for (int j = 0; j < NX; ++j) {
          double u = 0.0;
          NOC_UNROLL for (int k = 0; k < NX; ++k) u += Phi(i, k) * oP(k, j);
          Pn(i, j) = u;
        }
      }
      Phi = Pn;
    }
  }
}
template <int NX, int L>
NOC_DEV void affine_prefix_sklansky(Mat<NX, NX>& Phi, Vec<NX>& phi) {
  static_assert(L >= 1 && L <= 64 && (L & (L - 1)) == 0, "segment width: a power of two <= 64");
  const int lane = (int)__lane_id();
  NOC_ISA_MARK("fwd", 0);
  sklansky_fwd_level<0, NX, L>(Phi, phi, lane);
  NOC_ISA_MARK("fwd", 1);
  sklansky_fwd_level<1, NX, L>(Phi, phi, lane);
  NOC_ISA_MARK("fwd", 2);
  sklansky_fwd_level<2, NX, L>(Phi, phi, lane);
  NOC_ISA_MARK("fwd", 3);
  sklansky_fwd_level<3, NX, L>(Phi, phi, lane);
  NOC_ISA_MARK("fwd", 4);
  sklansky_fwd_level<4, NX, L>(Phi, phi, lane);
  NOC_ISA_MARK("fwd", 5);
  sklansky_fwd_level<5, NX, L>(Phi, phi, lane);
  NOC_ISA_MARK("fwd", 6);
}

// ---------------------------------------------------------------------------------------------
// LDL' factorisation + solve of a small symmetric system (no pivoting).  Returns true iff the
// matrix is positive definite (all D > 0, Sylvester), which is the eigh(Quu) > 0 test of
// noc/seq_interior_point_newton.py:52-53.  Y (N x NR) is overwritten by W^{-1} Y.
template <int N, int NR>
NOC_DEV bool ldl_solve(const Sym<N>& W, double (&Y)[N][NR]) {
  if constexpr (N == 1) {
    const double w = W(0, 0);
    const double iw = 1.0 / w;
    NOC_UNROLL for (int j = 0; j < NR; ++j) Y[0][j] *= iw;
    return w > 0.0;
  } else {
    double D[N], iD[N];
    double Lm[N][N];
    bool pd = true;
    NOC_UNROLL for (int j = 0; j < N; ++j) {
      double dj = W(j, j);
      NOC_UNROLL for (int t = 0; t < j; ++t) dj -= Lm[j][t] * Lm[j][t] * D[t];
      D[j] = dj;
      iD[j] = 1.0 / dj;
      pd = pd && (dj > 0.0);
      NOC_UNROLL for (int i = j + 1; i < N; ++i) {
        double s = W(i, j);
        NOC_UNROLL for (int t = 0; t < j; ++t) s -= Lm[i][t] * Lm[j][t] * D[t];
        Lm[i][j] = s * iD[j];
      }
    }
    // L z = y
    NOC_UNROLL for (int i = 0; i < N; ++i)
      NOC_UNROLL for (int t = 0; t < i; ++t)
        NOC_UNROLL for (int j = 0; j < NR; ++j) Y[i][j] -= Lm[i][t] * Y[t][j];
    NOC_UNROLL for (int i = 0; i < N; ++i) NOC_UNROLL for (int j = 0; j < NR; ++j) Y[i][j] *= iD[i];
    // L' x = z
    NOC_UNROLL for (int i = N - 1; i >= 0; --i)
      NOC_UNROLL for (int t = i + 1; t < N; ++t)
        NOC_UNROLL for (int j = 0; j < NR; ++j) Y[i][j] -= Lm[t][i] * Y[t][j];
    return pd;
  }
}

// Gaussian elimination WITHOUT row exchanges, accepted only if every pivot passes the
// threshold-pivoting test |p_k| >= tau * max_{i>=k} |x_ik| (tau = 1/2 bounds element growth like
// partial pivoting does, within a factor (1+1/tau)^(N-1)).  Returns false (X, Y garbage) if a
// pivot fails; the caller then redoes the solve with lu_pp_solve.  No selects: ~1/3 fewer VALU
// instructions than the pivoting solve.
template <int N, int NR>
NOC_DEV bool lu_np_solve(double (&X)[N][N], double (&Y)[N][NR]) {
  bool ok = true;
  NOC_UNROLL for (int k = 0; k < N; ++k) {
    double colmax = fabs(X[k][k]);
    NOC_UNROLL for (int i = k + 1; i < N; ++i) colmax = fmax(colmax, fabs(X[i][k]));
    ok = ok && (fabs(X[k][k]) >= 0.5 * colmax) && (colmax > 0.0);
    const double inv = 1.0 / X[k][k];
    X[k][k] = inv;
    NOC_UNROLL for (int i = k + 1; i < N; ++i) {
      const double lik = X[i][k] * inv;
      NOC_UNROLL for (int j = k + 1; j < N; ++j) X[i][j] -= lik * X[k][j];
      NOC_UNROLL for (int j = 0; j < NR; ++j) Y[i][j] -= lik * Y[k][j];
    }
  }
  NOC_UNROLL for (int k = N - 1; k >= 0; --k) {
    NOC_UNROLL for (int j = 0; j < NR; ++j) {
      double s = Y[k][j];
      NOC_UNROLL for (int t = k + 1; t < N; ++t) s -= X[k][t] * Y[t][j];
      Y[k][j] = s * X[k][k];
    }
  }
  return ok;
}

// Gaussian elimination with partial pivoting (row swaps as selects, so everything stays in
// VGPRs).  X (N x N) is destroyed; Y (N x NR) becomes X^{-1} Y.
template <int N, int NR>
NOC_DEV void lu_pp_solve(double (&X)[N][N], double (&Y)[N][NR]) {
  NOC_UNROLL for (int k = 0; k < N; ++k) {
    if constexpr (N > 1) {
      int piv = k;
      double best = fabs(X[k][k]);
      NOC_UNROLL for (int i = k + 1; i < N; ++i) {
        const double a = fabs(X[i][k]);
        const bool better = a > best;
        best = better ? a : best;
        piv = better ? i : piv;
      }
      NOC_UNROLL for (int i = k + 1; i < N; ++i) {
        const bool sw = (piv == i);
        NOC_UNROLL for (int j = k; j < N; ++j) {
          const double a = X[k][j], b = X[i][j];
          X[k][j] = sw ? b : a;
          X[i][j] = sw ? a : b;
        }
        NOC_UNROLL for (int j = 0; j < NR; ++j) {
          const double a = Y[k][j], b = Y[i][j];
          Y[k][j] = sw ? b : a;
          Y[i][j] = sw ? a : b;
        }
      }
    }
    const double inv = 1.0 / X[k][k];
    X[k][k] = inv;
    NOC_UNROLL for (int i = k + 1; i < N; ++i) {
      const double lik = X[i][k] * inv;
      NOC_UNROLL for (int j = k + 1; j < N; ++j) X[i][j] -= lik * X[k][j];
      NOC_UNROLL for (int j = 0; j < NR; ++j) Y[i][j] -= lik * Y[k][j];
    }
  }
  NOC_UNROLL for (int k = N - 1; k >= 0; --k) {
    NOC_UNROLL for (int j = 0; j < NR; ++j) {
      double s = Y[k][j];
      NOC_UNROLL for (int t = k + 1; t < N; ++t) s -= X[k][t] * Y[t][j];
      Y[k][j] = s * X[k][k];
    }
  }
}

// Y <- X^{-1} Y for a 2 x 2 X in closed form: one division (the adjugate over det), no pivoting.
// Used for the combine's X = I + C1 J2.  C1 (a controllability Gramian) is PSD, but the value
// Hessian J2 is not in general: Q = cxx + lambda.fxx, or a traced user cost, can make it
// indefinite, and then det(X) = 1 + tr(C1 J2) + det(C1) det(J2) can be small or zero.  Nothing is
// checked here: an exactly singular X gives inf / NaN in the step (reported as data, never a
// fault).  For n = 2 Cramer's rule is as accurate as elimination with partial pivoting, so a
// nearly singular X costs no more accuracy than the pivoting path would (tests/test_kkt_gpu.py:
// indefinite Q at nx = 2 against the oracle).
template <int NR>
NOC_DEV void solve2_closed(const double (&X)[2][2], double (&Y)[2][NR]) {
  const double det = X[0][0] * X[1][1] - X[0][1] * X[1][0];
  const double id = 1.0 / det;
  const double a = X[1][1] * id, b = -X[0][1] * id, c = -X[1][0] * id, d = X[0][0] * id;
  NOC_UNROLL for (int j = 0; j < NR; ++j) {
    const double y0 = Y[0][j], y1 = Y[1][j];
    Y[0][j] = a * y0 + b * y1;
    Y[1][j] = c * y0 + d * y1;
  }
}

}  // namespace noc
