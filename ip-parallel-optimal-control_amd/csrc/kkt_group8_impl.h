// nx = 8, nu = 4 horizon-sequential group KKT solve with LDS-DMA stage prefetch (fp64, gfx950).
//
// Same algorithm and lane mapping as kkt_group_kernel (kkt_group_impl.h: 8 trajectories per wave,
// lane q of a group owns state column q), but the backward sweep is latency-hidden: while stage s
// is computed from LDS buffer s&1, `global_load_lds_dwordx4` (no VGPR destination) streams stage
// s-1's blocks of the wave's 8 trajectories into the other buffer (grouped layout 9.1 KB: A 4 KB,
// B 2 KB, packed Q 2.25 KB, packed R 640 B, r 256 B; two buffers = 18.25 KB, so 8 waves fit a CU's
// 160 KB).  Lanes then read operands from LDS.  M is not staged: lane q needs only its row M[q, :]
// (32 contiguous bytes), which is prefetched one stage ahead into registers instead.  The LDS image of A, B, Q, R is
// row-rotated by the trajectory's slot g in the wave (row k of trajectory g stored at row slot
// (k + g) mod rows), chosen on the SOURCE address of the DMA, so the column reads A[:, q] of the
// 8 groups fall into different bank quarters (2-way instead of 8-way conflicts).
// Contract of this path: Q and R are read through their upper triangle (lane q forms S_new[:, q]
// from column q; the gathered S keeps entries i <= j), i.e. they are taken as symmetric.
// The forward sweep keeps kFwdDepth stages of its row loads in flight in registers.
// Two input layouts: natural (the ABI's [b][k][...]; each trajectory's 512/256/128 B blocks are
// N*sz apart) and grouped (tiled with lanes = 1, small_linalg.h group_base: the wave's 8
// trajectories of one stage contiguous per field, Q/R packed) -- what the IPM linearisation writes
// for nx = 8.  Measured c4 (grouped): 5.69 ms with M staged in LDS (7 waves/CU), 4.78 ms with the
// M row loaded per lane (8 waves/CU).
#pragma once
#include <hip/hip_runtime.h>

#include "kkt_group_impl.h"

#ifndef NOC_GROUP8_WAVES_PER_SIMD
#define NOC_GROUP8_WAVES_PER_SIMD 2
#endif

namespace noc {

namespace g8 {
constexpr int NX = 8, NU = 4, TPW = 8;  // trajectories per wave (== GROUP_T)
// Byte offsets of the fields inside one LDS stage buffer (8 trajectories each).  Natural layout:
// Q, R as full matrices; grouped (tiled, lanes = 1) layout: Q, R packed symmetric.
template <bool TILED>
struct Lds {
  static constexpr int QB = TILED ? 288 : 512;  // bytes of Q per trajectory
  static constexpr int RB = TILED ? 80 : 128;   // bytes of R per trajectory
  static constexpr int OA = 0, OB = 4096, OQ = 6144, OR = OQ + 8 * QB, ORV = OR + 8 * RB,
                       OC = ORV + 256, OQV = OC + 512;
  static constexpr int BUF_PLAIN = OC;        // A..r
  static constexpr int BUF_AFF = OQV + 512;   // + c, q
};
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

// One DMA instruction's per-lane source offset (bytes, relative to field + traj0*N*sz, stage 0):
// the row-rotated granule of trajectory t = traj0 + (wave-local slot).  sz: bytes per
// trajectory-stage, rb: bytes per row, rows: rows per block (rotation modulus; 0 = none), i: the
// instruction's index within the field.  Tail waves clamp t to the last trajectory (results of
// clamped groups are never stored).
// grouped: the 8 trajectories' blocks are contiguous (stride sz; padding records cover the tail).
NOC_DEV unsigned dma_off(int sz, int rb, int rows, int i, int lane, int traj0, int B, int N,
                         bool grouped) {
  const int gbyte = i * 1024 + lane * 16;  // byte offset inside the wave's field image
  int t = gbyte / sz;
  const int p = gbyte % sz;
  const int slot = p / rb, off = p % rb;
  const int row = rows ? ((slot - t) & (rows - 1)) : slot;
  t = t < TPW ? t : TPW - 1;
  if (grouped) return (unsigned)(t * sz + row * rb + off);
  t = (traj0 + t < B) ? t : B - 1 - traj0;
  return (unsigned)((size_t)t * N * sz + row * rb + off);
}

// AUX: the DMA's cache policy bits -- kLastUse (nt) for the backward sweep's last read of a field
template <int AUX = 0>
NOC_DEV void glds16(const char* src, char* lds_dst) {
  __builtin_amdgcn_global_load_lds((glb_void*)src, (lds_void*)lds_dst, 16, 0, AUX);
}
// Q, R, M, r, q are read for the last time by the backward sweep (the forward sweep re-reads A, B,
// c): non-temporal, so their lines do not displace A, B, c from the caches before that re-read
constexpr int kLastUse = 2;

// stages of the forward sweep's loads in flight per wave (deeper rings spill)
constexpr int kFwdDepth = 2;
// Broadcast lane J of every 8-lane group to the whole group on the VALU (DPP row_newbcast: lane n
// of each 16-lane row to the row; bank_mask 0x3 writes lanes 0-7 of the row from row lane J, 0xC
// lanes 8-15 from row lane 8+J) instead of a ds_bpermute through the LDS pipe, which the backward
// sweep saturates (SQ_INSTS_LDS).  Every lane of the wave must be active.
template <int J>
NOC_DEV double bcast8(double x) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  int rlo = __builtin_amdgcn_update_dpp(0, lo, 0x150 + J, 0xF, 0x3, false);
  int rhi = __builtin_amdgcn_update_dpp(0, hi, 0x150 + J, 0xF, 0x3, false);
  rlo = __builtin_amdgcn_update_dpp(rlo, lo, 0x158 + J, 0xF, 0xC, false);
  rhi = __builtin_amdgcn_update_dpp(rhi, hi, 0x158 + J, 0xF, 0xC, false);
  return __hiloint2double(rhi, rlo);
}
// group broadcast with a (post-unrolling) constant source lane
NOC_DEV double gb(double x, int j) {
  switch (j) {
    case 0: return bcast8<0>(x);
    case 1: return bcast8<1>(x);
    case 2: return bcast8<2>(x);
    case 3: return bcast8<3>(x);
    case 4: return bcast8<4>(x);
    case 5: return bcast8<5>(x);
    case 6: return bcast8<6>(x);
    default: return bcast8<7>(x);
  }
}
}  // namespace g8

// FWD: the forward sweep alone (MODE_FWD: paroc.par_fwd_pass, the gains are inputs); no LDS.
template <bool AFF, bool TILED, bool FWD = false>
__global__ __launch_bounds__(64, NOC_GROUP8_WAVES_PER_SIMD) void kkt_group8_kernel(KKTArgs a) {
  using namespace g8;
  using LD = Lds<TILED>;
  constexpr int G = NX;
  constexpr int BUF = AFF ? LD::BUF_AFF : LD::BUF_PLAIN;
  constexpr int OA = LD::OA, OB = LD::OB, OQ = LD::OQ, OR = LD::OR, ORV = LD::ORV,
                OC = LD::OC, OQV = LD::OQV;
  extern __shared__ __attribute__((aligned(16))) double noc_smem[];
  char* lds = reinterpret_cast<char*>(noc_smem);
  const int lane = threadIdx.x;
  const int g = lane / G;
  const int q = lane % G;
  const int uq = q % NU;
  const int traj0 = blockIdx.x * TPW;
  const int traj = traj0 + g;
  const bool valid = traj < a.B && !(a.active && a.active[traj] == 0);
  if (!__any(valid)) return;  // wave-uniform: nothing to do for this wave
  const int N = a.N;
  const size_t tN = (size_t)traj * N;
  const int trajc = traj < a.B ? traj : a.B - 1;  // clamped index for loads of tail groups

  // ablation bit 6 (timing only): skip the backward sweep, the forward sweep reads the K, d a
  // previous full solve left in the output buffers (tools/kkt_ablate.py, lanes 1)
  if (!FWD && a.mode != MODE_FWD && !(a.ablate & 64)) {
    // per-lane DMA source offsets (A and Q share theirs; the stage step is uniform)
    unsigned oA[4], oB[2], oQ[4];
    NOC_UNROLL for (int i = 0; i < 4; ++i) {
      oA[i] = dma_off(512, 64, 8, i, lane, traj0, a.B, N, TILED);
      // natural Q: full rows, rotated like A; grouped Q: packed (288 B), 3 instructions
      oQ[i] = TILED ? dma_off(LD::QB, LD::QB, 0, i, lane, traj0, a.B, N, true) : oA[i];
    }
    NOC_UNROLL for (int i = 0; i < 2; ++i) oB[i] = dma_off(256, 32, 8, i, lane, traj0, a.B, N, TILED);
    const unsigned oR = TILED ? dma_off(LD::RB, LD::RB, 0, 0, lane < 40 ? lane : 0, traj0, a.B, N, true)
                              : dma_off(128, 32, 4, 0, lane, traj0, a.B, N, false);
    const unsigned orv = dma_off(32, 32, 0, 0, lane < 16 ? lane : 0, traj0, a.B, N, TILED);
    const unsigned ocq = dma_off(64, 64, 0, 0, lane < 32 ? lane : 0, traj0, a.B, N, TILED);
    // wave-uniform bases of stage s: trajectory traj0 (natural) or the wave's record (grouped)
    auto ubase = [&](const double* f, int sz, int s) {
      const size_t rec = TILED ? ((size_t)(traj0 / TPW) * N + s) * TPW * sz
                               : ((size_t)traj0 * N + s) * sz;
      return reinterpret_cast<const char*>(f) + rec;
    };
    auto issue = [&](int s, int buf) {
      char* base = lds + buf * BUF;
      const char* bA = ubase(a.A, 512, s);
      const char* bQ = ubase(a.Q, LD::QB, s);
      const char* bB = ubase(a.Bm, 256, s);
      NOC_UNROLL for (int i = 0; i < 4; ++i) glds16(bA + oA[i], base + OA + i * 1024);
      if constexpr (TILED) {
        glds16<kLastUse>(bQ + oQ[0], base + OQ);
        glds16<kLastUse>(bQ + oQ[1], base + OQ + 1024);
        if (lane < 16) glds16<kLastUse>(bQ + oQ[2], base + OQ + 2048);
      } else {
        NOC_UNROLL for (int i = 0; i < 4; ++i) glds16<kLastUse>(bQ + oQ[i], base + OQ + i * 1024);
      }
      NOC_UNROLL for (int i = 0; i < 2; ++i) glds16(bB + oB[i], base + OB + i * 1024);
      if (!TILED || lane < 40) glds16<kLastUse>(ubase(a.R, LD::RB, s) + oR, base + OR);
      if (lane < 16) glds16<kLastUse>(ubase(a.r, 32, s) + orv, base + ORV);
      if constexpr (AFF) {
        if (lane < 32) {
          glds16(ubase(a.c ? a.c : a.A, 64, s) + ocq, base + OC);
          glds16<kLastUse>(ubase(a.q ? a.q : a.A, 64, s) + ocq, base + OQV);
        }
      }
    };
    const double reg = valid ? (a.reg ? a.reg[traj] : 0.0) : 0.0;
    Sym<NX> S;
    Vec<NX> v;
    gload_sym<NX>(a.P + (size_t)trajc * NX * NX, S);
    set_zero(v);
    if constexpr (AFF) { if (a.p) gload<NX>(a.p + (size_t)trajc * NX, v.v); }
    if (valid && a.S) {
      const double* Pp = a.P + (size_t)traj * NX * NX;
      double* dst = a.S + ((tN + traj + N) * NX + q) * NX;
      NOC_UNROLL for (int i = 0; i < NX; ++i) dst[i] = 0.5 * (Pp[q * NX + i] + Pp[i * NX + q]);
    }
    if (valid && a.v) a.v[(tN + traj + N) * NX + q] = (AFF && a.p) ? a.p[(size_t)traj * NX + q] : 0.0;
    double pred = 0.0;
    int feas = 1;
    // row q of M (stage s) straight into registers, one stage ahead like the DMA
    auto load_mrow = [&](int s, double* m) {
      const size_t mb = TILED ? group_base(NX * NU, N, trajc, s) : ((size_t)trajc * N + s) * (NX * NU);
      const noc_dbl2* mp = reinterpret_cast<const noc_dbl2*>(a.M + mb + q * NU);  // last use: nt
      NOC_UNROLL for (int i = 0; i < NU / 2; ++i) {
        const noc_dbl2 t = __builtin_nontemporal_load(mp + i);
        m[2 * i] = t.x;
        m[2 * i + 1] = t.y;
      }
    };
    // The M row is prefetched a stage ahead like the DMA and lands with it.  (Loaded at the top
    // of its own stage, its first use waited vmcnt(0): the compiler does not count the LDS-DMA
    // instructions issued next to it, so that wait also drained the next stage's DMA, which then
    // overlapped only the first GEMVs of the stage instead of all of it.)
    double mrow[NU], mnext[NU];
    load_mrow(N - 1, mrow);
    issue(N - 1, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int s = N - 1; s >= 0; --s) {
      const int buf = (N - 1 - s) & 1;
      if (s > 0) {  // next stage streams in while this one is computed
        load_mrow(s - 1, mnext);
        issue(s - 1, buf ^ 1);
      }
      const char* base = lds + buf * BUF;
      // row-rotated LDS images of trajectory g (see header)
      auto Arow = [&](int k) { return reinterpret_cast<const double*>(base + OA + g * 512 + ((k + g) & 7) * 64); };
      auto Brow = [&](int k) { return reinterpret_cast<const double*>(base + OB + g * 256 + ((k + g) & 7) * 32); };
      // Q[i][q] and R[u][uq] (natural: row-rotated full matrices; grouped: packed upper triangle)
      auto Qiq = [&](int i) {
        if constexpr (TILED) return reinterpret_cast<const double*>(base + OQ + g * LD::QB)[Sym<NX>::idx(i, q)];
        else return reinterpret_cast<const double*>(base + OQ + g * 512 + ((i + g) & 7) * 64)[q];
      };
      auto Ruq = [&](int u) {
        if constexpr (TILED) return reinterpret_cast<const double*>(base + OR + g * LD::RB)[Sym<NU>::idx(u, uq)];
        else return reinterpret_cast<const double*>(base + OR + g * 128 + ((u + g) & 3) * 32)[uq];
      };
      const double* rg = reinterpret_cast<const double*>(base + ORV + g * 32);
      double aq[NX], bq[NX], cc[NX];
      NOC_UNROLL for (int k = 0; k < NX; ++k) {
        aq[k] = Arow(k)[q];
        bq[k] = Brow(k)[uq];
        cc[k] = 0.0;
      }
      if constexpr (AFF) {
        const double* cg = reinterpret_cast<const double*>(base + OC + g * 64);
        if (a.c) NOC_UNROLL for (int k = 0; k < NX; ++k) cc[k] = cg[k];
      }
      double saq[NX], w[NX], gg[NX];
      NOC_UNROLL for (int i = 0; i < NX; ++i) {
        double t0 = 0.0, t1 = 0.0, t2 = v[i];
        NOC_UNROLL for (int k = 0; k < NX; ++k) {
          t0 += S(i, k) * aq[k];
          t1 += S(i, k) * bq[k];
          if constexpr (AFF) t2 += S(i, k) * cc[k];
        }
        saq[i] = t0;
        w[i] = t1;
        gg[i] = t2;
      }
      // Quu[:, uq] = R[:, uq] + reg e_uq + B' w ;  Qux[:, q] = M[q, :]' + B' SA_q ;  Qu = r + B' g
      double quc[NU], qux[NU], qu[NU];
      NOC_UNROLL for (int u = 0; u < NU; ++u) {
        quc[u] = Ruq(u) + (u == uq ? reg : 0.0);
        qux[u] = mrow[u];
        qu[u] = rg[u];
      }
      NOC_UNROLL for (int k = 0; k < NX; ++k) {
        const double* br = Brow(k);
        NOC_UNROLL for (int u = 0; u < NU; ++u) {
          const double bku = br[u];
          quc[u] += bku * w[k];
          qux[u] += bku * saq[k];
          qu[u] += bku * gg[k];
        }
      }
      Sym<NU> Quu;
      NOC_UNROLL for (int i = 0; i < NU; ++i)
        NOC_UNROLL for (int j = i; j < NU; ++j) Quu(i, j) = gb(quc[i], j);
      double Y[NU][2];
      NOC_UNROLL for (int u = 0; u < NU; ++u) {
        Y[u][0] = qux[u];
        Y[u][1] = qu[u];
      }
      feas &= ldl_solve<NU, 2>(Quu, Y) ? 1 : 0;
      double Kq[NU], dd[NU];
      NOC_UNROLL for (int u = 0; u < NU; ++u) {
        Kq[u] = -Y[u][0];
        dd[u] = -Y[u][1];
      }
      const size_t si = tN + s;
      if (valid) {
        const size_t kb = TILED ? group_base(NU * NX, N, traj, s) : si * (NU * NX);
        const size_t db = TILED ? group_base(NU, N, traj, s) : si * NU;
        NOC_UNROLL for (int u = 0; u < NU; ++u) a.K[kb + u * NX + q] = Kq[u];
        if (q == 0) gstore<NU>(a.d + db, dd);
      }
      NOC_UNROLL for (int i = 0; i < NU; ++i) {  // dV = d'Qu + 1/2 d'Quu d  (S:63)
        double t = 0.0;
        NOC_UNROLL for (int j = 0; j < NU; ++j) t += Quu(i, j) * dd[j];
        pred += dd[i] * qu[i] + 0.5 * dd[i] * t;
      }
      // v_new[q] = q_q + A[:, q]' g + Qux[:, q]' d
      double vq = 0.0;
      if constexpr (AFF) {
        if (a.q) vq = reinterpret_cast<const double*>(base + OQV + g * 64)[q];
      }
      NOC_UNROLL for (int k = 0; k < NX; ++k) vq += aq[k] * gg[k];
      NOC_UNROLL for (int u = 0; u < NU; ++u) vq += qux[u] * dd[u];
      // S_new[:, q] = Q[:, q] + A' SA_q + Qux' K[:, q]
      double sn[NX];
      NOC_UNROLL for (int i = 0; i < NX; ++i) sn[i] = Qiq(i);
      NOC_UNROLL for (int k = 0; k < NX; ++k) {
        const double* ar = Arow(k);
        NOC_UNROLL for (int i = 0; i < NX; ++i) sn[i] += ar[i] * saq[k];
      }
      NOC_UNROLL for (int u = 0; u < NU; ++u) {
        NOC_UNROLL for (int i = 0; i < NX; ++i) sn[i] += gb(qux[u], i) * Kq[u];
      }
      NOC_UNROLL for (int i = 0; i < NX; ++i)
        NOC_UNROLL for (int j = i; j < NX; ++j) S(i, j) = gb(sn[i], j);
      NOC_UNROLL for (int i = 0; i < NX; ++i) v[i] = gb(vq, i);
      if (valid && a.S) gstore<NX>(a.S + ((tN + traj + s) * NX + q) * NX, sn);
      if (valid && a.v) a.v[(tN + traj + s) * NX + q] = vq;
      // stage s-1 has landed in the other buffer (and this stage's reads of `buf` are done
      // before the DMA after next overwrites it: the loads above were all consumed)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (s > 0) NOC_UNROLL for (int u = 0; u < NU; ++u) mrow[u] = mnext[u];
    }
    if (valid && q == 0) {
      if (a.pred) a.pred[traj] = pred;
      if (a.feasible) a.feasible[traj] = feas;
    }
    if (a.mode == MODE_BWD || (a.ablate & 2)) return;  // ablation bit 1: no forward sweep
    __threadfence_block();  // this group's K, d stores are visible to its other lanes below
  }

  // ---------------- forward rollout of the closed loop (kFwdDepth stages in flight) ----
  const size_t tNc = (size_t)trajc * N;
  Vec<NX> x;
  set_zero(x);
  if (a.x0) gload<NX>(a.x0 + (size_t)trajc * NX, x.v);
  if (valid && a.dx) a.dx[(tN + traj) * NX + q] = a.x0 ? a.x0[(size_t)traj * NX + q] : 0.0;
  auto load_f = [&](int s, double* kr, double* ar, double* br, double& dv, double& cv) {
    if constexpr (TILED) {
      gload<NX>(a.K + group_base(NU * NX, N, trajc, s) + uq * NX, kr);
      gload<NX>(a.A + group_base(NX * NX, N, trajc, s) + q * NX, ar);
      gload<NU>(a.Bm + group_base(NX * NU, N, trajc, s) + q * NU, br);
      dv = a.d[group_base(NU, N, trajc, s) + uq];
      cv = (AFF && a.c) ? a.c[group_base(NX, N, trajc, s) + q] : 0.0;
    } else {
      const size_t si = tNc + s;
      gload<NX>(a.K + si * (NU * NX) + uq * NX, kr);
      gload<NX>(a.A + si * (NX * NX) + q * NX, ar);
      gload<NU>(a.Bm + si * (NX * NU) + q * NU, br);
      dv = a.d[si * NU + uq];
      cv = (AFF && a.c) ? a.c[si * NX + q] : 0.0;
    }
  };
  // Ring of kFwdDepth stage buffers, the loop unrolled by the depth so every buffer has a
  // fixed register home: stage s is computed from buffer s % DEPTH, which is then refilled with
  // stage s + DEPTH.  (A rotating k0 <- k1 copy reads the prefetch registers and makes the
  // compiler wait for the newest loads -- a vmcnt(0) per stage that left one stage of latency
  // hiding: the forward sweep then ran at 4.4 TB/s, 2.19 ms of c4's 4.68.)
  struct FwdStage {
    double k[NX], a[NX], b[NU], d, c;
  };
  auto load_fs = [&](int s, FwdStage& f) { load_f(s, f.k, f.a, f.b, f.d, f.c); };
  auto step_fs = [&](int s, const FwdStage& f) {
    double uu = f.d;
    NOC_UNROLL for (int k = 0; k < NX; ++k) uu += f.k[k] * x[k];
    double u[NU];
    NOC_UNROLL for (int j = 0; j < NU; ++j) u[j] = gb(uu, j);
    double xn = f.c;
    NOC_UNROLL for (int k = 0; k < NX; ++k) xn += f.a[k] * x[k];
    NOC_UNROLL for (int j = 0; j < NU; ++j) xn += f.b[j] * u[j];
    const size_t si = tN + s;
    if (valid && a.du && q < NU) a.du[si * NU + q] = uu;
    if (valid && a.dx) a.dx[(tN + traj + s + 1) * NX + q] = xn;
    NOC_UNROLL for (int i = 0; i < NX; ++i) x[i] = gb(xn, i);
  };
  // The refill loads are unconditional (stage index clamped to N - 1; the surplus reads are
  // never used): a data-dependent skip would leave the compiler unsure how many memory ops follow
  // a buffer's loads, and it then waits for all of them (vmcnt(0)) before every use.
  constexpr int D = kFwdDepth;
  auto clamp_s = [&](int t) { return t < N ? t : N - 1; };
  FwdStage fb[D];
  NOC_UNROLL for (int j = 0; j < D; ++j) load_fs(clamp_s(j), fb[j]);
  int s = 0;
#pragma unroll 1
  for (; s + D <= N; s += D) {
    NOC_UNROLL for (int j = 0; j < D; ++j) {
      step_fs(s + j, fb[j]);
      load_fs(clamp_s(s + j + D), fb[j]);
      // keep each refill after its own step: the scheduler hoisting later steps' loads above
      // this point multiplies the live prefetch registers (spills at depth >= 3)
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  NOC_UNROLL for (int j = 0; j < D; ++j)
    if (s + j < N) step_fs(s + j, fb[j]);
}

template <bool FWD>
static void launch_g8(const KKTArgs& a, unsigned grid, hipStream_t stream) {
  using LN = g8::Lds<false>;
  using LT = g8::Lds<true>;
  const bool aff = a.q || a.c || a.p;
  const size_t lds = FWD ? 0 : 2 * (a.tiled ? (aff ? LT::BUF_AFF : LT::BUF_PLAIN)
                                            : (aff ? LN::BUF_AFF : LN::BUF_PLAIN));
  if (a.tiled) {
    if (aff) hipLaunchKernelGGL((kkt_group8_kernel<true, true, FWD>), dim3(grid), dim3(64), lds, stream, a);
    else hipLaunchKernelGGL((kkt_group8_kernel<false, true, FWD>), dim3(grid), dim3(64), lds, stream, a);
  } else {
    if (aff) hipLaunchKernelGGL((kkt_group8_kernel<true, false, FWD>), dim3(grid), dim3(64), lds, stream, a);
    else hipLaunchKernelGGL((kkt_group8_kernel<false, false, FWD>), dim3(grid), dim3(64), lds, stream, a);
  }
}

[[maybe_unused]] static hipError_t launch_kkt_group8(const KKTArgs& a, hipStream_t stream) {
  if (!a.K || !a.d) return hipErrorInvalidValue;
  const unsigned grid = (unsigned)((a.B + g8::TPW - 1) / g8::TPW);
  if (a.mode == MODE_FWD) launch_g8<true>(a, grid, stream);
  else launch_g8<false>(a, grid, stream);
  return hipGetLastError();
}

}  // namespace noc
