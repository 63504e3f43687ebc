// Batched horizon-sequential KKT solve, one trajectory per NX-lane group (fp64, gfx950).
//
// The work-efficient variant of the KKT solve for batches that fill the chip on their own (c4:
// nx = 8, nu = 4, N = 512, B = 16384 -> 2048 waves): no horizon scan, the plain backward Riccati
// recursion and forward rollout of seq_interior_point_newton.bwd_pass / fwd_pass
// (noc/seq_interior_point_newton.py:42-90) with the trajectory's nx x nx algebra spread over NX
// lanes instead of one lane's registers (an nx = 8 scan element does not fit in 256 VGPRs).
//
// Lane q of a group owns state column q:
//   * every lane holds the full symmetric value Hessian S (packed) and v;
//   * backward stage:  SA_q = S A[:,q],  w = S B[:,q mod nu]  (local GEMVs);
//                      Quu[:,q mod nu], Qux[:,q], Qu  (stream B rows; local);
//                      gather Quu (nu(nu+1)/2 shuffles), LDL' solve -> K[:,q], d;
//                      gather Qux (nu*nx shuffles);
//                      S_new[:,q] = Q[:,q] + A' SA_q + Qux' K[:,q];  v_new[q] = q + A[:,q]'g + Qux[:,q]'d;
//                      gather S_new (nx(nx+1)/2 shuffles) and v_new (nx shuffles);
//   * forward stage:   u_j = K[j,:] x + d_j (lane j < nu), gather u; x_new[q] = A[q,:] x + B[q,:] u + c_q,
//                      gather x.
// The gains K, d go through HBM (they are outputs of par_bwd_pass and inputs of par_fwd_pass).
// Conventions: include/noc_hip.h (natural layout only).
#pragma once
#include <hip/hip_runtime.h>

#include "small_linalg.h"
#include "noc_internal.h"

namespace noc {

// value `x` held by lane `src` of this lane's G-lane group
NOC_DEV double gshfl(double x, int src, int G) { return __shfl(x, src, G); }

template <int NX, int NU, bool AFF>
__global__ __launch_bounds__(64, 2) void kkt_group_kernel(KKTArgs a) {
  constexpr int G = NX;
  static_assert(64 % G == 0 && NU <= NX, "group shape");
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int traj = tid / G;
  const int q = tid % G;
  const int uq = q % NU;
  if (traj >= a.B) return;                     // uniform over the group
  if (a.active && a.active[traj] == 0) return;  // uniform over the group
  const int N = a.N;
  const size_t tN = (size_t)traj * N;

  if (a.mode != MODE_FWD) {
    const double reg = a.reg ? a.reg[traj] : 0.0;
    Sym<NX> S;
    Vec<NX> v;
    gload_sym<NX>(a.P + (size_t)traj * NX * NX, S);
    set_zero(v);
    if constexpr (AFF) { if (a.p) gload<NX>(a.p + (size_t)traj * NX, v.v); }
    // Value outputs: lane q writes row q of S (its own column, S symmetric up to rounding) and
    // v[q].  Only lane-own scalars are stored: a register array indexed by the lane id would be
    // demoted to scratch / LDS by the compiler.
    if (a.S) {
      const double* Pp = a.P + (size_t)traj * NX * NX;
      double* dst = a.S + ((tN + traj + N) * NX + q) * NX;
      NOC_UNROLL for (int i = 0; i < NX; ++i) dst[i] = 0.5 * (Pp[q * NX + i] + Pp[i * NX + q]);
    }
    if (a.v) a.v[(tN + traj + N) * NX + q] = (AFF && a.p) ? a.p[(size_t)traj * NX + q] : 0.0;
    double pred = 0.0;
    int feas = 1;
    for (int s = N - 1; s >= 0; --s) {
      const size_t si = tN + s;
      const double* Ap = a.A + si * (NX * NX);
      const double* Bp = a.Bm + si * (NX * NU);
      const double* Qp = a.Q + si * (NX * NX);
      const double* Rp = a.R + si * (NU * NU);
      const double* Mp = a.M + si * (NX * NU);
      // columns q of A and q mod nu of B
      double aq[NX], bq[NX];
      NOC_UNROLL for (int k = 0; k < NX; ++k) {
        aq[k] = Ap[k * NX + q];
        bq[k] = Bp[k * NU + uq];
      }
      double saq[NX], w[NX], g[NX];
      Vec<NX> cc;
      set_zero(cc);
      if constexpr (AFF) { if (a.c) gload<NX>(a.c + si * NX, cc.v); }
      NOC_UNROLL for (int i = 0; i < NX; ++i) {
        double t0 = 0.0, t1 = 0.0, t2 = v[i];
        NOC_UNROLL for (int k = 0; k < NX; ++k) {
          t0 += S(i, k) * aq[k];
          t1 += S(i, k) * bq[k];
          if constexpr (AFF) t2 += S(i, k) * cc[k];
        }
        saq[i] = t0;
        w[i] = t1;
        g[i] = t2;
      }
      __builtin_amdgcn_sched_barrier(0);  // keep later sections' loads from piling up here
      // Quu[:, uq] = R[:, uq] + reg e_uq + B' w ;  Qux[:, q] = M[q, :]' + B' SA_q ;  Qu = r + B' g
      double quc[NU], qux[NU], qu[NU];
      NOC_UNROLL for (int u = 0; u < NU; ++u) {
        quc[u] = 0.5 * (Rp[u * NU + uq] + Rp[uq * NU + u]) + (u == uq ? reg : 0.0);
        qux[u] = Mp[q * NU + u];
        qu[u] = a.r[si * NU + u];
      }
      NOC_UNROLL for (int k = 0; k < NX; ++k) {
        double brow[NU];
        gload<NU>(Bp + k * NU, brow);
        NOC_UNROLL for (int u = 0; u < NU; ++u) {
          quc[u] += brow[u] * w[k];
          qux[u] += brow[u] * saq[k];
          qu[u] += brow[u] * g[k];
        }
      }
      Sym<NU> Quu;
      NOC_UNROLL for (int i = 0; i < NU; ++i)
        NOC_UNROLL for (int j = i; j < NU; ++j) Quu(i, j) = gshfl(quc[i], j, G);
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
      NOC_UNROLL for (int u = 0; u < NU; ++u) a.K[si * (NU * NX) + u * NX + q] = Kq[u];
      if (q == 0) gstore<NU>(a.d + si * NU, dd);
      // dV = d'Qu + 1/2 d'Quu d  (noc/seq_interior_point_newton.py:63)
      NOC_UNROLL for (int i = 0; i < NU; ++i) {
        double t = 0.0;
        NOC_UNROLL for (int j = 0; j < NU; ++j) t += Quu(i, j) * dd[j];
        pred += dd[i] * qu[i] + 0.5 * dd[i] * t;
      }
      __builtin_amdgcn_sched_barrier(0);
      // v_new[q] = q_q + A[:, q]' g + Qux[:, q]' d
      double vq = 0.0;
      if constexpr (AFF) { if (a.q) vq = a.q[si * NX + q]; }
      NOC_UNROLL for (int k = 0; k < NX; ++k) vq += aq[k] * g[k];
      NOC_UNROLL for (int u = 0; u < NU; ++u) vq += qux[u] * dd[u];
      // S_new[:, q] = Q[:, q] + A' SA_q + Qux' K[:, q]
      double sn[NX];
      NOC_UNROLL for (int i = 0; i < NX; ++i) sn[i] = 0.5 * (Qp[i * NX + q] + Qp[q * NX + i]);
      NOC_UNROLL for (int k = 0; k < NX; ++k) {
        double arow[NX];
        gload<NX>(Ap + k * NX, arow);
        NOC_UNROLL for (int i = 0; i < NX; ++i) sn[i] += arow[i] * saq[k];
      }
      __builtin_amdgcn_sched_barrier(0);
      NOC_UNROLL for (int u = 0; u < NU; ++u) {
        NOC_UNROLL for (int i = 0; i < NX; ++i) sn[i] += gshfl(qux[u], i, G) * Kq[u];
      }
      NOC_UNROLL for (int i = 0; i < NX; ++i)
        NOC_UNROLL for (int j = i; j < NX; ++j) S(i, j) = gshfl(sn[i], j, G);
      NOC_UNROLL for (int i = 0; i < NX; ++i) v[i] = gshfl(vq, i, G);
      if (a.S) gstore<NX>(a.S + ((tN + traj + s) * NX + q) * NX, sn);
      if (a.v) a.v[(tN + traj + s) * NX + q] = vq;
    }
    if (q == 0) {
      if (a.pred) a.pred[traj] = pred;
      if (a.feasible) a.feasible[traj] = feas;
    }
    if (a.mode == MODE_BWD) return;
    __threadfence_block();  // this group's K, d stores are visible to its other lanes below
  }

  // ---------------- forward rollout of the closed loop ----------------
  Vec<NX> x;
  set_zero(x);
  if (a.x0) gload<NX>(a.x0 + (size_t)traj * NX, x.v);
  if (a.dx) a.dx[(tN + traj) * NX + q] = a.x0 ? a.x0[(size_t)traj * NX + q] : 0.0;
  for (int s = 0; s < N; ++s) {
    const size_t si = tN + s;
    double krow[NX], arow[NX], brow[NU];
    gload<NX>(a.K + si * (NU * NX) + uq * NX, krow);
    gload<NX>(a.A + si * (NX * NX) + q * NX, arow);
    gload<NU>(a.Bm + si * (NX * NU) + q * NU, brow);
    double uu = a.d[si * NU + uq];
    NOC_UNROLL for (int k = 0; k < NX; ++k) uu += krow[k] * x[k];
    double u[NU];
    NOC_UNROLL for (int j = 0; j < NU; ++j) u[j] = gshfl(uu, j, G);
    double xn = 0.0;
    if constexpr (AFF) { if (a.c) xn = a.c[si * NX + q]; }
    NOC_UNROLL for (int k = 0; k < NX; ++k) xn += arow[k] * x[k];
    NOC_UNROLL for (int j = 0; j < NU; ++j) xn += brow[j] * u[j];
    if (a.du && q < NU) a.du[si * NU + q] = uu;
    if (a.dx) a.dx[(tN + traj + s + 1) * NX + q] = xn;
    NOC_UNROLL for (int i = 0; i < NX; ++i) x[i] = gshfl(xn, i, G);
  }
}

template <int NX, int NU>
static hipError_t launch_kkt_group(const KKTArgs& a, hipStream_t stream) {
  if (a.tiled) return hipErrorInvalidValue;   // natural layout only
  if (!a.K || !a.d) return hipErrorInvalidValue;
  const long long threads = (long long)a.B * NX;
  const int block = 64;
  const unsigned grid = (unsigned)((threads + block - 1) / block);
  const bool aff = a.q || a.c || a.p;
  if (aff)
    hipLaunchKernelGGL((kkt_group_kernel<NX, NU, true>), dim3(grid), dim3(block), 0, stream, a);
  else
    hipLaunchKernelGGL((kkt_group_kernel<NX, NU, false>), dim3(grid), dim3(block), 0, stream, a);
  return hipGetLastError();
}

}  // namespace noc
