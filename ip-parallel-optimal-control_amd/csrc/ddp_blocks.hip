// The reference DDP module's building blocks as standalone batched kernels (the whole-solve DDP
// kernel, ddp_persistent.hip, inlines them):
//   bwd_pass        D:28-70   second-order backward pass with the Vx . fxx terms
//   nonlin_rollout  D:73-90   (== P:87-104) the closed-loop nonlinear rollout of a gain set
// Both recursions are horizon-sequential (the backward one is nonlinear in V), so one thread per
// trajectory walks the horizon; natural layout, fp64.
#include <hip/hip_runtime.h>

#include "../../include/noc_hip.h"
#include "ipm_family.h"
#include "noc_internal.h"
#include "small_linalg.h"

namespace noc {

// D:37-56 per stage, D:58-70 around it.  reg = reg_param * ||cu||_F (D:34-35).  Quu's positive
// definiteness (eigh > 0, D:47-48) by the LDL' pivots (Sylvester); the solves with the same
// factorisation.  Vxx is propagated as the reference writes it (no symmetrisation).
template <int NX, int NU>
__global__ __launch_bounds__(64) void ddp_bwd_kernel(DdpBwdArgs a) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  const int N = a.N;
  const size_t bN = (size_t)b * N;
  double g2 = 0.0;
  for (int t = 0; t < N * NU; ++t) g2 += a.cu[bN * NU + t] * a.cu[bN * NU + t];
  const double reg = a.reg_param[b] * sqrt(g2);
  double Vx[NX], Vxx[NX * NX];
  NOC_UNROLL for (int i = 0; i < NX; ++i) Vx[i] = a.Vx[(size_t)b * NX + i];
  NOC_UNROLL for (int i = 0; i < NX * NX; ++i) Vxx[i] = a.Vxx[(size_t)b * NX * NX + i];
  double pred = 0.0;
  bool feas = true;
  for (int t = N - 1; t >= 0; --t) {
    const size_t bt = bN + t;
    const double* fx = a.fx + bt * NX * NX;
    const double* fu = a.fu + bt * NX * NU;
    // Qx = cx + fx'Vx, Qu = cu + fu'Vx (D:41-42)
    double Qx[NX], Qu[NU];
    NOC_UNROLL for (int j = 0; j < NX; ++j) {
      double s = a.cx[bt * NX + j];
      NOC_UNROLL for (int i = 0; i < NX; ++i) s += fx[i * NX + j] * Vx[i];
      Qx[j] = s;
    }
    NOC_UNROLL for (int j = 0; j < NU; ++j) {
      double s = a.cu[bt * NU + j];
      NOC_UNROLL for (int i = 0; i < NX; ++i) s += fu[i * NU + j] * Vx[i];
      Qu[j] = s;
    }
    // W = Vxx fx, Z = Vxx fu
    double W[NX * NX], Z[NX * NU];
    NOC_UNROLL for (int i = 0; i < NX; ++i) {
      NOC_UNROLL for (int j = 0; j < NX; ++j) {
        double s = 0.0;
        NOC_UNROLL for (int m = 0; m < NX; ++m) s += Vxx[i * NX + m] * fx[m * NX + j];
        W[i * NX + j] = s;
      }
      NOC_UNROLL for (int j = 0; j < NU; ++j) {
        double s = 0.0;
        NOC_UNROLL for (int m = 0; m < NX; ++m) s += Vxx[i * NX + m] * fu[m * NU + j];
        Z[i * NU + j] = s;
      }
    }
    // Qxx = cxx + fx'Vxx fx + Vx.fxx, Qxu = cxu + fx'Vxx fu + Vx.fxu, Quu = cuu + fu'Vxx fu +
    // Vx.fuu + reg I (D:43-46; tensordot over the dynamics' output axis)
    double Qxx[NX * NX], Qxu[NX * NU];
    Sym<NU> Quu;
    NOC_UNROLL for (int i = 0; i < NX; ++i) {
      NOC_UNROLL for (int j = 0; j < NX; ++j) {
        double s = a.cxx[bt * NX * NX + i * NX + j];
        NOC_UNROLL for (int m = 0; m < NX; ++m) s += fx[m * NX + i] * W[m * NX + j];
        NOC_UNROLL for (int m = 0; m < NX; ++m) s += Vx[m] * a.fxx[(bt * NX + m) * NX * NX + i * NX + j];
        Qxx[i * NX + j] = s;
      }
      NOC_UNROLL for (int j = 0; j < NU; ++j) {
        double s = a.cxu[bt * NX * NU + i * NU + j];
        NOC_UNROLL for (int m = 0; m < NX; ++m) s += fx[m * NX + i] * Z[m * NU + j];
        NOC_UNROLL for (int m = 0; m < NX; ++m) s += Vx[m] * a.fxu[(bt * NX + m) * NX * NU + i * NU + j];
        Qxu[i * NU + j] = s;
      }
    }
    NOC_UNROLL for (int i = 0; i < NU; ++i)
      NOC_UNROLL for (int j = i; j < NU; ++j) {
        double s = a.cuu[bt * NU * NU + i * NU + j];
        NOC_UNROLL for (int m = 0; m < NX; ++m) s += fu[m * NU + i] * Z[m * NU + j];
        NOC_UNROLL for (int m = 0; m < NX; ++m) s += Vx[m] * a.fuu[(bt * NX + m) * NU * NU + i * NU + j];
        Quu(i, j) = s + (i == j ? reg : 0.0);
      }
    // Quu^-1 [Qu | Qxu'] (D:50-55)
    double Y[NU][NX + 1];
    NOC_UNROLL for (int i = 0; i < NU; ++i) {
      Y[i][0] = Qu[i];
      NOC_UNROLL for (int j = 0; j < NX; ++j) Y[i][1 + j] = Qxu[j * NU + i];
    }
    feas = ldl_solve<NU, NX + 1>(Quu, Y) && feas;
    NOC_UNROLL for (int i = 0; i < NU; ++i) {
      a.k[bt * NU + i] = -Y[i][0];                                           // D:50
      NOC_UNROLL for (int j = 0; j < NX; ++j) a.K[(bt * NU + i) * NX + j] = -Y[i][1 + j];  // D:51
      a.Hu[bt * NU + i] = Qu[i];                                             // D:56
      pred += -0.5 * Qu[i] * Y[i][0];                                        // D:53
    }
    NOC_UNROLL for (int j = 0; j < NX; ++j) {                                // D:54
      double s = Qx[j];
      NOC_UNROLL for (int i = 0; i < NU; ++i) s -= Qu[i] * Y[i][1 + j];
      Vx[j] = s;
    }
    NOC_UNROLL for (int i = 0; i < NX; ++i)                                  // D:55
      NOC_UNROLL for (int j = 0; j < NX; ++j) {
        double s = Qxx[i * NX + j];
        NOC_UNROLL for (int m = 0; m < NU; ++m) s -= Qxu[i * NU + m] * Y[m][1 + j];
        Vxx[i * NX + j] = s;
      }
  }
  a.pred[b] = pred;
  a.feasible[b] = feas ? 1 : 0;
}

hipError_t ddp_bwd_pass(int nx, int nu, const DdpBwdArgs& a, hipStream_t s) {
#define NOC_KKT_SHAPE(X, U)                                                                      \
  if (nx == X && nu == U) {                                                                      \
    hipLaunchKernelGGL((ddp_bwd_kernel<X, U>), dim3((a.B + 63) / 64), dim3(64), 0, s, a);        \
    return hipGetLastError();                                                                    \
  }
#include NOC_KKT_SHAPES_DEF
#undef NOC_KKT_SHAPE
  return hipErrorInvalidValue;
}

// D:73-90: x_hat_0 = x_0; u_hat_s = u_s + k_s + K_s (x_hat_s - x_s); x_hat_{s+1} = f(x_hat_s, u_hat_s)
template <int KIND, int NX, int NU>
__global__ __launch_bounds__(64) void nonlin_rollout_kernel(noc_family prm, int N, int B,
                                                            const double* K, const double* k,
                                                            const double* x, const double* u,
                                                            double* xn, double* un) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const Fam<KIND, NX, NU> f(prm);
  const size_t bx = (size_t)b * (N + 1) * NX, bu = (size_t)b * N * NU;
  double xh[NX];
  NOC_UNROLL for (int i = 0; i < NX; ++i) xh[i] = x[bx + i];
  for (int t = 0; t < N; ++t) {
    double uh[NU];
    NOC_UNROLL for (int i = 0; i < NU; ++i) {
      double s = u[bu + (size_t)t * NU + i] + k[bu + (size_t)t * NU + i];
      NOC_UNROLL for (int j = 0; j < NX; ++j)
        s += K[(bu + (size_t)t * NU + i) * NX + j] * (xh[j] - x[bx + (size_t)t * NX + j]);
      uh[i] = s;
    }
    NOC_UNROLL for (int i = 0; i < NX; ++i) xn[bx + (size_t)t * NX + i] = xh[i];
    NOC_UNROLL for (int i = 0; i < NU; ++i) un[bu + (size_t)t * NU + i] = uh[i];
    double nx_[NX];
    f.step(xh, uh, nx_);
    NOC_UNROLL for (int i = 0; i < NX; ++i) xh[i] = nx_[i];
  }
  NOC_UNROLL for (int i = 0; i < NX; ++i) xn[bx + (size_t)N * NX + i] = xh[i];
}

hipError_t nonlin_rollout(const noc_family& p, int N, int B, const double* K, const double* k,
                          const double* x, const double* u, double* xn, double* un, hipStream_t s) {
#define NOC_FAMILY(KD, X, U)                                                                    \
  if (p.kind == KD && p.nx == X && p.nu == U) {                                                 \
    hipLaunchKernelGGL((nonlin_rollout_kernel<KD, X, U>), dim3((B + 63) / 64), dim3(64), 0, s, p, \
                       N, B, K, k, x, u, xn, un);                                               \
    return hipGetLastError();                                                                   \
  }
#include NOC_FAMILIES_DEF
#undef NOC_FAMILY
  return hipErrorInvalidValue;
}

}  // namespace noc
