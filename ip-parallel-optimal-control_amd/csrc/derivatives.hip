// The reference's building blocks of one Newton step as standalone batched kernels -- the API the
// fused interior-point kernels (ipm_kernels.hip, ipm_persistent.hip) inline:
//   compute_derivatives  P:13-28 == S:10-25   per-stage grad / Hessian of the stage cost and
//                                             Jacobian / second derivatives of the dynamics
//   grad / hessian of final_cost              C:35, S:66 (the terminal costate / value Hessian)
//   par_costates / seq_costates  C:34-54      lambda_k = cx_k + fx_k' lambda_{k+1}, lambda_N given
//   compute_lqr_params   P:31-42 == S:28-39   ru, Q, R, M from lambda and the derivatives
// All arrays natural layout (leading batch axis B, then the reference's shapes), fp64.
#include <hip/hip_runtime.h>

#include "../../include/noc_hip.h"
#include "ipm_family.h"
#include "noc_internal.h"
#include "small_linalg.h"

namespace noc {

// one thread per (trajectory, stage)
template <int KIND, int NX, int NU>
__global__ __launch_bounds__(256) void derivatives_kernel(noc_family prm, DerivArgs a) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)a.B * a.N) return;
  const int N = a.N;
  const long long b = t / N;
  const size_t bk = (size_t)t;  // b * N + k
  const int k = (int)(t - b * N);
  Fam<KIND, NX, NU> f(prm);
  double x[NX], u[NU];
  NOC_UNROLL for (int i = 0; i < NX; ++i) x[i] = a.x[((size_t)b * (N + 1) + k) * NX + i];
  NOC_UNROLL for (int j = 0; j < NU; ++j) u[j] = a.u[bk * NU + j];
  const double bp = a.bp[b];
  double cx[NX], cu[NU];
  f.stage_grad(x, u, bp, cx, cu);
  NOC_UNROLL for (int i = 0; i < NX; ++i) a.cx[bk * NX + i] = cx[i];
  NOC_UNROLL for (int j = 0; j < NU; ++j) a.cu[bk * NU + j] = cu[j];
  // cxx, cuu, cxu: the stage cost's Hessian (ipm_family.h: stage_hess; for the quadratic-plus-
  // log-barrier cost of PR:40-50 / CR:36-45 diag(wx), diag(wu + barrier), 0 -- the wrapped
  // coordinate's mod has derivative 1)
  {
    double cxx[NX * NX], cuu[NU * NU], cxu[NX * NU];
    f.stage_hess(x, u, bp, cxx, cuu, cxu);
    NOC_UNROLL for (int i = 0; i < NX * NX; ++i) a.cxx[bk * NX * NX + i] = cxx[i];
    NOC_UNROLL for (int i = 0; i < NU * NU; ++i) a.cuu[bk * NU * NU + i] = cuu[i];
    NOC_UNROLL for (int i = 0; i < NX * NU; ++i) a.cxu[bk * NX * NU + i] = cxu[i];
  }
  double fx[NX * NX], fu[NX * NU];
  f.jac(x, u, fx, fu);
  NOC_UNROLL for (int i = 0; i < NX * NX; ++i) a.fx[bk * NX * NX + i] = fx[i];
  NOC_UNROLL for (int i = 0; i < NX * NU; ++i) a.fu[bk * NX * NU + i] = fu[i];
  // fxx[i] = d2 f_i / dx dx etc. (jacrev(jacrev(dynamics)) shapes (nx, nx, nx), (nx, nu, nu),
  // (nx, nx, nu)): the lambda-contracted Hessian at lambda = e_i
  NOC_UNROLL for (int i = 0; i < NX; ++i) {
    double l[NX], Hxx[NX * NX], Huu[NU * NU], Hxu[NX * NU];
    NOC_UNROLL for (int m = 0; m < NX; ++m) l[m] = (m == i) ? 1.0 : 0.0;
    NOC_UNROLL for (int m = 0; m < NX * NX; ++m) Hxx[m] = 0.0;
    NOC_UNROLL for (int m = 0; m < NU * NU; ++m) Huu[m] = 0.0;
    NOC_UNROLL for (int m = 0; m < NX * NU; ++m) Hxu[m] = 0.0;
    f.add_hess_l(x, u, l, Hxx, Huu, Hxu);
    NOC_UNROLL for (int m = 0; m < NX * NX; ++m) a.fxx[(bk * NX + i) * NX * NX + m] = Hxx[m];
    NOC_UNROLL for (int m = 0; m < NU * NU; ++m) a.fuu[(bk * NX + i) * NU * NU + m] = Huu[m];
    NOC_UNROLL for (int m = 0; m < NX * NU; ++m) a.fxu[(bk * NX + i) * NX * NU + m] = Hxu[m];
  }
}

// grad / hessian of final_cost at x_N (one thread per trajectory)
template <int KIND, int NX, int NU>
__global__ __launch_bounds__(256) void final_derivs_kernel(noc_family prm, int B, const double* xN,
                                                           double* grad, double* hess) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  Fam<KIND, NX, NU> f(prm);
  double x[NX];
  NOC_UNROLL for (int i = 0; i < NX; ++i) x[i] = xN[(size_t)b * NX + i];
  double g[NX];
  f.final_grad(x, g);
  NOC_UNROLL for (int i = 0; i < NX; ++i) grad[(size_t)b * NX + i] = g[i];
  if (hess) {
    double H[NX * NX];
    f.final_hess(x, H);
    NOC_UNROLL for (int i = 0; i < NX * NX; ++i) hess[(size_t)b * NX * NX + i] = H[i];
  }
}

template <int KIND, int NX, int NU>
static hipError_t derivs_family(const noc_family& p, const DerivArgs& a, hipStream_t s) {
  const long long n = (long long)a.B * a.N;
  hipLaunchKernelGGL((derivatives_kernel<KIND, NX, NU>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     s, p, a);
  return hipGetLastError();
}

hipError_t derivatives(const noc_family& p, const DerivArgs& a, hipStream_t s) {
#define NOC_FAMILY(K, X, U) \
  if (p.kind == K && p.nx == X && p.nu == U) return derivs_family<K, X, U>(p, a, s);
#include NOC_FAMILIES_DEF
#undef NOC_FAMILY
  return hipErrorInvalidValue;
}

hipError_t final_cost_derivs(const noc_family& p, int B, const double* xN, double* grad,
                             double* hess, hipStream_t s) {
#define NOC_FAMILY(K, X, U)                                                                     \
  if (p.kind == K && p.nx == X && p.nu == U) {                                                  \
    hipLaunchKernelGGL((final_derivs_kernel<K, X, U>), dim3((B + 255) / 256), dim3(256), 0, s, \
                       p, B, xN, grad, hess);                                                   \
    return hipGetLastError();                                                                   \
  }
#include NOC_FAMILIES_DEF
#undef NOC_FAMILY
  return hipErrorInvalidValue;
}

// ------------------------------------------------------------------------------------------------
// check_traj_feasibility (P:45-47) / check_feasibility (S:93-95): all(constraints(x_k, u_k) <= 0)
// over k < N -- the family's whole constraint vector (the u box of the built-ins, a registered
// family's traced constraints(x, u) incl. state constraints; NaN compares false, as jnp's <= does).
// One wave64 per trajectory, lanes stride the stages, the verdict is the wave's vote.
template <int KIND, int NX, int NU>
__global__ __launch_bounds__(64) void feasibility_kernel(noc_family prm, int N, int B,
                                                         const double* x, const double* u, int* ok) {
  const int b = blockIdx.x;
  if (b >= B) return;
  Fam<KIND, NX, NU> f(prm);
  bool good = true;
  for (int k = threadIdx.x; k < N; k += 64) {
    double xk[NX], uk[NU];
    NOC_UNROLL for (int i = 0; i < NX; ++i) xk[i] = x[((size_t)b * (N + 1) + k) * NX + i];
    NOC_UNROLL for (int j = 0; j < NU; ++j) uk[j] = u[((size_t)b * N + k) * NU + j];
    good = good && f.feasible(xk, uk);
  }
  const bool all = __all(good);
  if (threadIdx.x == 0) ok[b] = all ? 1 : 0;
}

hipError_t traj_feasibility(const noc_family& p, int N, int B, const double* x, const double* u,
                            int* ok, hipStream_t s) {
#define NOC_FAMILY(K, X, U)                                                                   \
  if (p.kind == K && p.nx == X && p.nu == U) {                                                \
    hipLaunchKernelGGL((feasibility_kernel<K, X, U>), dim3(B), dim3(64), 0, s, p, N, B, x, u, \
                       ok);                                                                   \
    return hipGetLastError();                                                                 \
  }
#include NOC_FAMILIES_DEF
#undef NOC_FAMILY
  return hipErrorInvalidValue;
}

// total_cost(x, u, bp) = final_cost(x_N) + sum_k stage_cost(x_k, u_k, bp) (PR:53-56, CR:48-51,
// LD:45-48; the OCP's own callable for a traced family).  One wave64 per trajectory, lanes
// stride the stages, the wave's butterfly sum; bp per trajectory.
template <int KIND, int NX, int NU>
__global__ __launch_bounds__(64) void total_cost_kernel(noc_family prm, int N, int B,
                                                        const double* x, const double* u,
                                                        const double* bp, double* cost) {
  const int b = blockIdx.x;
  if (b >= B) return;
  Fam<KIND, NX, NU> f(prm);
  const double bpb = bp[b];
  double s = 0.0;
  for (int k = threadIdx.x; k < N; k += 64) {
    double xk[NX], uk[NU];
    NOC_UNROLL for (int i = 0; i < NX; ++i) xk[i] = x[((size_t)b * (N + 1) + k) * NX + i];
    NOC_UNROLL for (int j = 0; j < NU; ++j) uk[j] = u[((size_t)b * N + k) * NU + j];
    s += f.stage_cost(xk, uk, bpb);
  }
  s = wave_sum(s);
  if (threadIdx.x == 0) {
    double xN[NX];
    NOC_UNROLL for (int i = 0; i < NX; ++i) xN[i] = x[((size_t)b * (N + 1) + N) * NX + i];
    cost[b] = f.final_cost(xN) + s;
  }
}

hipError_t total_cost(const noc_family& p, int N, int B, const double* x, const double* u,
                      const double* bp, double* cost, hipStream_t s) {
#define NOC_FAMILY(K, X, U)                                                                    \
  if (p.kind == K && p.nx == X && p.nu == U) {                                                 \
    hipLaunchKernelGGL((total_cost_kernel<K, X, U>), dim3(B), dim3(64), 0, s, p, N, B, x, u, bp, \
                       cost);                                                                  \
    return hipGetLastError();                                                                  \
  }
#include NOC_FAMILIES_DEF
#undef NOC_FAMILY
  return hipErrorInvalidValue;
}

// ------------------------------------------------------------------------------------------------
// costates lambda_k = cx_k + fx_k' lambda_{k+1} (C:43-54), lambda_N = lamT.
// sequential (seq_costates, lax.scan): one thread per trajectory, the recurrence in stage order.
template <int NX>
__global__ __launch_bounds__(64) void costates_seq_kernel(int N, int B, const double* lamT,
                                                          const double* cx, const double* fx,
                                                          double* lam) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double l[NX];
  NOC_UNROLL for (int i = 0; i < NX; ++i) l[i] = lamT[(size_t)b * NX + i];
  double* L = lam + (size_t)b * (N + 1) * NX;
  NOC_UNROLL for (int i = 0; i < NX; ++i) L[(size_t)N * NX + i] = l[i];
  for (int k = N - 1; k >= 0; --k) {
    const double* F = fx + ((size_t)b * N + k) * NX * NX;
    const double* c = cx + ((size_t)b * N + k) * NX;
    double ln[NX];
    NOC_UNROLL for (int i = 0; i < NX; ++i) {
      double t = c[i];
      NOC_UNROLL for (int m = 0; m < NX; ++m) t += F[m * NX + i] * l[m];
      ln[i] = t;
    }
    NOC_UNROLL for (int i = 0; i < NX; ++i) { l[i] = ln[i]; L[(size_t)k * NX + i] = ln[i]; }
  }
}

// parallel (par_costates, lax.associative_scan of the affine maps, C:6-40): one wave per
// trajectory, lane l composes its horizon chunk's map lambda_start = G lambda_end + g, a reverse
// Hillis-Steele scan over the 64 lanes gives every chunk its true end costate, then each lane
// sweeps its chunk.
template <int NX>
__global__ __launch_bounds__(64) void costates_par_kernel(int N, int B, const double* lamT,
                                                          const double* cx, const double* fx,
                                                          double* lam) {
  constexpr int L = 64;
  const int b = blockIdx.x, l = threadIdx.x;
  if (b >= B) return;
  const Chunks ch(N, L);
  const int start = ch.start(l), len = ch.len(l);
  const bool last = (l == L - 1);
  double lamN[NX];
  NOC_UNROLL for (int i = 0; i < NX; ++i) lamN[i] = lamT[(size_t)b * NX + i];
  auto Fk = [&](int k) { return fx + ((size_t)b * N + k) * NX * NX; };
  auto ck = [&](int k) { return cx + ((size_t)b * N + k) * NX; };
  Mat<NX, NX> G;
  Vec<NX> g;
  set_identity(G);
  set_zero(g);
  for (int k = start + len - 1; k >= start; --k) {
    const double* F = Fk(k);
    const double* c = ck(k);
    Mat<NX, NX> Gn;
    Vec<NX> gn;
    NOC_UNROLL for (int i = 0; i < NX; ++i) {
      double t = c[i];
      NOC_UNROLL for (int m = 0; m < NX; ++m) t += F[m * NX + i] * g[m];
      gn[i] = t;
      NOC_UNROLL for (int j = 0; j < NX; ++j) {
        double u = 0.0;
        NOC_UNROLL for (int m = 0; m < NX; ++m) u += F[m * NX + i] * G(m, j);
        Gn(i, j) = u;
      }
    }
    G = Gn;
    g = gn;
  }
  if (last) {
    NOC_UNROLL for (int i = 0; i < NX; ++i) {
      double t = g[i];
      NOC_UNROLL for (int m = 0; m < NX; ++m) t += G(i, m) * lamN[m];
      g[i] = t;
    }
    set_zero(G);
  }
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
  double lm[NX];
  shfl_down_arr<NX>(g.v, lm, 1, L);
  if (last) NOC_UNROLL for (int i = 0; i < NX; ++i) lm[i] = lamN[i];
  double* LAM = lam + (size_t)b * (N + 1) * NX;
  if (last) NOC_UNROLL for (int i = 0; i < NX; ++i) LAM[(size_t)N * NX + i] = lamN[i];
  for (int k = start + len - 1; k > start; --k) {
    const double* F = Fk(k);
    const double* c = ck(k);
    double ln[NX];
    NOC_UNROLL for (int i = 0; i < NX; ++i) {
      double t = c[i];
      NOC_UNROLL for (int m = 0; m < NX; ++m) t += F[m * NX + i] * lm[m];
      ln[i] = t;
    }
    NOC_UNROLL for (int i = 0; i < NX; ++i) { lm[i] = ln[i]; LAM[(size_t)k * NX + i] = ln[i]; }
  }
  // the chunk start's costate is the scan's value (what the previous lane used as its end)
  if (len > 0) NOC_UNROLL for (int i = 0; i < NX; ++i) LAM[(size_t)start * NX + i] = g[i];
}

template <int NX>
static hipError_t costates_nx(int N, int B, const double* lamT, const double* cx, const double* fx,
                              double* lam, int sequential, hipStream_t s) {
  if (sequential)
    hipLaunchKernelGGL((costates_seq_kernel<NX>), dim3((B + 63) / 64), dim3(64), 0, s, N, B, lamT,
                       cx, fx, lam);
  else
    hipLaunchKernelGGL((costates_par_kernel<NX>), dim3(B), dim3(64), 0, s, N, B, lamT, cx, fx, lam);
  return hipGetLastError();
}

hipError_t costates(int nx, int N, int B, const double* lamT, const double* cx, const double* fx,
                    double* lam, int sequential, hipStream_t s) {
  switch (nx) {
    case 1: return costates_nx<1>(N, B, lamT, cx, fx, lam, sequential, s);
    case 2: return costates_nx<2>(N, B, lamT, cx, fx, lam, sequential, s);
    case 3: return costates_nx<3>(N, B, lamT, cx, fx, lam, sequential, s);
    case 4: return costates_nx<4>(N, B, lamT, cx, fx, lam, sequential, s);
    case 5: return costates_nx<5>(N, B, lamT, cx, fx, lam, sequential, s);
    case 6: return costates_nx<6>(N, B, lamT, cx, fx, lam, sequential, s);
    case 7: return costates_nx<7>(N, B, lamT, cx, fx, lam, sequential, s);
    case 8: return costates_nx<8>(N, B, lamT, cx, fx, lam, sequential, s);
    default: return hipErrorInvalidValue;
  }
}

// ------------------------------------------------------------------------------------------------
// compute_lqr_params (P:31-42): one thread per (trajectory, stage), l = lambda_{k+1}
//   ru = cu + fu' l,  Q = cxx + l . fxx,  R = cuu + l . fuu,  M = cxu + l . fxu
__global__ __launch_bounds__(256) void lqr_params_kernel(LqrArgs a) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)a.B * a.N) return;
  const int nx = a.nx, nu = a.nu, N = a.N;
  const long long b = t / N;
  const size_t bk = (size_t)t;
  const int k = (int)(t - b * N);
  const double* l = a.lam + ((size_t)b * (N + 1) + k + 1) * nx;
  for (int j = 0; j < nu; ++j) {
    double s = a.cu[bk * nu + j];
    for (int i = 0; i < nx; ++i) s += a.fu[(bk * nx + i) * nu + j] * l[i];
    a.ru[bk * nu + j] = s;
  }
  for (int i = 0; i < nx; ++i)
    for (int j = 0; j < nx; ++j) {
      double s = a.cxx[(bk * nx + i) * nx + j];
      for (int m = 0; m < nx; ++m) s += l[m] * a.fxx[((bk * nx + m) * nx + i) * nx + j];
      a.Q[(bk * nx + i) * nx + j] = s;
    }
  for (int i = 0; i < nu; ++i)
    for (int j = 0; j < nu; ++j) {
      double s = a.cuu[(bk * nu + i) * nu + j];
      for (int m = 0; m < nx; ++m) s += l[m] * a.fuu[((bk * nx + m) * nu + i) * nu + j];
      a.R[(bk * nu + i) * nu + j] = s;
    }
  for (int i = 0; i < nx; ++i)
    for (int j = 0; j < nu; ++j) {
      double s = a.cxu[(bk * nx + i) * nu + j];
      for (int m = 0; m < nx; ++m) s += l[m] * a.fxu[((bk * nx + m) * nx + i) * nu + j];
      a.M[(bk * nx + i) * nu + j] = s;
    }
}

hipError_t lqr_params(const LqrArgs& a, hipStream_t s) {
  const long long n = (long long)a.B * a.N;
  hipLaunchKernelGGL(lqr_params_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace noc
