// Interior-point DDP on the MI355X: the reference's third solver
// (noc/differential_dynamic_programming.py, "D"), the whole barrier schedule of every trajectory
// in ONE launch.
//
// DDP's backward pass is NOT the KKT scan: its Q-function carries the second-order dynamics terms
// Vx . fxx evaluated with the pass's own value gradient Vx_{k+1} (D:43-45), so the recursion is
// nonlinear in V and has no associative form; the forward pass is the nonlinear closed-loop
// rollout (D:73-90).  Both are horizon-sequential per trajectory, so the mapping is one lane per
// trajectory: the stage derivatives are evaluated on the fly from the nominal (x, u) (the same
// sympy-generated family code as the Newton solvers; Vx . fxx is add_hess_l with l = Vx), nothing
// is materialised but the gains k, K and the trial trajectory.  Every lane runs its own reference
// control flow (outer Newton loop D:105-170, retry loop D:114-152, barrier loop D:189-208).
// Layout: natural, per trajectory contiguous (x (Bt, N+1, nx), u (Bt, N, nu)); workspace
// include/noc_hip.h noc_ddp_work_doubles.
#include <hip/hip_runtime.h>

#include <cmath>

#include "../../include/noc_hip.h"
#include "ipm_family.h"
#include "noc_internal.h"

namespace noc {

struct DdpArgs {
  int N, Bt, max_passes;
  double bp0;
  const double* x0;
  double* u;
  double *X, *TX, *TU, *k, *K;
  int *iterations, *passes, *done;
};

template <int KIND, int NX, int NU>
__global__ __launch_bounds__(64) void ddp_solve_kernel(noc_family prm, DdpArgs a) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.Bt) return;
  const Fam<KIND, NX, NU> f(prm);
  const int N = a.N;
  double* ubuf = a.u + (size_t)b * N * NU;
  double* U = ubuf;
  double* TU = a.TU + (size_t)b * N * NU;
  double* X = a.X + (size_t)b * (N + 1) * NX;
  double* TX = a.TX + (size_t)b * (N + 1) * NX;
  double* kk = a.k + (size_t)b * N * NU;
  double* KK = a.K + (size_t)b * N * NU * NX;
  const double* x0 = a.x0 + (size_t)b * NX;

  // ocp.total_cost (PR:53-56 / CR:48-51): stage costs in stage order, then the final cost
  auto total_cost = [&](const double* Xs, const double* Us, double bp) {
    double c = 0.0;
    for (int t = 0; t < N; ++t) c += f.stage_cost(Xs + (size_t)t * NX, Us + (size_t)t * NU, bp);
    return c + f.final_cost(Xs + (size_t)N * NX);
  };

  double bp = a.bp0;
  int total_it = 0, passes = 0;
  bool capped = false;
  while (bp > 1e-4 && !capped) {  // ---------------- barrier schedule (D:189-208) ----------------
    // rollout of the current controls (D:101, U:57-63)
    {
      double x[NX];
      NOC_UNROLL for (int i = 0; i < NX; ++i) { x[i] = x0[i]; X[i] = x[i]; }
      for (int t = 0; t < N; ++t) {
        double xn[NX];
        f.step(x, U + (size_t)t * NU, xn);
        NOC_UNROLL for (int i = 0; i < NX; ++i) { x[i] = xn[i]; X[(size_t)(t + 1) * NX + i] = xn[i]; }
      }
    }
    double reg_param = 1.0, reg_inc = 2.0, hu_norm = 1.0;  // D:102-103, D:183
    int it = 0;
    while (!(hu_norm < 1e-4 || it > 500)) {  // ---------------- DDP iterations (D:167-170) -------
      const double cost = total_cost(X, U, bp);  // D:109
      // reg = rp * ||cu||_F of the nominal derivatives (D:34-35)
      double g2 = 0.0;
      for (int t = 0; t < N; ++t) {
        double cx[NX], cu[NU];
        f.stage_grad(X + (size_t)t * NX, U + (size_t)t * NU, bp, cx, cu);
        NOC_UNROLL for (int j = 0; j < NU; ++j) g2 += cu[j] * cu[j];
      }
      const double gnorm = sqrt(g2);
      double rp = reg_param, r_inc = reg_inc, hn = 0.0;
      int inner = 0;
      bool success = false;
      for (;;) {  // ---------------- retry loop (D:114-152) ----------------
        // backward pass (D:37-70): Vx_N, Vxx_N = grad, hessian of the final cost (D:58-59)
        const double reg = rp * gnorm;
        double Vx[NX], Vxx[NX * NX];
        {
          const double* xN = X + (size_t)N * NX;
          NOC_UNROLL for (int i = 0; i < NX; ++i) {
            Vx[i] = prm.wf[i] * f.err(xN, i);
            NOC_UNROLL for (int j = 0; j < NX; ++j) Vxx[i * NX + j] = (i == j) ? prm.wf[i] : 0.0;
          }
        }
        double pred = 0.0;
        bool feas = true;
        hn = 0.0;
        for (int t = N - 1; t >= 0; --t) {
          double x[NX], u[NU];
          NOC_UNROLL for (int i = 0; i < NX; ++i) x[i] = X[(size_t)t * NX + i];
          NOC_UNROLL for (int j = 0; j < NU; ++j) u[j] = U[(size_t)t * NU + j];
          double fx[NX * NX], fu[NX * NU], cx[NX], cu[NU];
          f.jac(x, u, fx, fu);
          f.stage_grad(x, u, bp, cx, cu);
          // cxx, cuu, cxu of the stage cost + the Vx-contracted dynamics Hessians (D:43-45)
          double Qxx[NX * NX], Quu[NU * NU], Qxu[NX * NU];
          NOC_UNROLL for (int i = 0; i < NX; ++i) NOC_UNROLL for (int j = 0; j < NX; ++j) Qxx[i * NX + j] = (i == j) ? prm.wx[i] : 0.0;
          NOC_UNROLL for (int i = 0; i < NU; ++i) NOC_UNROLL for (int j = 0; j < NU; ++j) Quu[i * NU + j] = (i == j) ? f.stage_cuu(u, bp, i) : 0.0;
          NOC_UNROLL for (int i = 0; i < NX * NU; ++i) Qxu[i] = 0.0;
          f.add_hess_l(x, u, Vx, Qxx, Quu, Qxu);
          // Qx = cx + fx'Vx, Qu = cu + fu'Vx (D:41-42); W = Vxx fx, Z = Vxx fu
          double Qx[NX], Qu[NU], W[NX * NX], Z[NX * NU];
          NOC_UNROLL for (int j = 0; j < NX; ++j) {
            double s = cx[j];
            NOC_UNROLL for (int i = 0; i < NX; ++i) s += fx[i * NX + j] * Vx[i];
            Qx[j] = s;
          }
          NOC_UNROLL for (int j = 0; j < NU; ++j) {
            double s = cu[j];
            NOC_UNROLL for (int i = 0; i < NX; ++i) s += fu[i * NU + j] * Vx[i];
            Qu[j] = s;
          }
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
          // Qxx += fx'Vxx fx, Qxu += fx'Vxx fu, Quu += fu'Vxx fu + reg I (D:43-46)
          NOC_UNROLL for (int i = 0; i < NX; ++i) {
            NOC_UNROLL for (int j = 0; j < NX; ++j) {
              double s = Qxx[i * NX + j];
              NOC_UNROLL for (int m = 0; m < NX; ++m) s += fx[m * NX + i] * W[m * NX + j];
              Qxx[i * NX + j] = s;
            }
            NOC_UNROLL for (int j = 0; j < NU; ++j) {
              double s = Qxu[i * NU + j];
              NOC_UNROLL for (int m = 0; m < NX; ++m) s += fx[m * NX + i] * Z[m * NU + j];
              Qxu[i * NU + j] = s;
            }
          }
          Sym<NU> Qs;
          NOC_UNROLL for (int i = 0; i < NU; ++i)
            NOC_UNROLL for (int j = i; j < NU; ++j) {
              double s = Quu[i * NU + j];
              NOC_UNROLL for (int m = 0; m < NX; ++m) s += fu[m * NU + i] * Z[m * NU + j];
              Qs(i, j) = s + (i == j ? reg : 0.0);
            }
          // Quu^-1 [Qu | Qux]; positive definiteness <=> eigh(Quu) > 0 (D:47-48, Sylvester)
          double Y[NU][NX + 1];
          NOC_UNROLL for (int i = 0; i < NU; ++i) {
            Y[i][0] = Qu[i];
            NOC_UNROLL for (int j = 0; j < NX; ++j) Y[i][1 + j] = Qxu[j * NU + i];
          }
          feas = ldl_solve<NU, NX + 1>(Qs, Y) && feas;
          // k = -Quu^-1 Qu, K = -Quu^-1 Qux (D:50-51); dV = -1/2 Qu'Quu^-1 Qu (D:53)
          NOC_UNROLL for (int i = 0; i < NU; ++i) {
            kk[(size_t)t * NU + i] = -Y[i][0];
            NOC_UNROLL for (int j = 0; j < NX; ++j) KK[((size_t)t * NU + i) * NX + j] = -Y[i][1 + j];
            pred += -0.5 * Qu[i] * Y[i][0];
            hn = fmax(hn, fabs(Qu[i]));  // Hu = Qu (D:56, D:120)
          }
          // Vx = Qx - Qu'Quu^-1 Qux, Vxx = Qxx - Qxu Quu^-1 Qux (D:54-55)
          NOC_UNROLL for (int j = 0; j < NX; ++j) {
            double s = Qx[j];
            NOC_UNROLL for (int i = 0; i < NU; ++i) s -= Qu[i] * Y[i][1 + j];
            Vx[j] = s;
          }
          NOC_UNROLL for (int i = 0; i < NX; ++i)
            NOC_UNROLL for (int j = 0; j < NX; ++j) {
              double s = Qxx[i * NX + j];
              NOC_UNROLL for (int m = 0; m < NU; ++m) s -= Qxu[i * NU + m] * Y[m][1 + j];
              Vxx[i * NX + j] = s;
            }
        }
        passes += 1;
        // nonlinear rollout of the closed loop (D:73-90) fused with check_feasibility (D:93-95)
        // and the trial cost (stage order, then the final cost, like total_cost above)
        bool ok = true;
        double tcost = 0.0;
        {
          double xh[NX];
          NOC_UNROLL for (int i = 0; i < NX; ++i) xh[i] = X[i];
          for (int t = 0; t < N; ++t) {
            double uh[NU], dxh[NX];
            NOC_UNROLL for (int i = 0; i < NX; ++i) dxh[i] = xh[i] - X[(size_t)t * NX + i];
            NOC_UNROLL for (int i = 0; i < NU; ++i) {
              double s = U[(size_t)t * NU + i] + kk[(size_t)t * NU + i];
              NOC_UNROLL for (int j = 0; j < NX; ++j) s += KK[((size_t)t * NU + i) * NX + j] * dxh[j];
              uh[i] = s;
            }
            NOC_UNROLL for (int i = 0; i < NX; ++i) TX[(size_t)t * NX + i] = xh[i];
            NOC_UNROLL for (int i = 0; i < NU; ++i) TU[(size_t)t * NU + i] = uh[i];
            ok = ok && f.feasible(uh);
            tcost += f.stage_cost(xh, uh, bp);
            double xn[NX];
            f.step(xh, uh, xn);
            NOC_UNROLL for (int i = 0; i < NX; ++i) xh[i] = xn[i];
          }
          NOC_UNROLL for (int i = 0; i < NX; ++i) TX[(size_t)N * NX + i] = xh[i];
          tcost += f.final_cost(xh);
        }
        const double new_cost = ok ? tcost : INFINITY;             // D:121-125
        const double gain = (new_cost - cost) / pred;               // D:126-127
        success = (gain > 0.0) && feas;                             // D:128
        rp = success ? rp * fmax(1.0 / 3.0, 1.0 - (2.0 * gain - 1.0) * (2.0 * gain - 1.0) * (2.0 * gain - 1.0))
                     : rp * reg_inc;                                // D:129-133: the OUTER reg_inc
        r_inc = success ? 2.0 : 2.0 * r_inc;                        // D:133
        rp = fmin(fmax(rp, 1e-16), 1e16);                           // D:135
        inner += 1;
        if (passes >= a.max_passes) capped = true;
        if (success || inner > 500 || capped) break;                // D:147-152
      }
      // the last trial becomes the nominal trajectory, accepted or not (D:154)
      double* t0 = X; X = TX; TX = t0;
      double* t1 = U; U = TU; TU = t1;
      reg_param = rp;
      reg_inc = r_inc;
      hu_norm = hn;
      it += 1;
      if (capped) break;
    }
    total_it += it;  // D:196
    bp = bp / 5.0;   // D:195
  }
  if (U != ubuf) {  // the final controls live in the trial buffer: copy them out
    for (int t = 0; t < N * NU; ++t) ubuf[t] = U[t];
  }
  if (X != a.X + (size_t)b * (N + 1) * NX) {  // and the final states into X
    double* Xo = a.X + (size_t)b * (N + 1) * NX;
    for (int t = 0; t < (N + 1) * NX; ++t) Xo[t] = X[t];
  }
  a.iterations[b] = total_it;
  a.passes[b] = passes;
  a.done[b] = capped ? 0 : 1;
}

template <int KIND, int NX, int NU>
static hipError_t ddp_t(const noc_family& p, const DdpArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((ddp_solve_kernel<KIND, NX, NU>), dim3((a.Bt + 63) / 64), dim3(64), 0, s, p, a);
  return hipGetLastError();
}

bool ddp_supported(const noc_family& p) {
  return family_supported(p) && p.nx <= 4;  // one lane holds the nx x nx value Hessian
}

hipError_t ddp_solve(const noc_family& p, int N, int Bt, const double* x0, double* u,
                     double* work, int* iterations, int* passes, int* done, double bp0,
                     int max_passes, hipStream_t s) {
  DdpArgs a{};
  a.N = N;
  a.Bt = Bt;
  a.max_passes = max_passes;
  a.bp0 = bp0;
  a.x0 = x0;
  a.u = u;
  const size_t nxs = (size_t)Bt * (N + 1) * p.nx, nus = (size_t)Bt * N * p.nu;
  a.X = work;
  a.TX = a.X + nxs;
  a.TU = a.TX + nxs;
  a.k = a.TU + nus;
  a.K = a.k + nus;
  a.iterations = iterations;
  a.passes = passes;
  a.done = done;
  switch (p.kind) {
    case NOC_FAMILY_PENDULUM:
      if (p.nx == 2 && p.nu == 1) return ddp_t<NOC_FAMILY_PENDULUM, 2, 1>(p, a, s);
      break;
    case NOC_FAMILY_CARTPOLE:
      if (p.nx == 4 && p.nu == 1) return ddp_t<NOC_FAMILY_CARTPOLE, 4, 1>(p, a, s);
      break;
    case NOC_FAMILY_LINEAR:
      if (p.nx == 2 && p.nu == 1) return ddp_t<NOC_FAMILY_LINEAR, 2, 1>(p, a, s);
      break;
    default: break;
  }
  return hipErrorInvalidValue;
}

}  // namespace noc
