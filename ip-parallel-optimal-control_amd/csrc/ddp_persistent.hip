// Interior-point DDP on the MI355X: the reference's third solver
// (noc/differential_dynamic_programming.py, "D"), the whole barrier schedule of every trajectory
// in ONE launch, one wave64 per trajectory.
//
// DDP's backward pass is NOT the KKT scan: its Q-function carries the second-order dynamics terms
// Vx . fxx evaluated with the pass's own value gradient Vx_{k+1} (D:43-45), so the recursion is
// nonlinear in V and has no associative form; the forward pass is the nonlinear closed-loop
// rollout (D:73-90).  Both recursions are horizon-sequential.  What is NOT sequential is the
// expensive part of a backward step -- the stage derivatives at the nominal (x, u) (the generated
// family code: sincos, divisions), which are the same for every retry of an iteration.  So:
//   * derivatives: the 64 lanes evaluate them stage-parallel once per DDP iteration into a
//     per-stage record (fx, fu, cx, cu, cuu and the full second-derivative tensors d2f_i, taken
//     as add_hess_l with l = e_i), written to HBM / L2;
//   * backward pass: wave-uniform (every lane runs the same recursion; lane 0 stores k, K),
//     reading the records -- only the Vx contraction and the Riccati-like algebra remain;
//   * rollouts: wave-uniform recurrence (lane 0 stores), then trial cost and feasibility
//     stage-parallel with wave reductions (cost summed chunk-wise in stage order, then across
//     lanes: the summation order of the multi-lane Newton kernels).
// Every wave follows its own trajectory's reference control flow (outer Newton loop D:105-170,
// retry loop D:114-152, barrier loop D:189-208).  Layout: natural, per trajectory contiguous
// (x (Bt, N+1, nx), u (Bt, N, nu)); workspace include/noc_hip.h noc_ddp_work_doubles.
#include <hip/hip_runtime.h>
#include <cstdlib>

#include <cmath>

#include "../../include/noc_hip.h"
#include "ipm_family.h"
#include "noc_internal.h"

namespace noc {

// Diagnostic per-pass trace of the DDP decisions (tools/ddp_trace_diff.py), set by the debug
// export noc_debug_set_ddp_trace (not part of the ABI header); NULL in product use.
__device__ double* g_ddp_trace = nullptr;
__device__ int g_ddp_trace_cap = 0;
__device__ int g_ddp_trace_traj = 0;

struct DdpArgs {
  int N, Bt, max_passes;
  int skip_repeats;  // account the identical retries at the rp clip without recomputing them
  int one_stage;     // NOC_DDP_ONE_STAGE: ddp(ocp, u, x0, bp) -- one barrier value (D:98-186)
  double bp0;
  const double* x0;
  double* u;
  double *X, *TX, *TU, *k, *K, *rec;
  int *iterations, *passes, *done;
};

// per-stage derivative record: fx | fu | cx | cu | cxx | cuu | cxu (the stage cost's full Hessian,
// D:43-45 -- a registered family's traced cost is not diagonal) | Hxx_i | Hxu_i | Huu_i (i < nx)
template <int NX, int NU>
struct Rec {
  static constexpr int FX = 0, FU = FX + NX * NX, CX = FU + NX * NU, CU = CX + NX, CXX = CU + NU,
                       CUU = CXX + NX * NX, CXU = CUU + NU * NU, HXX = CXU + NX * NU,
                       HXU = HXX + NX * NX * NX, HUU = HXU + NX * NX * NU,
                       SIZE = HUU + NX * NU * NU;
};

NOC_DEV void ddp_fence() { __threadfence_block(); }  // this wave's global stores before its loads

template <int KIND, int NX, int NU>
__global__ __launch_bounds__(64) void ddp_solve_kernel(noc_family prm, DdpArgs a) {
  using R = Rec<NX, NU>;
  const int b = blockIdx.x;  // one wave per trajectory
  const int l = threadIdx.x;
  if (b >= a.Bt) return;
  const Fam<KIND, NX, NU> f(prm);
  const int N = a.N;
  const Chunks ch(N, 64);
  const int start = ch.start(l), len = ch.len(l);
  double* const ubuf = a.u + (size_t)b * N * NU;
  double* const xbuf = a.X + (size_t)b * (N + 1) * NX;
  double* U = ubuf;
  double* TU = a.TU + (size_t)b * N * NU;
  double* X = xbuf;
  double* TX = a.TX + (size_t)b * (N + 1) * NX;
  double* kk = a.k + (size_t)b * N * NU;
  double* KK = a.K + (size_t)b * N * NU * NX;
  double* rec = a.rec + (size_t)b * N * R::SIZE;
  const double* x0 = a.x0 + (size_t)b * NX;
  const bool lead = (l == 0);

  // ocp.total_cost (PR:53-56 / CR:48-51) and check_feasibility (D:93-95) of (Xs, Us), lane-parallel
  auto cost_feas = [&](const double* Xs, const double* Us, double bp, bool& feasible) {
    double c = 0.0;
    bool ok = true;
    for (int t = start; t < start + len; ++t) {
      ok = ok && f.feasible(Xs + (size_t)t * NX, Us + (size_t)t * NU);
      c += f.stage_cost(Xs + (size_t)t * NX, Us + (size_t)t * NU, bp);
    }
    feasible = __all(ok);
    return wave_sum(c) + f.final_cost(Xs + (size_t)N * NX);
  };

  double bp = a.bp0;
  int total_it = 0, passes = 0;
  bool capped = false;
  // ddp() at one barrier value (NOC_DDP_ONE_STAGE) runs whatever that value is (D:98-186)
  while ((a.one_stage || bp > 1e-4) && !capped) {  // ------- barrier schedule (D:189-208) -------
    // rollout of the current controls (D:101, U:57-63): wave-uniform recurrence, lane 0 stores
    {
      double x[NX];
      NOC_UNROLL for (int i = 0; i < NX; ++i) x[i] = x0[i];
      if (lead) NOC_UNROLL for (int i = 0; i < NX; ++i) X[i] = x[i];
      for (int t = 0; t < N; ++t) {
        double xn[NX];
        f.step(x, U + (size_t)t * NU, xn);
        NOC_UNROLL for (int i = 0; i < NX; ++i) x[i] = xn[i];
        if (lead) NOC_UNROLL for (int i = 0; i < NX; ++i) X[(size_t)(t + 1) * NX + i] = xn[i];
      }
    }
    ddp_fence();
    double reg_param = 1.0, reg_inc = 2.0, hu_norm = 1.0;  // D:102-103, D:183
    int it = 0;
    while (!(hu_norm < 1e-4 || it > 500)) {  // ---------------- DDP iterations (D:167-170) -------
      bool unused;
      const double cost = cost_feas(X, U, bp, unused);  // D:109
      // stage derivatives at the nominal trajectory (D:112), stage-parallel; ||cu||_F (D:34)
      double g2 = 0.0;
      for (int t = start; t < start + len; ++t) {
        const double* x = X + (size_t)t * NX;
        const double* u = U + (size_t)t * NU;
        double* r = rec + (size_t)t * R::SIZE;
        double fx[NX * NX], fu[NX * NU], cx[NX], cu[NU];
        f.jac(x, u, fx, fu);
        f.stage_grad(x, u, bp, cx, cu);
        NOC_UNROLL for (int i = 0; i < NX * NX; ++i) r[R::FX + i] = fx[i];
        NOC_UNROLL for (int i = 0; i < NX * NU; ++i) r[R::FU + i] = fu[i];
        NOC_UNROLL for (int i = 0; i < NX; ++i) r[R::CX + i] = cx[i];
        NOC_UNROLL for (int j = 0; j < NU; ++j) {
          r[R::CU + j] = cu[j];
          g2 += cu[j] * cu[j];
        }
        if constexpr (Fam<KIND, NX, NU>::kGenCost) {  // cxx, cuu, cxu of a traced cost
          double cxx[NX * NX], cuu[NU * NU], cxu[NX * NU];
          f.stage_hess(x, u, bp, cxx, cuu, cxu);
          NOC_UNROLL for (int i = 0; i < NX * NX; ++i) r[R::CXX + i] = cxx[i];
          NOC_UNROLL for (int i = 0; i < NU * NU; ++i) r[R::CUU + i] = cuu[i];
          NOC_UNROLL for (int i = 0; i < NX * NU; ++i) r[R::CXU + i] = cxu[i];
        } else {  // the parametrised cost: only the cuu diagonal varies along the trajectory
          NOC_UNROLL for (int j = 0; j < NU; ++j) r[R::CUU + j * NU + j] = f.stage_cuu(u, bp, j);
        }
        if constexpr (KIND != NOC_FAMILY_LINEAR) {  // d2 f_i = add_hess_l with l = e_i
          NOC_UNROLL for (int i = 0; i < NX; ++i) {
            double e[NX], hxx[NX * NX], huu[NU * NU], hxu[NX * NU];
            NOC_UNROLL for (int m = 0; m < NX; ++m) e[m] = (m == i) ? 1.0 : 0.0;
            NOC_UNROLL for (int m = 0; m < NX * NX; ++m) hxx[m] = 0.0;
            NOC_UNROLL for (int m = 0; m < NU * NU; ++m) huu[m] = 0.0;
            NOC_UNROLL for (int m = 0; m < NX * NU; ++m) hxu[m] = 0.0;
            f.add_hess_l(x, u, e, hxx, huu, hxu);
            NOC_UNROLL for (int m = 0; m < NX * NX; ++m) r[R::HXX + i * NX * NX + m] = hxx[m];
            NOC_UNROLL for (int m = 0; m < NX * NU; ++m) r[R::HXU + i * NX * NU + m] = hxu[m];
            NOC_UNROLL for (int m = 0; m < NU * NU; ++m) r[R::HUU + i * NU * NU + m] = huu[m];
          }
        }
      }
      const double gnorm = sqrt(wave_sum(g2));
      ddp_fence();
      double rp = reg_param, r_inc = reg_inc, hn = 0.0;
      int inner = 0;
      bool success = false;
      for (;;) {  // ---------------- retry loop (D:114-152) ----------------
        // backward pass (D:37-70), wave-uniform: Vx_N, Vxx_N = grad, hessian of the final cost
        const double reg = rp * gnorm;
        double Vx[NX], Vxx[NX * NX];
        {
          const double* xN = X + (size_t)N * NX;
          f.final_grad(xN, Vx);
          f.final_hess(xN, Vxx);
        }
        double pred = 0.0;
        bool feas = true;
        hn = 0.0;
        for (int t = N - 1; t >= 0; --t) {
          const double* r = rec + (size_t)t * R::SIZE;
          double fx[NX * NX], fu[NX * NU];
          NOC_UNROLL for (int i = 0; i < NX * NX; ++i) fx[i] = r[R::FX + i];
          NOC_UNROLL for (int i = 0; i < NX * NU; ++i) fu[i] = r[R::FU + i];
          // cxx, cxu, cuu (the stage cost's Hessian); + Vx . d2f (D:43-45).  The parametrised cost's
          // Hessian is diag(wx), 0, diag(cuu): formed from the descriptor and the cuu diagonal
          // (the same values as the record's, without loading them on this sequential path)
          double Qxx[NX * NX], Quu[NU * NU], Qxu[NX * NU];
          if constexpr (Fam<KIND, NX, NU>::kGenCost) {
            NOC_UNROLL for (int i = 0; i < NX * NX; ++i) Qxx[i] = r[R::CXX + i];
            NOC_UNROLL for (int i = 0; i < NU * NU; ++i) Quu[i] = r[R::CUU + i];
            NOC_UNROLL for (int i = 0; i < NX * NU; ++i) Qxu[i] = r[R::CXU + i];
          } else {
            NOC_UNROLL for (int i = 0; i < NX; ++i) NOC_UNROLL for (int j = 0; j < NX; ++j) Qxx[i * NX + j] = (i == j) ? prm.wx[i] : 0.0;
            NOC_UNROLL for (int i = 0; i < NU; ++i) NOC_UNROLL for (int j = 0; j < NU; ++j) Quu[i * NU + j] = (i == j) ? r[R::CUU + i * NU + i] : 0.0;
            NOC_UNROLL for (int i = 0; i < NX * NU; ++i) Qxu[i] = 0.0;
          }
          if constexpr (KIND != NOC_FAMILY_LINEAR) {
            NOC_UNROLL for (int i = 0; i < NX; ++i) {
              NOC_UNROLL for (int m = 0; m < NX * NX; ++m) Qxx[m] += Vx[i] * r[R::HXX + i * NX * NX + m];
              NOC_UNROLL for (int m = 0; m < NX * NU; ++m) Qxu[m] += Vx[i] * r[R::HXU + i * NX * NU + m];
              NOC_UNROLL for (int m = 0; m < NU * NU; ++m) Quu[m] += Vx[i] * r[R::HUU + i * NU * NU + m];
            }
          }
          // Qx = cx + fx'Vx, Qu = cu + fu'Vx (D:41-42); W = Vxx fx, Z = Vxx fu
          double Qx[NX], Qu[NU], W[NX * NX], Z[NX * NU];
          NOC_UNROLL for (int j = 0; j < NX; ++j) {
            double s = r[R::CX + j];
            NOC_UNROLL for (int i = 0; i < NX; ++i) s += fx[i * NX + j] * Vx[i];
            Qx[j] = s;
          }
          NOC_UNROLL for (int j = 0; j < NU; ++j) {
            double s = r[R::CU + j];
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
            if (lead) {
              kk[(size_t)t * NU + i] = -Y[i][0];
              NOC_UNROLL for (int j = 0; j < NX; ++j) KK[((size_t)t * NU + i) * NX + j] = -Y[i][1 + j];
            }
            pred += -0.5 * Qu[i] * Y[i][0];
            hn = nan_max(hn, fabs(Qu[i]));  // Hu = Qu (D:56, D:120)
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
        ddp_fence();
        // nonlinear rollout of the closed loop (D:73-90): wave-uniform, lane 0 stores
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
            if (lead) {
              NOC_UNROLL for (int i = 0; i < NX; ++i) TX[(size_t)t * NX + i] = xh[i];
              NOC_UNROLL for (int i = 0; i < NU; ++i) TU[(size_t)t * NU + i] = uh[i];
            }
            double xn[NX];
            f.step(xh, uh, xn);
            NOC_UNROLL for (int i = 0; i < NX; ++i) xh[i] = xn[i];
          }
          if (lead) NOC_UNROLL for (int i = 0; i < NX; ++i) TX[(size_t)N * NX + i] = xh[i];
        }
        ddp_fence();
        bool ok;
        const double tcost = cost_feas(TX, TU, bp, ok);
        const double new_cost = ok ? tcost : INFINITY;             // D:121-125
        const double gain = (new_cost - cost) / pred;               // D:126-127
        success = (gain > 0.0) && feas;                             // D:128
        const double rp_used = rp;
        rp = success ? rp * rp_shrink(gain)
                     : rp * reg_inc;                                // D:129-133: the OUTER reg_inc
        r_inc = success ? 2.0 : 2.0 * r_inc;                        // D:133
        rp = fmin(fmax(rp, 1e-16), 1e16);                           // D:135
        inner += 1;
        // identical retries at the rp clip (the par rule, noc_internal.h par_retry_repeats): a
        // rejected pass at rp = 1e16 leaves every input of the next pass unchanged (records, X, U,
        // rp; reg_inc is the outer one), so the retries up to the cap repeat it bit for bit
        if (a.skip_repeats && !g_ddp_trace && !success && rp == rp_used && inner <= 500) {
          const int room = a.max_passes - passes;
          const int k = (501 - inner) < room ? (501 - inner) : (room > 0 ? room : 0);
          inner += k;
          passes += k;
          r_inc = ldexp(r_inc, k);  // D:133 per retry
        }
        if (g_ddp_trace && lead && b < g_ddp_trace_traj && passes <= g_ddp_trace_cap) {
          // diagnostic trace (noc_debug_set_ddp_trace; off in product use): one record per pass
          double* tr = g_ddp_trace + ((size_t)b * g_ddp_trace_cap + (passes - 1)) * 10;
          tr[0] = bp; tr[1] = it; tr[2] = inner; tr[3] = pred; tr[4] = gain;
          tr[5] = success ? 1.0 : 0.0; tr[6] = rp; tr[7] = hn; tr[8] = cost; tr[9] = new_cost;
        }
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
    if (a.one_stage) break;
  }
  // the final controls / states may live in the trial buffers: copy them out (lane-parallel)
  if (U != ubuf) for (int i = l; i < N * NU; i += 64) ubuf[i] = U[i];
  if (X != xbuf) for (int i = l; i < (N + 1) * NX; i += 64) xbuf[i] = X[i];
  if (lead) {
    a.iterations[b] = total_it;
    a.passes[b] = passes;
    a.done[b] = capped ? 0 : 1;
  }
}

template <int KIND, int NX, int NU>
static hipError_t ddp_t(const noc_family& p, const DdpArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((ddp_solve_kernel<KIND, NX, NU>), dim3(a.Bt), dim3(64), 0, s, p, a);
  return hipGetLastError();
}

// instances for nx <= 4 only (a template: the others are never instantiated)
template <int K, int X, int U>
static hipError_t ddp_family(const noc_family& p, const DdpArgs& a, hipStream_t s) {
  if constexpr (X <= 4) return ddp_t<K, X, U>(p, a, s);
  else return hipErrorInvalidValue;
}

bool ddp_supported(const noc_family& p) {
  // any registered family's cost (parametrised or traced: the record holds the full Hessian);
  // nx <= 4: every lane holds the value Hessian and the stage's Q blocks in registers
  return family_supported(p) && p.nx <= 4;
}

long long ddp_record_doubles(int nx, int nu) {
  return (long long)nx * nx + nx * nu + nx + nu + (long long)nx * nx + nu * nu + nx * nu +
         (long long)nx * (nx * nx + nx * nu + nu * nu);
}

hipError_t ddp_solve(const noc_family& p, int N, int Bt, const double* x0, double* u,
                     double* work, int* iterations, int* passes, int* done, double bp0,
                     int max_passes, int flags, hipStream_t s) {
  DdpArgs a{};
  a.one_stage = (flags & NOC_DDP_ONE_STAGE) ? 1 : 0;
  a.N = N;
  a.Bt = Bt;
  a.max_passes = max_passes;
  const char* no_skip = std::getenv("NOC_DDP_NO_REPEAT_SKIP");  // 1: recompute every retry
  a.skip_repeats = !(no_skip && no_skip[0] == '1');
  a.bp0 = bp0;
  a.x0 = x0;
  a.u = u;
  const size_t nxs = (size_t)Bt * (N + 1) * p.nx, nus = (size_t)Bt * N * p.nu;
  a.X = work;
  a.TX = a.X + nxs;
  a.TU = a.TX + nxs;
  a.k = a.TU + nus;
  a.K = a.k + nus;
  a.rec = a.K + nus * p.nx;
  a.iterations = iterations;
  a.passes = passes;
  a.done = done;
#define NOC_FAMILY(K, X, U) \
  if (p.kind == K && p.nx == X && p.nu == U) return ddp_family<K, X, U>(p, a, s);
#include NOC_FAMILIES_DEF
#undef NOC_FAMILY
  return hipErrorInvalidValue;
}

}  // namespace noc

// debug export: trace buffer of traj x cap x 10 doubles (bp, it, inner, pred, gain, success, rp,
// |Hu|, cost, new_cost per backward pass) for the first `traj` trajectories; buf = NULL disables
extern "C" int noc_debug_set_ddp_trace(double* buf, int cap, int traj) {
  if (hipMemcpyToSymbol(HIP_SYMBOL(noc::g_ddp_trace), &buf, sizeof(buf)) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(noc::g_ddp_trace_cap), &cap, sizeof(cap)) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(noc::g_ddp_trace_traj), &traj, sizeof(traj)) != hipSuccess) return -1;
  return 0;
}
