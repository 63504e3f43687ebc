// Registered problem families (dynamics, derivatives, costs) and wave helpers shared by the
// interior-point kernels (ipm_kernels.hip: one launch per phase; ipm_persistent.hip: the whole
// solve in one launch).  Restates examples/pendulum_runtime.py:19-72, cartpole_runtime.py:18-82,
// linear_mpc_parallel.py:24-63 and noc/utils.py:8-63.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#include "../../include/noc_hip.h"
#include "families_gen.h"
#include "small_linalg.h"
#ifdef NOC_CUSTOM_FAMILY
// a custom-family build (noc.families.register_family): the generated ODE / discrete map of the
// registered problem, its Jacobian and lambda-contracted Hessian (noc/_codegen.py), found first
// on the include path
#include "custom_family_gen.h"
#endif

namespace noc {

constexpr double kTwoPi = 6.283185307179586;  // 2.0 * jnp.pi

// noc/utils.py:8-10 with jnp.remainder semantics (C fmod, + divisor if the sign differs).
// fmod is exact, and so is its value on the two innermost periods: fmod(a, 2 pi) == a for
// |a| < 2 pi, and a - sign(a) 2 pi for 2 pi <= |a| < 4 pi (Sterbenz: the subtraction of two
// doubles within a factor of two is exact, so this IS fmod's result bit for bit).  The general
// fmod routine (a loop of ~100s of instructions) runs only beyond 4 pi, behind a branch.  The
// cart-pole's angle lives around 2 pi (examples/cartpole_runtime.py: the pole hangs at 0 = 2 pi
// and swings up to pi), so before round 6 every stage cost, gradient and trial point of a typical
// trajectory took the loop -- 2/3 of the trial phase.
NOC_DEV double wrap_angle(double a) {
  double r = a;
  const double fa = fabs(a);
  if (fa >= kTwoPi) {
    if (__builtin_expect(fa < 2.0 * kTwoPi, 1)) r = a - copysign(kTwoPi, a);
    else r = fmod(a, kTwoPi);
  }
  return (r != 0.0 && r < 0.0) ? r + kTwoPi : r;
}

template <int KIND, int NX, int NU>
struct Fam {
  const noc_family& p;
  NOC_DEV explicit Fam(const noc_family& prm) : p(prm) {}

  // A registered custom family either gives a continuous-time ODE (Euler-discretised here like
  // the built-ins, noc/utils.py:50-54) or the discrete map x+ = F(x, u) itself (kDiscrete).
#ifdef NOC_CUSTOM_FAMILY
  static constexpr bool kDiscrete = (KIND == NOC_FAMILY_CUSTOM) && gen::kCustomDiscrete;
  // the family's own stage cost / final cost / constraints, traced from the user's callables
  // (noc.families.register_family(stage_cost=..., final_cost=..., constraints=...)), instead of
  // the parametrised quadratic tracking cost with a box log barrier on u
  static constexpr bool kGenCost = (KIND == NOC_FAMILY_CUSTOM) && gen::kCustomCost;
#else
  static constexpr bool kDiscrete = false;
  static constexpr bool kGenCost = false;
#endif
  // generated right-hand side / Jacobian J = d rhs / d[x; u] / lambda-contracted Hessian
  NOC_DEV static void rhs(const double* x, const double* u, double* f) {
    if constexpr (KIND == NOC_FAMILY_PENDULUM) gen::pendulum_ode(x, u, f);
    else if constexpr (KIND == NOC_FAMILY_CARTPOLE) gen::cartpole_ode(x, u, f);
#ifdef NOC_CUSTOM_FAMILY
    else if constexpr (KIND == NOC_FAMILY_CUSTOM) gen::custom_ode(x, u, f);
#endif
  }
  NOC_DEV static void rhs_jac(const double* x, const double* u, double* J) {
    if constexpr (KIND == NOC_FAMILY_PENDULUM) gen::pendulum_ode_jac(x, u, J);
    else if constexpr (KIND == NOC_FAMILY_CARTPOLE) gen::cartpole_ode_jac(x, u, J);
#ifdef NOC_CUSTOM_FAMILY
    else if constexpr (KIND == NOC_FAMILY_CUSTOM) gen::custom_ode_jac(x, u, J);
#endif
  }
  NOC_DEV static void rhs_hess_l(const double* x, const double* u, const double* l, double* H) {
    if constexpr (KIND == NOC_FAMILY_PENDULUM) gen::pendulum_ode_hess_l(x, u, l, H);
    else if constexpr (KIND == NOC_FAMILY_CARTPOLE) gen::cartpole_ode_hess_l(x, u, l, H);
#ifdef NOC_CUSTOM_FAMILY
    else if constexpr (KIND == NOC_FAMILY_CUSTOM) gen::custom_ode_hess_l(x, u, l, H);
#endif
  }

  // ------------------------------------------------------------------ dynamics
  NOC_DEV void step(const double* x, const double* u, double* xn) const {
    if constexpr (KIND == NOC_FAMILY_LINEAR) {
      NOC_UNROLL for (int i = 0; i < NX; ++i) {
        double t = 0.0;
        NOC_UNROLL for (int k = 0; k < NX; ++k) t += p.A[i * NX + k] * x[k];
        NOC_UNROLL for (int j = 0; j < NU; ++j) t += p.B[i * NU + j] * u[j];
        xn[i] = t;
      }
    } else if constexpr (kDiscrete) {
      rhs(x, u, xn);
    } else {
      double f[NX];
      rhs(x, u, f);
      NOC_UNROLL for (int i = 0; i < NX; ++i) xn[i] = x[i] + p.dt * f[i];  // noc/utils.py:50-54
    }
  }
  NOC_DEV void jac(const double* x, const double* u, double* fx, double* fu) const {
    if constexpr (KIND == NOC_FAMILY_LINEAR) {
      NOC_UNROLL for (int i = 0; i < NX * NX; ++i) fx[i] = p.A[i];
      NOC_UNROLL for (int i = 0; i < NX * NU; ++i) fu[i] = p.B[i];
    } else {
      constexpr int NZ = NX + NU;
      double J[NX * NZ];
      rhs_jac(x, u, J);
      NOC_UNROLL for (int i = 0; i < NX; ++i) {
        if constexpr (kDiscrete) {
          NOC_UNROLL for (int j = 0; j < NX; ++j) fx[i * NX + j] = J[i * NZ + j];
          NOC_UNROLL for (int j = 0; j < NU; ++j) fu[i * NU + j] = J[i * NZ + NX + j];
        } else {
          NOC_UNROLL for (int j = 0; j < NX; ++j) fx[i * NX + j] = (i == j ? 1.0 : 0.0) + p.dt * J[i * NZ + j];
          NOC_UNROLL for (int j = 0; j < NU; ++j) fu[i * NU + j] = p.dt * J[i * NZ + NX + j];
        }
      }
    }
  }
  // sum_i lam_i d2 f_i (Euler: dt * ode Hessians); adds into Hxx (NXxNX), Huu, Hxu (NXxNU)
  NOC_DEV void add_hess_l(const double* x, const double* u, const double* lam, double* Hxx,
                          double* Huu, double* Hxu) const {
    if constexpr (KIND != NOC_FAMILY_LINEAR) {
      constexpr int NZ = NX + NU;
      double H[NZ * NZ];
      rhs_hess_l(x, u, lam, H);
      const double s = kDiscrete ? 1.0 : p.dt;
      NOC_UNROLL for (int i = 0; i < NX; ++i) {
        NOC_UNROLL for (int j = 0; j < NX; ++j) Hxx[i * NX + j] += s * H[i * NZ + j];
        NOC_UNROLL for (int j = 0; j < NU; ++j) Hxu[i * NU + j] += s * H[i * NZ + NX + j];
      }
      NOC_UNROLL for (int i = 0; i < NU; ++i)
        NOC_UNROLL for (int j = 0; j < NU; ++j) Huu[i * NU + j] += s * H[(NX + i) * NZ + NX + j];
    }
  }

  // ------------------------------------------------------------------ costs
  NOC_DEV double err(const double* x, int i) const {
    const double xi = (i == p.wrap_index) ? wrap_angle(x[i]) : x[i];
    return xi - p.goal[i];
  }
  NOC_DEV bool barrier() const { return p.u_bound > 0.0; }
  // stage cost (PR:40-50 / CR:36-45 / LD:34-37)
  NOC_DEV double stage_cost(const double* x, const double* u, double bp) const {
#ifdef NOC_CUSTOM_FAMILY
    if constexpr (kGenCost) return gen::custom_stage_cost(x, u, bp);
#endif
    double c = 0.0;
    NOC_UNROLL for (int i = 0; i < NX; ++i) { const double e = err(x, i); c += p.wx[i] * e * e; }
    c *= 0.5;
    double cu = 0.0;
    NOC_UNROLL for (int j = 0; j < NU; ++j) cu += p.wu[j] * u[j] * u[j];
    c += 0.5 * cu;
    if (barrier()) {
      double lb = 0.0;
      NOC_UNROLL for (int j = 0; j < NU; ++j) lb += log(p.u_bound - u[j]) + log(u[j] + p.u_bound);
      c -= bp * lb;
    }
    return c;
  }
  NOC_DEV void stage_grad(const double* x, const double* u, double bp, double* cx,
                          double* cu) const {
#ifdef NOC_CUSTOM_FAMILY
    if constexpr (kGenCost) {
      gen::custom_stage_grad(x, u, bp, cx, cu);
      return;
    }
#endif
    NOC_UNROLL for (int i = 0; i < NX; ++i) cx[i] = p.wx[i] * err(x, i);
    NOC_UNROLL for (int j = 0; j < NU; ++j) {
      double g = p.wu[j] * u[j];
      if (barrier()) g += bp / (p.u_bound - u[j]) - bp / (u[j] + p.u_bound);
      cu[j] = g;
    }
  }
  NOC_DEV double stage_cuu(const double* u, double bp, int j) const {
    double h = p.wu[j];
    if (barrier()) {
      const double a = p.u_bound - u[j], b = u[j] + p.u_bound;
      h += bp / (a * a) + bp / (b * b);
    }
    return h;
  }
  // hessian of the stage cost (P:19-21: cxx, cuu, cxu), full row-major matrices
  NOC_DEV void stage_hess(const double* x, const double* u, double bp, double* Q, double* R,
                          double* M) const {
#ifdef NOC_CUSTOM_FAMILY
    if constexpr (kGenCost) {
      gen::custom_stage_hess(x, u, bp, Q, R, M);
      return;
    }
#endif
    (void)x;
    NOC_UNROLL for (int i = 0; i < NX; ++i) NOC_UNROLL for (int j = 0; j < NX; ++j) Q[i * NX + j] = (i == j) ? p.wx[i] : 0.0;
    NOC_UNROLL for (int i = 0; i < NU; ++i) NOC_UNROLL for (int j = 0; j < NU; ++j) R[i * NU + j] = (i == j) ? stage_cuu(u, bp, i) : 0.0;
    NOC_UNROLL for (int i = 0; i < NX * NU; ++i) M[i] = 0.0;
  }
  // all(constraints(x, u) <= 0) (P:45-47)
  NOC_DEV bool feasible(const double* x, const double* u) const {
#ifdef NOC_CUSTOM_FAMILY
    if constexpr (kGenCost) return gen::custom_feasible(x, u);
#endif
    (void)x;
    if (!barrier()) return true;
    bool ok = true;
    NOC_UNROLL for (int j = 0; j < NU; ++j) ok = ok && (u[j] - p.u_bound <= 0.0) && (-u[j] - p.u_bound <= 0.0);
    return ok;
  }
  NOC_DEV double final_cost(const double* x) const {
#ifdef NOC_CUSTOM_FAMILY
    if constexpr (kGenCost) return gen::custom_final_cost(x);
#endif
    double c = 0.0;
    NOC_UNROLL for (int i = 0; i < NX; ++i) { const double e = err(x, i); c += p.wf[i] * e * e; }
    return 0.5 * c;
  }
  // grad(final_cost) (C:35: the terminal costate) and hessian(final_cost) (S:66)
  NOC_DEV void final_grad(const double* x, double* g) const {
#ifdef NOC_CUSTOM_FAMILY
    if constexpr (kGenCost) {
      gen::custom_final_grad(x, g);
      return;
    }
#endif
    NOC_UNROLL for (int i = 0; i < NX; ++i) g[i] = p.wf[i] * err(x, i);
  }
  NOC_DEV void final_hess(const double* x, double* H) const {
#ifdef NOC_CUSTOM_FAMILY
    if constexpr (kGenCost) {
      gen::custom_final_hess(x, H);
      return;
    }
#endif
    (void)x;
    NOC_UNROLL for (int i = 0; i < NX; ++i) NOC_UNROLL for (int j = 0; j < NX; ++j) H[i * NX + j] = (i == j) ? p.wf[i] : 0.0;
  }
};

// ------------------------------------------------------------------------------------------------
NOC_DEV double readlane_d(double v, int lane) {  // wave-uniform broadcast of one lane's double
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(bits & 0xffffffffLL), lane);
  const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// max that propagates NaN like jnp.max (fmax drops it): a NaN |Hu| must fail the < 1e-4 stop
// test exactly as in the reference (P:158, P:199; D:120)
NOC_DEV double nan_max(double a, double b) { return (a != a || b != b) ? NAN : fmax(a, b); }

// The phase a persistent solve resumes at (NOC_WS_RESUME) from a workspace phase, including the
// two-stream driver's intermediate ones: ROLLED (states current) continues with a new Newton
// iteration, ROLLOUT_PENDING with the rollout.
NOC_DEV int resume_phase(int ph) {
  if (ph == NOC_PHASE_ROLLED) return NOC_PHASE_LINEARIZE;
  if (ph == NOC_PHASE_ROLLOUT_PENDING) return NOC_PHASE_ROLLOUT;
  return ph;
}

// wave-wide sum, every lane the same value: the __shfl_xor butterfly (off = 32 .. 1) with VALU
// partners (small_linalg.h: segment_allreduce), bit-identical to the shuffle loop
NOC_DEV double wave_sum(double v) {
  return segment_allreduce<64>(v, (int)__lane_id(), [](double a, double b) { return a + b; });
}

}  // namespace noc
