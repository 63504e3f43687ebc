// Structure-aware LQ blocks of the persistent interior-point solver.
//
// For the generated families most entries of a stage's blocks are the same for every (x, u, lambda,
// bp): cart-pole's A = I + dt fx has 4 entries that depend on the state (of 16), B = dt fu 2 (of 4),
// Q = cxx + lambda.fxx 3 (of 10 packed), M = cxu + lambda.fxu 1 (of 4) -- 12 variable doubles of 36
// per stage with R and r (examples/cartpole_runtime.py:54-81 through noc/par_interior_point_newton.py:
// 13-42).  The generator knows which (noc/_codegen.py: {name}_jac_var / _const, {name}_hess_nz,
// custom_cost_hess_var / _const), so the persistent solver
//   * stores only the variable entries of A, B, Q, R, M (the "compact" tiled fields: the tiled
//     layout of include/noc_hip.h with E = the field's variable count), and
//   * rebuilds the constant entries where the blocks are read, from literals (0, 1), the family's
//     parameters (dt, wx, the linear family's A, B: kernel arguments, so scalar operands) and the
//     generator's constants -- the same doubles the dense path computes, e.g. 1 + dt * 0 == 1 and
//     0 + dt * 1 == dt for a finite dt -- and skips the products with a structural zero (nzA / nzB,
//     used by the KKT scan's arithmetic, kkt_scan_impl.h).
// A skipped term s += a * 0 leaves s unchanged where the dense path adds an exact zero (the same
// double up to the sign of a zero sum), so the results equal the dense instance's (tested bit for
// bit: tests/test_ipm_gpu.py).  BlockStruct<..., false> is the dense layout (every entry
// variable), the instance NOC_PERSIST_STRUCT=0 selects.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

#include "ipm_family.h"

namespace noc {

// compile-time loop: f(std::integral_constant<int, 0>) ... f(std::integral_constant<int, N - 1>)
template <class F, int... I>
NOC_DEV void static_for_seq(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
NOC_DEV void static_for(F&& f) {
  static_for_seq(f, std::make_integer_sequence<int, N>{});
}

// how a block entry is obtained
enum BlockKind : int {
  BK_VAR = 0,  // stored (depends on x, u, lambda or bp)
  BK_ZERO,     // 0
  BK_ONE,      // 1
  BK_DT,       // 0 + dt * 1
  BK_EXPR_A,   // delta + dt * c (Euler A entry with a constant ODE Jacobian entry c)
  BK_EXPR_B,   // dt * c
  BK_LIT,      // c (discrete map Jacobian entry, traced cost Hessian entry)
  BK_PA,       // the linear family's A[idx]
  BK_PB,       // the linear family's B[idx]
  BK_WX        // the parametrised cost's wx[idx]
};

template <int N>
struct KindTable {
  int kind[N] = {};
  int pos[N] = {};   // BK_VAR: index in the compact record
  int idx[N] = {};   // BK_PA / BK_PB / BK_WX: parameter index
  double lit[N] = {};
  double delta[N] = {};
  int nv = 0;        // variable entries = the compact field's doubles per stage
};

// The generator's patterns of a family (families_gen.h / a custom build's custom_family_gen.h)
template <int KIND, int NX, int NU>
struct GenPattern {
  static constexpr int NZ = NX + NU;
  static constexpr bool kLinear = KIND == NOC_FAMILY_LINEAR;
  static constexpr bool kDiscrete = Fam<KIND, NX, NU>::kDiscrete;
  static constexpr bool kGenCost = Fam<KIND, NX, NU>::kGenCost;
  // ODE (or discrete map) Jacobian entry k of [fx | fu] (row-major NX x NZ)
  static constexpr bool jvar(int k) {
    if constexpr (KIND == NOC_FAMILY_PENDULUM) return gen::pendulum_jac_var[k] != 0;
    else if constexpr (KIND == NOC_FAMILY_CARTPOLE) return gen::cartpole_jac_var[k] != 0;
#ifdef NOC_CUSTOM_FAMILY
    else if constexpr (KIND == NOC_FAMILY_CUSTOM) return gen::custom_jac_var[k] != 0;
#endif
    else return true;
  }
  static constexpr double jconst(int k) {
    if constexpr (KIND == NOC_FAMILY_PENDULUM) return gen::pendulum_jac_const[k];
    else if constexpr (KIND == NOC_FAMILY_CARTPOLE) return gen::cartpole_jac_const[k];
#ifdef NOC_CUSTOM_FAMILY
    else if constexpr (KIND == NOC_FAMILY_CUSTOM) return gen::custom_jac_const[k];
#endif
    else return 0.0;
  }
  // lambda-contracted Hessian entry k (NZ x NZ) not identically zero
  static constexpr bool hnz(int k) {
    if constexpr (kLinear) return false;
    else if constexpr (KIND == NOC_FAMILY_PENDULUM) return gen::pendulum_hess_nz[k] != 0;
    else if constexpr (KIND == NOC_FAMILY_CARTPOLE) return gen::cartpole_hess_nz[k] != 0;
#ifdef NOC_CUSTOM_FAMILY
    else if constexpr (KIND == NOC_FAMILY_CUSTOM) return gen::custom_hess_nz[k] != 0;
#endif
    else return true;
  }
  // traced stage-cost Hessian [Q (NX*NX) | R (NU*NU) | M (NX*NU)] entry k
  static constexpr bool cvar(int k) {
#ifdef NOC_CUSTOM_FAMILY
    if constexpr (kGenCost) return gen::custom_cost_hess_var[k] != 0;
#endif
    (void)k;
    return true;
  }
  static constexpr double cconst(int k) {
#ifdef NOC_CUSTOM_FAMILY
    if constexpr (kGenCost) return gen::custom_cost_hess_const[k];
#endif
    (void)k;
    return 0.0;
  }
};

enum BlockField : int { BF_A = 0, BF_B, BF_Q, BF_R, BF_M };

template <int N>
constexpr void kt_set(KindTable<N>& t, int e, int kind, double lit = 0.0, int idx = 0, double delta = 0.0) {
  t.kind[e] = kind;
  t.lit[e] = lit;
  t.idx[e] = idx;
  t.delta[e] = delta;
  if (kind == BK_VAR) t.pos[e] = t.nv++;
}

// A = fx (NX x NX): Euler I + dt J_x, a discrete map's J_x, or the linear family's A
template <int KIND, int NX, int NU, bool ON>
constexpr KindTable<NX * NX> table_A() {
  using G = GenPattern<KIND, NX, NU>;
  KindTable<NX * NX> t{};
  for (int i = 0; i < NX; ++i)
    for (int j = 0; j < NX; ++j) {
      const int e = i * NX + j, k = i * G::NZ + j;
      if (!ON) kt_set(t, e, BK_VAR);
      else if (G::kLinear) kt_set(t, e, BK_PA, 0.0, e);
      else if (G::jvar(k)) kt_set(t, e, BK_VAR);
      else if (G::kDiscrete) {
        const double c = G::jconst(k);
        kt_set(t, e, c == 0.0 ? BK_ZERO : (c == 1.0 ? BK_ONE : BK_LIT), c);
      } else {
        const double c = G::jconst(k);
        if (c == 0.0) kt_set(t, e, i == j ? BK_ONE : BK_ZERO);
        else if (i != j && c == 1.0) kt_set(t, e, BK_DT);
        else kt_set(t, e, BK_EXPR_A, c, 0, i == j ? 1.0 : 0.0);
      }
    }
  return t;
}
// B = fu (NX x NU)
template <int KIND, int NX, int NU, bool ON>
constexpr KindTable<NX * NU> table_B() {
  using G = GenPattern<KIND, NX, NU>;
  KindTable<NX * NU> t{};
  for (int i = 0; i < NX; ++i)
    for (int j = 0; j < NU; ++j) {
      const int e = i * NU + j, k = i * G::NZ + NX + j;
      if (!ON) kt_set(t, e, BK_VAR);
      else if (G::kLinear) kt_set(t, e, BK_PB, 0.0, e);
      else if (G::jvar(k)) kt_set(t, e, BK_VAR);
      else {
        const double c = G::jconst(k);
        if (c == 0.0) kt_set(t, e, BK_ZERO);
        else if (G::kDiscrete) kt_set(t, e, c == 1.0 ? BK_ONE : BK_LIT, c);
        else kt_set(t, e, c == 1.0 ? BK_DT : BK_EXPR_B, c);
      }
    }
  return t;
}
// Q (packed symmetric, Sym<NX> order): cxx + s lambda.fxx, symmetrised
template <int KIND, int NX, int NU, bool ON>
constexpr KindTable<Sym<NX>::SZ> table_Q() {
  using G = GenPattern<KIND, NX, NU>;
  KindTable<Sym<NX>::SZ> t{};
  for (int i = 0; i < NX; ++i)
    for (int j = i; j < NX; ++j) {
      const int e = Sym<NX>::idx(i, j);
      const bool h = G::hnz(i * G::NZ + j) || G::hnz(j * G::NZ + i);
      if (!ON || h) kt_set(t, e, BK_VAR);
      else if (G::kGenCost) {
        if (G::cvar(i * NX + j) || G::cvar(j * NX + i)) kt_set(t, e, BK_VAR);
        else if (i == j) kt_set(t, e, BK_LIT, G::cconst(i * NX + i));
        else kt_set(t, e, BK_LIT, 0.5 * (G::cconst(i * NX + j) + G::cconst(j * NX + i)));
      } else {
        if (i == j) kt_set(t, e, BK_WX, 0.0, i);
        else kt_set(t, e, BK_ZERO);
      }
    }
  return t;
}
// R (packed symmetric, Sym<NU> order): cuu (+ the log barrier: always stored on the diagonal) + s
// lambda.fuu
template <int KIND, int NX, int NU, bool ON>
constexpr KindTable<Sym<NU>::SZ> table_R() {
  using G = GenPattern<KIND, NX, NU>;
  KindTable<Sym<NU>::SZ> t{};
  for (int i = 0; i < NU; ++i)
    for (int j = i; j < NU; ++j) {
      const int e = Sym<NU>::idx(i, j);
      const bool h = G::hnz((NX + i) * G::NZ + NX + j) || G::hnz((NX + j) * G::NZ + NX + i);
      const int ci = NX * NX + i * NU + j, cj = NX * NX + j * NU + i;
      if (!ON || h || i == j) kt_set(t, e, BK_VAR);
      else if (G::kGenCost) {
        if (G::cvar(ci) || G::cvar(cj)) kt_set(t, e, BK_VAR);
        else kt_set(t, e, BK_LIT, 0.5 * (G::cconst(ci) + G::cconst(cj)));
      } else {
        kt_set(t, e, BK_ZERO);
      }
    }
  return t;
}
// M (NX x NU): cxu + s lambda.fxu
template <int KIND, int NX, int NU, bool ON>
constexpr KindTable<NX * NU> table_M() {
  using G = GenPattern<KIND, NX, NU>;
  KindTable<NX * NU> t{};
  for (int i = 0; i < NX; ++i)
    for (int j = 0; j < NU; ++j) {
      const int e = i * NU + j, ck = NX * NX + NU * NU + e;
      if (!ON || G::hnz(i * G::NZ + NX + j)) kt_set(t, e, BK_VAR);
      else if (G::kGenCost) {
        if (G::cvar(ck)) kt_set(t, e, BK_VAR);
        else kt_set(t, e, BK_LIT, G::cconst(ck));
      } else {
        kt_set(t, e, BK_ZERO);
      }
    }
  return t;
}

template <int N>
constexpr uint64_t nz_mask(const KindTable<N>& t) {
  uint64_t m = 0;
  for (int e = 0; e < N; ++e)
    if (t.kind[e] != BK_ZERO) m |= (uint64_t)1 << e;
  return m;
}

template <int KIND, int NX, int NU, bool ON>
struct BlockStruct {
  static_assert(NX * NX <= 64, "structure masks hold up to 64 entries");
  static constexpr bool kOn = ON;
  template <int F>
  static constexpr auto table() {
    if constexpr (F == BF_A) return table_A<KIND, NX, NU, ON>();
    else if constexpr (F == BF_B) return table_B<KIND, NX, NU, ON>();
    else if constexpr (F == BF_Q) return table_Q<KIND, NX, NU, ON>();
    else if constexpr (F == BF_R) return table_R<KIND, NX, NU, ON>();
    else return table_M<KIND, NX, NU, ON>();
  }
  template <int F>
  static constexpr int size() {
    if constexpr (F == BF_A) return NX * NX;
    else if constexpr (F == BF_B || F == BF_M) return NX * NU;
    else if constexpr (F == BF_Q) return Sym<NX>::SZ;
    else return Sym<NU>::SZ;
  }
  // doubles per stage of each compact field
  template <int F>
  static constexpr int nv() { return table<F>().nv; }
  static constexpr uint64_t kNzA = nz_mask(table_A<KIND, NX, NU, ON>());
  static constexpr uint64_t kNzB = nz_mask(table_B<KIND, NX, NU, ON>());
  // may A(k, j) / B(k, j) be nonzero (the scan's arithmetic skips the products with the others)
  static constexpr bool nzA(int k, int j) { return ((kNzA >> (k * NX + j)) & 1) != 0; }
  static constexpr bool nzB(int k, int j) { return ((kNzB >> (k * NU + j)) & 1) != 0; }

  template <int K>
  NOC_DEV static double value(const noc_family& p, double lit, int idx, double delta) {
    if constexpr (K == BK_ZERO) return 0.0;
    else if constexpr (K == BK_ONE) return 1.0;
    else if constexpr (K == BK_DT) return p.dt;
    else if constexpr (K == BK_EXPR_A) return delta + p.dt * lit;  // Fam::jac's expression
    else if constexpr (K == BK_EXPR_B) return p.dt * lit;
    else if constexpr (K == BK_LIT) return lit;
    else if constexpr (K == BK_PA) return p.A[idx];
    else if constexpr (K == BK_PB) return p.B[idx];
    else return p.wx[idx];  // BK_WX
  }
  // full field <- compact record v (variable entries) + the constants
  template <int F>
  NOC_DEV static void expand(const noc_family& p, const double* v, double* full) {
    static_for<size<F>()>([&](auto E) {
      constexpr auto T = table<F>();
      constexpr int e = decltype(E)::value;
      constexpr int k = T.kind[e];
      if constexpr (k == BK_VAR) {
        constexpr int pos = T.pos[e];
        full[e] = v[pos];
      } else {
        full[e] = value<k>(p, T.lit[e], T.idx[e], T.delta[e]);
      }
    });
  }
  // the constant entries of a computed full field replaced by their structural values (the same
  // doubles for a finite dt; the compiler then drops their computation and folds them)
  template <int F>
  NOC_DEV static void fold_consts(const noc_family& p, double* full) {
    static_for<size<F>()>([&](auto E) {
      constexpr auto T = table<F>();
      constexpr int e = decltype(E)::value;
      constexpr int k = T.kind[e];
      if constexpr (k != BK_VAR) full[e] = value<k>(p, T.lit[e], T.idx[e], T.delta[e]);
    });
  }
  // compact record v <- the variable entries of a full field
  template <int F>
  NOC_DEV static void compress(const double* full, double* v) {
    static_for<size<F>()>([&](auto E) {
      constexpr auto T = table<F>();
      constexpr int e = decltype(E)::value;
      if constexpr (T.kind[e] == BK_VAR) {
        constexpr int pos = T.pos[e];
        v[pos] = full[e];
      }
    });
  }
};

}  // namespace noc
