// Internal (non-ABI) declarations shared by the HIP translation units of libnoc_hip.so.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "../../include/noc_hip.h"

// The family / KKT-shape lists the dispatchers expand (X-macros).  A custom-family build points
// these at its generated lists (an absolute path: a quoted include would otherwise find the
// default list next to the source first).
#ifndef NOC_FAMILIES_DEF
#define NOC_FAMILIES_DEF "families.def"
#endif
#ifndef NOC_KKT_SHAPES_DEF
#define NOC_KKT_SHAPES_DEF "kkt_shapes.def"
#endif

// gfx950 (MI355X) only: the launchers size LDS budgets for its 160 KB per CU (the 40 KB per wave
// of the one-wave-per-SIMD instances, kkt_scan_impl.h: AB) and the cache policy for its 256 MiB
// memory-side cache (kkt_nt3); on another target those sizes would be wrong, so refuse to build.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "libnoc_hip targets gfx950 (MI355X) only: LDS budgets and cache policies are sized for it"
#endif

namespace noc {

enum KKTMode : int { MODE_FULL = 0, MODE_BWD = 1, MODE_FWD = 2 };

// Kernel argument block of the KKT scan (passed by value).  Layouts: include/noc_hip.h.
struct KKTArgs {
  int N, B, mode;
  int ab_slots; // set by the launcher: chunk slots whose A, B stay in LDS (kkt_scan_impl.h: AB)
  const double *A, *Bm, *Q, *R, *M, *r, *q, *c, *P, *p, *x0, *reg;
  const int* active;
  double *dx, *du, *pred, *K, *d, *S, *v;
  int* feasible;
  int ablate;  // timing-only ablation bits (tools/kkt_ablate.py); 0 in every product call
  int tiled;   // 1: A, B, Q, R, M, r, q, c, K, d in the tiled layout (Q, R packed symmetric)
  int lds_out; // set by the launcher: dx/du staged through LDS and written as contiguous rows
  int lds_base; // set by the launcher: LDS offset (doubles) of the A, B slot region
  // (ab_slots and lds_base sit in what was alignment padding: the struct -- the scan kernels'
  // argument block -- keeps its round-4 size)
};

// On-chip staging of the KKT scan (kkt_scan_impl.h): per trajectory N slots of nu*(nx+1) doubles
// (K_s, d_s, later overwritten by dx_s, du_s) + dx_N, one region per L-lane segment of the
// 64-thread block (L = 128: one per 128-thread block).  Staged when the region fits in 20 KB per
// wave (8 resident waves per CU).
// SIMDs of the current device (4 per CU); 1024 (MI355X: 256 CUs) when no device is visible.
inline int kkt_device_simds() {
  static int simds = 0;
  if (simds == 0) {
    int n = 0, dev = 0, cus = 0;
    if (hipGetDeviceCount(&n) == hipSuccess && n > 0 && hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
      simds = 4 * cus;
    else
      simds = 1024;
    (void)hipGetLastError();
  }
  return simds;
}

// Independent waves per workgroup of the L <= 64 scan (the measured A/B,
// profiles/r03/waves_per_block/): four while the batch's waves fit one per SIMD (fewer workgroups
// to place: c2 7.98 -> 7.73 us), two beyond (c3 90.4 -> 89.0 us; two-wave groups at one wave per
// SIMD were slower: c2 9.9 us).  NOC_KKT_WPB = 1 | 2 | 4 overrides (read once); capped so a
// workgroup's on-chip slots stay within 64 KB.
inline int kkt_waves_per_block(long waves, size_t lds_per_wave) {
  static const int forced = [] {
    const char* e = std::getenv("NOC_KKT_WPB");
    const int v = e ? std::atoi(e) : 0;
    return (v == 1 || v == 2 || v == 4) ? v : 0;
  }();
  int w = forced ? forced : (waves <= kkt_device_simds() ? 4 : 2);
  while (w > 1 && lds_per_wave * w > 65536) w /= 2;
  return w;
}

// The one-wave-per-SIMD (512-register) L = 64 scan instance for batches whose waves fit one per
// SIMD (kkt_scan_impl.h: BIG); NOC_KKT_BIG=0 turns it off (read once).
inline bool kkt_big_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("NOC_KKT_BIG");
    return !(e && e[0] == '0');
  }();
  return on;
}

// The A, B slots of the SIMD-owning scan instances (kkt_scan_impl.h: AB); NOC_KKT_AB=0 turns
// them off (read once)
inline bool kkt_ab_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("NOC_KKT_AB");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Cache policy of the scan's phase-3 re-reads (the last use of Q, R, M, r, q; tiled layout):
// non-temporal or the default.  Measured, same build, bench lines (profiles/r05/nt3/):
// non-temporal pays where a launch's blocks overflow the 256 MiB memory-side cache by far -- their
// lines would only displace the A, B, c that phase 4 and the other waves' phase 3 still re-read
// (c5, 577 MB: -4.2 %; N = 300, 432 MB: -0.9 %; 16 384 cart-poles: -1.3 %) -- and in the
// two-wave segments of the 512 shard, whose re-reads are cache hits (-2.0 %); it costs where a
// good part of the batch survives in that cache from one launch to the next (c3, 288 MB: +0.8 %;
// 4096 cart-poles at N = 100, 144 MB: +2.8 %).  The 512-register instances stay at the default
// (1024 shard 0; 2048 shard -1.0 % as a run-time choice inside one kernel, +1.5 % as an instance
// of its own).  So the two-wave (L = 128) instance is built non-temporal, and the L = 32 instance
// of larger batches exists in both forms, chosen here by the blocks' size: non-temporal beyond
// 1.5x the cache.  NOC_KKT_NT3=0 | 1 forces that choice (read once).
inline bool kkt_nt3(int B, int N, int nx, int nu) {
  static const int forced = [] {
    const char* e = std::getenv("NOC_KKT_NT3");
    return e ? (e[0] == '1' ? 1 : 0) : -1;
  }();
  if (forced >= 0) return forced == 1;
  const double stage = 8.0 * (nx * nx + 2 * nx * nu + nx * (nx + 1) / 2 + nu * (nu + 1) / 2 + nu + 2 * nx);
  const double mall = 256.0 * 1024 * 1024;  // MI355X Infinity Cache
  return (double)B * N * stage > 1.5 * mall;
}

inline size_t kkt_lds_bytes_rt(int nx, int nu, int N, int L) {
  if (L < 8) return 0;  // lanes = 1 (group solve): gains go through HBM
  const size_t per_traj = (size_t)(((long long)N * nu * (nx + 1) + nx + 1) & ~1LL);
  const size_t segs = L >= 64 ? 1 : 64 / L;  // trajectories per workgroup (L = 128: two waves)
  const size_t bytes = segs * per_traj * sizeof(double);
  return bytes <= 20480 * (size_t)(L > 64 ? L / 64 : 1) ? bytes : 0;
}

// The regularisation shrink factor max(1/3, 1 - (2 gain - 1)^3) of P:169 / S:141 / D:131 with
// JAX's rounding: `x ** 3` with an int exponent is lax.integer_pow, x * (x * x), and 1 - that
// rounds once more -- so no FMA contraction here (it would fuse the last multiply with the
// subtraction: one rounding instead of two, a last-bit difference in rp that steers every later
// step).  oracle/noc_oracle.py: _cube; tests/test_ipm_gpu.py checks every accepted step's rp.
__device__ __forceinline__ double rp_shrink(double gain) {
#pragma clang fp contract(off)
  const double c = 2.0 * gain - 1.0;
  return fmax(1.0 / 3.0, 1.0 - c * (c * c));
}

// Retry fixed point of the par inner loop (P:151-188).  A rejected trial whose rp was already at
// the upper clip (P:173: rp * r_inc clipped back to 1e16) leaves every input of the next par_Newton
// call unchanged -- x, u, the LQ blocks, rp -- so every remaining retry of the iteration repeats
// this trial bit for bit (deterministic kernels) until the retry cap keeps it (P:175-184).  Returns
// how many of those identical retries to account for without recomputing them (each one: a KKT
// solve, inner += 1, r_inc *= 2), at most `room` (a max_solves cap); 0 when the shortcut is off.
__device__ __forceinline__ int par_retry_repeats(const noc_ipm_ws& w, bool success, double rp_used,
                                                 double rp_new, int inner, int room) {
  if ((w.flags & NOC_WS_NO_REPEAT_SKIP) || success || rp_new != rp_used || inner > 500) return 0;
  const int k = 501 - inner;
  return room < k ? (room > 0 ? room : 0) : k;
}

// Diagnostic decision trace of the persistent interior-point solvers (built only with
// -DNOC_DECISION_TRACE: `make trace-lib`, read by tools/flip_probe.py).  One record of
// kTraceFields doubles per computed KKT solve of trajectories b < ntraj, indexed by the solve
// count before the solve: bp, it, inner, cost, new_cost, pred, gain, success, rp, r_inc, |Hu|,
// bwd feasible -- the inputs and the outcome of the accept test (P:159-173).  The product library
// has no such code; noc_debug_set_decision_trace then returns 0.
constexpr int kTraceFields = 12;
struct DecisionTrace {
  double* buf;
  int cap, ntraj;
};
#define NOC_TRACE_DECISION(T, b, idx, bp, it, inner, cost, new_cost, pred, gain, success, rp,    \
                           rinc, hu, bwd_ok)                                                      \
  do {                                                                                          \
    if ((T).buf && (b) < (T).ntraj && (idx) < (T).cap) {                                        \
      double* r_ = (T).buf + ((size_t)(b) * (T).cap + (idx)) * kTraceFields;                    \
      r_[0] = (bp); r_[1] = (it); r_[2] = (inner); r_[3] = (cost); r_[4] = (new_cost);           \
      r_[5] = (pred); r_[6] = (gain); r_[7] = (success) ? 1.0 : 0.0; r_[8] = (rp);               \
      r_[9] = (rinc); r_[10] = (hu); r_[11] = (bwd_ok) ? 1.0 : 0.0;                              \
    }                                                                                           \
  } while (0)
int wide_set_decision_trace(const DecisionTrace& t);  // ipm_wide.hip's copy of the pointer
int debug_set_decision_trace(double* buf, int cap, int ntraj);  // both kernels (ipm_persistent.hip)

// standalone building blocks (derivatives.hip)
struct DerivArgs {
  int N, B;
  const double *x, *u, *bp;
  double *cx, *cu, *cxx, *cuu, *cxu, *fx, *fu, *fxx, *fuu, *fxu;
};
struct LqrArgs {
  int nx, nu, N, B;
  const double *lam, *cu, *cxx, *cuu, *cxu, *fu, *fxx, *fuu, *fxu;
  double *ru, *Q, *R, *M;
};
hipError_t derivatives(const noc_family& p, const DerivArgs& a, hipStream_t s);
hipError_t final_cost_derivs(const noc_family& p, int B, const double* xN, double* grad,
                             double* hess, hipStream_t s);
hipError_t costates(int nx, int N, int B, const double* lamT, const double* cx, const double* fx,
                    double* lam, int sequential, hipStream_t s);
hipError_t lqr_params(const LqrArgs& a, hipStream_t s);
hipError_t traj_feasibility(const noc_family& p, int N, int B, const double* x, const double* u,
                            int* ok, hipStream_t s);
hipError_t total_cost(const noc_family& p, int N, int B, const double* x, const double* u,
                      const double* bp, double* cost, hipStream_t s);

hipError_t kkt_dispatch(int nx, int nu, const KKTArgs& a, int lanes, hipStream_t stream);
// lanes == 1: horizon-sequential solve, one trajectory per nx-lane group (kkt_group_impl.h)
hipError_t kkt_group_dispatch(int nx, int nu, const KKTArgs& a, hipStream_t stream);
// the scan for one (nx, nu) of kkt_shapes.def; instantiated in that shape's translation unit
// (kkt_scan_<nx>x<nu>.hip, or csrc/custom/kkt_scan_custom.hip in a custom-family build)
template <int NX, int NU>
hipError_t kkt_dispatch_shape(const KKTArgs& a, int lanes, hipStream_t stream);
bool kkt_supported(int nx, int nu);
int kkt_default_lanes(int nx, int nu, int N);
int kkt_pick_lanes(int nx, int nu, int N, int B);

hipError_t ipm_prepare(const noc_family& p, const noc_ipm_ws& w, int mode, int terminal,
                       hipStream_t s);
hipError_t ipm_trial(const noc_family& p, const noc_ipm_ws& w, int mode, hipStream_t s);
hipError_t ipm_rollout(const noc_family& p, const noc_ipm_ws& w, hipStream_t s);
hipError_t ipm_prepare_main(const noc_family& p, const noc_ipm_ws& w, int mode, int terminal,
                            hipStream_t s);
hipError_t ipm_promote(const noc_ipm_ws& w, hipStream_t s);
hipError_t ipm_init(const noc_ipm_ws& w, double bp0, hipStream_t s);
// persistent whole-solve kernel (ipm_persistent.hip)
bool ipm_solve_supported(const noc_family& p, int N, int lanes);
// interior-point DDP (ddp_persistent.hip)
bool ddp_supported(const noc_family& p);
long long ddp_record_doubles(int nx, int nu);
hipError_t ddp_solve(const noc_family& p, int N, int Bt, const double* x0, double* u,
                     double* work, int* iterations, int* passes, int* done, double bp0,
                     int max_passes, int flags, hipStream_t s);
// DDP building blocks (ddp_blocks.hip)
struct DdpBwdArgs {
  int N, B;
  const double *Vx, *Vxx, *reg_param;
  const double *cx, *cu, *cxx, *cuu, *cxu, *fx, *fu, *fxx, *fuu, *fxu;
  double *k, *K, *pred, *Hu;
  int* feasible;
};
hipError_t ddp_bwd_pass(int nx, int nu, const DdpBwdArgs& a, hipStream_t s);
hipError_t nonlin_rollout(const noc_family& p, int N, int B, const double* K, const double* k,
                          const double* x, const double* u, double* xn, double* un, hipStream_t s);
int debug_phase_cycles(long long* out, int n, int reset);
int debug_traj_times(long long* out, int n);
hipError_t ipm_solve(const noc_family& p, const noc_ipm_ws& w, int mode, int terminal, double bp0,
                     int max_solves, hipStream_t s);
// wide whole-solve kernel (ipm_wide.hip): one 4-wave workgroup per trajectory, LDS-resident
bool ipm_wide_supported(const noc_family& p, int N);
size_t wide_lds_bytes(const noc_family& p, int N, int W);
int wide_waves(const noc_family& p, const noc_ipm_ws& w, int cus);
int debug_wide_cycles(long long* out, int n, int reset);
// grid workgroups solve trajectories idx[0 .. *count) (idx == NULL: 0 .. Bt-1, count ignored)
hipError_t ipm_solve_wide(const noc_family& p, const noc_ipm_ws& w, int mode, int terminal,
                          double bp0, int max_solves, const int* idx, const int* count, int grid,
                          int W, hipStream_t s);
hipError_t relayout(int direction, int E, int sym_n, int N, int Bt, int L, const double* src,
                    double* dst, hipStream_t s);
bool family_supported(const noc_family& p);

}  // namespace noc
