// extern "C" entry points of libnoc_hip.so (declared in include/noc_hip.h).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/noc_hip.h"
#include "noc_internal.h"
#include "small_linalg.h"

namespace noc {
static std::string kkt_shapes_str();
}

namespace {
thread_local std::string g_last_error;
int g_ablate = 0;  // timing-only phase ablation (noc_debug_set_ablation); never set in product use

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

// align: 16 where the kernels read / write the array with 16-byte vector accesses (the fp64 KKT
// fields), the natural alignment (8 for fp64, 4 for int32) elsewhere
int check_ptr(const void* p, const char* name, bool required, unsigned align = 16) {
  if (!p) return required ? fail(-2, std::string("required pointer is NULL: ") + name) : 0;
  if (reinterpret_cast<uintptr_t>(p) & (align - 1))
    return fail(-3, std::string("pointer not ") + std::to_string(align) + "-byte aligned: " + name);
  return 0;
}

int hip_status(hipError_t e, const char* where) {
  if (e == hipSuccess) return 0;
  return fail(-10, std::string(where) + ": " + hipGetErrorString(e));
}

int check_dims(int nx, int nu, int N, int B, int lanes) {
  if (!noc::kkt_supported(nx, nu))
    return fail(-1, "unsupported (nx, nu) = (" + std::to_string(nx) + ", " + std::to_string(nu) +
                        "); supported: " + noc::kkt_shapes_str());
  if (N < 1) return fail(-1, "horizon N must be >= 1");
  if (B < 0) return fail(-1, "batch B must be >= 0");
  if (lanes != 0 && lanes != 1 && lanes != 8 && lanes != 16 && lanes != 32 && lanes != 64 &&
      lanes != 128)
    return fail(-1, "lanes must be 0, 1, 8, 16, 32, 64 or 128");
  return 0;
}
}  // namespace

namespace noc {
bool kkt_supported(int nx, int nu) {
#define NOC_KKT_SHAPE(X, U) if (nx == X && nu == U) return true;
#include NOC_KKT_SHAPES_DEF
#undef NOC_KKT_SHAPE
  return false;
}

static std::string kkt_shapes_str() {
  std::string s;
#define NOC_KKT_SHAPE(X, U) s += std::string(s.empty() ? "" : " ") + "(" #X "," #U ")";
#include NOC_KKT_SHAPES_DEF
#undef NOC_KKT_SHAPE
  return s;
}

hipError_t kkt_dispatch(int nx, int nu, const KKTArgs& a, int lanes, hipStream_t stream) {
  if (lanes == 1) return kkt_group_dispatch(nx, nu, a, stream);
#define NOC_KKT_SHAPE(X, U) if (nx == X && nu == U) return kkt_dispatch_shape<X, U>(a, lanes, stream);
#include NOC_KKT_SHAPES_DEF
#undef NOC_KKT_SHAPE
  return hipErrorInvalidValue;
}

// lanes per trajectory chosen from the measured sweep (profiles/r01/kkt_lanes_sweep_tiled.log):
// long horizons amortise the cross-lane scan over longer chunks (L = 32 at c3, N = 200); short
// horizons need the lanes for parallelism (L = 64 at c2, N = 100).
int kkt_default_lanes(int nx, int nu, int N) {
  (void)nu;
  // nx = 8: the horizon-sequential group solve (lanes 1) -- c4: 6.1 ms vs 47-55 ms for the scan,
  // whose nx = 8 element spills (profiles/r01/session2/r9_sweep_c4.log, bench_c4_dma.log)
  if (nx >= 8) return 1;
  return N >= 160 ? 32 : 64;
}


// Batch-aware lanes per trajectory (the measured lanes x horizon x batch sweep,
// profiles/r01/session4/lanes_policy/): (1) the longest-parallel split whose chunks still hold
// >= cmin stages (the cross-lane combine is amortised over the chunk: nx = 2 needs 3, nx = 4 four;
// shorter chunks are combine-bound, longer ones serialise the lane and, at L = 32 and N >= 300,
// the on-chip gains cap residency at 6 waves/CU), then (2) double L while the batch gives fewer
// waves than the device has SIMDs (a half-empty chip loses more than a short chunk costs), up to
// two waves per trajectory.
int kkt_pick_lanes(int nx, int nu, int N, int B) {
  if (nx >= 8) return kkt_default_lanes(nx, nu, N);
  const int cmin = nx <= 2 ? 3 : 4;
  int L = 8;
  for (int c = 64; c >= 8; c /= 2)
    if (N >= cmin * c) { L = c; break; }
  const long simds = kkt_device_simds();
  // (3) two waves per trajectory (L = 128, nx <= 4) only when the horizon gives every lane of
  // both waves a stage and the whole batch is resident at once: that instance runs one wave per
  // SIMD (kkt_scan_kernel), so B * 2 waves must not exceed the SIMDs
  while ((long)B * L < 64 * simds &&
         (L < 64 || (L == 64 && nx <= 4 && N >= 128 && (long)B * 2 <= simds)))
    L *= 2;
  return L;
}
}  // namespace noc

// sha256 (16 hex digits) of the sources, from the Makefile (-DNOC_BUILD_HASH); include/noc_hip.h
#ifndef NOC_BUILD_HASH
#define NOC_BUILD_HASH "unknown"
#endif

extern "C" {

int noc_abi_version(void) { return NOC_ABI_VERSION; }
const char* noc_build_hash(void) { return NOC_BUILD_HASH; }
void noc_debug_set_ablation(int bits) { g_ablate = bits; }
const char* noc_last_error(void) { return g_last_error.c_str(); }
int noc_kkt_supported(int nx, int nu) { return noc::kkt_supported(nx, nu) ? 1 : 0; }
int noc_kkt_default_lanes(int nx, int nu, int N) { return noc::kkt_default_lanes(nx, nu, N); }
int noc_kkt_pick_lanes(int nx, int nu, int N, int B) {
  if (check_dims(nx, nu, N, B, 0)) return -1;
  return noc::kkt_pick_lanes(nx, nu, N, B);
}
int noc_kkt_gains_on_chip(int nx, int nu, int N, int lanes) {
  if (check_dims(nx, nu, N, 1, lanes)) return 0;
  const int L = lanes ? lanes : noc::kkt_default_lanes(nx, nu, N);
  return noc::kkt_lds_bytes_rt(nx, nu, N, L) > 0 ? 1 : 0;
}

static int kkt_common(int mode, int tiled, int nx, int nu, int N, int B, int lanes, const double* A,
                      const double* Bm, const double* Q, const double* R, const double* M,
                      const double* r, const double* q, const double* c, const double* P,
                      const double* p, const double* x0, const double* reg, const int* active,
                      double* dx, double* du, double* pred, int* feasible, double* K, double* d,
                      double* S, double* v, void* stream) {
  int rc = check_dims(nx, nu, N, B, lanes);
  if (rc) return rc;
  const bool bwd = mode != noc::MODE_FWD;
  const bool fwd = mode != noc::MODE_BWD;
  if ((rc = check_ptr(A, "A", true))) return rc;
  if ((rc = check_ptr(Bm, "B", true))) return rc;
  if ((rc = check_ptr(Q, "Q", bwd))) return rc;
  if ((rc = check_ptr(R, "R", bwd))) return rc;
  if ((rc = check_ptr(M, "M", bwd))) return rc;
  if ((rc = check_ptr(r, "r", bwd))) return rc;
  if ((rc = check_ptr(P, "P", bwd))) return rc;
  if ((rc = check_ptr(q, "q", false))) return rc;
  if ((rc = check_ptr(c, "c", false))) return rc;
  if ((rc = check_ptr(p, "p", false))) return rc;
  if ((rc = check_ptr(x0, "x0", false))) return rc;
  if ((rc = check_ptr(K, "K", false))) return rc;
  if ((rc = check_ptr(d, "d", false))) return rc;
  if ((rc = check_ptr(S, "S", false))) return rc;
  if ((rc = check_ptr(v, "v", false))) return rc;
  if ((rc = check_ptr(dx, "dx", false))) return rc;
  if ((rc = check_ptr(du, "du", false))) return rc;
  if ((rc = check_ptr(reg, "reg", false, 8))) return rc;
  if ((rc = check_ptr(pred, "pred", false, 8))) return rc;
  if ((rc = check_ptr(feasible, "feasible", false, 4))) return rc;
  if ((rc = check_ptr(active, "active", false, 4))) return rc;
  if (B == 0) return 0;
  noc::KKTArgs a{};
  a.N = N;
  a.B = B;
  a.mode = mode;
  a.A = A; a.Bm = Bm; a.Q = Q; a.R = R; a.M = M; a.r = r; a.q = q; a.c = c;
  a.P = P; a.p = p; a.x0 = x0; a.reg = reg; a.active = active;
  a.dx = dx; a.du = du; a.pred = pred; a.K = K; a.d = d; a.S = S; a.v = v;
  a.feasible = feasible;
  a.ablate = g_ablate;
  a.tiled = tiled;
  if (tiled && lanes == 0) return fail(-1, "the tiled layout needs an explicit lanes value");
  if (tiled && lanes == 1 && !(nx == 8 && nu == 4))
    return fail(-1, "the grouped (lanes = 1) tiled layout is supported for (nx, nu) = (8, 4)");
  if (lanes == 1 && !(64 % nx == 0 && nu <= nx))
    return fail(-1, "the group solve (lanes = 1) needs nx dividing 64 and nu <= nx");
  (void)bwd;
  (void)fwd;
  const int L = lanes ? lanes : noc::kkt_default_lanes(nx, nu, N);
  const bool on_chip = mode == noc::MODE_FULL && (dx || du) && noc::kkt_lds_bytes_rt(nx, nu, N, L) > 0;
  if ((!K || !d) && !on_chip)
    return fail(-2, "K and d are required (workspace) unless noc_kkt_gains_on_chip() is 1");
  return hip_status(noc::kkt_dispatch(nx, nu, a, L, static_cast<hipStream_t>(stream)),
                    "kkt_scan launch");
}

int noc_kkt_solve(int nx, int nu, int N, int B, int lanes, const double* A, const double* Bm,
                  const double* Q, const double* R, const double* M, const double* r,
                  const double* q, const double* c, const double* P, const double* p,
                  const double* x0, const double* reg, const int* active, double* dx, double* du,
                  double* pred, int* feasible, double* K, double* d, double* S, double* v,
                  void* stream) {
  return kkt_common(noc::MODE_FULL, 0, nx, nu, N, B, lanes, A, Bm, Q, R, M, r, q, c, P, p, x0, reg,
                    active, dx, du, pred, feasible, K, d, S, v, stream);
}

int noc_kkt_solve_tiled(int nx, int nu, int N, int B, int lanes, const double* A,
                        const double* Bm, const double* Q, const double* R, const double* M,
                        const double* r, const double* q, const double* c, const double* P,
                        const double* p, const double* x0, const double* reg, const int* active,
                        double* dx, double* du, double* pred, int* feasible, double* K, double* d,
                        double* S, double* v, void* stream) {
  return kkt_common(noc::MODE_FULL, 1, nx, nu, N, B, lanes, A, Bm, Q, R, M, r, q, c, P, p, x0,
                    reg, active, dx, du, pred, feasible, K, d, S, v, stream);
}

long long noc_tiled_doubles(int N, int B, int lanes, int E) {
  if (N < 1 || B < 0 || lanes < 1 || E < 1) return -1;
  if (lanes == 1)  // grouped layout: whole records of GROUP_T trajectories
    return (long long)((B + noc::GROUP_T - 1) / noc::GROUP_T) * noc::GROUP_T * N * E;
  const long long cmax = (N + lanes - 1) / lanes;
  return (long long)B * cmax * E * lanes;
}

int noc_relayout(int direction, int E, int sym_n, int N, int B, int lanes, const double* src,
                 double* dst, void* stream) {
  if (direction != 0 && direction != 1) return fail(-1, "direction must be 0 or 1");
  if (N < 1 || B < 0 || E < 1) return fail(-1, "bad dims");
  if (lanes != 1 && lanes != 8 && lanes != 16 && lanes != 32 && lanes != 64 && lanes != 128)
    return fail(-1, "lanes must be 1/8/16/32/64/128");
  if (sym_n > 0 && E != sym_n * (sym_n + 1) / 2) return fail(-1, "E must be sym_n(sym_n+1)/2");
  if (!src || !dst) return fail(-2, "NULL pointer");
  return hip_status(noc::relayout(direction, E, sym_n, N, B, lanes, src, dst,
                                  static_cast<hipStream_t>(stream)), "relayout");
}

int noc_par_bwd_pass(int nx, int nu, int N, int B, int lanes, const double* A, const double* Bm,
                     const double* Q, const double* R, const double* M, const double* r,
                     const double* q, const double* c, const double* P, const double* p,
                     const double* reg, const int* active, double* K, double* d, double* S,
                     double* v, double* pred, int* feasible, void* stream) {
  return kkt_common(noc::MODE_BWD, 0, nx, nu, N, B, lanes, A, Bm, Q, R, M, r, q, c, P, p, nullptr,
                    reg, active, nullptr, nullptr, pred, feasible, K, d, S, v, stream);
}

int noc_par_fwd_pass(int nx, int nu, int N, int B, int lanes, const double* A, const double* Bm,
                     const double* c, const double* x0, const double* K, const double* d,
                     const int* active, double* du, double* dx, void* stream) {
  return kkt_common(noc::MODE_FWD, 0, nx, nu, N, B, lanes, A, Bm, nullptr, nullptr, nullptr,
                    nullptr, nullptr, c, nullptr, nullptr, x0, nullptr, active, dx, du, nullptr,
                    nullptr, const_cast<double*>(K), const_cast<double*>(d), nullptr, nullptr,
                    stream);
}

int noc_family_supported(const noc_family* fam) {
  return (fam && noc::family_supported(*fam)) ? 1 : 0;
}

static int check_ipm(const noc_family* fam, const noc_ipm_ws* ws) {
  if (!ws) return fail(-2, "workspace is NULL");
  if (ws->Bt < 0 || ws->N < 1) return fail(-1, "workspace dims: need Bt >= 0, N >= 1");
  if (ws->lanes != 1 && ws->lanes != 8 && ws->lanes != 16 && ws->lanes != 32 && ws->lanes != 64)
    return fail(-1, "workspace lanes must be 1, 8, 16, 32 or 64");
  if (ws->lanes == 1 && fam && !(fam->nx == 8 && fam->nu == 4))
    return fail(-1, "workspace lanes = 1 (grouped layout) is supported for nx = 8, nu = 4");
  if (fam && !noc::family_supported(*fam))
    return fail(-1, "unsupported problem family (kind/nx/nu)");
  const void* req[] = {ws->x, ws->u, ws->x0, ws->A, ws->B, ws->Q, ws->R, ws->M, ws->r, ws->P,
                       ws->cx, ws->cu, ws->lc, ws->lam, ws->dx, ws->du, ws->pred, ws->K, ws->d,
                       ws->feasible, ws->phase, ws->kkt_active, ws->it, ws->inner, ws->total_it,
                       ws->kkt_solves, ws->bp, ws->rp, ws->rinc, ws->cost, ws->hu, ws->gnorm,
                       ws->reg};
  for (const void* p : req)
    if (!p) return fail(-2, "a required workspace pointer is NULL");
  if (ws->flags & ~(NOC_WS_ONE_STAGE | NOC_WS_RESUME | NOC_WS_NO_REPEAT_SKIP))
    return fail(-1, "workspace flags: unknown bits set (NOC_WS_ONE_STAGE | NOC_WS_RESUME | "
                    "NOC_WS_NO_REPEAT_SKIP are defined)");
  return 0;
}

int noc_ipm_init(const noc_ipm_ws* ws, double bp0, void* stream) {
  int rc = check_ipm(nullptr, ws);
  if (rc) return rc;
  if (ws->Bt == 0) return 0;
  return hip_status(noc::ipm_init(*ws, bp0, static_cast<hipStream_t>(stream)), "ipm_init");
}

int noc_ipm_prepare(const noc_family* fam, const noc_ipm_ws* ws, int mode, int terminal,
                    void* stream) {
  if (!fam) return fail(-2, "family is NULL");
  int rc = check_ipm(fam, ws);
  if (rc) return rc;
  if (mode != NOC_MODE_PAR && mode != NOC_MODE_SEQ) return fail(-1, "bad mode");
  if (terminal != NOC_TERMINAL_FINAL_COST && terminal != NOC_TERMINAL_STAGE0)
    return fail(-1, "bad terminal option");
  if (ws->Bt == 0) return 0;
  return hip_status(noc::ipm_prepare(*fam, *ws, mode, terminal, static_cast<hipStream_t>(stream)),
                    "ipm_prepare");
}

int noc_ipm_trial(const noc_family* fam, const noc_ipm_ws* ws, int mode, void* stream) {
  if (!fam) return fail(-2, "family is NULL");
  int rc = check_ipm(fam, ws);
  if (rc) return rc;
  if (mode != NOC_MODE_PAR && mode != NOC_MODE_SEQ) return fail(-1, "bad mode");
  if (ws->Bt == 0) return 0;
  return hip_status(noc::ipm_trial(*fam, *ws, mode, static_cast<hipStream_t>(stream)), "ipm_trial");
}

int noc_total_cost(const noc_family* fam, int N, int B, const double* x, const double* u,
                   const double* bp, double* cost, void* stream) {
  if (!fam) return fail(-2, "family is NULL");
  if (!noc::family_supported(*fam)) return fail(-1, "unsupported problem family (kind/nx/nu)");
  if (N < 1 || B < 0) return fail(-1, "need N >= 1, B >= 0");
  int rc = 0;
  if ((rc = check_ptr(x, "x", true, 8)) || (rc = check_ptr(u, "u", true, 8)) ||
      (rc = check_ptr(bp, "bp", true, 8)) || (rc = check_ptr(cost, "cost", true, 8)))
    return rc;
  if (B == 0) return 0;
  return hip_status(noc::total_cost(*fam, N, B, x, u, bp, cost, static_cast<hipStream_t>(stream)),
                    "total_cost");
}

static int kkt_and_trial(const noc_family* fam, const noc_ipm_ws* ws, int mode, void* stream);

int noc_ipm_step(const noc_family* fam, const noc_ipm_ws* ws, int mode, int terminal, int lanes,
                 void* stream) {
  // lanes: 0 = the workspace's; any other value must equal it (the blocks are laid out for it)
  if (ws && lanes != 0 && lanes != ws->lanes)
    return fail(-1, "noc_ipm_step: lanes (" + std::to_string(lanes) + ") differs from the workspace's (" +
                        std::to_string(ws->lanes) + "); pass 0 or ws->lanes");
  int rc = noc_ipm_prepare(fam, ws, mode, terminal, stream);
  if (rc) return rc;
  return kkt_and_trial(fam, ws, mode, stream);
}

int noc_ipm_rollout(const noc_family* fam, const noc_ipm_ws* ws, void* stream) {
  if (!fam) return fail(-2, "family is NULL");
  int rc = check_ipm(fam, ws);
  if (rc) return rc;
  if (ws->Bt == 0) return 0;
  return hip_status(noc::ipm_rollout(*fam, *ws, static_cast<hipStream_t>(stream)), "ipm_rollout");
}

int noc_ipm_promote(const noc_ipm_ws* ws, void* stream) {
  int rc = check_ipm(nullptr, ws);
  if (rc) return rc;
  if (ws->Bt == 0) return 0;
  return hip_status(noc::ipm_promote(*ws, static_cast<hipStream_t>(stream)), "ipm_promote");
}

int noc_ipm_step_main(const noc_family* fam, const noc_ipm_ws* ws, int mode, int terminal,
                      void* stream) {
  if (!fam) return fail(-2, "family is NULL");
  int rc = check_ipm(fam, ws);
  if (rc) return rc;
  if (mode != NOC_MODE_PAR && mode != NOC_MODE_SEQ) return fail(-1, "bad mode");
  if (terminal != NOC_TERMINAL_FINAL_COST && terminal != NOC_TERMINAL_STAGE0)
    return fail(-1, "bad terminal option");
  if (ws->Bt == 0) return 0;
  rc = hip_status(noc::ipm_prepare_main(*fam, *ws, mode, terminal, static_cast<hipStream_t>(stream)),
                  "ipm_prepare_main");
  if (rc) return rc;
  return kkt_and_trial(fam, ws, mode, stream);
}

int noc_debug_phase_cycles(long long* out, int n, int reset) {
  if (!out || n < 0) return fail(-2, "out is NULL");
  return noc::debug_phase_cycles(out, n, reset) == 0 ? 0 : fail(-10, "hipMemcpyFromSymbol failed");
}

// Diagnostic export (not in include/noc_hip.h; tools/flip_probe.py): the decision-trace buffer of
// the persistent solvers, (ntraj, cap, 12) doubles; NULL switches it off.  Returns 1 if this build
// records (make trace-lib), 0 if it has no trace code.
extern "C" int noc_debug_set_decision_trace(double* buf, int cap, int ntraj) {
  if (cap < 0 || ntraj < 0) return fail(-1, "cap, ntraj must be >= 0");
  const int rc = noc::debug_set_decision_trace(buf, cap, ntraj);
  return rc < 0 ? fail(-10, "hipMemcpyToSymbol failed") : rc;
}

int noc_debug_traj_times(long long* out, int n) {
  if (!out || n < 0) return fail(-2, "out is NULL");
  return noc::debug_traj_times(out, n) == 0 ? 0 : fail(-10, "hipMemcpyFromSymbol failed");
}

int noc_ipm_solve_supported(const noc_family* fam, int N, int lanes) {
  return (fam && N >= 1 && noc::ipm_solve_supported(*fam, N, lanes)) ? 1 : 0;
}

int noc_ipm_solve(const noc_family* fam, const noc_ipm_ws* ws, int mode, int terminal, double bp0,
                  int max_solves, void* stream) {
  if (!fam) return fail(-2, "family is NULL");
  int rc = check_ipm(fam, ws);
  if (rc) return rc;
  if (mode != NOC_MODE_PAR && mode != NOC_MODE_SEQ) return fail(-1, "bad mode");
  if (terminal != NOC_TERMINAL_FINAL_COST && terminal != NOC_TERMINAL_STAGE0)
    return fail(-1, "bad terminal option");
  if (!(bp0 > 0.0)) return fail(-1, "bp0 must be > 0");
  if (max_solves < 1) return fail(-1, "max_solves must be >= 1");
  if (!noc::ipm_solve_supported(*fam, ws->N, ws->lanes))
    return fail(-1, "persistent solve needs workspace lanes = 64 and a step that fits in LDS "
                    "(noc_ipm_solve_supported)");
  if (ws->Bt == 0) return 0;
  return hip_status(noc::ipm_solve(*fam, *ws, mode, terminal, bp0, max_solves,
                                   static_cast<hipStream_t>(stream)), "ipm_solve");
}

long long noc_ddp_work_doubles(int nx, int nu, int N, int Bt) {
  if (nx < 1 || nu < 1 || N < 1 || Bt < 0) return -1;
  const long long b = Bt, n = N;
  // X, TX, TU, k, K and the per-stage derivative records
  return b * (2 * (n + 1) * nx + 2 * n * nu + n * nu * nx + n * noc::ddp_record_doubles(nx, nu));
}

int noc_ddp_supported(const noc_family* fam) { return (fam && noc::ddp_supported(*fam)) ? 1 : 0; }

int noc_ddp_solve(const noc_family* fam, int N, int Bt, const double* x0, double* u, double* work,
                  int* iterations, int* passes, int* done, double bp0, int max_passes,
                  void* stream) {
  return noc_ddp_solve_ex(fam, N, Bt, x0, u, work, iterations, passes, done, bp0, max_passes, 0,
                          stream);
}

int noc_ddp_solve_ex(const noc_family* fam, int N, int Bt, const double* x0, double* u,
                     double* work, int* iterations, int* passes, int* done, double bp0,
                     int max_passes, int flags, void* stream) {
  if (flags & ~NOC_DDP_ONE_STAGE) return fail(-1, "ddp flags: only NOC_DDP_ONE_STAGE is defined");
  if (!fam) return fail(-2, "family is NULL");
  if (!noc::ddp_supported(*fam))
    return fail(-1, "DDP supports the registered families with nx <= 4 (noc_ddp_supported)");
  if (N < 1) return fail(-1, "horizon N must be >= 1");
  if (Bt < 0) return fail(-1, "batch Bt must be >= 0");
  // any finite bp0 >= 0, like the reference ddp (D:98, no check on bp): bp0 = 0 is the
  // unconstrained one-stage solve; the schedule (no NOC_DDP_ONE_STAGE) runs no stage for
  // bp0 <= 1e-4, as interior_point_ddp's while loop (D:194) -- the same rule as the nx > 4 host loop
  if (!(bp0 >= 0.0) || !(bp0 < INFINITY)) return fail(-1, "bp0 must be finite and >= 0");
  if (max_passes < 1) return fail(-1, "max_passes must be >= 1");
  int rc = 0;
  if ((rc = check_ptr(x0, "x0", true, 8)) || (rc = check_ptr(u, "u", true, 8)) ||
      (rc = check_ptr(work, "work", true, 8)) || (rc = check_ptr(iterations, "iterations", true, 4)) ||
      (rc = check_ptr(passes, "passes", true, 4)) || (rc = check_ptr(done, "done", true, 4)))
    return rc;
  if (Bt == 0) return 0;
  return hip_status(noc::ddp_solve(*fam, N, Bt, x0, u, work, iterations, passes, done, bp0,
                                   max_passes, flags, static_cast<hipStream_t>(stream)), "ddp_solve");
}

int noc_ddp_bwd_pass(int nx, int nu, int N, int B, const double* Vx, const double* Vxx,
                     const double* reg_param, const double* cx, const double* cu,
                     const double* cxx, const double* cuu, const double* cxu, const double* fx,
                     const double* fu, const double* fxx, const double* fuu, const double* fxu,
                     double* k, double* K, double* pred, int* feasible, double* Hu, void* stream) {
  if (!noc::kkt_supported(nx, nu))
    return fail(-1, "noc_ddp_bwd_pass: unsupported (nx, nu); supported: " + noc::kkt_shapes_str());
  if (N < 1 || B < 0) return fail(-1, "need N >= 1, B >= 0");
  const void* req[] = {Vx, Vxx, reg_param, cx, cu, cxx, cuu, cxu, fx, fu, fxx, fuu, fxu, k, K,
                       pred, Hu};
  for (const void* p : req) {
    int rc = check_ptr(p, "ddp_bwd_pass argument", true, 8);
    if (rc) return rc;
  }
  int rc = check_ptr(feasible, "feasible", true, 4);
  if (rc) return rc;
  if (B == 0) return 0;
  noc::DdpBwdArgs a{N, B, Vx, Vxx, reg_param, cx, cu, cxx, cuu, cxu, fx, fu, fxx, fuu, fxu,
                    k, K, pred, Hu, feasible};
  return hip_status(noc::ddp_bwd_pass(nx, nu, a, static_cast<hipStream_t>(stream)), "ddp_bwd_pass");
}

int noc_nonlin_rollout(const noc_family* fam, int N, int B, const double* K, const double* k,
                       const double* x, const double* u, double* x_new, double* u_new,
                       void* stream) {
  if (!fam) return fail(-2, "family is NULL");
  if (!noc::family_supported(*fam)) return fail(-1, "unsupported problem family (kind/nx/nu)");
  if (N < 1 || B < 0) return fail(-1, "need N >= 1, B >= 0");
  const void* req[] = {K, k, x, u, x_new, u_new};
  for (const void* p : req) {
    int rc = check_ptr(p, "nonlin_rollout argument", true, 8);
    if (rc) return rc;
  }
  if (B == 0) return 0;
  return hip_status(noc::nonlin_rollout(*fam, N, B, K, k, x, u, x_new, u_new,
                                        static_cast<hipStream_t>(stream)), "nonlin_rollout");
}

int noc_derivatives(const noc_family* fam, int N, int B, const double* x, const double* u,
                    const double* bp, double* cx, double* cu, double* cxx, double* cuu,
                    double* cxu, double* fx, double* fu, double* fxx, double* fuu, double* fxu,
                    void* stream) {
  if (!fam) return fail(-2, "family is NULL");
  if (!noc::family_supported(*fam)) return fail(-1, "unsupported problem family (kind/nx/nu)");
  if (N < 1 || B < 0) return fail(-1, "need N >= 1, B >= 0");
  const void* req[] = {x, u, bp, cx, cu, cxx, cuu, cxu, fx, fu, fxx, fuu, fxu};
  for (const void* p : req) {
    int rc = check_ptr(p, "derivatives argument", true, 8);
    if (rc) return rc;
  }
  if (B == 0) return 0;
  noc::DerivArgs a{N, B, x, u, bp, cx, cu, cxx, cuu, cxu, fx, fu, fxx, fuu, fxu};
  return hip_status(noc::derivatives(*fam, a, static_cast<hipStream_t>(stream)), "derivatives");
}

int noc_final_cost_derivs(const noc_family* fam, int B, const double* xN, double* grad,
                          double* hess, void* stream) {
  if (!fam) return fail(-2, "family is NULL");
  if (!noc::family_supported(*fam)) return fail(-1, "unsupported problem family (kind/nx/nu)");
  if (B < 0) return fail(-1, "need B >= 0");
  int rc = 0;
  if ((rc = check_ptr(xN, "xN", true, 8)) || (rc = check_ptr(grad, "grad", true, 8)) ||
      (rc = check_ptr(hess, "hess", false, 8)))
    return rc;
  if (B == 0) return 0;
  return hip_status(noc::final_cost_derivs(*fam, B, xN, grad, hess, static_cast<hipStream_t>(stream)),
                    "final_cost_derivs");
}

int noc_costates(int nx, int N, int B, const double* lamT, const double* cx, const double* fx,
                 double* lam, int sequential, void* stream) {
  if (nx < 1 || nx > 8) return fail(-1, "costates support 1 <= nx <= 8");
  if (N < 1 || B < 0) return fail(-1, "need N >= 1, B >= 0");
  int rc = 0;
  if ((rc = check_ptr(lamT, "lamT", true, 8)) || (rc = check_ptr(cx, "cx", true, 8)) ||
      (rc = check_ptr(fx, "fx", true, 8)) || (rc = check_ptr(lam, "lam", true, 8)))
    return rc;
  if (B == 0) return 0;
  return hip_status(noc::costates(nx, N, B, lamT, cx, fx, lam, sequential,
                                  static_cast<hipStream_t>(stream)), "costates");
}

int noc_lqr_params(int nx, int nu, int N, int B, const double* lam, const double* cu,
                   const double* cxx, const double* cuu, const double* cxu, const double* fu,
                   const double* fxx, const double* fuu, const double* fxu, double* ru, double* Q,
                   double* R, double* M, void* stream) {
  if (nx < 1 || nx > 8 || nu < 1 || nu > 8) return fail(-1, "lqr_params support nx, nu <= 8");
  if (N < 1 || B < 0) return fail(-1, "need N >= 1, B >= 0");
  const void* req[] = {lam, cu, cxx, cuu, cxu, fu, fxx, fuu, fxu, ru, Q, R, M};
  for (const void* p : req) {
    int rc = check_ptr(p, "lqr_params argument", true, 8);
    if (rc) return rc;
  }
  if (B == 0) return 0;
  noc::LqrArgs a{nx, nu, N, B, lam, cu, cxx, cuu, cxu, fu, fxx, fuu, fxu, ru, Q, R, M};
  return hip_status(noc::lqr_params(a, static_cast<hipStream_t>(stream)), "lqr_params");
}

int noc_check_feasibility(const noc_family* fam, int N, int B, const double* x, const double* u,
                          int* feasible, void* stream) {
  if (!fam) return fail(-2, "family is NULL");
  if (!noc::family_supported(*fam)) return fail(-1, "unsupported problem family (kind/nx/nu)");
  if (N < 1 || B < 0) return fail(-1, "need N >= 1, B >= 0");
  int rc = 0;
  if ((rc = check_ptr(x, "x", true, 8)) || (rc = check_ptr(u, "u", true, 8)) ||
      (rc = check_ptr(feasible, "feasible", true, 4)))
    return rc;
  if (B == 0) return 0;
  return hip_status(noc::traj_feasibility(*fam, N, B, x, u, feasible,
                                          static_cast<hipStream_t>(stream)), "check_feasibility");
}

static int kkt_and_trial(const noc_family* fam, const noc_ipm_ws* ws, int mode, void* stream) {
  // the trial step needs dx, du only: gains stay on chip when they fit (ws->K, ws->d otherwise)
  const bool on_chip = noc_kkt_gains_on_chip(fam->nx, fam->nu, ws->N, ws->lanes) == 1;
  int rc = noc_kkt_solve_tiled(fam->nx, fam->nu, ws->N, ws->Bt, ws->lanes, ws->A, ws->B, ws->Q,
                               ws->R, ws->M, ws->r, nullptr, nullptr, ws->P, nullptr, nullptr,
                               ws->reg, ws->kkt_active, ws->dx, ws->du, ws->pred, ws->feasible,
                               on_chip ? nullptr : ws->K, on_chip ? nullptr : ws->d, nullptr,
                               nullptr, stream);
  if (rc) return rc;
  return noc_ipm_trial(fam, ws, mode, stream);
}

}  // extern "C"
