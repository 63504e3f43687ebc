/* noc_hip.h -- C-ABI of libnoc_hip.so, the MI355X (gfx950) hot path of the interior-point
 * trajectory optimiser.  Plain pointers and sizes only; all arrays are fp64 device pointers
 * (hipMalloc / torch data_ptr), row-major, contiguous, 16-byte aligned; every call is
 * asynchronous on `stream` (a hipStream_t, NULL = default stream) and never synchronises.
 *
 * Return value: 0 on success, < 0 on an argument or HIP error (noc_last_error() explains).
 * Numerical trouble is data, never an error: feasible[b] = 0, pred NaN/inf, exactly like the
 * reference's jnp.where / NaN semantics (noc/par_interior_point_newton.py:159-173).
 *
 * LQ sub-problem solved per trajectory b (shapes per trajectory; leading batch axis B):
 *   stage k < N : 1/2 x'Q_k x + x'M_k u + 1/2 u'(R_k + reg_b I)u + r_k'u + q_k'x
 *   dynamics    : x_{k+1} = A_k x_k + Bm_k u_k + c_k,   x_0 = x0
 *   terminal    : 1/2 x_N'P x_N + p'x_N
 *   A [B][N][nx][nx]  Bm [B][N][nx][nu]  Q [B][N][nx][nx]  R [B][N][nu][nu]  M [B][N][nx][nu]
 *   r [B][N][nu]      q, c [B][N][nx] (NULL = 0)   P [B][nx][nx]   p, x0 [B][nx] (NULL = 0)
 *   reg [B] (NULL = 0)                              active [B] int32 (NULL = all; 0 = skip)
 * Outputs:
 *   dx [B][N+1][nx]  du [B][N][nu]  pred [B]  feasible [B] int32
 *   K [B][N][nu][nx] d [B][N][nu]   (du_k = K_k dx_k + d_k); NULL = not written, allowed in
 *                                   the fused solves when noc_kkt_gains_on_chip() is 1 (the
 *                                   gains then never leave the CU: par_Newton discards them)
 *   S [B][N+1][nx][nx]  v [B][N+1][nx]  (V_k(x) = 1/2 x'S_k x + v_k'x; NULL = not written)
 *   pred = sum_k d_k'Qu_k + 1/2 d_k'Quu_k d_k,  feasible = all_k Quu_k > 0
 *
 * Supported (nx, nu): (2,1) pendulum, (4,1) cart-pole, (8,4) stacked double integrators.
 * `lanes` = lanes of a wave64 per trajectory (64, 32, 16, 8: parallel-in-time scan over the
 * horizon, chunked over the lanes; 128: two waves per trajectory joined through LDS, nx <= 4, for
 * batches too small to give every SIMD a wave); 1 = horizon-sequential Riccati with the
 * trajectory's algebra spread over an nx-lane group (work-efficient; for batches that fill the
 * GPU by themselves, natural layout, gains through HBM); 0 = library default.
 */
#ifndef NOC_HIP_H
#define NOC_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

#define NOC_ABI_VERSION 5 /* 2: noc_ipm_ws gained `repeats`; 3: `order`; 4: noc_check_feasibility,
                             noc_ddp_solve_ex, noc_ddp_bwd_pass, noc_nonlin_rollout (additive);
                             5: noc_total_cost (additive) */

/* Library identity / diagnostics. */
int noc_abi_version(void);
/* Provenance of the binary: the first 16 hex digits of sha256 over the sources it was compiled
 * from (the .hip, .h and .def files of csrc/ and csrc/custom/ in name order, then this header), baked in by
 * the Makefile.  The Python host refuses a library whose hash differs from the tree's
 * (noc/_lib.py: load), so a stale binary cannot pass for the current sources. */
const char* noc_build_hash(void);
const char* noc_last_error(void);
int noc_kkt_supported(int nx, int nu);
/* Lanes per trajectory used when a solve is called with lanes = 0 (batch-agnostic). */
int noc_kkt_default_lanes(int nx, int nu, int N);
/* Batch-aware choice for B trajectories on the current device (chunks of >= 3-4 stages per lane,
 * then enough waves to fill every SIMD); what the Python host passes explicitly.  -1 on bad
 * dimensions.  A caller that uses it passes the result as `lanes` to every call of the solve
 * (including noc_kkt_gains_on_chip and the tiled-layout helpers). */
int noc_kkt_pick_lanes(int nx, int nu, int N, int B);
/* 1 if the fused solve (noc_kkt_solve / _tiled) with these sizes keeps the gains K, d in LDS
 * between its backward and forward phases, so K and d may be passed as NULL. */
int noc_kkt_gains_on_chip(int nx, int nu, int N, int lanes);
/* Timing-only phase ablation of the KKT scan (bit0: skip the cross-lane scan, bit1: skip the
 * forward pass, bit2: stop after the in-chunk elements, bit3: stream the chunk from memory in
 * every phase instead of the register-cached chunk; bit 3 alone keeps results exact).  Results of
 * bits 0-2 are WRONG while set; used by
 * tools/kkt_ablate.py to attribute kernel time to phases.  0 (default) in every product call. */
void noc_debug_set_ablation(int bits);

/* Fused batched KKT solve of one Newton step: par_bwd_pass + par_fwd_pass.
 * Replaces par_Newton's solver calls, noc/par_interior_point_newton.py:119-123
 * (paroc.par_bwd_pass(lqt) -> Kx, d, S, v, pred, feasible; paroc.par_fwd_pass(lqt, 0, Kx, d)). */
int noc_kkt_solve(int nx, int nu, int N, int B, int lanes,
                  const double* A, const double* Bm, const double* Q, const double* R,
                  const double* M, const double* r, const double* q, const double* c,
                  const double* P, const double* p, const double* x0, const double* reg,
                  const int* active,
                  double* dx, double* du, double* pred, int* feasible,
                  double* K, double* d, double* S, double* v, void* stream);

/* ---- tiled ("lane-interleaved") block layout ------------------------------------------------
 * For `lanes` = L lanes per trajectory, stage s of an N-stage horizon belongs to chunk lane l at
 * chunk position j (lanes l < N % L own N/L + 1 stages, the others N/L; chunks are contiguous in
 * time, cmax = ceil(N/L)).  A field with E doubles per stage is stored, per trajectory b, as
 *   E even: [b][j][e/2][l][2]      E odd: [b][j][e][l]
 * (noc_tiled_doubles() doubles per field).  Q and R are stored PACKED symmetric (upper triangle,
 * row-major: E = n(n+1)/2).  Every wave-wide access of the KKT scan is then L*16 contiguous
 * bytes.  The interior-point workspace (noc_ipm_ws) always uses this layout. */
long long noc_tiled_doubles(int N, int B, int lanes, int E);
/* direction 0: natural (B,N,E) -> tiled; 1: tiled -> natural.  sym_n > 0: the natural field is a
 * full sym_n x sym_n matrix per stage and the tiled one packed (E must be sym_n(sym_n+1)/2). */
int noc_relayout(int direction, int E, int sym_n, int N, int B, int lanes, const double* src,
                 double* dst, void* stream);
/* noc_kkt_solve with A, Bm, Q(packed), R(packed), M, r, q, c, K, d in the tiled layout of
 * `lanes` (required, 8/16/32/64/128); P, p, x0, reg, dx, du, S, v natural. */
int noc_kkt_solve_tiled(int nx, int nu, int N, int B, int lanes,
                        const double* A, const double* Bm, const double* Q, const double* R,
                        const double* M, const double* r, const double* q, const double* c,
                        const double* P, const double* p, const double* x0, const double* reg,
                        const int* active,
                        double* dx, double* du, double* pred, int* feasible,
                        double* K, double* d, double* S, double* v, void* stream);

/* Backward pass only: replaces paroc.par_bwd_pass (call sites
 * noc/par_interior_point_newton.py:120, examples/linear_mpc_parallel.py:68). */
int noc_par_bwd_pass(int nx, int nu, int N, int B, int lanes,
                     const double* A, const double* Bm, const double* Q, const double* R,
                     const double* M, const double* r, const double* q, const double* c,
                     const double* P, const double* p, const double* reg, const int* active,
                     double* K, double* d, double* S, double* v, double* pred, int* feasible,
                     void* stream);

/* Forward pass only: replaces paroc.par_fwd_pass(lqt, x0, Kx, d) -> (u, x) (call sites
 * noc/par_interior_point_newton.py:121-123, examples/linear_mpc_parallel.py:69).
 * K and d are inputs here. */
int noc_par_fwd_pass(int nx, int nu, int N, int B, int lanes,
                     const double* A, const double* Bm, const double* c, const double* x0,
                     const double* K, const double* d, const int* active,
                     double* du, double* dx, void* stream);

/* ------------------------------------------------------------------------------------------
 * Batched interior-point driver kernels for registered problem families.
 * Replaces the device-side body of par_interior_point_optimal_control / newton_oc
 * (noc/par_interior_point_newton.py:127-254) and, with mode NOC_MODE_SEQ, of
 * seq_interior_point_optimal_control (noc/seq_interior_point_newton.py:108-202).
 * The host loop calls noc_ipm_step until no trajectory's phase is NOC_PHASE_DONE-pending.
 * ------------------------------------------------------------------------------------------ */
#define NOC_FAMILY_PENDULUM 1 /* examples/pendulum_runtime.py:19-72 */
#define NOC_FAMILY_CARTPOLE 2 /* examples/cartpole_runtime.py:18-82 */
#define NOC_FAMILY_LINEAR 3   /* examples/linear_mpc_parallel.py:24-63, linear_demo_cuda.py */
#define NOC_FAMILY_CUSTOM 4   /* a family registered at run time (noc.families.register_family):
                                 supported only by that family's own build of this library */

#define NOC_PHASE_ROLLOUT 0
#define NOC_PHASE_LINEARIZE 1
#define NOC_PHASE_SOLVE 2
#define NOC_PHASE_DONE 3
#define NOC_PHASE_ROLLED 4 /* rolled out, waiting to be promoted to LINEARIZE (two-stream loop) */
#define NOC_PHASE_ROLLOUT_PENDING 5 /* a barrier stage ended in the last trial; noc_ipm_promote (or
                                       the single-stream noc_ipm_step) starts its rollout */

#define NOC_MODE_PAR 0 /* par_interior_point_newton semantics (retry loop, reg = rp*|cu|) */
#define NOC_MODE_SEQ 1 /* seq_interior_point_newton semantics (one accept/reject, reg = mu) */

#define NOC_TERMINAL_FINAL_COST 0 /* terminal Hessian = hessian(final_cost)(x_N)  (S:66) */
#define NOC_TERMINAL_STAGE0 1     /* the reference par path's XT = Q[0]           (P:73) */

/* Problem family descriptor.  Stage cost:
 *   1/2 sum_i wx_i e_i^2 + 1/2 sum_j wu_j u_j^2 - bp sum_j [log(ub - u_j) + log(u_j + ub)]
 * with e = x - goal (state wrap_index taken mod 2*pi first); the barrier term is absent when
 * u_bound <= 0.  Terminal cost 1/2 sum_i wf_i e_i^2.  Dynamics: Euler(ode, dt) for the pendulum
 * and cart-pole, x+ = A x + B u for LINEAR. */
typedef struct noc_family {
  int kind, nx, nu, wrap_index;
  double dt, u_bound;
  double goal[8], wx[8], wu[4], wf[8];
  double A[64], B[32];
} noc_family;

/* Workspace of device pointers (all fp64 unless noted; Bt trajectories, horizon N). */
#define NOC_WS_ONE_STAGE 1 /* flags bit: stop after ONE barrier stage (newton_oc, P:127-225 /
                              S:108-177) instead of running the schedule while bp > 1e-4 */
#define NOC_WS_RESUME 2    /* flags bit (noc_ipm_solve): continue every trajectory from the state
                              held in the workspace (bp, rp, r_inc, cost, hu, gnorm, it, inner,
                              total_it, kkt_solves, x, u) at its phase -- ROLLOUT: a new barrier
                              stage, LINEARIZE: a new Newton iteration, SOLVE: a retry on the
                              current blocks, DONE: nothing -- instead of starting at bp0 */
#define NOC_WS_NO_REPEAT_SKIP 4 /* flags bit: recompute every retry of the par inner loop, even the
                              repeats at the rp clip that the solvers otherwise account without
                              recomputing (ws->repeats; same results bit for bit either way) */
/* Any other flags bit is rejected (-1) by every noc_ipm_* entry point. */
typedef struct noc_ipm_ws {
  int Bt, N;
  int lanes;                           /* tiled layout of A,B,Q,R,M,r,K,d (8/16/32/64)  */
  int flags;                           /* NOC_WS_* bits (0 = the whole barrier schedule) */
  double *x, *u, *x0;                  /* (Bt,N+1,nx) (Bt,N,nu) (Bt,nx)           */
  double *A, *B, *Q, *R, *M, *r, *P;   /* LQ blocks: tiled (P natural).  noc_ipm_solve
                                          keeps only their variable entries here (compact
                                          records, csrc/block_struct.h): scratch after it */
  double *cx, *cu, *lc, *lam;          /* cx, cu, lc tiled (E = nx, nu, 1); lam (Bt,N+1,nx).
                                          cx, cu, lam: written by the launch-per-phase driver
                                          only (noc_ipm_solve keeps them in registers) */
  double *dx, *du, *pred, *K, *d;      /* KKT outputs (dx, du natural; K, d tiled)  */
  int *feasible;                       /* (Bt) int32                               */
  int *phase, *kkt_active, *it, *inner, *total_it, *kkt_solves; /* (Bt) int32     */
  int *repeats;                        /* (Bt) int32 or NULL: of kkt_solves, the retries that
                                          repeat a rejected trial at the rp clip exactly and were
                                          accounted without recomputation (par mode, P:151-188) */
  const int *order;                    /* (Bt) int32 or NULL: noc_ipm_solve's one-wave kernel
                                          starts trajectory order[i] as its i-th workgroup.  MUST
                                          be a permutation of 0..Bt-1 (the caller's contract: the
                                          library cannot check it without a device sync; an entry
                                          outside 0..Bt-1 is skipped, a repeated one makes two
                                          workgroups race on one trajectory).  Results per
                                          trajectory are the same for any order -- only the
                                          schedule changes.  The wide kernel (B <= #CUs) ignores it:
                                          it runs one trajectory per CU at once anyway. */
  double *bp, *rp, *rinc, *cost, *hu, *gnorm, *reg;              /* (Bt)           */
} noc_ipm_ws;

int noc_family_supported(const noc_family* fam);
/* state <- start of the barrier schedule (bp = bp0, rp = 1, r_inc = 2, phase ROLLOUT). */
int noc_ipm_init(const noc_ipm_ws* ws, double bp0, void* stream);
/* rollout (phase ROLLOUT) + linearise / costates / LQ blocks (phase LINEARIZE) -> phase SOLVE. */
int noc_ipm_prepare(const noc_family* fam, const noc_ipm_ws* ws, int mode, int terminal,
                    void* stream);
/* trial point, gain ratio, regularisation update, accept, stop test, barrier schedule. */
int noc_ipm_trial(const noc_family* fam, const noc_ipm_ws* ws, int mode, void* stream);
/* one device iteration: prepare + noc_kkt_solve(active = phase SOLVE) + trial.  lanes must be 0
 * or ws->lanes (the workspace's tiled layout fixes it); anything else is rejected. */
int noc_ipm_step(const noc_family* fam, const noc_ipm_ws* ws, int mode, int terminal, int lanes,
                 void* stream);
/* Two-stream form of one iteration (rollouts overlap the other trajectories' Newton step):
 *   roll stream : wait(prev main event); noc_ipm_rollout      (ROLLOUT -> ROLLED)
 *   main stream : noc_ipm_step_main (LINEARIZE..SOLVE..trial); wait(roll event);
 *                 noc_ipm_promote                              (ROLLED  -> LINEARIZE)
 * The trial marks a trajectory whose barrier stage ended NOC_PHASE_ROLLOUT_PENDING; only promote
 * (after the main stream waited on the roll event) turns that into ROLLOUT, so a rollout never
 * runs concurrently with the trial that writes its controls.
 * Every trajectory still performs exactly its own reference sequence of operations. */
int noc_ipm_rollout(const noc_family* fam, const noc_ipm_ws* ws, void* stream);
int noc_ipm_step_main(const noc_family* fam, const noc_ipm_ws* ws, int mode, int terminal,
                      void* stream);
int noc_ipm_promote(const noc_ipm_ws* ws, void* stream);

/* Persistent solve: the WHOLE barrier schedule (rollout, Newton / retry loops, barrier updates)
 * of every trajectory in ONE launch, one wave64 per trajectory running its own reference control
 * flow back to back (no per-step launches, no host polls, no lockstep across trajectories).
 * Same arithmetic and results as the noc_ipm_init + noc_ipm_step loop at lanes = 64 -- except that
 * a batch of at most one trajectory per CU with N > 128 runs the wide kernel (four waves per
 * trajectory, blocks in LDS; same control flow, the scans associate differently, so iterates agree
 * to fp64 rounding, not bitwise); the environment variable NOC_PERSIST_WIDE=0 forces the one-wave
 * kernel.  Cart-pole batches of at most half as many trajectories as SIMDs with N <= 320 instead
 * run two or four waves per trajectory, each solving one candidate regularisation of the retry
 * chain ahead of the accept test (speculative retries): the one-wave kernel's results bit for bit
 * (NOC_PERSIST_SPEC=1 forces one wave).  Requires
 * ws->lanes == 64 and a KKT step that fits in LDS (noc_ipm_solve_supported).  A trajectory that
 * reaches max_solves KKT solves stops with phase != NOC_PHASE_DONE.  On return (stream order)
 * u, x, bp, rp, r_inc, cost, hu, it, total_it, kkt_solves and phase hold the final state. */
int noc_ipm_solve_supported(const noc_family* fam, int N, int lanes);
/* Timing-only: per-phase cycle counters of the persistent solver's workgroup 0 (rollout,
 * linearise, costate + blocks, KKT scan, trial, Newton iterations; n up to 16: slots 8..14 split
 * the wide kernel's KKT solve into prepend, in-wave scan, cross-wave join, Riccati, pred
 * reduction, forward scan, propagate); all zero unless the library was built with
 * -DNOC_PERSIST_PROFILE.  reset != 0 zeroes them after reading.  Synchronous. */
int noc_debug_phase_cycles(long long* out, int n, int reset);
/* Timing-only: start / end stamps (s_memrealtime, 100 MHz) of trajectories 0..n-1 of the last
 * one-wave persistent solve, out[2b], out[2b+1] (n <= 16384); zeros unless the library was built
 * with -DNOC_PERSIST_PROFILE.  Synchronous. */
int noc_debug_traj_times(long long* out, int n);
int noc_ipm_solve(const noc_family* fam, const noc_ipm_ws* ws, int mode, int terminal, double bp0,
                  int max_solves, void* stream);

/* ---- building blocks of one Newton step: the reference's API functions as standalone batched
 * kernels (the fused solvers above inline them).  Natural layout, leading batch axis B. ---------
 * compute_derivatives (P:13-28 == S:10-25, D:10-25) of a family at (x (B,N+1,nx), u (B,N,nu)),
 * barrier parameter bp (B): cx (B,N,nx) cu (B,N,nu) cxx (B,N,nx,nx) cuu (B,N,nu,nu)
 * cxu (B,N,nx,nu) fx (B,N,nx,nx) fu (B,N,nx,nu) fxx (B,N,nx,nx,nx) fuu (B,N,nx,nu,nu)
 * fxu (B,N,nx,nx,nu) -- jax.grad / hessian / jacrev shapes. */
int noc_derivatives(const noc_family* fam, int N, int B, const double* x, const double* u,
                    const double* bp, double* cx, double* cu, double* cxx, double* cuu,
                    double* cxu, double* fx, double* fu, double* fxx, double* fuu, double* fxu,
                    void* stream);
/* grad(final_cost)(xN) (B,nx) and hessian(final_cost)(xN) (B,nx,nx; NULL = skip), C:35 / S:66. */
int noc_final_cost_derivs(const noc_family* fam, int B, const double* xN, double* grad,
                          double* hess, void* stream);
/* costates lambda (B,N+1,nx): lambda_N = lamT (B,nx), lambda_k = cx_k + fx_k' lambda_{k+1}.
 * sequential = 1: seq_costates (C:43-54, one recursion per trajectory); 0: par_costates (C:34-40,
 * the affine associative scan).  nx <= 8. */
int noc_costates(int nx, int N, int B, const double* lamT, const double* cx, const double* fx,
                 double* lam, int sequential, void* stream);
/* compute_lqr_params (P:31-42 == S:28-39) with l = lambda[:, 1:]: ru (B,N,nu) = cu + fu' l,
 * Q = cxx + l.fxx, R = cuu + l.fuu, M = cxu + l.fxu.  nx <= 8, nu <= 8. */
int noc_lqr_params(int nx, int nu, int N, int B, const double* lam, const double* cu,
                   const double* cxx, const double* cuu, const double* cxu, const double* fu,
                   const double* fxx, const double* fuu, const double* fxu, double* ru, double* Q,
                   double* R, double* M, void* stream);

/* check_traj_feasibility (noc/par_interior_point_newton.py:45-47) == check_feasibility
 * (noc/seq_interior_point_newton.py:93-95): feasible[b] = all_k constraints(x_k, u_k) <= 0 over
 * k < N, with the family's whole constraint vector (the built-ins' box on u; a registered family's
 * own constraints(x, u), state constraints included).  x (B, N+1, nx), u (B, N, nu), feasible (B)
 * int32 (1 / 0; a NaN entry is infeasible).  One wave64 per trajectory. */
int noc_check_feasibility(const noc_family* fam, int N, int B, const double* x, const double* u,
                          int* feasible, void* stream);

/* The OCP's total_cost(x, u, bp) = final_cost(x_N) + sum_k stage_cost(x_k, u_k, bp)
 * (examples/pendulum_runtime.py:53-56, examples/cartpole_runtime.py:48-51,
 * examples/linear_demo_cuda.py:149-152; a registered family's own traced costs), evaluated where
 * the reference's DDP evaluates it (noc/differential_dynamic_programming.py:108, 123-127).
 * x (B, N+1, nx), u (B, N, nu), bp (B) barrier parameter per trajectory, cost (B).  One wave64
 * per trajectory; an infeasible point's log barrier gives NaN, as jnp.log does. */
int noc_total_cost(const noc_family* fam, int N, int B, const double* x, const double* u,
                   const double* bp, double* cost, void* stream);

/* Interior-point DDP (noc/differential_dynamic_programming.py: interior_point_ddp, D:189-208):
 * the whole barrier schedule of DDP iterations (second-order backward pass with the Vx . fxx
 * terms, nonlinear closed-loop rollout, retry loop) of every trajectory in ONE launch, one wave64
 * per trajectory (stage derivatives lane-parallel, the recursions wave-uniform).  Natural layout: x0 (Bt, nx), u (Bt, N, nu) = initial controls on entry, final
 * controls on return.  work: noc_ddp_work_doubles(nx, nu, N, Bt) doubles (on return it starts
 * with the final states (Bt, N+1, nx)).  iterations[b] = total DDP iterations (the reference's
 * return value), passes[b] = backward passes incl. rejected retries, done[b] = 0 if max_passes
 * stopped the trajectory early.  Families with nx <= 4 (noc_ddp_supported). */
long long noc_ddp_work_doubles(int nx, int nu, int N, int Bt);
int noc_ddp_supported(const noc_family* fam);
int noc_ddp_solve(const noc_family* fam, int N, int Bt, const double* x0, double* u, double* work,
                  int* iterations, int* passes, int* done, double bp0, int max_passes,
                  void* stream);
/* noc_ddp_solve with flags: NOC_DDP_ONE_STAGE = ddp(ocp, controls, initial_state, barrier_param)
 * (noc/differential_dynamic_programming.py:98-186): the DDP iterations at bp0 only, no barrier
 * schedule; iterations[b] = that stage's DDP iterations, work starts with its final states.
 * bp0: any finite value >= 0 (the reference's ddp has no check on it, D:98; 0 = the unconstrained
 * stage); the schedule (flags = 0) runs no stage for bp0 <= 1e-4 (D:194).  NaN, inf and negative
 * values are rejected -- the same rule as the nx > 4 host loop of the Python module. */
#define NOC_DDP_ONE_STAGE 1
int noc_ddp_solve_ex(const noc_family* fam, int N, int Bt, const double* x0, double* u,
                     double* work, int* iterations, int* passes, int* done, double bp0,
                     int max_passes, int flags, void* stream);
/* bwd_pass(final_cost, final_state, d, reg_param) of the DDP module
 * (noc/differential_dynamic_programming.py:28-70): the second-order backward pass (Q-function
 * with the Vx . fxx / fxu / fuu terms) from Vx = grad(final_cost)(x_N) (B, nx), Vxx =
 * hessian(final_cost)(x_N) (B, nx, nx) (noc_final_cost_derivs) over the Derivatives arrays of
 * noc_derivatives (natural layout, B leading); reg = reg_param[b] * ||cu_b||_F added to Quu.
 * Outputs ffgain k (B, N, nu), gain K (B, N, nu, nx), pred (B) = sum dV, feasible (B) int32 =
 * all eigh(Quu) > 0, Hu (B, N, nu) = Qu.  (nx, nu) as noc_kkt_supported; one thread per
 * trajectory (the recursion is nonlinear in V: no scan).  Quu = cuu + fu'Vxx fu + Vx.fuu + reg I
 * is READ AS SYMMETRIC: only its upper triangle is formed (cuu[i][j], fuu[m][i][j] with i <= j)
 * and factorised LDL' (the pivots give the eigh > 0 test).  The reference (D:45-51) solves with
 * the full Quu; the two agree whenever cuu and fuu are symmetric (Hessians) and Vxx is -- Vxx is
 * propagated unsymmetrised as D:55 writes it, so a caller-supplied asymmetric Vxx or cuu / fuu
 * gives k, K that differ from the reference by more than rounding. */
int noc_ddp_bwd_pass(int nx, int nu, int N, int B, const double* Vx, const double* Vxx,
                     const double* reg_param, const double* cx, const double* cu,
                     const double* cxx, const double* cuu, const double* cxu, const double* fx,
                     const double* fu, const double* fxx, const double* fuu, const double* fxu,
                     double* k, double* K, double* pred, int* feasible, double* Hu, void* stream);
/* nonlin_rollout(ocp, gain, ffgain, nominal_states, nominal_controls)
 * (noc/differential_dynamic_programming.py:73-90 == noc/par_interior_point_newton.py:87-104):
 * x_hat_0 = x_0, u_hat_s = u_s + k_s + K_s (x_hat_s - x_s), x_hat_{s+1} = dynamics(x_hat_s,
 * u_hat_s).  K (B, N, nu, nx), k (B, N, nu), x (B, N+1, nx), u (B, N, nu) -> x_new, u_new. */
int noc_nonlin_rollout(const noc_family* fam, int N, int B, const double* K, const double* k,
                       const double* x, const double* u, double* x_new, double* u_new,
                       void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NOC_HIP_H */
