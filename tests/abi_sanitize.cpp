// Host-side argument validation of the C-ABI (include/noc_hip.h) under AddressSanitizer and
// UndefinedBehaviorSanitizer (test infrastructure: `make -C ip-parallel-optimal-control_amd
// abi-sanitize`, run by tests/test_sanitizers.py; no GPU needed -- every call here is rejected
// before a kernel launch, or fails cleanly at the launch when no device is visible).  Checks that
// each invalid argument returns a negative status with a message, never touches memory it must
// not, and that the queries stay in range.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../include/noc_hip.h"

static int fails = 0;
#define EXPECT(cond)                                                               \
  do {                                                                             \
    if (!(cond)) {                                                                 \
      std::fprintf(stderr, "FAILED %s:%d: %s (%s)\n", __FILE__, __LINE__, #cond,   \
                   noc_last_error());                                              \
      ++fails;                                                                     \
    }                                                                              \
  } while (0)

int main() {
  EXPECT(noc_abi_version() == NOC_ABI_VERSION);
  EXPECT(noc_kkt_supported(4, 1) == 1 && noc_kkt_supported(3, 1) == 0);
  EXPECT(noc_kkt_pick_lanes(4, 1, 200, 4096) > 0);
  EXPECT(noc_kkt_pick_lanes(3, 1, 200, 4096) == -1);
  EXPECT(noc_kkt_pick_lanes(4, 1, 0, 4096) == -1);
  EXPECT(noc_kkt_gains_on_chip(4, 1, 200, 32) == 1);
  EXPECT(noc_kkt_gains_on_chip(4, 1, 200, 7) == 0);
  EXPECT(noc_tiled_doubles(0, 1, 32, 4) == -1 && noc_tiled_doubles(10, 1, 32, 4) > 0);

  std::vector<double> f(1 << 16, 0.0);
  double* p = f.data();
  int fe[8] = {0};
  // noc_kkt_solve: bad shape, bad N, bad B, bad lanes, NULL required block, misaligned pointer,
  // missing K/d workspace where the gains do not fit on chip
  EXPECT(noc_kkt_solve(3, 1, 10, 1, 0, p, p, p, p, p, p, 0, 0, p, 0, 0, 0, 0, p, p, p, fe, p, p, 0, 0, 0) < 0);
  EXPECT(noc_kkt_solve(4, 1, 0, 1, 0, p, p, p, p, p, p, 0, 0, p, 0, 0, 0, 0, p, p, p, fe, p, p, 0, 0, 0) < 0);
  EXPECT(noc_kkt_solve(4, 1, 10, -1, 0, p, p, p, p, p, p, 0, 0, p, 0, 0, 0, 0, p, p, p, fe, p, p, 0, 0, 0) < 0);
  EXPECT(noc_kkt_solve(4, 1, 10, 1, 5, p, p, p, p, p, p, 0, 0, p, 0, 0, 0, 0, p, p, p, fe, p, p, 0, 0, 0) < 0);
  EXPECT(noc_kkt_solve(4, 1, 10, 1, 0, nullptr, p, p, p, p, p, 0, 0, p, 0, 0, 0, 0, p, p, p, fe, p, p, 0, 0, 0) < 0);
  EXPECT(noc_kkt_solve(4, 1, 10, 1, 0, p + 1, p, p, p, p, p, 0, 0, p, 0, 0, 0, 0, p, p, p, fe, p, p, 0, 0, 0) < 0);
  EXPECT(noc_kkt_solve(8, 4, 4000, 1, 64, p, p, p, p, p, p, 0, 0, p, 0, 0, 0, 0, p, p, p, fe, 0, 0, 0, 0, 0) < 0);
  EXPECT(std::strlen(noc_last_error()) > 0);
  // the tiled entry needs explicit lanes; the grouped layout only for (8, 4)
  EXPECT(noc_kkt_solve_tiled(4, 1, 10, 1, 0, p, p, p, p, p, p, 0, 0, p, 0, 0, 0, 0, p, p, p, fe, p, p, 0, 0, 0) < 0);
  EXPECT(noc_kkt_solve_tiled(4, 1, 10, 1, 1, p, p, p, p, p, p, 0, 0, p, 0, 0, 0, 0, p, p, p, fe, p, p, 0, 0, 0) < 0);
  EXPECT(noc_relayout(2, 4, 0, 10, 1, 32, p, p, 0) < 0);
  EXPECT(noc_relayout(0, 4, 3, 10, 1, 32, p, p, 0) < 0);   // E != sym_n (sym_n + 1) / 2
  EXPECT(noc_relayout(0, 4, 0, 10, 1, 12, p, p, 0) < 0);   // lanes
  EXPECT(noc_relayout(0, 4, 0, 10, 1, 32, nullptr, p, 0) < 0);
  EXPECT(noc_par_bwd_pass(4, 1, 10, 1, 3, p, p, p, p, p, p, 0, 0, p, 0, 0, 0, p, p, 0, 0, p, fe, 0) < 0);
  EXPECT(noc_par_fwd_pass(4, 1, 10, 1, 0, p, p, 0, 0, nullptr, p, 0, p, p, 0) < 0);

  // interior-point entry points: NULL workspace / family, bad lanes, unknown flag bits, bad mode
  noc_family fam;
  std::memset(&fam, 0, sizeof(fam));
  fam.kind = NOC_FAMILY_CARTPOLE;
  fam.nx = 4;
  fam.nu = 1;
  fam.dt = 0.005;
  fam.u_bound = 50.0;
  EXPECT(noc_family_supported(&fam) == 1);
  EXPECT(noc_family_supported(nullptr) == 0);
  noc_ipm_ws ws;
  std::memset(&ws, 0, sizeof(ws));
  ws.Bt = 1;
  ws.N = 10;
  ws.lanes = 64;
  EXPECT(noc_ipm_init(nullptr, 0.1, 0) < 0);
  EXPECT(noc_ipm_init(&ws, 0.1, 0) < 0);  // required pointers NULL
  double** fields[] = {&ws.x, &ws.u, &ws.x0, &ws.A, &ws.B, &ws.Q, &ws.R, &ws.M, &ws.r, &ws.P,
                       &ws.cx, &ws.cu, &ws.lc, &ws.lam, &ws.dx, &ws.du, &ws.pred, &ws.K, &ws.d,
                       &ws.bp, &ws.rp, &ws.rinc, &ws.cost, &ws.hu, &ws.gnorm, &ws.reg};
  for (double** fp : fields) *fp = p;
  int ints[8][4] = {{0}};
  ws.feasible = ints[0]; ws.phase = ints[1]; ws.kkt_active = ints[2]; ws.it = ints[3];
  ws.inner = ints[4]; ws.total_it = ints[5]; ws.kkt_solves = ints[6]; ws.repeats = ints[7];
  ws.flags = 8;  // not a defined bit
  EXPECT(noc_ipm_init(&ws, 0.1, 0) < 0);
  ws.flags = 0;
  ws.lanes = 12;
  EXPECT(noc_ipm_init(&ws, 0.1, 0) < 0);
  ws.lanes = 64;
  EXPECT(noc_ipm_step(&fam, &ws, 7, NOC_TERMINAL_STAGE0, 0, 0) < 0);          // mode
  EXPECT(noc_ipm_step(&fam, &ws, NOC_MODE_PAR, 5, 0, 0) < 0);                 // terminal
  EXPECT(noc_ipm_step(&fam, &ws, NOC_MODE_PAR, NOC_TERMINAL_STAGE0, 32, 0) < 0);  // lanes
  EXPECT(noc_ipm_solve(&fam, &ws, NOC_MODE_PAR, NOC_TERMINAL_STAGE0, 0.0, 10, 0) < 0);  // bp0
  EXPECT(noc_ipm_solve(&fam, &ws, NOC_MODE_PAR, NOC_TERMINAL_STAGE0, 0.1, 0, 0) < 0);   // cap
  EXPECT(noc_ipm_solve(nullptr, &ws, NOC_MODE_PAR, NOC_TERMINAL_STAGE0, 0.1, 10, 0) < 0);
  // round-4 building blocks: NULL family / pointers, bad sizes, misaligned, unknown flags; an
  // empty batch is a no-op
  double* ph = p + 1;  // misaligned for doubles
  EXPECT(noc_check_feasibility(nullptr, 10, 1, p, p, fe, 0) < 0);
  EXPECT(noc_check_feasibility(&fam, 0, 1, p, p, fe, 0) < 0);
  EXPECT(noc_check_feasibility(&fam, 10, 1, p, nullptr, fe, 0) < 0);
  EXPECT(noc_check_feasibility(&fam, 10, 0, p, p, fe, 0) == 0);
  EXPECT(noc_total_cost(nullptr, 10, 1, p, p, p, p, 0) < 0);
  EXPECT(noc_total_cost(&fam, 10, -1, p, p, p, p, 0) < 0);
  EXPECT(noc_total_cost(&fam, 10, 1, p, p, nullptr, p, 0) < 0);
  EXPECT(noc_total_cost(&fam, 10, 1, p, p, p, ph, 0) < 0);
  EXPECT(noc_total_cost(&fam, 10, 0, p, p, p, p, 0) == 0);
  EXPECT(noc_nonlin_rollout(&fam, 10, 1, p, p, p, nullptr, p, p, 0) < 0);
  EXPECT(noc_nonlin_rollout(&fam, 0, 1, p, p, p, p, p, p, 0) < 0);
  EXPECT(noc_ddp_bwd_pass(3, 1, 10, 1, p, p, p, p, p, p, p, p, p, p, p, p, p, p, p, p, fe, p, 0) < 0);
  EXPECT(noc_ddp_bwd_pass(4, 1, 10, 1, p, p, p, p, nullptr, p, p, p, p, p, p, p, p, p, p, p, fe, p, 0) < 0);
  EXPECT(noc_ddp_solve_ex(&fam, 10, 1, p, p, p, fe, fe, fe, 0.1, 10, 2, 0) < 0);  // flag bit
  EXPECT(noc_ddp_solve_ex(&fam, 10, 1, p, p, p, fe, fe, fe, -1.0, 10, 1, 0) < 0);  // bp0 < 0
  EXPECT(noc_ddp_solve_ex(&fam, 10, 1, p, p, p, fe, fe, fe, NAN, 10, 1, 0) < 0);  // bp0 NaN
  fam.nx = 3;
  EXPECT(noc_total_cost(&fam, 10, 1, p, p, p, p, 0) < 0);  // family
  EXPECT(noc_ipm_prepare(&fam, &ws, NOC_MODE_PAR, NOC_TERMINAL_STAGE0, 0) < 0);  // family
  EXPECT(noc_ddp_work_doubles(0, 1, 10, 1) == -1 && noc_ddp_work_doubles(4, 1, 10, 2) > 0);
  EXPECT(noc_debug_phase_cycles(nullptr, 4, 0) < 0);
  std::printf("abi sanitizer run: %s\n", fails ? "FAILED" : "ok");
  return fails ? 1 : 0;
}
