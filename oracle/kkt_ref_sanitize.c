/* ORACLE test driver (test infrastructure only): oracle/kkt_ref.c built with AddressSanitizer and
 * UndefinedBehaviorSanitizer (make -C oracle sanitize).  Random LQ problems of every supported
 * shape and the edge cases (N = 1, one trajectory, an empty batch, an indefinite Quu, the
 * invalid dimensions the entry point must reject), each checked for dynamics consistency
 * dx_{k+1} = A dx_k + B du_k; any out-of-bounds access or undefined behaviour aborts the run. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

int kkt_ref_solve(int nx, int nu, int N, int Bt, int threads, const double* A, const double* B,
                  const double* Q, const double* R, const double* M, const double* r,
                  const double* P, const double* reg, double* dx, double* du, double* pred,
                  int* feasible, double* K, double* d);

static double urand(unsigned* s) {
  *s = *s * 1103515245u + 12345u;
  return ((*s >> 8) & 0xFFFFFF) / (double)0x1000000 - 0.5;
}

/* exact-size heap buffers, so any overrun is an ASan report */
static double* buf(size_t n) { return (double*)malloc((n ? n : 1) * sizeof(double)); }

static int run(int nx, int nu, int N, int Bt, unsigned seed, int indefinite) {
  const size_t sN = (size_t)Bt * N;
  double *A = buf(sN * nx * nx), *B = buf(sN * nx * nu), *Q = buf(sN * nx * nx),
         *R = buf(sN * nu * nu), *M = buf(sN * nx * nu), *r = buf(sN * nu), *P = buf((size_t)Bt * nx * nx),
         *reg = buf(Bt), *dx = buf((size_t)Bt * (N + 1) * nx), *du = buf(sN * nu), *pred = buf(Bt),
         *K = buf(sN * nu * nx), *d = buf(sN * nu);
  int* feas = (int*)malloc((Bt ? Bt : 1) * sizeof(int));
  for (size_t k = 0; k < sN; ++k) {
    for (int i = 0; i < nx; ++i) {
      for (int j = 0; j < nx; ++j) {
        A[k * nx * nx + i * nx + j] = (i == j ? 1.0 : 0.0) + 0.1 * urand(&seed);
        Q[k * nx * nx + i * nx + j] = (i == j ? 1.0 : 0.0);
      }
      for (int j = 0; j < nu; ++j) {
        B[k * nx * nu + i * nu + j] = urand(&seed);
        M[k * nx * nu + i * nu + j] = 0.1 * urand(&seed);
      }
    }
    for (int i = 0; i < nu; ++i) {
      for (int j = 0; j < nu; ++j) R[k * nu * nu + i * nu + j] = (i == j ? 1.0 : 0.0);
      r[k * nu + i] = urand(&seed);
    }
  }
  for (int b = 0; b < Bt; ++b) {
    for (int i = 0; i < nx * nx; ++i) P[(size_t)b * nx * nx + i] = (i % (nx + 1) == 0) ? 2.0 : 0.0;
    reg[b] = 0.01 * b;
  }
  if (indefinite && Bt > 0) R[0] = -50.0;  /* Quu < 0 at stage 0 of trajectory 0 */
  if (kkt_ref_solve(nx, nu, N, Bt, 2, A, B, Q, R, M, r, P, reg, dx, du, pred, feas, K, d) != 0) {
    fprintf(stderr, "rc != 0 for a valid problem (%d %d %d %d)\n", nx, nu, N, Bt);
    return 1;
  }
  int bad = 0;
  for (int b = 0; b < Bt; ++b) {
    if (indefinite && b == 0) {
      if (feas[0] != 0) bad = 1;
      continue;
    }
    for (int k = 0; k < N; ++k) {
      const size_t s = (size_t)b * N + k;
      for (int i = 0; i < nx; ++i) {
        double v = 0.0;
        for (int j = 0; j < nx; ++j) v += A[s * nx * nx + i * nx + j] * dx[((size_t)b * (N + 1) + k) * nx + j];
        for (int j = 0; j < nu; ++j) v += B[s * nx * nu + i * nu + j] * du[s * nu + j];
        if (fabs(v - dx[((size_t)b * (N + 1) + k + 1) * nx + i]) > 1e-9 * (1.0 + fabs(v))) bad = 1;
      }
    }
    if (!feas[b] || !isfinite(pred[b])) bad = 1;
  }
  free(A); free(B); free(Q); free(R); free(M); free(r); free(P); free(reg); free(dx); free(du);
  free(pred); free(K); free(d); free(feas);
  if (bad) fprintf(stderr, "check failed (%d %d %d %d)\n", nx, nu, N, Bt);
  return bad;
}

int main(void) {
  int fails = 0;
  const int shapes[][2] = {{2, 1}, {4, 1}, {8, 4}, {3, 2}};
  const int Ns[] = {1, 2, 7, 64};
  const int Bts[] = {0, 1, 5};
  for (int s = 0; s < 4; ++s)
    for (int n = 0; n < 4; ++n)
      for (int b = 0; b < 3; ++b) fails += run(shapes[s][0], shapes[s][1], Ns[n], Bts[b], 7u * s + n + b, 0);
  fails += run(4, 1, 30, 3, 11u, 1);
  /* invalid dimensions: rejected before any access */
  double z = 0.0;
  int zi = 0;
  if (kkt_ref_solve(9, 1, 5, 1, 1, &z, &z, &z, &z, &z, &z, &z, &z, &z, &z, &z, &zi, &z, &z) == 0) ++fails;
  if (kkt_ref_solve(4, 5, 5, 1, 1, &z, &z, &z, &z, &z, &z, &z, &z, &z, &z, &z, &zi, &z, &z) == 0) ++fails;
  if (kkt_ref_solve(4, 1, 0, 1, 1, &z, &z, &z, &z, &z, &z, &z, &z, &z, &z, &z, &zi, &z, &z) == 0) ++fails;
  if (kkt_ref_solve(4, 1, 5, -1, 1, &z, &z, &z, &z, &z, &z, &z, &z, &z, &z, &z, &zi, &z, &z) == 0) ++fails;
  printf("kkt_ref sanitizer run: %s\n", fails ? "FAILED" : "ok");
  return fails ? 1 : 0;
}
