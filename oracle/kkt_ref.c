/* ORACLE (test infrastructure / CPU baseline only) -- plain-C restatement of the reference's
 * sequential KKT solve, noc/seq_interior_point_newton.py:42-90 (bwd_pass + fwd_pass), batched
 * over trajectories with OpenMP.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  Parity unpinned (see oracle/noc_oracle.py header).
 *
 * Per trajectory (layouts as include/noc_hip.h, q = c = p = 0, x0 = 0 as in the Newton step):
 *   Vxx = P, Vx = 0;  for k = N-1..0:                                         (S:45-74)
 *     Qxx = Q + A'Vxx A ; Quu = R + B'Vxx B + reg I ; Qxu = M + A'Vxx B
 *     Qu = r + B'Vx ; Qx = A'Vx ; feasible &= Quu > 0 (Cholesky; eigh > 0 in S:52-53)
 *     k = -Quu^-1 Qu ; K = -Quu^-1 Qxu' ; Vx = Qx + Qxu k ; Vxx = Qxx + Qxu K
 *     pred += k'Qu + 1/2 k'Quu k
 *   dx_0 = 0 ; du_k = K dx_k + k ; dx_{k+1} = A dx_k + B du_k                    (S:78-90)
 * Build: make -C oracle   (gcc -O3 -march=x86-64-v3 -fopenmp -shared; portable to the GPU box host)
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MAXN 8

/* Cholesky of the nu x nu matrix W (in place, lower); returns 1 iff positive definite. */
static int chol(int n, double* W) {
  for (int j = 0; j < n; ++j) {
    double s = W[j * n + j];
    for (int t = 0; t < j; ++t) s -= W[j * n + t] * W[j * n + t];
    if (!(s > 0.0)) return 0;
    const double l = sqrt(s);
    W[j * n + j] = l;
    for (int i = j + 1; i < n; ++i) {
      double v = W[i * n + j];
      for (int t = 0; t < j; ++t) v -= W[i * n + t] * W[j * n + t];
      W[i * n + j] = v / l;
    }
  }
  return 1;
}

/* General solve W X = Y (Gaussian elimination with partial pivoting), nrhs columns. */
static void gsolve(int n, const double* Win, double* Y, int nrhs) {
  double W[MAXN * MAXN];
  memcpy(W, Win, sizeof(double) * n * n);
  for (int k = 0; k < n; ++k) {
    int p = k;
    for (int i = k + 1; i < n; ++i)
      if (fabs(W[i * n + k]) > fabs(W[p * n + k])) p = i;
    if (p != k) {
      for (int j = 0; j < n; ++j) { double t = W[k * n + j]; W[k * n + j] = W[p * n + j]; W[p * n + j] = t; }
      for (int j = 0; j < nrhs; ++j) { double t = Y[k * nrhs + j]; Y[k * nrhs + j] = Y[p * nrhs + j]; Y[p * nrhs + j] = t; }
    }
    for (int i = k + 1; i < n; ++i) {
      const double l = W[i * n + k] / W[k * n + k];
      for (int j = k; j < n; ++j) W[i * n + j] -= l * W[k * n + j];
      for (int j = 0; j < nrhs; ++j) Y[i * nrhs + j] -= l * Y[k * nrhs + j];
    }
  }
  for (int k = n - 1; k >= 0; --k)
    for (int j = 0; j < nrhs; ++j) {
      double s = Y[k * nrhs + j];
      for (int t = k + 1; t < n; ++t) s -= W[k * n + t] * Y[t * nrhs + j];
      Y[k * nrhs + j] = s / W[k * n + k];
    }
}

static void solve_one(int nx, int nu, int N, const double* A, const double* B, const double* Q,
                      const double* R, const double* M, const double* r, const double* P,
                      double reg, double* dx, double* du, double* pred, int* feasible, double* K,
                      double* d) {
  double Vxx[MAXN * MAXN], Vx[MAXN];
  memcpy(Vxx, P, sizeof(double) * nx * nx);
  memset(Vx, 0, sizeof(Vx));
  double pr = 0.0;
  int feas = 1;
  for (int k = N - 1; k >= 0; --k) {
    const double* Ak = A + (size_t)k * nx * nx;
    const double* Bk = B + (size_t)k * nx * nu;
    const double* Qk = Q + (size_t)k * nx * nx;
    const double* Rk = R + (size_t)k * nu * nu;
    const double* Mk = M + (size_t)k * nx * nu;
    const double* rk = r + (size_t)k * nu;
    double VA[MAXN * MAXN], VB[MAXN * 4], Qxx[MAXN * MAXN], Quu[16], Qxu[MAXN * 4], Qu[4], Qx[MAXN];
    for (int i = 0; i < nx; ++i) {
      for (int j = 0; j < nx; ++j) { double s = 0; for (int t = 0; t < nx; ++t) s += Vxx[i * nx + t] * Ak[t * nx + j]; VA[i * nx + j] = s; }
      for (int j = 0; j < nu; ++j) { double s = 0; for (int t = 0; t < nx; ++t) s += Vxx[i * nx + t] * Bk[t * nu + j]; VB[i * nu + j] = s; }
    }
    for (int i = 0; i < nx; ++i) {
      for (int j = 0; j < nx; ++j) { double s = Qk[i * nx + j]; for (int t = 0; t < nx; ++t) s += Ak[t * nx + i] * VA[t * nx + j]; Qxx[i * nx + j] = s; }
      for (int j = 0; j < nu; ++j) { double s = Mk[i * nu + j]; for (int t = 0; t < nx; ++t) s += Ak[t * nx + i] * VB[t * nu + j]; Qxu[i * nu + j] = s; }
      double s = 0; for (int t = 0; t < nx; ++t) s += Ak[t * nx + i] * Vx[t]; Qx[i] = s;
    }
    for (int i = 0; i < nu; ++i) {
      for (int j = 0; j < nu; ++j) { double s = Rk[i * nu + j] + (i == j ? reg : 0.0); for (int t = 0; t < nx; ++t) s += Bk[t * nu + i] * VB[t * nu + j]; Quu[i * nu + j] = s; }
      double s = rk[i]; for (int t = 0; t < nx; ++t) s += Bk[t * nu + i] * Vx[t]; Qu[i] = s;
    }
    double Wc[16];
    memcpy(Wc, Quu, sizeof(double) * nu * nu);
    feas &= chol(nu, Wc);
    /* Y = [Qu | Qxu'] -> Quu^-1 Y */
    const int nr = nx + 1;
    double Y[4 * (MAXN + 1)];
    for (int i = 0; i < nu; ++i) { Y[i * nr] = Qu[i]; for (int j = 0; j < nx; ++j) Y[i * nr + 1 + j] = Qxu[j * nu + i]; }
    gsolve(nu, Quu, Y, nr);
    double kk[4], KK[4 * MAXN];
    for (int i = 0; i < nu; ++i) { kk[i] = -Y[i * nr]; for (int j = 0; j < nx; ++j) KK[i * nx + j] = -Y[i * nr + 1 + j]; }
    for (int i = 0; i < nx; ++i) {
      double s = Qx[i]; for (int t = 0; t < nu; ++t) s += Qxu[i * nu + t] * kk[t]; Vx[i] = s;
      for (int j = 0; j < nx; ++j) { double v = Qxx[i * nx + j]; for (int t = 0; t < nu; ++t) v += Qxu[i * nu + t] * KK[t * nx + j]; Vxx[i * nx + j] = v; }
    }
    for (int i = 0; i < nu; ++i) {
      double qk = 0; for (int j = 0; j < nu; ++j) qk += Quu[i * nu + j] * kk[j];
      pr += kk[i] * Qu[i] + 0.5 * kk[i] * qk;
    }
    memcpy(K + (size_t)k * nu * nx, KK, sizeof(double) * nu * nx);
    memcpy(d + (size_t)k * nu, kk, sizeof(double) * nu);
  }
  /* forward pass */
  double x[MAXN];
  memset(x, 0, sizeof(x));
  memcpy(dx, x, sizeof(double) * nx);
  for (int k = 0; k < N; ++k) {
    const double* Ak = A + (size_t)k * nx * nx;
    const double* Bk = B + (size_t)k * nx * nu;
    const double* KK = K + (size_t)k * nu * nx;
    double u[4], xn[MAXN];
    for (int i = 0; i < nu; ++i) { double s = d[(size_t)k * nu + i]; for (int j = 0; j < nx; ++j) s += KK[i * nx + j] * x[j]; u[i] = s; }
    for (int i = 0; i < nx; ++i) { double s = 0; for (int j = 0; j < nx; ++j) s += Ak[i * nx + j] * x[j]; for (int j = 0; j < nu; ++j) s += Bk[i * nu + j] * u[j]; xn[i] = s; }
    memcpy(du + (size_t)k * nu, u, sizeof(double) * nu);
    memcpy(x, xn, sizeof(double) * nx);
    memcpy(dx + (size_t)(k + 1) * nx, x, sizeof(double) * nx);
  }
  *pred = pr;
  *feasible = feas;
}

int kkt_ref_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* Batched entry: arrays as include/noc_hip.h, host memory; threads <= 0 = OpenMP default. */
int kkt_ref_solve(int nx, int nu, int N, int Bt, int threads, const double* A, const double* B,
                  const double* Q, const double* R, const double* M, const double* r,
                  const double* P, const double* reg, double* dx, double* du, double* pred,
                  int* feasible, double* K, double* d) {
  if (nx < 1 || nx > MAXN || nu < 1 || nu > 4 || N < 1 || Bt < 0) return -1;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(static)
#endif
  for (int b = 0; b < Bt; ++b) {
    const size_t sN = (size_t)b * N;
    solve_one(nx, nu, N, A + sN * nx * nx, B + sN * nx * nu, Q + sN * nx * nx, R + sN * nu * nu,
              M + sN * nx * nu, r + sN * nu, P + (size_t)b * nx * nx, reg ? reg[b] : 0.0,
              dx + (size_t)b * (N + 1) * nx, du + sN * nu, pred + b, feasible + b,
              K + sN * nu * nx, d + sN * nu);
  }
  return 0;
}
