// Natural <-> tiled (lane-interleaved) relayout of per-stage block fields (include/noc_hip.h).
#include <hip/hip_runtime.h>

#include "noc_internal.h"
#include "small_linalg.h"

namespace noc {

// packed upper-triangle index e of an n x n symmetric matrix -> (i, k), i <= k
NOC_DEV void unpack_sym(int n, int e, int& i, int& k) {
  i = 0;
  while (e >= n - i) { e -= n - i; ++i; }
  k = i + e;
}

__global__ __launch_bounds__(256) void relayout_kernel(int dir, int E, int sym_n, int N, int Bt, int L,
                                                       const double* __restrict__ src,
                                                       double* __restrict__ dst) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)Bt * N * E;
  if (t >= total) return;
  const int b = (int)(t / ((long long)N * E));
  const int rest = (int)(t % ((long long)N * E));
  const int s = rest / E, e = rest % E;
  const Chunks ch(N, L);
  int l, j;
  ch.owner(s, l, j);
  const size_t ti = tile_index(E, L, ch.cmax, b, j, l, e);
  if (sym_n > 0) {
    int i, k;
    unpack_sym(sym_n, e, i, k);
    const size_t nat = ((size_t)b * N + s) * sym_n * sym_n;
    if (dir == 0) {
      dst[ti] = (i == k) ? src[nat + i * sym_n + i] : 0.5 * (src[nat + i * sym_n + k] + src[nat + k * sym_n + i]);
    } else {
      const double v = src[ti];
      dst[nat + i * sym_n + k] = v;
      dst[nat + k * sym_n + i] = v;
    }
  } else {
    const size_t nat = ((size_t)b * N + s) * E + e;
    if (dir == 0) dst[ti] = src[nat];
    else dst[nat] = src[ti];
  }
}

hipError_t relayout(int direction, int E, int sym_n, int N, int Bt, int L, const double* src,
                    double* dst, hipStream_t s) {
  const long long total = (long long)Bt * N * E;
  if (total == 0) return hipSuccess;
  const unsigned grid = (unsigned)((total + 255) / 256);
  hipLaunchKernelGGL(relayout_kernel, dim3(grid), dim3(256), 0, s, direction, E, sym_n, N, Bt, L,
                     src, dst);
  return hipGetLastError();
}

}  // namespace noc
