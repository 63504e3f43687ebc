// Memory-side cache probe for the KKT scan's re-read pattern (tools only; not on the product path).
//
// Each lane streams its chunk of S stages (E doubles per stage, tiled like the scan's layout:
// one wave-wide 16-byte-per-lane load per granule), then streams the same chunk again either in
// the SAME order (what phases 1 and 3 of the scan do) or REVERSED.  With LRU-like replacement and a
// re-read distance close to the cache size, the reversed order should hit for its first part.
// Occupancy is pinned to 8 waves/CU (2 per SIMD) with 20 KB of LDS per one-wave block, like c3.
// Build: hipcc -O3 --offload-arch=gfx950 tools/reread_probe.hip -o tools/reread_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int E2 = 18;  // double2 granules per stage (36 doubles = one cart-pole stage, 288 B)
constexpr int S = 7;    // stages per lane (N = 200 over 32 lanes: 6-7)

template <int MODE>  // 0: one pass, 1: two passes same order, 2: second pass reversed
__global__ __launch_bounds__(64) void probe(const double2* __restrict__ x, double* out, int waves) {
  extern __shared__ double lds[];
  const int w = blockIdx.x, l = threadIdx.x;
  if (w >= waves) return;
  const double2* base = x + (size_t)w * S * E2 * 64 + l;
  double acc = 0.0;
  for (int s = S - 1; s >= 0; --s)
    for (int e = 0; e < E2; ++e) {
      const double2 v = base[((size_t)s * E2 + e) * 64];
      acc = acc * 0.5 + v.x + v.y;
    }
  if (MODE == 1) {
    for (int s = S - 1; s >= 0; --s)
      for (int e = 0; e < E2; ++e) {
        const double2 v = base[((size_t)s * E2 + e) * 64];
        acc = acc * 0.25 + v.x - v.y;
      }
  } else if (MODE == 2) {
    for (int s = 0; s < S; ++s)
      for (int e = 0; e < E2; ++e) {
        const double2 v = base[((size_t)s * E2 + e) * 64];
        acc = acc * 0.25 + v.x - v.y;
      }
  }
  lds[l] = acc;
  __syncthreads();
  out[(size_t)w * 64 + l] = lds[(l + 1) & 63];
}

int main(int argc, char** argv) {
  const int waves = argc > 1 ? atoi(argv[1]) : 2048;
  const size_t n2 = (size_t)waves * S * E2 * 64;
  double2* x;
  double* out;
  if (hipMalloc(&x, n2 * sizeof(double2)) != hipSuccess || hipMalloc(&out, (size_t)waves * 64 * 8) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  hipMemset(x, 0, n2 * sizeof(double2));
  const size_t lds = 20 * 1024;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[3] = {"one_pass", "two_pass_same_order", "two_pass_reversed"};
  for (int round = 0; round < 2; ++round) {
    for (int mode = 0; mode < 3; ++mode) {
      auto launch = [&]() {
        if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(waves), dim3(64), lds, 0, x, out, waves);
        if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(waves), dim3(64), lds, 0, x, out, waves);
        if (mode == 2) hipLaunchKernelGGL(probe<2>, dim3(waves), dim3(64), lds, 0, x, out, waves);
      };
      for (int i = 0; i < 3; ++i) launch();
      hipEventRecord(a, 0);
      const int reps = 20;
      for (int i = 0; i < reps; ++i) launch();
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms = 0.f;
      hipEventElapsedTime(&ms, a, b);
      const double us = 1e3 * ms / reps;
      const double mb = n2 * 16.0 / 1e6;
      printf("{\"mode\": \"%s\", \"waves\": %d, \"chunk_MB\": %.1f, \"us\": %.2f, \"GBs_per_pass\": %.0f}\n",
             names[mode], waves, mb, us, mb * 1e-3 / (us * 1e-6) * (mode ? 2 : 1));
    }
  }
  hipFree(x);
  hipFree(out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
