// FETCH_SIZE / WRITE_SIZE calibration for the access widths of the KKT scan (the microarch guide
// calibrates only 16-B-per-lane streaming reads / writes; others must be calibrated on a known
// byte count).  Each kernel moves exactly BYTES bytes with one access pattern; rocprofv3 --pmc
// FETCH_SIZE (one pass) and WRITE_SIZE (another) per dispatch give the counter-to-bytes factor.
//   read16   : global_load_dwordx4, lane-contiguous (the scan's even-E fields, tload)
//   read8    : global_load_dwordx2, lane-contiguous 512 B per wave-instruction
//   read8_l32: the scan's odd-E tiled fields at L = 32: per wave-instruction two 256 B pieces
//   write16 / write8 : the same for stores
// Build: hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o tools/pmc_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr size_t BYTES = 512ull << 20;  // 512 MiB: far beyond L2, about the memory-side cache

__global__ void read16(const double2* __restrict__ src, double* out, size_t n2) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
    const double2 v = src[i];
    s += v.x + v.y;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void read8(const double* __restrict__ src, double* out, size_t n) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    s += src[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// lanes 0-31 and 32-63 of a wave read two separate 256 B pieces (L = 32 segments of different
// trajectories in the tiled layout): piece of segment g at wave w, step t = 
// base + ((t * nwaves + w) * 2 + g) * 32 + lane%32 -- every byte read once
__global__ void read8_l32(const double* __restrict__ src, double* out, size_t n) {
  const size_t nw = (size_t)gridDim.x * blockDim.x / 64;
  const size_t w = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) / 64;
  const int lane = threadIdx.x & 63, g = lane >> 5, l = lane & 31;
  double s = 0.0;
  for (size_t t = 0;; ++t) {
    const size_t i = (((t * nw + w) * 2 + g) * 32) + l;
    if (i >= n) break;
    s += src[i];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void write16(double2* __restrict__ dst, size_t n2) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = make_double2((double)i, 1.0);
}
__global__ void write8(double* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = (double)i;
}

int main() {
  double *buf, *out;
  CHECK(hipMalloc(&buf, BYTES));
  CHECK(hipMalloc(&out, 1 << 24));
  CHECK(hipMemset(buf, 0, BYTES));
  const size_t n = BYTES / 8;
  const dim3 grid(2048), block(256);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(read16, grid, block, 0, 0, (const double2*)buf, out, n / 2);
    hipLaunchKernelGGL(read8, grid, block, 0, 0, buf, out, n);
    hipLaunchKernelGGL(read8_l32, grid, block, 0, 0, buf, out, n);
    hipLaunchKernelGGL(write16, grid, block, 0, 0, (double2*)buf, n / 2);
    hipLaunchKernelGGL(write8, grid, block, 0, 0, buf, n);
  }
  CHECK(hipDeviceSynchronize());
  printf("{\"bytes_per_kernel\": %zu}\n", BYTES);
  return 0;
}
