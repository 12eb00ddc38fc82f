// tools/fetch_calib.hip — calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on
// gfx950 for the access widths the executor kernels use (measurement only).
// Reads a 1 GiB buffer (well past the 256 MiB Infinity Cache) once with
// 4 B per lane (global_load_dword, the batched executor's plane reads) and
// once with 16 B per lane (the width the microarch guide calibrates), and
// writes 256 MiB with 4 B per lane; each kernel is its own dispatch, so the
// per-dispatch counters divide by the known byte counts.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/build/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__global__ void k_read4(const uint32_t* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if (acc == 0x9E3779B9u) out[0] = acc;  // keeps the loads live
}
__global__ void k_read16(const uint4* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) out[0] = acc;
}
__global__ void k_write4(uint32_t* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)i;
}

int main() {
  const size_t bytes = 1ull << 30, wbytes = 1ull << 28;
  uint32_t *buf = nullptr, *out = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  if (hipMemset(buf, 1, bytes) != hipSuccess) return 1;
  const dim3 grid(256 * 8), block(256);
  hipLaunchKernelGGL(k_read4, grid, block, 0, 0, buf, bytes / 4, out);
  hipLaunchKernelGGL(k_read16, grid, block, 0, 0, (const uint4*)buf, bytes / 16, out);
  hipLaunchKernelGGL(k_write4, grid, block, 0, 0, buf, wbytes / 4);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("k_read4 %zu B, k_read16 %zu B, k_write4 %zu B\n", bytes, bytes, wbytes);
  hipFree(buf);
  hipFree(out);
  return 0;
}
