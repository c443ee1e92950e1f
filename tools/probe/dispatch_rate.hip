// Workgroup dispatch-rate probe: how long do N short workgroups take, empty and with an 8 KB store each
// (the output tile of a 64x64 bf16 conv tile)?  Decides whether the 1x1 conv layers (16k+ tiny tiles per
// launch) are bound by workgroup turnover rather than by memory.
//   hipcc --offload-arch=gfx950 -O3 dispatch_rate.hip -o dispatch_rate && ./dispatch_rate
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) p[0] = 1;
}

__global__ void store_kernel(uint4* __restrict__ y) {   // 256 threads x 2 x 16 B = 8 KB per workgroup
  const size_t base = (size_t)blockIdx.x * 512;
  y[base + threadIdx.x] = make_uint4(threadIdx.x, 1, 2, 3);
  y[base + 256 + threadIdx.x] = make_uint4(threadIdx.x, 4, 5, 6);
}

__global__ void __launch_bounds__(256) store_loop_kernel(uint4* __restrict__ y, int tiles) {   // persistent
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const size_t base = (size_t)t * 512;
    y[base + threadIdx.x] = make_uint4(threadIdx.x, 1, 2, 3);
    y[base + 256 + threadIdx.x] = make_uint4(threadIdx.x, 4, 5, 6);
  }
}

int main() {
  uint4* y;
  const int maxN = 65536;
  if (hipMalloc(&y, (size_t)maxN * 8192) != hipSuccess) return 1;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int threads : {64, 256}) {
    for (int n : {4096, 16384, 65536}) {
      hipLaunchKernelGGL(empty_kernel, dim3(n), dim3(threads), 0, 0, nullptr);
      hipEventRecord(a);
      for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(empty_kernel, dim3(n), dim3(threads), 0, 0, nullptr);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      printf("empty   %6d WGs x %3d threads: %8.2f us/launch  (%.1f ns per WG)\n", n, threads, ms * 1e3 / 20,
             ms * 1e6 / 20 / n);
    }
  }
  for (int n : {4096, 16384, 65536}) {
    hipLaunchKernelGGL(store_kernel, dim3(n), dim3(256), 0, 0, y);
    hipEventRecord(a);
    for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(store_kernel, dim3(n), dim3(256), 0, 0, y);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("store8k %6d WGs: %8.2f us/launch  %.2f TB/s\n", n, ms * 1e3 / 20, (double)n * 8192 / (ms / 20 * 1e-3) / 1e12);
    for (int grid : {1024, 2048, 4096}) {
      hipLaunchKernelGGL(store_loop_kernel, dim3(grid), dim3(256), 0, 0, y, n);
      hipEventRecord(a);
      for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(store_loop_kernel, dim3(grid), dim3(256), 0, 0, y, n);
      hipEventRecord(b);
      hipEventSynchronize(b);
      hipEventElapsedTime(&ms, a, b);
      printf("  persistent grid %4d over %6d tiles: %8.2f us/launch  %.2f TB/s\n", grid, n, ms * 1e3 / 20,
             (double)n * 8192 / (ms / 20 * 1e-3) / 1e12);
    }
  }
  hipFree(y);
  return 0;
}
