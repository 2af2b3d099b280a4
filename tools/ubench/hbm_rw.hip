// HBM stream rates on one MI355X (dev microbenchmark): write-only, read-only and copy of large buffers with 16-byte
// accesses from a grid-stride loop, the K1 panel's store shape (every lane a 16-byte store, whole 128-byte lines per
// 8 lanes).  The write-only rate is K1's ceiling: K1 writes 22.3 KB per Spot sample and reads 0.57 KB.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench/hbm_rw tools/ubench/hbm_rw.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void __launch_bounds__(256) k_write(double2* __restrict__ p, size_t n, double v) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    p[i] = make_double2(v, v + 1.0);
}

__global__ void __launch_bounds__(256) k_read(const double2* __restrict__ p, size_t n, double* __restrict__ out) {
  double a = 0.0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const double2 x = p[i];
    a += x.x + x.y;
  }
  if (a == 12345.678) out[0] = a;  // keeps the loads
}

__global__ void __launch_bounds__(256) k_copy(const double2* __restrict__ s, double2* __restrict__ d, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) d[i] = s[i];
}

int main(int argc, char** argv) {
  const size_t mb = argc > 1 ? std::atoll(argv[1]) : 2048;
  const size_t bytes = mb << 20, n = bytes / 16;
  double2 *a = nullptr, *b = nullptr;
  double* o = nullptr;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess || hipMalloc(&o, 8) != hipSuccess) {
    std::printf("alloc failed\n");
    return 1;
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int grid : {1024, 2048, 4096, 8192}) {
    float best[3] = {1e9f, 1e9f, 1e9f};
    for (int it = 0; it < 12; ++it) {
      for (int k = 0; k < 3; ++k) {
        (void)hipEventRecord(e0);
        if (k == 0) hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, a, n, (double)it);
        if (k == 1) hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a, n, o);
        if (k == 2) hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, a, b, n);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (it >= 2 && ms < best[k]) best[k] = ms;
      }
    }
    std::printf("%zu MB grid %5d: write %.0f GB/s  read %.0f GB/s  copy %.0f GB/s (read+write bytes)\n", mb, grid,
                bytes / (best[0] * 1e-3) / 1e9, bytes / (best[1] * 1e-3) / 1e9, 2.0 * bytes / (best[2] * 1e-3) / 1e9);
  }
  return 0;
}
