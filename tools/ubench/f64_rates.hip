// Microbenchmark: fp64 MFMA (v_mfma_f64_16x16x4_f64) and fp64 VALU FMA throughput on one MI355X.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dbl4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void mfma_loop(double* out, int iters) {
  dbl4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = dbl4{0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = 1.0 + blockIdx.x * 1e-6;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void fma_loop(double* out, int iters) {
  double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  const double a = 0.999999, b = 1e-7;
  for (int it = 0; it < iters; ++it) {
    x0 = fma(x0, a, b); x1 = fma(x1, a, b); x2 = fma(x2, a, b); x3 = fma(x3, a, b);
    x4 = fma(x4, a, b); x5 = fma(x5, a, b); x6 = fma(x6, a, b); x7 = fma(x7, a, b);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

int main() {
  double* out;
  hipMalloc(&out, 1 << 26);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 20000;
  for (int wpb : {4, 8, 16}) {
    const int blocks = 256 * 1;
    hipLaunchKernelGGL(mfma_loop<4>, dim3(blocks), dim3(64 * wpb), 0, 0, out, 100);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_loop<4>, dim3(blocks), dim3(64 * wpb), 0, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double flops = 2.0 * 16 * 16 * 4 * 4 * (double)iters * blocks * wpb;
    printf("MFMA f64 16x16x4: %2d waves/CU  %.2f TFLOP/s  (%.1f cycles/MFMA/SIMD at 2.4GHz)\n", wpb, flops / ms / 1e9,
           (ms * 1e-3 * 2.4e9) / ((double)iters * 4 * wpb / 4));
  }
  for (int wpb : {4, 8, 16}) {
    const int blocks = 256;
    hipLaunchKernelGGL(fma_loop, dim3(blocks), dim3(64 * wpb), 0, 0, out, 100);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(fma_loop, dim3(blocks), dim3(64 * wpb), 0, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double flops = 2.0 * 8 * (double)iters * blocks * wpb * 64;
    printf("VALU f64 FMA:     %2d waves/CU  %.2f TFLOP/s\n", wpb, flops / ms / 1e9);
  }
  return 0;
}
