// Microbenchmark: fp64 MFMA shapes on one MI355X: v_mfma_f64_16x16x4_f64 (one 16x16 block, 2048 flops) against
// v_mfma_f64_4x4x4_f64 (four 4x4 blocks, 512 flops), independent accumulators, 4 / 8 / 16 waves per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dbl4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void mfma16(double* out, int iters) {
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

template <int NACC>
__global__ void mfma4(double* out, int iters) {
  double acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = 0.0;
  double a = threadIdx.x * 1e-3, b = 1.0 + blockIdx.x * 1e-6;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static void run(const char* name, K kern, int nacc, double flops_per_inst, double* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 20000, blocks = 256;
  for (int wpb : {4, 8, 16}) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * wpb), 0, 0, out, 100);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * wpb), 0, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double insts = (double)iters * nacc * blocks * wpb;  // per wave
    printf("%-22s %2d waves/CU  %6.2f TFLOP/s  %5.1f cycles/inst/SIMD at 2.4 GHz\n", name, wpb,
           flops_per_inst * insts / ms / 1e9, (ms * 1e-3 * 2.4e9) / ((double)iters * nacc * wpb / 4));
  }
}

int main() {
  double* out;
  hipMalloc(&out, 1 << 26);
  run("f64 16x16x4 (2048)", mfma16<4>, 4, 2.0 * 16 * 16 * 4, out);
  run("f64 4x4x4 4-block (512)", mfma4<8>, 8, 2.0 * 4 * 4 * 4 * 4, out);
  run("f64 4x4x4 4-block x16", mfma4<16>, 16, 2.0 * 4 * 4 * 4 * 4, out);
  return 0;
}
