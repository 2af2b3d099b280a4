// Microbenchmark: how fast can v_mfma_f64_16x16x4_f64 run when its operands come from LDS the way K2 feeds them?
//   (a) registers only (the f64_rates baseline, 8 accumulators per wave)
//   (b) 8 ds_read_b64 fragments per k-step, 8 MFMAs (two 2x2 super-tiles), single register set
//   (c) (b) with the next k-step's fragments read while the MFMAs issue (two register sets)
//   (d) (c) plus a workgroup barrier every 8 k-steps (K2's per-chunk barrier, without staging)
// and which SIMD each wave of an 8-wave workgroup lands on (HW_REG_HW_ID simd_id).
// Build: hipcc --offload-arch=gfx950 -O3 -o k2_feed k2_feed.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dbl4 __attribute__((ext_vector_type(4)));

constexpr int STRIDE = 176;
constexpr int KC = 32;

template <int MODE>
__global__ void __launch_bounds__(512, 2) feed(double* out, int iters, int* simd) {
  __shared__ double lds[KC * STRIDE];
  for (int x = threadIdx.x; x < KC * STRIDE; x += 512) lds[x] = 1e-3 * (x & 255);
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0 && blockIdx.x == 0) simd[wave] = (__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11)) >> 4) & 3;
  int foff[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) foff[u] = (lane >> 4) * STRIDE + 16 * ((wave + 3 * u) % 10) + (lane & 15);
  dbl4 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = dbl4{0, 0, 0, 0};
  constexpr int AB[8][2] = {{0, 2}, {0, 3}, {1, 2}, {1, 3}, {4, 6}, {4, 7}, {5, 6}, {5, 7}};
  double a = lane * 1e-3, b = 1.0;
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int kk = 0; kk < KC; kk += 4)
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[t], 0, 0, 0);
    } else if constexpr (MODE == 1) {
#pragma unroll
      for (int kk = 0; kk < KC; kk += 4) {
        double x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = lds[foff[u] + kk * STRIDE];
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(x[AB[t][0]], x[AB[t][1]], acc[t], 0, 0, 0);
      }
    } else {
      double x[2][8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[0][u] = lds[foff[u]];
#pragma unroll
      for (int kk = 0; kk < KC; kk += 4) {
        const int bb = (kk >> 2) & 1;
        if (kk + 4 < KC) {
#pragma unroll
          for (int u = 0; u < 8; ++u) x[bb ^ 1][u] = lds[foff[u] + (kk + 4) * STRIDE];
        }
#pragma unroll
        for (int t = 0; t < 8; ++t)
          acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(x[bb][AB[t][0]], x[bb][AB[t][1]], acc[t], 0, 0, 0);
      }
      if constexpr (MODE == 3) __syncthreads();
    }
  }
  double s = 0;
#pragma unroll
  for (int t = 0; t < 8; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
void run(const char* name, double* out, int* simd) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256, iters = 400;
  hipLaunchKernelGGL(feed<MODE>, dim3(blocks), dim3(512), 0, 0, out, 10, simd);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  hipLaunchKernelGGL(feed<MODE>, dim3(blocks), dim3(512), 0, 0, out, iters, simd);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double mfma = (double)iters * (KC / 4) * 8 * 8 * blocks;  // per launch
  printf("%-34s %.3f ms  %.2f TFLOP/s  %.1f cycles/MFMA/SIMD at 2.4 GHz\n", name, ms, mfma * 2048 / ms / 1e9,
         ms * 1e-3 * 2.4e9 / (mfma / (blocks * 4)));
}

int main() {
  double* out;
  int* simd;
  hipMalloc(&out, 1 << 24);
  hipMallocManaged(&simd, 64);
  run<0>("(a) registers only", out, simd);
  run<1>("(b) LDS fragments, one set", out, simd);
  run<2>("(c) LDS fragments, two sets", out, simd);
  run<3>("(d) (c) + barrier per 8 k-steps", out, simd);
  printf("SIMD of waves 0..7 of block 0:");
  for (int w = 0; w < 8; ++w) printf(" %d", simd[w]);
  printf("\n");
  return 0;
}
