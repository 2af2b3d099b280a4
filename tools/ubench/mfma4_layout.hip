// Probe: operand / result lane layout of v_mfma_f64_4x4x4_4b_f64.  For each A lane L (A = e_L, B = lane + 1), print
// the result lanes that are nonzero and their values (= 1 + the B lane multiplied).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(double* out) {
  const int l = threadIdx.x;
  for (int L = 0; L < 64; ++L) {
    const double a = l == L ? 1.0 : 0.0, b = 1.0 + l;
    const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    out[L * 64 + l] = d;
  }
}
int main() {
  double* d;
  (void)hipMalloc(&d, 64 * 64 * sizeof(double));
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  double h[64 * 64];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int L = 0; L < 64; ++L) {
    printf("A lane %2d ->", L);
    for (int m = 0; m < 64; ++m)
      if (h[L * 64 + m] != 0.0) printf(" D%d=B%d", m, (int)h[L * 64 + m] - 1);
    printf("\n");
  }
  return 0;
}
