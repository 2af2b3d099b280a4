// Micro-test (dev tool): can a running kernel observe a flag written by another stream while it runs?
// A spinning kernel (grid G workgroups of 256 threads, every lane polling) waits for flag >= 1; another stream
// then writes the flag by (w) hipStreamWriteValue32, (c) a 4-byte hipMemcpyAsync from pinned host memory, or
// (h) the host itself (fine-grained host memory, plain store).  Prints what each waiter saw and how long it took.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/ubench/stream_flag tools/ubench/stream_flag.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

__global__ void spin(const unsigned* flag, unsigned* out, long long max_spins) {
  long long n = 0;
  unsigned v = 0;
  while ((v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) < 1u && n < max_spins) {
    __builtin_amdgcn_s_sleep(8);
    ++n;
  }
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = v;
    out[2 * blockIdx.x + 1] = (unsigned)(n > 0xffffffffll ? 0xffffffffu : n);
  }
}

#define CK(x) do { hipError_t r_ = (x); if (r_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(r_)); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int G = argc > 1 ? atoi(argv[1]) : 1;
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  unsigned *d_out, *h_one, *h_out;
  CK(hipMalloc(&d_out, 2 * G * sizeof(unsigned)));
  CK(hipHostMalloc(&h_one, sizeof(unsigned), hipHostMallocDefault));
  CK(hipHostMalloc(&h_out, 2 * G * sizeof(unsigned), hipHostMallocDefault));
  *h_one = 1;
  const char* modes[] = {"writevalue/uncached", "writevalue/coarse", "memcpy/uncached", "memcpy/coarse", "host/finegrained"};
  for (int m = 0; m < 5; ++m) {
    unsigned* flag = nullptr;
    if (m == 0 || m == 2) CK(hipExtMallocWithFlags((void**)&flag, 256, hipDeviceMallocUncached));
    else if (m == 1 || m == 3) CK(hipMalloc(&flag, 256));
    else CK(hipHostMalloc(&flag, 256, hipHostMallocCoherent));
    if (m < 4) CK(hipMemset(flag, 0, 256)); else *flag = 0;
    CK(hipDeviceSynchronize());
    const auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(spin, dim3(G), dim3(256), 0, a, flag, d_out, 20000000ll);
    CK(hipGetLastError());
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
    if (m == 0 || m == 1) CK(hipStreamWriteValue32(b, flag, 1u, 0));
    else if (m == 2 || m == 3) CK(hipMemcpyAsync(flag, h_one, sizeof(unsigned), hipMemcpyHostToDevice, b));
    else __atomic_store_n(flag, 1u, __ATOMIC_SEQ_CST);
    CK(hipStreamSynchronize(b));
    const double tb = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    CK(hipStreamSynchronize(a));
    const double ta = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    CK(hipMemcpy(h_out, d_out, 2 * G * sizeof(unsigned), hipMemcpyDeviceToHost));
    unsigned seen = 0, maxspin = 0;
    for (int g = 0; g < G; ++g) {
      seen += h_out[2 * g] >= 1;
      maxspin = h_out[2 * g + 1] > maxspin ? h_out[2 * g + 1] : maxspin;
    }
    printf("%-22s grid %4d: writer stream done %.3f ms, kernel done %.3f ms, %u/%d waiters saw the flag, max spins %u\n",
           modes[m], G, tb, ta, seen, G, maxspin);
    if (m < 4) CK(hipFree(flag)); else CK(hipHostFree(flag));
  }
  return 0;
}
