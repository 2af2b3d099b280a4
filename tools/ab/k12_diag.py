# Diagnostic patch (tools/build_patched.sh): per-wave records of the fused K1 + Gram kernel in a device array,
# read back with sysid_debug_k12_diag(out, n).  Record of wave w of workgroup b at [(b * 8 + w) * 10]:
#   K1 wave:   [1, t_start, t_end, ready[w] at exit, f0, f1, 0, 0, 0, 0]
#   Gram wave: [2, t_start, t_end, bad, np, nfast, ready[0..3] at exit]
# (times: s_memrealtime, 100 MHz).  Diagnostics only, never the product.
k = open("sysid_kernels.h").read()


def rep(old, new):
    global k
    assert k.count(old) == 1, old
    k = k.replace(old, new)


rep("constexpr int K12_NTC = 10;", "__device__ long long k12_diag[256 * 8 * 10];\nconstexpr int K12_NTC = 10;")
rep("""  double* o = slab + ((size_t)blockIdx.x * K12_NSLOTS + R.base) * 256;
""", """  if (lane == 0 && blockIdx.x < 256) {
    long long* d = k12_diag + ((int64_t)blockIdx.x * 8 + K1_WAVES + W) * 10;
    d[2] = (long long)__builtin_amdgcn_s_memrealtime();
    d[3] = bad ? 1 : 0;
    d[4] = np;
    d[5] = nfast;
    for (int v = 0; v < 4; ++v) d[6 + v] = __hip_atomic_load(k12_ready + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  double* o = slab + ((size_t)blockIdx.x * K12_NSLOTS + R.base) * 256;
""")
rep("""  const int wave = threadIdx.x >> 6;
  if (wave < K1_WAVES) {
    if constexpr (RING > 0) {""", """  const int wave = threadIdx.x >> 6;
  const long long t_start = (long long)__builtin_amdgcn_s_memrealtime();
  long long* dg = k12_diag + ((int64_t)blockIdx.x * 8 + wave) * 10;
  if ((threadIdx.x & 63) == 0 && blockIdx.x < 256) {
    dg[0] = wave < K1_WAVES ? 1 : 2;
    dg[1] = t_start;
  }
  if (wave < K1_WAVES) {
    if constexpr (RING > 0) {""")
rep("""      k1_body<MAXCH, NVC, SPW, double, 0, 0, 0, 1>(kp, mimg_g, in, N, ld, panel, ldp, nullptr, nullptr, nullptr,
                                                   ready, f0, f1);
    }
""", """      k1_body<MAXCH, NVC, SPW, double, 0, 0, 0, 1>(kp, mimg_g, in, N, ld, panel, ldp, nullptr, nullptr, nullptr,
                                                   ready, f0, f1);
    }
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 256) {
      dg[2] = (long long)__builtin_amdgcn_s_memrealtime();
      dg[3] = __hip_atomic_load(ready + wave, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      dg[4] = f0;
      dg[5] = f1;
    }
""")
open("sysid_kernels.h", "w").write(k)
e = open("sysid_k12_inst.hip").read()
e += '''
extern "C" int32_t sysid_debug_k12_diag(long long* out, int32_t n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(sysid_dev::k12_diag), (size_t)n * sizeof(long long)) == hipSuccess ? 0 : -1;
}
'''
open("sysid_k12_inst.hip", "w").write(e)
