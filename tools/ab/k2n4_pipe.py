"""Patch (tools/build_patched.sh): the N4 narrow K2's k-loop reads k-step kk + 4's operands before issuing k-step
kk's MFMAs (one step of register double-buffering; the compiler barrier then sits after the MFMAs, so reads run at
most one step ahead)."""
k = open("sysid_kernels.h").read()
old_start = "    auto mfma_chunk = [&](const T* cur) {\n#pragma unroll\n      for (int kk = 0; kk < KC; kk += 4) {\n        T x[4] = {0, 0, 0, 0};\n        if constexpr (uA0) x[0] = cur[foff[0] + kk * STRIDE];"
assert k.count(old_start) == 1
a = k.index(old_start)
end_marker = "    constexpr std::integral_constant<int, 0> A{};"
b = k.index(end_marker, a)
new = r'''    auto mfma_chunk = [&](const T* cur) {
      constexpr int NOP = 4 + 2 * (NS > 0 ? NS : 1);
      auto rd = [&](int kk, T* o) {
        o[0] = uA0 ? cur[foff[0] + kk * STRIDE] : (T)0;
        o[1] = uA1 ? cur[foff[1] + kk * STRIDE] : (T)0;
        o[2] = uB0 ? cur[foff[2] + kk * STRIDE] : (T)0;
        o[3] = uB1 ? cur[foff[3] + kk * STRIDE] : (T)0;
#pragma unroll
        for (int n = 0; n < NS; ++n) {
          o[4 + 2 * n] = cur[aoff[n] + kk * STRIDE];
          o[5 + 2 * n] = cur[boff[n] + kk * STRIDE];
        }
      };
      auto mm = [&](const T* x) {
        auto tile = [&](auto tc) {
          constexpr int t = decltype(tc)::value;
          if constexpr (((M >> t) & 1) != 0) {
            if constexpr (sizeof(T) == 8)
              acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(x[t >> 1], x[2 + (t & 1)], acc[t], 0, 0, 0);
            else
              acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[t >> 1], x[2 + (t & 1)], acc[t], 0, 0, 0);
          }
        };
        tile(std::integral_constant<int, 0>{});
        tile(std::integral_constant<int, 1>{});
        tile(std::integral_constant<int, 2>{});
        tile(std::integral_constant<int, 3>{});
        if constexpr (N4) {
#pragma unroll
          for (int n = 0; n < NS; ++n)
            acc4[n] = __builtin_amdgcn_mfma_f64_4x4x4f64(x[4 + 2 * n], x[5 + 2 * n], acc4[n], 0, 0, 0);
        }
      };
      if constexpr (N4) {
        T xc[NOP], xn[NOP];
        rd(0, xc);
#pragma unroll
        for (int kk = 0; kk < KC; kk += 4) {
          if (kk + 4 < KC) rd(kk + 4, xn);
          mm(xc);
          asm volatile("" ::: "memory");
#pragma unroll
          for (int u = 0; u < NOP; ++u) xc[u] = xn[u];
        }
      } else {
#pragma unroll
        for (int kk = 0; kk < KC; kk += 4) {
          T x[NOP];
          rd(kk, x);
          mm(x);
        }
      }
    };
'''
k = k[:a] + new + k[b:]
open("sysid_kernels.h", "w").write(k)
# with one step of double-buffering, at most 10 operand reads per k-step (12 spilled)
k = open("sysid_kernels.h").read()
old = "  return (12 - k2_mask_frags(m)) / 2 < K2N4_MAXNS ? (12 - k2_mask_frags(m)) / 2 : K2N4_MAXNS;"
assert k.count(old) == 1
k = k.replace(old, "  return (10 - k2_mask_frags(m)) / 2 < K2N4_MAXNS ? (10 - k2_mask_frags(m)) / 2 : K2N4_MAXNS;")
open("sysid_kernels.h", "w").write(k)
