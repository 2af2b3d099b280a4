"""A/B patch (tools/build_patched.sh): the narrow register-staged K2 writes the next chunk's staged rows to LDS after
the first two k-steps of the current chunk instead of after all of them, so the ds_write latency is off the
per-chunk barrier's critical path (the buffer written was last read before the previous barrier)."""
k = open("sysid_kernels.h").read()
old = """    auto mfma_chunk = [&](const T* cur) {
#pragma unroll
      for (int kk = 0; kk < KC; kk += 4) {"""
new = """    auto mfma_chunk = [&](const T* cur, auto k0c, auto k1c) {
      constexpr int K0 = decltype(k0c)::value, K1E = decltype(k1c)::value;
#pragma unroll
      for (int kk = K0; kk < K1E; kk += 4) {"""
assert old in k
k = k.replace(old, new)
old = """    for (; c + 1 < nfull; c += 2) {  // chunks c (buffer 0, set A) and c + 1 (buffer 1, set B)
      load_full(c + 2, A);
      mfma_chunk(lds);
      store_set(B, lds + BUF);
      __syncthreads();
      load_full(c + 3, B);
      mfma_chunk(lds + BUF);
      if (c + 2 < nfull) store_set(A, lds);
      __syncthreads();
    }
    if (c < nfull) {  // an odd last full chunk, already in buffer 0
      mfma_chunk(lds);
      __syncthreads();
    }
    if (r0 + nfull * KC < r1) {  // the panel's partial last chunk
      load_chunk(r0 + nfull * KC);
      store_chunk(lds);
      __syncthreads();
      mfma_chunk(lds);
    }"""
new = """    constexpr std::integral_constant<int, 0> KS0{};
    constexpr std::integral_constant<int, KSPLIT> KSM{};
    constexpr std::integral_constant<int, KC> KSE{};
    for (; c + 1 < nfull; c += 2) {  // chunks c (buffer 0, set A) and c + 1 (buffer 1, set B)
      load_full(c + 2, A);
      mfma_chunk(lds, KS0, KSM);
      store_set(B, lds + BUF);  // buffer 1's last reads retired at the previous barrier
      mfma_chunk(lds, KSM, KSE);
      __syncthreads();
      load_full(c + 3, B);
      mfma_chunk(lds + BUF, KS0, KSM);
      if (c + 2 < nfull) store_set(A, lds);
      mfma_chunk(lds + BUF, KSM, KSE);
      __syncthreads();
    }
    if (c < nfull) {  // an odd last full chunk, already in buffer 0
      mfma_chunk(lds, KS0, KSE);
      __syncthreads();
    }
    if (r0 + nfull * KC < r1) {  // the panel's partial last chunk
      load_chunk(r0 + nfull * KC);
      store_chunk(lds);
      __syncthreads();
      mfma_chunk(lds, KS0, KSE);
    }"""
assert old in k
k = k.replace(old, new)
old = """  typedef typename K2Acc<T>::type accT;
  constexpr int K2W = k2_waves(NTC), K2S = k2_slots<T>(NTC);
  constexpr int STRIDE = k2_stride(NTC);
  constexpr int BUF = KC * STRIDE;                       // elements per LDS buffer"""
new = """  typedef typename K2Acc<T>::type accT;
  constexpr int K2W = k2_waves(NTC), K2S = k2_slots<T>(NTC);
  constexpr int STRIDE = k2_stride(NTC);
  constexpr int BUF = KC * STRIDE;                       // elements per LDS buffer
  constexpr int KSPLIT = SYSID_K2_EARLY;                 // rows of a chunk multiplied before the next chunk's LDS writes"""
assert old in k
k = k.replace(old, new)
open("sysid_kernels.h", "w").write(k)
