# A/B patch: K1 at one 4-wave workgroup per CU (one wave per SIMD), by inflating its dynamic LDS request.
# Question answered: how much of K1's time is latency that a second wave per SIMD hides (the fused K1+K2 design
# leaves K1 one wave per SIMD beside one MFMA wave).
import re
p = "sysid_engine.hip"
s = open(p).read()
old = "const size_t lds = (size_t)(MI.ndbl + wv * k1_spw(vars[c]) * wls[c].total) * sizeof(double);"
assert old in s
s = s.replace(old, "const size_t lds = std::max<size_t>((size_t)(MI.ndbl + wv * k1_spw(vars[c]) * wls[c].total) * sizeof(double), 100 * 1024);")
open(p, "w").write(s)
