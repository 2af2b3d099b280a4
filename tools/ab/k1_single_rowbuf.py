# A/B patch (tools/build_patched.sh): the quadruped K1's Y rows with ONE row-load register set (no prefetch of row
# rho + 1 while row rho is multiplied): 18 fewer live VGPRs in the Y phase, the LDS latency of each row's loads exposed.
p = "sysid_kernels.h"
s = open(p).read()
old = """        int rho = 0;
#pragma unroll 1
        for (; rho + 1 < rh; rho += 2) {
          row_load(g * rh + rho + 1, hB, pB);
          yrow(rho, hn, pn);
          if (rho + 2 < rh) row_load(g * rh + rho + 2, hn, pn);
          yrow(rho + 1, hB, pB);
        }
        if (rho < rh) yrow(rho, hn, pn);"""
new = """#pragma unroll 1
        for (int rho = 0; rho < rh; ++rho) {
          if (rho > 0) row_load(g * rh + rho, hn, pn);
          yrow(rho, hn, pn);
        }"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
