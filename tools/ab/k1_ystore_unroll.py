"""A/B patch (tools/build_patched.sh): the quadruped Y row's store loop unrolled over its at most five 32-lane
passes (n2 <= 160 pairs), one staged pair read and stored per pass with a compiler barrier between passes (no
batching of reads: the batched form spilled).  Passes 0-2 are always whole (n2 >= 110: 11..16 bodies, and wy2 >= 55
when only the first group is stored), passes 3-4 store a lane's pair of pass 0 again (same data, same address) when
theirs is past the row: no exec-masked branch per pass."""
k = open("sysid_kernels.h").read()
old = """          for (int x = hl; x < n2v; x += HW) {
            const uint32_t off = yhoff + (uint32_t)((2 * x + (x >= wy2 ? dg : 0)) * (int)sizeof(OutT));
            panel_store(reinterpret_cast<OutT*>(rb + off), s2[x].x, s2[x].y);
          }"""
new = """          constexpr int NST = (160 + HW - 1) / HW;
          int hx = hl;  // opaque: the passes' offsets are recomputed per row, not held across the row loop
          asm volatile("" : "+v"(hx));
          if (n2v > 0) {
#pragma unroll
            for (int u = 0; u < NST; ++u) {
              int x = hx + HW * u;
              if (u >= 3) x = x < n2v ? x : hx;
              const uint32_t off = yhoff + (uint32_t)((2 * x + (x >= wy2 ? dg : 0)) * (int)sizeof(OutT));
              const double2 v = s2[x];
              panel_store(reinterpret_cast<OutT*>(rb + off), v.x, v.y);
              asm volatile("" ::: "memory");
            }
          }"""
assert old in k
k = k.replace(old, new)
open("sysid_kernels.h", "w").write(k)
