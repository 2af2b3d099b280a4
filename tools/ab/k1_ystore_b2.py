"""A/B patch (tools/build_patched.sh): the quadruped Y row's store loop reads its staged pairs two at a time (two LDS
reads in flight per wait instead of one); a lane without a second pair stores its first one twice (same data, same
address), so the loop has no branch."""
k = open("sysid_kernels.h").read()
old = """          for (int x = hl; x < n2v; x += HW) {
            const uint32_t off = yhoff + (uint32_t)((2 * x + (x >= wy2 ? dg : 0)) * (int)sizeof(OutT));
            panel_store(reinterpret_cast<OutT*>(rb + off), s2[x].x, s2[x].y);
          }"""
new = """          for (int x = hl; x < n2v; x += 2 * HW) {
            const int x1 = x + HW < n2v ? x + HW : x;
            const double2 v0 = s2[x], v1 = s2[x1];
            const uint32_t off = yhoff + (uint32_t)((2 * x + (x >= wy2 ? dg : 0)) * (int)sizeof(OutT));
            const uint32_t off1 = yhoff + (uint32_t)((2 * x1 + (x1 >= wy2 ? dg : 0)) * (int)sizeof(OutT));
            panel_store(reinterpret_cast<OutT*>(rb + off), v0.x, v0.y);
            panel_store(reinterpret_cast<OutT*>(rb + off1), v1.x, v1.y);
          }"""
assert old in k
k = k.replace(old, new)
open("sysid_kernels.h", "w").write(k)
