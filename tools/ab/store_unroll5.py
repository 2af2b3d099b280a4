# A/B patch: the Spot staged-row store loop fully unrolled (all LDS reads of a row issued before its stores)
k = open("sysid_kernels.h").read()
old = '''          double2 cur = s2[hl];  // (staged slots past n2v hold finite values; unused)
          for (int x = hl; x < n2v; x += HW) {
            const double2 nxt = s2[x + HW < n2v ? x + HW : x];  // clamped index: no pointer select
            const uint32_t off = yhoff + (uint32_t)((2 * x + (x >= wy2 ? dg : 0)) * (int)sizeof(OutT));
            panel_store(reinterpret_cast<OutT*>(rb + off), cur.x, cur.y);
            cur = nxt;
          }'''
new = '''          constexpr int NS = (2 * 80 + HW - 1) / HW;  // staged pairs per lane (<= 16 bodies)
          double2 v[NS];
#pragma unroll
          for (int t = 0; t < NS; ++t) {
            const int x = hl + HW * t;
            v[t] = s2[x < n2v ? x : hl];
          }
#pragma unroll
          for (int t = 0; t < NS; ++t) {
            const int x = hl + HW * t;
            if (x < n2v) {
              const uint32_t off = yhoff + (uint32_t)((2 * x + (x >= wy2 ? dg : 0)) * (int)sizeof(OutT));
              panel_store(reinterpret_cast<OutT*>(rb + off), v[t].x, v[t].y);
            }
          }'''
assert old in k
k = k.replace(old, new)
open("sysid_kernels.h", "w").write(k)
