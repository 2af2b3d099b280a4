"""A/B patch (tools/build_patched.sh): the quadruped K1's friction / torque columns with every row's LDS reads issued
up front (9 rows per lane for Spot / Solo: two 16-lane groups), instead of a rolled loop that waits per row."""
k = open("sysid_kernels.h").read()
old = """        } else {
          for (int r = fg; r < nrows; r += NG, po += pstep) {
            const double* pr = Ps + r * nv + bd;
            const double t = tps[r];
            double v2[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) v2[u] = fcol[u] ? pr[jc[u]] * sc[u] : (tcol[u] ? t : 0.0);  // pad: whole lines
            panel_store(po, v2[0], v2[1]);
          }
        }"""
new = """        } else if (NVC == 18 && HW == 32 && !CMP && NG == 2) {
          constexpr int NR = NVC > 0 ? NVC / 2 : 1;
          double pv[NR][2], tv[NR];
#pragma unroll
          for (int i = 0; i < NR; ++i) {
            const int r = fg + 2 * i;
            const double* pr = Ps + r * NVC + bd;
            pv[i][0] = pr[jc[0]];
            pv[i][1] = pr[jc[1]];
            tv[i] = tps[r];
          }
#pragma unroll
          for (int i = 0; i < NR; ++i) {
            double v2[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) v2[u] = fcol[u] ? pv[i][u] * sc[u] : (tcol[u] ? tv[i] : 0.0);
            panel_store(po + i * pstep, v2[0], v2[1]);
          }
        } else {
          for (int r = fg; r < nrows; r += NG, po += pstep) {
            const double* pr = Ps + r * nv + bd;
            const double t = tps[r];
            double v2[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) v2[u] = fcol[u] ? pr[jc[u]] * sc[u] : (tcol[u] ? t : 0.0);  // pad: whole lines
            panel_store(po, v2[0], v2[1]);
          }
        }"""
assert old in k
k = k.replace(old, new)
open("sysid_kernels.h", "w").write(k)
