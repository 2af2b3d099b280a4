"""A/B patch (tools/build_patched.sh): the quadruped K1's staged panel rows double-buffered in LDS — row rho's pieces
go to buffer rho & 1 (the joint records, or the dead [J_w, P) region: tp and dq move before J_w in the layout), and
the previous row's buffer is read back before this row's arithmetic and stored after it, so the read-back's LDS
latency hides behind the row's FMAs instead of sitting between the staging stores and the panel stores."""
k = open("sysid_kernels.h").read()
def rep(old, new):
    global k
    assert old in k, old[:80]
    k = k.replace(old, new)
rep("""  l.Jw = take(nv * 6);          // spatial axis of every dof [linear at origin; angular]
  l.tp = take(nv);              // P S^T tau
  l.dqs = take(nv);             // dq for the friction columns (`in` takes the next sample's inputs mid-step)""",
"""  l.tp = take(nv);              // P S^T tau
  l.dqs = take(nv);             // dq for the friction columns (`in` takes the next sample's inputs mid-step)
  l.Jw = take(nv * 6);          // spatial axis of every dof [linear at origin; angular] (before J_c: the quadruped
                                // K1 stages panel rows in [J_w, P) once the axes are in registers)""")
rep("""        wsync();
        if (valid) {
          const double2* s2 = reinterpret_cast<const double2*>(stg);
          char* rb = ybase + (int64_t)rho * ldp * (int64_t)sizeof(OutT);
          // nullspace mode: the rows past nrows of either group are not stored
          const int n2v = !CMP ? n2 : rh + rho < nrows ? n2 : rho < nrows ? wy2 : 0;
          for (int x = hl; x < n2v; x += HW) {
            const uint32_t off = yhoff + (uint32_t)((2 * x + (x >= wy2 ? dg : 0)) * (int)sizeof(OutT));
            panel_store(reinterpret_cast<OutT*>(rb + off), s2[x].x, s2[x].y);
          }
        }
        wsync();
      };""",
"""      };
      (void)0;""")
# replace stg usage with a per-row buffer and the pipelined read-back
rep("""      double* stg = body;  // [row group][wy]""",
"""      double* stg0 = body;            // [row group][wy], even rows
      double* stg1 = wr + L.Jw;       // odd rows ([J_w, P) is dead once the axes are in registers)
      constexpr int NRB = (2 * 80 + 31) / 32;  // read-back pieces per lane (rg * wy / 2 <= 160 pairs)""")
rep("""          double2* sp = reinterpret_cast<double2*>(stg + g * kp.wy + 10 * (i - 1));""",
    """          double2* sp = reinterpret_cast<double2*>(((rho & 1) ? stg1 : stg0) + g * kp.wy + 10 * (i - 1));""")
# after the yrow lambda (now compute+stage only) define the pipelined driver
rep("""      if constexpr (CMP) {
#pragma unroll 1
        for (int rho = 0; rho < rh; rho += 2) {
          row_load(g * rh + rho + 1, hB, pB);
          yrow(rho, hn, pn);
          row_load(g * rh + rho + 2, hn, pn);
          yrow(rho + 1, hB, pB);
        }
      } else {
        int rho = 0;
#pragma unroll 1
        for (; rho + 1 < rh; rho += 2) {
          row_load(g * rh + rho + 1, hB, pB);
          yrow(rho, hn, pn);
          if (rho + 2 < rh) row_load(g * rh + rho + 2, hn, pn);
          yrow(rho + 1, hB, pB);
        }
        if (rho < rh) yrow(rho, hn, pn);
      }""",
"""      auto rb_issue = [&](int rho, double2 (&rv)[NRB]) {
        const double2* s2 = reinterpret_cast<const double2*>((rho & 1) ? stg1 : stg0);
#pragma unroll
        for (int u = 0; u < NRB; ++u) rv[u] = s2[hl + HW * u];  // past n2: unused values inside the buffer
      };
      auto rb_store = [&](int rho, const double2 (&rv)[NRB]) {
        char* rb = ybase + (int64_t)rho * ldp * (int64_t)sizeof(OutT);
        // nullspace mode: the rows past nrows of either group are not stored
        const int n2v = !CMP ? n2 : rh + rho < nrows ? n2 : rho < nrows ? wy2 : 0;
#pragma unroll
        for (int u = 0; u < NRB; ++u) {
          const int x = hl + HW * u;
          if (x < n2v) {
            const uint32_t off = yhoff + (uint32_t)((2 * x + (x >= wy2 ? dg : 0)) * (int)sizeof(OutT));
            panel_store(reinterpret_cast<OutT*>(rb + off), rv[u].x, rv[u].y);
          }
        }
      };
      // row rho: the previous row's staged pieces are read back before its arithmetic and stored after it
      auto ystep = [&](int rho, const double* hc, const double* pc) {
        double2 rv[NRB];
        rb_issue(rho + 1, rv);  // (rho - 1) & 1 == (rho + 1) & 1; row 0 reads unused values
        yrow(rho, hc, pc);
        if (rho > 0 && valid) rb_store(rho - 1, rv);
        wsync();  // this row's pieces are staged; the previous row's buffer has been read
      };
      if constexpr (CMP) {
#pragma unroll 1
        for (int rho = 0; rho < rh; rho += 2) {
          row_load(g * rh + rho + 1, hB, pB);
          ystep(rho, hn, pn);
          row_load(g * rh + rho + 2, hn, pn);
          ystep(rho + 1, hB, pB);
        }
      } else {
        int rho = 0;
#pragma unroll 1
        for (; rho + 1 < rh; rho += 2) {
          row_load(g * rh + rho + 1, hB, pB);
          ystep(rho, hn, pn);
          if (rho + 2 < rh) row_load(g * rh + rho + 2, hn, pn);
          ystep(rho + 1, hB, pB);
        }
        if (rho < rh) ystep(rho, hn, pn);
      }
      if (valid) {
        double2 rv[NRB];
        rb_issue(rh - 1, rv);
        rb_store(rh - 1, rv);
      }
      wsync();""")
open("sysid_kernels.h", "w").write(k)
