"""A/B patch (tools/build_patched.sh), on top of k1_ystage_pipe.py: one H1 / P register set instead of two; row rho's
H1 / P reads and the previous row's staged read-back are issued together, so one LDS latency per row is exposed
instead of the row-load wait and the read-back wait in turn."""
import runpy
runpy.run_path("/root/repo/tools/ab/k1_ystage_pipe.py")
k = open("sysid_kernels.h").read()
def rep(old, new):
    global k
    assert old in k, old[:80]
    k = k.replace(old, new)
rep("""      auto ystep = [&](int rho, const double* hc, const double* pc) {
        double2 rv[NRB];
        rb_issue(rho + 1, rv);  // (rho - 1) & 1 == (rho + 1) & 1; row 0 reads unused values
        yrow(rho, hc, pc);""","""      auto ystep = [&](int rho, const double* hc, const double* pc) {
        double2 rv[NRB];
        rb_issue(rho + 1, rv);  // (rho - 1) & 1 == (rho + 1) & 1; row 0 reads unused values
        row_load(g * rh + rho, hn, pn);
        yrow(rho, hn, pn);""")
rep("""      if constexpr (CMP) {
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
      }""","""#pragma unroll 1
      for (int rho = 0; rho < rh; ++rho) ystep(rho, hn, pn);""")
rep("""      row_load(g * rh, hn, pn);
      wsync();  // every read of the joint records precedes the first staging store""",
    """      wsync();  // every read of the joint records precedes the first staging store""")
rep("""      double hB[6], pB[MAXCH];
""", "")
open("sysid_kernels.h", "w").write(k)
