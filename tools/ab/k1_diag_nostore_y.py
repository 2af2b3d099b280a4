"""Diagnostic patch (tools/build_patched.sh): the quadruped K1's staged Y-row global stores are kept behind a
never-true test on the staged value (the LDS staging and its reads stay), so the time difference against the product
build is the cost of the Y phase's global stores."""
k = open("sysid_kernels.h").read()
old = """            panel_store(reinterpret_cast<OutT*>(rb + off), s2[x].x, s2[x].y);"""
new = """            const double2 v = s2[x];
            if (v.x == -1.25e300) panel_store(reinterpret_cast<OutT*>(rb + off), v.x, v.y);"""
assert old in k
k = k.replace(old, new)
open("sysid_kernels.h", "w").write(k)
