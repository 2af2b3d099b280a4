"""Diagnostic patch: as k1_diag_nostore_y.py, plus the quadruped friction / torque columns' stores behind a
never-true test: K1 without any panel store."""
exec(open(__file__.replace("nostore_all", "nostore_y")).read())
k = open("sysid_kernels.h").read()
old = """            panel_store(po + i * pstep, v2[0], v2[1]);"""
new = """            if (v2[0] == -1.25e300) panel_store(po + i * pstep, v2[0], v2[1]);"""
assert old in k
k = k.replace(old, new)
open("sysid_kernels.h", "w").write(k)
