"""A/B patch (tools/build_patched.sh): the quadruped K1 (NVC = 18) compiled without the paths it never runs for its
models -- the full-force mode (kp.full treated as 0), the LDS Gram-Schmidt fallback (2k > 32 lanes: more than 5
contact frames) and the generic friction loops (NG != 2) -- to see whether the dead code's register pressure (126 SGPR
spill slots) costs time."""
import re
k = open("sysid_kernels.h").read()
i = k.index("__device__ __forceinline__ void k1_body(")
j = k.index("\ntemplate <int MAXCH, int NVC, int SPW, typename OutT, int POV = 0, int CMP = 0, int QF = 0>\n// Two-sample", i)
body = k[i:j]
n = body.count("kp.full")
body = body.replace("kp.full", "kfull")
old = "  const int nv = NVC > 0 ? NVC : kp.nv;\n"
assert old in body
body = body.replace(old, old + "  const int kfull = NVC == 18 ? 0 : kp.full;  // A/B: the quadruped kernel never runs the full mode\n", 1)
old = """        } else {
          mgs_lds();
        }
      } else if (8 * k <= HW && nv <= 8 * K1_MGS_NU) {"""
assert old in body
body = body.replace(old, """        }
      } else if (8 * k <= HW && nv <= 8 * K1_MGS_NU) {""")
old = """    if (npair <= 32) {"""
assert old in body
body = body.replace(old, """    if (NVC == 18 || npair <= 32) {""")
old = """        } else if (NVC == 18 && HW == 32 && !CMP && NG == 2) {"""
assert old in body
body = body.replace(old, """        } else if constexpr (NVC == 18 && HW == 32 && !CMP) {""")
k = k[:i] + body + k[j:]
open("sysid_kernels.h", "w").write(k)
print("kp.full uses replaced:", n)
