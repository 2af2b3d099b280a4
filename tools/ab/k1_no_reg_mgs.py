"""A/B patch (tools/build_patched.sh): the runtime-nv kernels' Gram-Schmidt through LDS (mgs_lds) instead of the
register-resident 8-lane-group form."""
k = open("sysid_kernels.h").read()
old = "      } else if (8 * k <= HW && nv <= 8 * K1_MGS_NU) {"
assert old in k
k = k.replace(old, "      } else if (false && 8 * k <= HW && nv <= 8 * K1_MGS_NU) {")
open("sysid_kernels.h", "w").write(k)
