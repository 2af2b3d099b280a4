"""A/B patch (tools/build_patched.sh): chain-product poses (the one-sample-wave kernels' form) for the two-sample
quadruped K1 too (HW = 32 lanes per sample, nb <= 16: one joint per lane)."""
k = open("sysid_kernels.h").read()
old = "    if constexpr (SPW == 1) {\n      // One-sample waves (every joint has its own lane: NJ <= 64)"
assert old in k
k = k.replace(old, "    if constexpr (true) {\n      // One-sample waves (every joint has its own lane: NJ <= 64)")
open("sysid_kernels.h", "w").write(k)
