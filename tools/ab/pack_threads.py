"""A/B patch (tools/build_patched.sh, -DSYSID_PACK_T=<n>): the host entry points' packing pool takes
min(n, OMP_NUM_THREADS - 1) threads instead of min(8, OMP_NUM_THREADS / 2) (the first staged chunk's packing is on
the Gram-only call's critical path)."""
k = open("sysid_engine.hip").read()
old = "      if (const char* v = std::getenv(\"OMP_NUM_THREADS\")) T = std::max(1, std::min(8, std::atoi(v) / 2));"
new = "      if (const char* v = std::getenv(\"OMP_NUM_THREADS\")) T = std::max(1, std::min(SYSID_PACK_T, std::atoi(v) - 1));"
assert old in k
k = k.replace(old, new)
open("sysid_engine.hip", "w").write(k)
