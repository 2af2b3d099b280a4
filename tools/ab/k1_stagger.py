"""A/B patch (tools/build_patched.sh): K1 waves of odd global index start late by SYSID_K1_STAGGER x s_sleep(127)
(~8k cycles each), so the waves' store-heavy column phases are out of phase with the others' store-free phases
instead of every wave of the chip writing the panel at the same time."""
k = open("sysid_kernels.h").read()
def rep(old, new, src="k"):
    global k
    assert old in k, old[:80]
    k = k.replace(old, new)
rep("""  int k12_spin_log2, k12_stall_polls;
};""", """  int k12_spin_log2, k12_stall_polls;
  int k1_stagger;
};""")
rep("""  int64_t s = claim_value(claim_issue());
  if (s < N) {""", """  if constexpr (!FUSED) {
    if (((blockIdx.x * (blockDim.x >> 6) + wave) & 1) != 0)
      for (int x = 0; x < kp.k1_stagger; ++x) __builtin_amdgcn_s_sleep(127);
  }
  int64_t s = claim_value(claim_issue());
  if (s < N) {""")
open("sysid_kernels.h", "w").write(k)
e = open("sysid_engine.hip").read()
old = """  kp.k12_stall_polls = 0;"""
assert old in e
e = e.replace(old, old + """
  kp.k1_stagger = 0;
  if (const char* v = std::getenv("SYSID_K1_STAGGER")) kp.k1_stagger = std::max(0, std::atoi(v));""")
open("sysid_engine.hip", "w").write(e)
