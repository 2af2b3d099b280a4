# A/B patch: the K1 publish adds an agent-scope release (buffer_wbl2) before the ready flag.
p = "sysid_kernels.h"
s = open(p).read()
old = """      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's panel stores have reached L2
      if (lane == 0) __hip_atomic_store(k12_ready + wave, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);"""
assert old in s
s = s.replace(old, """      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(k12_ready + wave, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);""")
open(p, "w").write(s)
