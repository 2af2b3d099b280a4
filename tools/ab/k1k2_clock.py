"""Diagnostic patch (tools/build_patched.sh): in-kernel clock of K1 and the narrow K2 (MI355X_MICROARCH.md 'DVFS
give-back' item 6): every workgroup stamps s_memtime and s_memrealtime (100 MHz) at its start and end; one lane per
workgroup adds the two deltas to a __device__ accumulator per kernel; sysid_debug_clock(out[4], reset) reads
{K1 core cycles, K1 realtime ticks, K2 core cycles, K2 realtime ticks}.  clock = cycles / ticks x 100 MHz."""
k = open("sysid_kernels.h").read()
def rep(old, new):
    global k
    assert k.count(old) == 1, old[:80]
    k = k.replace(old, new)
rep("namespace sysid_dev {\n", "namespace sysid_dev {\n__device__ unsigned long long dbg_clock[4];\n")
# K1: around the whole body
rep("""  k1_body<MAXCH, NVC, SPW, OutT, POV, CMP, QF>(kp, mimg_g, in, N, ld, panel, ldp, work, dbg, rcount);""",
    """  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  k1_body<MAXCH, NVC, SPW, OutT, POV, CMP, QF>(kp, mimg_g, in, N, ld, panel, ldp, work, dbg, rcount);
  const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { atomicAdd(&dbg_clock[0], c1 - c0); atomicAdd(&dbg_clock[1], r1 - r0); }""")
rep("""  k2_syrk_body<T, NTC, KC, false>(panel, rows, ldp, supers, ngroups, ksplit, nslots, accumulate, slab, nullptr,
                                  nullptr);""",
    """  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  k2_syrk_body<T, NTC, KC, false>(panel, rows, ldp, supers, ngroups, ksplit, nslots, accumulate, slab, nullptr,
                                  nullptr);
  const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { atomicAdd(&dbg_clock[2], c1 - c0); atomicAdd(&dbg_clock[3], r1 - r0); }""")
open("sysid_kernels.h", "w").write(k)
# readers: the f64 K1 unit holds K1's copy of the accumulator, the f64 narrow K2 unit K2's (each unit has its own)
for f, cond, lo in (("sysid_k1_inst.hip", "SYSID_PREC == 0 && SYSID_CMP == 0", 0),
                    ("sysid_k2_inst.hip", "SYSID_PREC == 0 && SYSID_WIDE == 0", 2)):
    e = open(f).read()
    e += f'''
#if {cond}
extern "C" int32_t sysid_debug_clock{lo}(unsigned long long* out2, int32_t reset) {{
  unsigned long long z[4] = {{0, 0, 0, 0}};
  if (reset) return hipMemcpyToSymbol(HIP_SYMBOL(sysid_dev::dbg_clock), z, sizeof z) == hipSuccess ? 0 : -1;
  if (hipMemcpyFromSymbol(z, HIP_SYMBOL(sysid_dev::dbg_clock), sizeof z) != hipSuccess) return -1;
  out2[0] = z[{lo}];
  out2[1] = z[{lo + 1}];
  return 0;
}}
#endif
'''
    open(f, "w").write(e)
