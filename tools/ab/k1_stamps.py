"""Patch (tools/build_patched.sh) for a K1 phase-time diagnostic build: s_memtime stamps at the top-level phase
boundaries of the sample loop, summed per wave in registers and added to a device array once per wave at the
end; sysid_debug_k1_stamps(out[10]) copies [9 phase sums, waves] to the host.  Diagnostics only, never the
product.  Phases: 0 loop top -> FK, 1 FK poses, 2 axes + contact points, 3 v / a_gf, 4 J_c, 5 Gram-Schmidt / P /
nullspace, 6 tp, H1, mid-step claim + commit, 7 Y_proj columns, 8 friction / torque columns."""
k = open("sysid_kernels.h").read()
def ins_before(anchor, text, count=1):
    global k
    assert anchor in k, anchor
    k = k.replace(anchor, text + anchor, count)
ins_before("template <int MAXCH, int NVC, int SPW, typename OutT, int POV = 0, int CMP = 0, int QF = 0, int FUSED = 0>",
           "__device__ unsigned long long k1_stamp_sum[16];\n")
ins_before("  while (s < N) {\n    // Quadruped variant (OPQ)",
           "  unsigned long long st_acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};\n"
           "  unsigned long long st_t = __builtin_readcyclecounter();\n"
           "#define K1STAMP(i) { const unsigned long long _t = __builtin_readcyclecounter(); st_acc[i] += _t - st_t; st_t = _t; }\n")
ins_before("    // ---- forward pass (computeJointTorqueRegressor forward step), in two parts ----", "    K1STAMP(0)\n")
ins_before("    // ---- world motion axes of every dof; contact points ----", "    K1STAMP(1)\n")
ins_before("    // ---- forward pass, part (2): body velocities and accelerations ----", "    K1STAMP(2)\n")
ins_before("    // ---- contact Jacobian (LOCAL_WORLD_ALIGNED, linear rows) ----", "    K1STAMP(3)\n")
ins_before("    // ---- tp = P S^T tau  (+ J_c^T lambda in the full mode) ;  H1 = P[:, ff] J_w[:, ff]^T ----", "    K1STAMP(5)\n")
ins_before("    // ---- projected regressor Y_proj: lane = (body i, row group g), all ten columns of body i ----", "    K1STAMP(6)\n")
ins_before("    // ---- [B_v | B_c | tau_proj | pad]: 16-byte stores of column pairs ----", "    K1STAMP(7)\n")
old = "    __builtin_amdgcn_s_setprio(2);\n    s = s1;\n    s1 = s2;\n    ++steps_done;\n  }\n  publish(steps_done);\n}\n"
assert old in k
k = k.replace(old, "    __builtin_amdgcn_s_setprio(2);\n    K1STAMP(8)\n    s = s1;\n    s1 = s2;\n    ++steps_done;\n  }\n"
              "  publish(steps_done);\n  if (lane == 0) {\n    for (int i = 0; i < 9; ++i) atomicAdd(&k1_stamp_sum[i], st_acc[i]);\n"
              "    atomicAdd(&k1_stamp_sum[9], 1ull);\n  }\n}\n")
# J_c -> Gram-Schmidt boundary: the first wsync after the J_c loop
anchor = "    // ---- contact Jacobian (LOCAL_WORLD_ALIGNED, linear rows) ----"
i = k.index(anchor)
j = k.index("    wsync();\n", i)
k = k[:j] + "    wsync();\n    K1STAMP(4)\n" + k[j + len("    wsync();\n"):]
open("sysid_kernels.h", "w").write(k)
# the readout lives in the translation unit of the f64 stacked-output K1 instantiations (sysid_k1_inst.hip with
# SYSID_PREC=0, SYSID_CMP=0): every unit has its own copy of the __device__ accumulator
import os
e = open("sysid_k1_inst.hip").read()
e = e.replace('#include "sysid_launch.h"', '#include "sysid_launch.h"\n#define STAMP_PREC ' + os.environ.get("STAMP_PREC", "0"), 1)
e += '''
#if SYSID_PREC == STAMP_PREC && SYSID_CMP == 0
extern "C" int32_t sysid_debug_k1_stamps(unsigned long long* out10, int32_t reset) {
  if (reset) {
    unsigned long long z[16] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(sysid_dev::k1_stamp_sum), z, sizeof z) == hipSuccess ? 0 : -1;
  }
  return hipMemcpyFromSymbol(out10, HIP_SYMBOL(sysid_dev::k1_stamp_sum), 10 * sizeof(unsigned long long)) == hipSuccess ? 0 : -1;
}
#endif
'''
open("sysid_k1_inst.hip", "w").write(e)
