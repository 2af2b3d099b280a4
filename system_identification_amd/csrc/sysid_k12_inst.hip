// sysid_k12_inst.hip — the fused K1 + Gram kernel (k12_fused_panel_gram) of the quadruped K1 variant: full outputs
// (ring = 0) and the Gram-only ring form (ring = K12_RING), and their launcher (sysid_launch.h).  Built by
// __graft_entry__.build() like the other instantiation units.
#define SYSID_TEMPLATE_TU 1
#include "sysid_launch.h"

namespace sysid_launch {

const void* k12_fn(int ring) {
  return ring ? reinterpret_cast<const void*>(sysid_dev::k12_fused_panel_gram<QCH, 18, SPW_QUAD, K12_RING>)
              : reinterpret_cast<const void*>(sysid_dev::k12_fused_panel_gram<QCH, 18, SPW_QUAD, 0>);
}

void k12_launch(int ring, dim3 g, size_t lds, hipStream_t st, const sysid_dev::K1Params& kp, const uint32_t* mimg,
                const double* d_in, int64_t N, int64_t ld, double* d_panel, int64_t ld_panel, double* slab) {
  const dim3 b(64 * (sysid_dev::K1_WAVES + sysid_dev::K12_GW));
  if (ring)
    hipLaunchKernelGGL((sysid_dev::k12_fused_panel_gram<QCH, 18, SPW_QUAD, K12_RING>), g, b, lds, st, kp, mimg, d_in,
                       N, ld, d_panel, ld_panel, slab);
  else
    hipLaunchKernelGGL((sysid_dev::k12_fused_panel_gram<QCH, 18, SPW_QUAD, 0>), g, b, lds, st, kp, mimg, d_in, N, ld,
                       d_panel, ld_panel, slab);
}

}  // namespace sysid_launch
