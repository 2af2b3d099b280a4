// sysid_k2_inst.hip — K2 (Gram SYRK) instantiations of one Gram arithmetic and width class.
// Built once per (SYSID_PREC, SYSID_WIDE) by __graft_entry__.build(); see sysid_launch.h.
#define SYSID_TEMPLATE_TU 1
#include "sysid_launch.h"

#ifndef SYSID_PREC
#error "SYSID_PREC (0 f64, 1 f32, 2 bf16) must be set"
#endif
#ifndef SYSID_WIDE
#error "SYSID_WIDE (0: 1..15 tile columns, 1: 16..24) must be set"
#endif

// rows per staged chunk of the 10-tile-column narrow Gram (Spot, solo12): 24 (K2 0.1640 ms) against 16 / 32 / 40 / 48
// (0.1662 / 0.1650 / slower / slower; profiles/r04_s8, r03_l) and 20 / 28 (+0.5% / +1.2%, r04_final2); -D for A/B
// builds only
#ifndef SYSID_K2_KC10
#define SYSID_K2_KC10 24
#endif

namespace sysid_launch {
using namespace sysid_dev;

// f64 / f32 Gram kernels: LDS-DMA staged (three buffers) for wide Grams, register-staged for narrow ones
// (measured, 20k samples: G1 K2 1.81 -> 1.66 ms with the DMA kernel; Spot 0.202 -> 0.213 ms, so not there);
// the register-blocked kernels for 16..23 tile columns; the gathered rows of the nullspace mode go through the
// DMA / blocked kernels.  bf16: the blocked kernel, the transposed-read kernel (wide or gathered) or the
// register-staged one.
template <int PREC, int NTC, int KC>
void k2_case(const K2Args& a) {
  const dim3 g2(a.ngroups * a.ks), b2(64 * k2_waves(NTC));
  const bool gather = a.rowlist != nullptr;
  const int2* T = a.d_tiles;
  if constexpr (PREC == 0 || PREC == 1) {
    typedef std::conditional_t<PREC == 0, double, float> E;
    const E* P = static_cast<const E*>(a.panel);
    constexpr int DKC = (PREC == 0 ? 1 : 2) * k2_dma_kc(NTC);  // f32: twice the rows in the same LDS bytes
    if constexpr (k2b_supported(NTC)) {
      if (gather)
        hipLaunchKernelGGL((k2_gram_syrk_blk<E, NTC, true>), g2, dim3(512), 0, a.st, P, a.rows, a.ld_panel, a.ks,
                           a.nslots, a.accumulate, a.slab, a.rowlist, a.d_rows);
      else
        hipLaunchKernelGGL((k2_gram_syrk_blk<E, NTC>), g2, dim3(512), 0, a.st, P, a.rows, a.ld_panel, a.ks, a.nslots,
                           a.accumulate, a.slab, nullptr, nullptr);
    } else if constexpr (NTC >= 16) {
      if (gather)
        hipLaunchKernelGGL((k2_gram_syrk_dma<E, NTC, DKC, true>), g2, b2, 0, a.st, P, a.rows, a.ld_panel, T,
                           a.ngroups, a.ks, a.nslots, a.accumulate, a.slab, a.rowlist, a.d_rows);
      else
        hipLaunchKernelGGL((k2_gram_syrk_dma<E, NTC, DKC>), g2, b2, 0, a.st, P, a.rows, a.ld_panel, T, a.ngroups,
                           a.ks, a.nslots, a.accumulate, a.slab, nullptr, nullptr);
    } else if (gather) {
      constexpr int RKC = (PREC == 0 ? 1 : 2) * KC;
      hipLaunchKernelGGL((k2_gram_syrk_gather<E, NTC, RKC>), g2, b2, 0, a.st, P, a.rows, a.ld_panel, T, a.ngroups,
                         a.ks, a.nslots, a.accumulate, a.slab, a.rowlist, a.d_rows);
    } else {
      constexpr int RKC = (PREC == 0 ? 1 : 2) * KC;
      hipLaunchKernelGGL((k2_gram_syrk<E, NTC, RKC>), g2, b2, 0, a.st, P, a.rows, a.ld_panel, T, a.ngroups, a.ks,
                         a.nslots, a.accumulate, a.slab);
    }
  } else {
    const __bf16* P = static_cast<const __bf16*>(a.panel);
    const dim3 b16(64 * K2_BF16_WAVES);
    if constexpr (k2b_supported(NTC)) {
      if (gather)
        hipLaunchKernelGGL((k2_gram_syrk_bf16_blk<NTC, true>), g2, b16, 0, a.st, P, a.rows, a.ld_panel, a.ks,
                           a.nslots, a.accumulate, a.slab, a.rowlist, a.d_rows);
      else
        hipLaunchKernelGGL((k2_gram_syrk_bf16_blk<NTC>), g2, b16, 0, a.st, P, a.rows, a.ld_panel, a.ks, a.nslots,
                           a.accumulate, a.slab, nullptr, nullptr);
    } else if (gather) {
      hipLaunchKernelGGL((k2_gram_syrk_bf16_tr<NTC, k2_bf16_tr_kc(NTC), true>), g2, b16, 0, a.st, P, a.rows,
                         a.ld_panel, T, a.ngroups, a.ks, a.nslots, a.accumulate, a.slab, a.rowlist, a.d_rows);
    } else if constexpr (NTC >= 16) {
      hipLaunchKernelGGL((k2_gram_syrk_bf16_tr<NTC, k2_bf16_tr_kc(NTC)>), g2, b16, 0, a.st, P, a.rows, a.ld_panel, T,
                         a.ngroups, a.ks, a.nslots, a.accumulate, a.slab, nullptr, nullptr);
    } else {
      hipLaunchKernelGGL((k2_gram_syrk_bf16<NTC, k2_bf16_kc(NTC)>), g2, b16, 0, a.st, P, a.rows, a.ld_panel, T,
                         a.ngroups, a.ks, a.nslots, a.accumulate, a.slab);
    }
  }
}

template <int PREC, int WIDE>
bool k2_launch(const K2Args& a) {
#define SYSID_K2_CASE(NTC, KC) \
  case NTC:                    \
    k2_case<PREC, NTC, KC>(a); \
    return true;
  switch (a.ntc) {
#if SYSID_WIDE
    SYSID_K2_CASE(16, 12) SYSID_K2_CASE(17, 12) SYSID_K2_CASE(18, 12) SYSID_K2_CASE(19, 12) SYSID_K2_CASE(20, 12)
    SYSID_K2_CASE(21, 8) SYSID_K2_CASE(22, 8) SYSID_K2_CASE(23, 8) SYSID_K2_CASE(24, 8)
#else
    SYSID_K2_CASE(1, 32) SYSID_K2_CASE(2, 32) SYSID_K2_CASE(3, 32) SYSID_K2_CASE(4, 32) SYSID_K2_CASE(5, 32)
    SYSID_K2_CASE(6, 32) SYSID_K2_CASE(7, 32) SYSID_K2_CASE(8, 32) SYSID_K2_CASE(9, 32) SYSID_K2_CASE(10, SYSID_K2_KC10)
    SYSID_K2_CASE(11, 24) SYSID_K2_CASE(12, 24) SYSID_K2_CASE(13, 24) SYSID_K2_CASE(14, 20) SYSID_K2_CASE(15, 20)
#endif
    default: return false;
  }
#undef SYSID_K2_CASE
}

template bool k2_launch<SYSID_PREC, SYSID_WIDE>(const K2Args&);

}  // namespace sysid_launch
