// sysid_k1_inst.hip — K1 (k1_regressor_panel) instantiations of one panel element type and row mode.
// Built once per (SYSID_PREC, SYSID_CMP) by __graft_entry__.build(); see sysid_launch.h.
#define SYSID_TEMPLATE_TU 1
#include "sysid_launch.h"

#ifndef SYSID_PREC
#error "SYSID_PREC (0 f64, 1 f32, 2 bf16) must be set"
#endif
#ifndef SYSID_CMP
#error "SYSID_CMP (0 projector rows, 1 nullspace rows) must be set"
#endif

namespace sysid_launch {
namespace {
using namespace sysid_dev;
template <int PREC>
using Elem = std::conditional_t<PREC == 0, double, std::conditional_t<PREC == 1, float, __bf16>>;

// The layout forms that exist per row mode: the nullspace rows run the plain layout only.
template <typename OutT, int CMP, int MAXCH, int NVC, int SPW, int POV, int QF>
const void* fn() {
  if constexpr (CMP && (POV || QF))
    return nullptr;
  else
    return reinterpret_cast<const void*>(k1_regressor_panel<MAXCH, NVC, SPW, OutT, POV, CMP, QF>);
}

template <typename OutT, int CMP, int MAXCH, int NVC, int SPW, int POV, int QF>
void launch(dim3 g, dim3 b, size_t lds, hipStream_t st, const K1Params& kp, const uint32_t* mimg, const double* d_in,
            int64_t N, int64_t ld, void* d_panel, int64_t ld_panel, unsigned long long* work, double* dbg,
            int* rcount) {
  if constexpr (!(CMP && (POV || QF)))
    hipLaunchKernelGGL((k1_regressor_panel<MAXCH, NVC, SPW, OutT, POV, CMP, QF>), g, b, lds, st, kp, mimg, d_in, N,
                       ld, static_cast<OutT*>(d_panel), ld_panel, work, dbg, rcount);
}
}  // namespace

#define SYSID_K1_VARIANTS(X)                                                                                      \
  X(K1_C4_NV18, QCH, 18, SPW_QUAD, 0, 0)                                                                          \
  X(K1_C4, 4, 0, SPW_GEN, 0, 0)                                                                                   \
  X(K1_C12, 12, 0, SPW_GEN, 0, 0)                                                                                 \
  X(K1_C16, 16, 0, SPW_GEN, 0, 0)                                                                                 \
  X(K1_C12P, 12, 0, SPW_GEN, 1, 0)                                                                                \
  X(K1_C16P, 16, 0, SPW_GEN, 1, 0)                                                                                \
  X(K1_C4Q, 4, 0, SPW_GEN, 0, 1)                                                                                  \
  X(K1_C12Q, 12, 0, SPW_GEN, 0, 1)                                                                                \
  X(K1_C16Q, 16, 0, SPW_GEN, 0, 1)

template <int PREC, int CMP>
const void* k1_fn(int variant) {
#define SYSID_FN_CASE(V, MAXCH, NVC, SPW, POV, QF) \
  case V: return fn<Elem<PREC>, CMP, MAXCH, NVC, SPW, POV, QF>();
  switch (variant) {
    SYSID_K1_VARIANTS(SYSID_FN_CASE)
    default: return nullptr;
  }
#undef SYSID_FN_CASE
}

template <int PREC, int CMP>
void k1_launch(int variant, dim3 g, dim3 b, size_t lds, hipStream_t st, const K1Params& kp, const uint32_t* mimg,
               const double* d_in, int64_t N, int64_t ld, void* d_panel, int64_t ld_panel, unsigned long long* work,
               double* dbg, int* rcount) {
#define SYSID_LAUNCH_CASE(V, MAXCH, NVC, SPW, POV, QF)                                                      \
  case V:                                                                                                   \
    launch<Elem<PREC>, CMP, MAXCH, NVC, SPW, POV, QF>(g, b, lds, st, kp, mimg, d_in, N, ld, d_panel, ld_panel, work, \
                                                      dbg, rcount);                                                \
    break;
  switch (variant) {
    SYSID_K1_VARIANTS(SYSID_LAUNCH_CASE)
    default: break;
  }
#undef SYSID_LAUNCH_CASE
}

template const void* k1_fn<SYSID_PREC, SYSID_CMP>(int);
template void k1_launch<SYSID_PREC, SYSID_CMP>(int, dim3, dim3, size_t, hipStream_t, const K1Params&, const uint32_t*,
                                               const double*, int64_t, int64_t, void*, int64_t, unsigned long long*,
                                               double*, int*);

}  // namespace sysid_launch
