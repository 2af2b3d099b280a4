// sysid_launch.h — the K1 / K2 instantiation launchers.
//
// The kernel templates have ~120 instantiations (K1: chain slots x layout form x panel type; K2: Gram width x
// arithmetic x staging form).  They are compiled in parallel translation units instead of inside
// sysid_engine.hip: sysid_k1_inst.hip is built once per (panel type, row mode) and sysid_k2_inst.hip once per
// (Gram arithmetic, narrow / wide), each with SYSID_PREC / SYSID_CMP / SYSID_WIDE set on the compile line
// (__graft_entry__.build()).  The engine calls the explicit instantiations declared here.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sysid_kernels.h"

namespace sysid_launch {

// K1 instantiations: chain slots x compile-time nv x samples per wave.  Quadrupeds (nv = 18) run two
// samples per wave; anything else one, with nv read at run time (a compile-time nv = 35 for the humanoid
// ran 1.8x slower, its unrolled serial phases being heavier than the saved address arithmetic).
constexpr int SPW_QUAD = 2, SPW_GEN = 1;
// Chain slots of the nv = 18 kernel: the quadrupeds' legs are 3 revolute joints deep (3 measured 2% faster
// than 4 on Spot: no dead slot in the column phase).
constexpr int QCH = 3;
// ...P: the P-overlay layout (wave_layout pov); ...Q: the Q-form (at most K1_QF_KMAX contact rows, no P)
enum { K1_C4_NV18, K1_C4, K1_C12, K1_C16, K1_C12P, K1_C16P, K1_C4Q, K1_C12Q, K1_C16Q };

// PREC: panel element 0 = f64, 1 = f32, 2 = bf16; CMP: the nullspace rows (Gram-only).
// k1_fn: the kernel of a variant, for occupancy queries and attributes (nullptr: no such instantiation).
template <int PREC, int CMP>
const void* k1_fn(int variant);
template <int PREC, int CMP>
void k1_launch(int variant, dim3 g, dim3 b, size_t lds, hipStream_t st, const sysid_dev::K1Params& kp,
               const uint32_t* mimg, const double* d_in, int64_t N, int64_t ld, void* d_panel, int64_t ld_panel,
               unsigned long long* work, double* dbg, int* rcount);

// One K2 launch: the Gram's tile columns, the deal (super-tile / tile-slot table of the arithmetic), the split
// and the rows (gathered through rowlist / d_rows in the nullspace mode).
struct K2Args {
  int ntc;
  const int2* d_tiles;
  int ngroups, nslots, blk;
  const void* panel;
  int64_t rows, ld_panel;
  int ks, accumulate;
  double* slab;
  hipStream_t st;
  const int* rowlist;
  const int* d_rows;
};
// WIDE: Gram widths of 16..24 tile columns (else 1..15).  Returns false for a width outside the unit's range.
template <int PREC, int WIDE>
bool k2_launch(const K2Args& a);

}  // namespace sysid_launch
