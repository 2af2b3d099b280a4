// sysid_kernels.h — device code of the MI355X identification-regressor engine (gfx950, wave64).
//
// Included by sysid_engine.hip (every kernel) and by the instantiation units sysid_k1_inst.hip /
// sysid_k2_inst.hip (SYSID_TEMPLATE_TU: the templates only, one panel type each).  Kernels:
//   k1_regressor_panel  per sample: forward kinematics, contact Jacobian, projector P, projected
//                       regressor / friction / torque columns -> panel [Y_proj | B_v | B_c | tau_proj].
//                       One wave = one sample; a workgroup holds 4 independent waves; no workgroup
//                       barrier inside the sample loop (wave-synchronous LDS); persistent waves walk
//                       contiguous sample ranges with the next sample's inputs prefetched.
//   k2_gram_syrk        split-K SYRK of the panel on v_mfma_f64_16x16x4_f64 (upper 16x16 tiles),
//                       8 waves, register-staged double-buffered row chunks in LDS.
//   k3_gram_reduce      deterministic one-pass sum of the K2 slabs -> symmetric Gram.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

namespace sysid_dev {

constexpr int JT_FREEFLYER = 1;
constexpr int JT_REVOLUTE = 2;
constexpr int K1_WAVES = 4;            // waves (= samples in flight) per K1 workgroup
constexpr int K1_SHARDS = 8;           // K1 sample ranges / claim counters (one per XCD), 128 B apart

// ------------------------------------------------------------------------------------------------
// layouts shared by host and device
// ------------------------------------------------------------------------------------------------

// Compact model image kept in LDS by every K1 workgroup.  Int section offsets are in 4-byte words,
// double section offsets in doubles from the image start.
struct MImg {
  int parent, jtype, idx_q, idx_v, depth, chain_len, chain, anc, dof_joint, dof_k, cjoint, csupp, nint;
  int axis, R0, t0, ct, ndbl;
};

__host__ __device__ inline MImg mimg_layout(int NJ, int nv, int nc, int maxch) {
  MImg m;
  int o = 0;
  m.parent = o; o += NJ;
  m.jtype = o; o += NJ;
  m.idx_q = o; o += NJ;
  m.idx_v = o; o += NJ;
  m.depth = o; o += NJ;
  m.chain_len = o; o += NJ;
  m.chain = o; o += NJ * maxch;
  m.anc = o; o += NJ * maxch;  // the joints of `chain` (dof_joint of each entry): the chain products' placements
  m.dof_joint = o; o += nv;
  m.dof_k = o; o += nv;
  m.cjoint = o; o += nc;
  o = (o + 1) & ~1;
  m.csupp = o; o += 2 * nc;
  m.nint = o;
  int d = o / 2;
  m.axis = d; d += 3 * NJ;
  m.R0 = d; d += 9 * NJ;
  m.t0 = d; d += 3 * NJ;
  m.ct = d; d += 3 * nc;
  m.ndbl = (d + 1) & ~1;  // image size in doubles (16-B aligned)
  return m;
}

// Row groups of K1's regressor-column phase: lanes = bodies x row groups, one pass of a sample's lanes.
__host__ __device__ inline int k1_row_groups(int NJ, int lanes) {
  const int nb = NJ - 1 > 0 ? NJ - 1 : 1;
  return lanes / nb > 1 ? lanes / nb : 1;
}

// Joint records in LDS are padded to 26 doubles (52 dwords): the 24-double stride put bodies i and i+4 on
// the same LDS banks (4-way conflicts when the lanes of the column phase read 13 different bodies).
constexpr int BODY_STRIDE = 26;

// Per-wave LDS region of K1 (doubles, every piece 16-B aligned).  The projector's working set
// D = [J_c | M | W,Pt,pf / Z] is dead once P is built, and holds its results too:
//   * H1 over J_c (stored after the tau column, which reads J_c in the full mode), or after everything
//     when J_c's slot is smaller;
//   * with `hw` > 0 (lanes per sample of a compile-time-nv kernel) P ends inside Z's slot: P is built
//     row-major, `hw` entries per wave pass, row a from Z row a (Z is stored transposed, stride 3 nc), so
//     a pass may overwrite the Z rows the passes before it consumed; P starts `margin` doubles before Z,
//     the largest lead of the written entries over the consumed Z rows (over M, dead after Z is built).
//     Spot: 1,582 -> 1,158 doubles per sample, so 8 two-sample waves share a CU's 160 KB (was 6).
//   * otherwise P follows D, or, with `pov` (P overlay, runtime-nv kernels whose H1 is read from P), P starts
//     at D and D's working set moves to the tail of P's slot: the P pass buffers the entries that land on it
//     in registers until every entry has been computed (K1_POV_BUF passes at most).  G1: 2,916 -> 2,452
//     doubles per sample, so one workgroup of 8 one-sample waves fits a CU's 160 KB (was 3 x 2 waves).
constexpr int K1_POV_BUF = 12;  // P passes (of 64 entries) a P overlay may hold in registers
// The bf16 Q-form's f32 row operands, by row pairs (rows 2p, 2p + 1 at 28 p floats): Q entries interleaved
// (2 j + (r & 1): Q_j of row r, zero past the sample's rows), then the motion axes as [J_r[0], J_r[1], J_r1[0], J_r1[1],
// J_r[3], J_r[4], J_r1[3], J_r1[4], J_r[2], J_r1[2], J_r[5], J_r1[5]] (r1 = r + 1), so a lane's operands of a pair are a
// few aligned 16- and 8-byte reads already in packed-FMA order.  One pair past the last is readable (the row loop's
// operand prefetch).
__host__ __device__ constexpr int k1q32_pairs(int nv) { return (nv + 1) / 2 + 1; }
__host__ __device__ constexpr int k1q32_doubles(int nv) { return k1q32_pairs(nv) * 14; }
struct WLay {
  int in, body, W, Pt, Jw, pf, Jc, M, P, H1, tp, dqs, Z, q32, total;
};

//   * with `nop` (the Q-form kernels, which never form P) there is no P slot at all.
__host__ __device__ inline WLay wave_layout(int in_rows, int nv, int NJ, int nc, int hw, int pov = 0, int nop = 0) {
  WLay l;
  const int k = 3 * nc;
  int o = 0;
  auto r2 = [](int n) { return (n + 1) & ~1; };
  auto take = [&](int n) { const int r = o; o += r2(n); return r; };
  auto grow = [&](int end) { if (o < end) o = end; };
  l.in = take(in_rows);
  l.body = take(NJ * BODY_STRIDE);  // per joint: oR(9) ot(3) v(6) a_gf(6), padded
  l.Jw = take(nv * 6);          // spatial axis of every dof [linear at origin; angular]
  l.tp = take(nv);              // P S^T tau
  l.dqs = take(nv);             // dq for the friction columns (`in` takes the next sample's inputs mid-step)
  const int D = o;
  l.Jc = take(k * nv);          // J_c
  int margin = 0;
  if (hw > 0)
    for (int E = hw; E < nv * nv; E += hw) {
      const int lead = E - k * (E / nv);
      if (lead > margin) margin = lead;
    }
  l.M = take(k * k);            // row norms of the Gram-Schmidt pass (k used)
  grow(l.M + r2(margin));
  const int u0 = o;
  l.W = take(nv * 3);           // direction of every dof's motion axis
  l.Pt = take(nv * 3);          // a point on it
  l.pf = take(nc * 3);          // contact points
  l.Z = u0;                     // Q^T (orthonormal rows of J_c's row space), row r at r * 3 nc (W, Pt, pf
                                // are dead by then)
  grow(u0 + r2(k * nv > k * k ? k * nv : k * k));
  l.q32 = 0;
  if (nop) {
    l.P = l.Jc;                 // unused
    l.H1 = D;                   // unused
    // f32 copies of every row's Q entries (8, zero past k) and motion axis (6) for the bf16 row loop: converted
    // once per sample instead of by every lane on every row
    l.q32 = take(k1q32_doubles(nv));
    l.total = o;
    return l;
  }
  if (hw > 0) {
    l.P = u0 - r2(margin);      // P = I - Q^T Q
    grow(l.P + r2(nv * nv));
  } else if (pov) {
    // D's working set [Jc .. end) moves to the tail of P's slot [D, D + r2(nv nv)) (the caller checked it fits)
    const int shift = r2(nv * nv) - (o - D);
    l.Jc += shift; l.M += shift; l.W += shift; l.Pt += shift; l.pf += shift; l.Z += shift;
    l.P = D;
    l.H1 = D;  // unused: H1 is read from P's free-flyer columns
    l.total = D + r2(nv * nv);
    return l;
  } else {
    l.P = take(nv * nv);
  }
  l.H1 = r2(nv * 6) <= r2(k * nv) ? D : take(nv * 6);  // P[:, ff] J_w[:, ff]^T
  l.total = o;
  return l;
}

struct K1Params {
  int nq, nv, NJ, nc, bd, nj, maxdepth, wy, w, ncol, in_rows, maxch, has_ff, ff0, mimg_dbl, wave_dbl;
  int out_cols;     // columns written per panel row (ncol rounded up to the panel's even stride)
  int in_lds;       // input channels the LDS layout holds (in_rows of the full-force mode)
  int full;         // 1: get_full_regressor_force mode (P = I, tau column = S^T tau + J_c^T lambda)
  int rg;           // row groups of the regressor-column phase (lanes = bodies x rg)
  int pov;          // 1: P overlays the projector's working set (wave_layout `pov`)
  double thr_rel;   // rank cut of the projector: remaining row norm <= thr_rel * the largest row norm
  double thr_rel2;  // thr_rel^2, formed on the host (a kernel argument stays in SGPRs; the product hoisted out of the
                    // sample loop took a VGPR pair, which the register-bound kernels spilled)
  double g0, g1, g2;  // gravity (a_gf[0] = -gravity)
};
constexpr int K1_QUAD_IN_MAX = 96;  // input channels of the quadruped K1 (nv = 18, two samples per wave)

// Start of claim shard x of N samples: multiples of 16 samples (one 128-byte line of a channel row), so with a
// 16-sample-aligned row pitch no line of the input block spans two shards.
__host__ __device__ inline int64_t k1_shard_begin(int64_t N, int x) {
  return x >= K1_SHARDS ? N : (N * x / K1_SHARDS) / 16 * 16;
}

// ------------------------------------------------------------------------------------------------
// small helpers (host+device so the CPU test-suite can exercise the same code)
// ------------------------------------------------------------------------------------------------
__host__ __device__ inline void mat3mul(const double* A, const double* B, double* C) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

__host__ __device__ inline void mat3vec(const double* A, const double* x, double* y) {
#pragma unroll
  for (int i = 0; i < 3; ++i) y[i] = A[3 * i] * x[0] + A[3 * i + 1] * x[1] + A[3 * i + 2] * x[2];
}

__host__ __device__ inline void mat3tvec(const double* A, const double* x, double* y) {
#pragma unroll
  for (int i = 0; i < 3; ++i) y[i] = A[i] * x[0] + A[3 + i] * x[1] + A[6 + i] * x[2];
}

__host__ __device__ inline void cross3(const double* a, const double* b, double* c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}

// SE3(R, t).actInv(motion m = [v; w])
__host__ __device__ inline void act_inv_motion(const double* R, const double* t, const double* m, double* out) {
  double tw[3], d[3];
  cross3(t, m + 3, tw);
  d[0] = m[0] - tw[0];
  d[1] = m[1] - tw[1];
  d[2] = m[2] - tw[2];
  mat3tvec(R, d, out);
  mat3tvec(R, m + 3, out + 3);
}

// Rotation about a unit axis; pinocchio's RX/RY/RZ closed forms for the aligned axes.
__device__ inline void axis_rotation(const double* a, double ang, double* R) {
  double s, c;
  sincos(ang, &s, &c);
  if (a[0] == 1.0 && a[1] == 0.0 && a[2] == 0.0) {
    R[0] = 1; R[1] = 0; R[2] = 0; R[3] = 0; R[4] = c; R[5] = -s; R[6] = 0; R[7] = s; R[8] = c;
  } else if (a[0] == 0.0 && a[1] == 1.0 && a[2] == 0.0) {
    R[0] = c; R[1] = 0; R[2] = s; R[3] = 0; R[4] = 1; R[5] = 0; R[6] = -s; R[7] = 0; R[8] = c;
  } else if (a[0] == 0.0 && a[1] == 0.0 && a[2] == 1.0) {
    R[0] = c; R[1] = -s; R[2] = 0; R[3] = s; R[4] = c; R[5] = 0; R[6] = 0; R[7] = 0; R[8] = 1;
  } else {
    const double C = 1.0 - c;
    const double x = a[0], y = a[1], z = a[2];
    R[0] = 1.0 + C * (x * x - 1.0); R[1] = -s * z + C * x * y;      R[2] = s * y + C * x * z;
    R[3] = s * z + C * x * y;       R[4] = 1.0 + C * (y * y - 1.0); R[5] = -s * x + C * y * z;
    R[6] = -s * y + C * x * z;      R[7] = s * x + C * y * z;       R[8] = 1.0 + C * (z * z - 1.0);
  }
}

// Eigen Quaternion::toRotationMatrix (no normalisation), q = (x, y, z, w).
__device__ inline void quat_to_matrix(double x, double y, double z, double w, double* R) {
  const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w;
  const double txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;         R[2] = txz + twy;
  R[3] = txy + twz;         R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy;         R[7] = tyz + twx;         R[8] = 1.0 - (txx + tyy);
}

__device__ inline double sign_of(double x) {
  return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : (x == x ? 0.0 : x));
}


// Wave-level ordering point for LDS traffic.  The LDS executes one wave's DS instructions in issue
// order, so a store by one lane is seen by a later load of any lane of the same wave; this only stops
// the compiler from moving memory operations across the point.
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// 1/sqrt(x) for x > 0: the hardware estimate refined by two Newton steps (~1 ulp; no division).
__device__ __forceinline__ double rsqrt_f64(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  y = y * (1.5 - h * y * y);
  y = y * (1.5 - h * y * y);
  return y;
}

// v + v of another lane, by a DPP lane pattern on both halves of the double (the partner lane must be
// active: callers keep whole lane groups together).
template <int CTRL>
__device__ __forceinline__ double dpp_add(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
  return v + __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double pair_sum(double v) { return dpp_add<0xB1>(v); }  // quad_perm [1,0,3,2]
// v of the partner lane (lane ^ 1)
__device__ __forceinline__ double pair_swap(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, 0xB1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0xB1, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Sum over an aligned group of `lpr` lanes (1, 2, 4 or 8; uniform over the group): lane ^ 1, lane ^ 2,
// then the half-row mirror (lane i <-> 7 - i pairs the two quads of an 8-lane group).
__device__ __forceinline__ double group_sum(double v, int lpr) {
  if (lpr >= 2) v = dpp_add<0xB1>(v);
  if (lpr >= 4) v = dpp_add<0x4E>(v);   // quad_perm [2,3,0,1]
  if (lpr >= 8) v = dpp_add<0x141>(v);  // row_half_mirror
  return v;
}

// v of lane `lane` (a wave-uniform index) in every lane.
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// |x|^2 of a row of nv doubles (three partial sums).
template <int NVC>
__device__ __forceinline__ double mgs_sqnorm(const double* x, int nv_rt) {
  const int nv = NVC > 0 ? NVC : nv_rt;
  double a[3] = {0.0, 0.0, 0.0};
#pragma unroll 6
  for (int r = 0; r < nv; ++r) a[r % 3] += x[r] * x[r];
  return (a[0] + a[1]) + a[2];
}

// One Gram-Schmidt step on a row x still in play, against the pivot row xp (q = xp / |xp|, inv2 =
// 1 / |xp|^2): x -= ((xp . x) inv2) xp = (q . x) q.  Returns x's new squared norm (recomputed, not
// downdated: the rank cut needs the small ones accurate).  The pivot row itself is not touched (its
// lane skips the step), so no load of xp can see a store of the pass.
// Runtime nv: a group of lpr lanes per row, lane h of the group taking entries h, h + lpr, ...; the dot
// product and the norm are completed across the group.  All lanes of the group return the new norm.
__device__ __forceinline__ double mgs_step_group(const double* xp, double* x, double inv2, int nv, int h, int lpr) {
  double c0 = 0.0, c1 = 0.0;
  for (int r = h; r < nv; r += 2 * lpr) {
    c0 += xp[r] * x[r];
    if (r + lpr < nv) c1 += xp[r + lpr] * x[r + lpr];
  }
  const double c = group_sum(c0 + c1, lpr) * inv2;
  double a0 = 0.0, a1 = 0.0;
  for (int r = h; r < nv; r += 2 * lpr) {
    const double v0 = x[r] - c * xp[r];
    x[r] = v0;
    a0 += v0 * v0;
    if (r + lpr < nv) {
      const double v1 = x[r + lpr] - c * xp[r + lpr];
      x[r + lpr] = v1;
      a1 += v1 * v1;
    }
  }
  return group_sum(a0 + a1, lpr);
}

// Compile-time nv = NVC: two lanes per row (lane pair 2j, 2j+1 takes entries [0, H) and [H, NVC) of
// row j, H = NVC/2 rounded up to even so both halves start 16-byte aligned); the dot product and the norm
// are completed across the pair with DPP.  Both lanes of a pair return the row's new squared norm.
template <int NVC>
__device__ __forceinline__ double mgs_step_pair(const double* xp, double* x, double inv2, int h) {
  constexpr int H = ((NVC + 1) / 2 + 1) & ~1;
  constexpr int H2 = H / 2;
  const double2* xp2 = reinterpret_cast<const double2*>(xp + h * H);
  double2* x2 = reinterpret_cast<double2*>(x + h * H);
  const int n2 = h == 0 ? H2 : (NVC - H) / 2;  // double2 entries of this lane's half (NVC even)
  double2 pv[H2], xv[H2];
#pragma unroll
  for (int u = 0; u < H2; ++u) {
    pv[u] = u < n2 ? xp2[u] : make_double2(0.0, 0.0);
    xv[u] = u < n2 ? x2[u] : make_double2(0.0, 0.0);
  }
  double c0 = 0.0, c1 = 0.0;
#pragma unroll
  for (int u = 0; u < H2; ++u) {
    c0 += pv[u].x * xv[u].x;
    c1 += pv[u].y * xv[u].y;
  }
  const double c = pair_sum(c0 + c1) * inv2;
  double a0 = 0.0, a1 = 0.0;
#pragma unroll
  for (int u = 0; u < H2; ++u) {
    xv[u].x -= c * pv[u].x;
    xv[u].y -= c * pv[u].y;
    a0 += xv[u].x * xv[u].x;
    a1 += xv[u].y * xv[u].y;
    if (u < n2) x2[u] = xv[u];
  }
  return pair_sum(a0 + a1);
}

// Panel stores (plain: non-temporal stores measured equal on Spot and 2.5x slower K1 on G1).  Two adjacent
// columns per store, in the panel's element type: f64 (the reference's outputs and the parity Gram) or, for
// the Gram-only chunk panel of a reduced-precision Gram, f32 / bf16 — rounded once
// here, so the Gram kernel stages 2x / 4x fewer bytes than from an f64 panel.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef double dbl4 __attribute__((ext_vector_type(4)));  // MFMA accumulators and fragments
typedef float flt4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void panel_store(double* p, double a, double b) {
  *reinterpret_cast<double2*>(p) = make_double2(a, b);
}
__device__ __forceinline__ void panel_store(float* p, double a, double b) {
  *reinterpret_cast<float2*>(p) = make_float2((float)a, (float)b);
}
__device__ __forceinline__ void panel_store(__bf16* p, double a, double b) {
  // RNE to f32, then RNE to bf16 (v_cvt_pk_bf16_f32).  The empty asm keeps the f32 values: without it the two
  // truncations fold into one f64 -> bf16 rounding, which the compiler emulates with a round-to-odd sequence
  // of ~10 VALU per value (G1's Q-form K1: ~1.7k VALU per sample)
  float fa = (float)a, fb = (float)b;
  asm volatile("" : "+v"(fa), "+v"(fb));
  bf16x2_t v;
  v[0] = (__bf16)fa;
  v[1] = (__bf16)fb;
  *reinterpret_cast<bf16x2_t*>(p) = v;
}
// bf16 store of two f32 values (the f32 row loop of the Q-form, below): one RNE conversion each
__device__ __forceinline__ void panel_store_f32(__bf16* p, float a, float b) {
  bf16x2_t v;
  v[0] = (__bf16)a;
  v[1] = (__bf16)b;
  *reinterpret_cast<bf16x2_t*>(p) = v;
}
// one column (the odd column of a lane's inertia triple in the f64 / f32 Q-form)
__device__ __forceinline__ void panel_store1(double* p, double a) { *p = a; }
__device__ __forceinline__ void panel_store1(float* p, double a) { *p = (float)a; }
typedef float f32x2_t __attribute__((ext_vector_type(2)));
// v of the partner lane (lane ^ 1), f32
__device__ __forceinline__ float pair_swap_f32(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}


// Columns 0..3 (m, mc) of the block: F[6c .. 6c+5] = [linear; angular] of column c.
__host__ __device__ inline void body_block_mass(const double* bi, double* F) {
  const double* R = bi;
  const double* t = bi + 9;
  const double* v = bi + 12;
  const double* w = bi + 15;
  const double* a = bi + 18;
  const double* dw = bi + 21;
  double ac[3], tmp[3];
  cross3(w, v, tmp);
  ac[0] = a[0] + tmp[0]; ac[1] = a[1] + tmp[1]; ac[2] = a[2] + tmp[2];
  // column 0 (mass): f = ac, n = 0
  {
    double Rf[3];
    mat3vec(R, ac, Rf);
    F[0] = Rf[0]; F[1] = Rf[1]; F[2] = Rf[2];
    cross3(t, Rf, F + 3);
  }
  // columns 1..3 (first moment e_k): f = dw x e + w x (w x e), n = e x ac
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double e[3] = {k == 0 ? 1.0 : 0.0, k == 1 ? 1.0 : 0.0, k == 2 ? 1.0 : 0.0};
    double x1[3], x2[3], x3[3], f[3], n[3], Rf[3], Rn[3], tf[3];
    cross3(dw, e, x1);
    cross3(w, e, x2);
    cross3(w, x2, x3);
    f[0] = x1[0] + x3[0]; f[1] = x1[1] + x3[1]; f[2] = x1[2] + x3[2];
    cross3(e, ac, n);
    mat3vec(R, f, Rf);
    mat3vec(R, n, Rn);
    cross3(t, Rf, tf);
    double* c = F + 6 * (k + 1);
    c[0] = Rf[0]; c[1] = Rf[1]; c[2] = Rf[2];
    c[3] = Rn[0] + tf[0]; c[4] = Rn[1] + tf[1]; c[5] = Rn[2] + tf[2];
  }
}

// Columns 4..9 (Ixx, Ixy, Iyy, Ixz, Iyz, Izz): f = 0, n = I dw + w x (I w); F[3q .. 3q+2] = angular part.
__host__ __device__ inline void body_block_inertia(const double* bi, double* F) {
  const double* R = bi;
  const double* w = bi + 15;
  const double* dw = bi + 21;
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const double s0 = q == 0, s1 = q == 1, s2 = q == 2, s3 = q == 3, s4 = q == 4, s5 = q == 5;
    double bdw[3], bw[3], x[3], n[3];
    bdw[0] = s0 * dw[0] + s1 * dw[1] + s3 * dw[2];
    bdw[1] = s1 * dw[0] + s2 * dw[1] + s4 * dw[2];
    bdw[2] = s3 * dw[0] + s4 * dw[1] + s5 * dw[2];
    bw[0] = s0 * w[0] + s1 * w[1] + s3 * w[2];
    bw[1] = s1 * w[0] + s2 * w[1] + s4 * w[2];
    bw[2] = s3 * w[0] + s4 * w[1] + s5 * w[2];
    cross3(w, bw, x);
    n[0] = bdw[0] + x[0]; n[1] = bdw[1] + x[1]; n[2] = bdw[2] + x[2];
    mat3vec(R, n, F + 3 * q);
  }
}

// All ten columns of pinocchio's bodyRegressor for body i, moved to the free-flyer frame, in a compact
// layout: columns 0..3 (m, mc) as [linear(3); angular(3)] in F[0..23]; columns 4..9 (inertia) have a
// zero force part, only their angular rows are kept in F[24..41].  bi = {oR(9), ot(3), v(6), a_gf(6)}.
constexpr int FBLK = 42;

__host__ __device__ inline void body_regressor_block(const double* bi, double* F) {
  body_block_mass(bi, F);
  body_block_inertia(bi, F + 24);
}

// Column p of the block as a 6-vector [linear; angular] (diagnostics and tests).
__host__ __device__ inline void block_column(const double* F, int p, double* fw) {
  if (p < 4) {
    for (int k = 0; k < 6; ++k) fw[k] = F[6 * p + k];
  } else {
    fw[0] = fw[1] = fw[2] = 0.0;
    for (int k = 0; k < 3; ++k) fw[3 + k] = F[24 + 3 * (p - 4) + k];
  }
}

// ------------------------------------------------------------------------------------------------
// K1
// ------------------------------------------------------------------------------------------------
// MAXCH: chain-slot count (>= longest revolute chain).  NVC: nv fixed at compile time (0 = read it
// from K1Params), so the row loops of the common robots unroll with immediate LDS offsets.
// SPW: samples per wave (1 or 2).  With SPW > 1 each 64/SPW-lane slice of the wave carries its own
// sample through every phase, so the lane-starved serial phases (forward pass, Gram-Schmidt steps) do SPW
// samples per instruction; each slice has its own LDS region.
// CMP: Gram-only nullspace mode (north_star "batched QR/nullspace"): instead of P·A (nv rows
// per sample) the sample emits Zᵀ·A, m = nv - rank(J_c) rows, with Zᵀ ((m x nv), orthonormal rows, ZᵀZ = P)
// completed from the Gram-Schmidt basis Q by Householder reconstruction (tests/alg_mirror.py nullspace_rows):
// Σ (ZᵀA)ᵀ(ZᵀA) = Σ AᵀPA = Σ (PA)ᵀ(PA), the same Gram from fewer rows.  Sample s keeps its rows at
// [s·nv, s·nv + m) of the chunk panel and records m in rcount[s], from which k1s_seg_sums / k1s_row_list build
// the list of live rows the Gram kernels gather.
constexpr int K1_SEG_LOG = 10;  // samples per row-count segment of the CMP mode (1024)
constexpr int K1S_ONEPASS_SEGS = 32;  // up to this many segments k1s_row_list sums the earlier counts itself
constexpr int K1_CMP_KMAX = 12;
  // CMP mode: at most 12 contact rows (4 contact frames; the host checks)
// QF: the Q-form of the runtime-nv kernel for at most K1_QF_KMAX contact rows (G1: 6): P = I - QᵀQ is never
// formed; the column phases use G_i[r] = [r in S_i] J_r - Σ_j Q_j[r] K_ij with K_ij = Σ_{d in S_i} Q_j[d] J_d
// (S_i: the free-flyer and chain dofs of body i), k reads per row instead of a chain of P entries and axes.
constexpr int K1_QF_KMAX = 6;
// Register-resident Gram-Schmidt of the runtime-nv kernels: at most 8 rows (one 8-lane group each) of nv <= 8 x
// K1_MGS_NU entries (G1: 35); larger models take the LDS form (mgs_lds)
constexpr int K1_MGS_NU = 5;
// K1's per-wave body (k1_regressor_panel): samples claimed from device counters.
template <int MAXCH, int NVC, int SPW, typename OutT, int POV = 0, int CMP = 0, int QF = 0>
__device__ __forceinline__ void k1_body(const K1Params& kp, const uint32_t* __restrict__ mimg_g,
                                        const double* __restrict__ in, int64_t N, int64_t ld,
                                        OutT* __restrict__ panel, int64_t ldp, unsigned long long* __restrict__ work,
                                        double* __restrict__ dbg, int* __restrict__ rcount) {
  static_assert(!(POV && CMP), "the nullspace mode runs the plain layout");
  static_assert(!QF || (NVC == 0 && !POV && !CMP), "the Q-form is a runtime-nv, plain-layout kernel");
  extern __shared__ double smem[];
  const MImg MI = mimg_layout(kp.NJ, kp.nv, kp.nc, kp.maxch);
  {
    uint32_t* mw = reinterpret_cast<uint32_t*>(smem);
    for (int x = threadIdx.x; x < 2 * kp.mimg_dbl; x += blockDim.x) mw[x] = mimg_g[x];
    __syncthreads();  // the only workgroup barrier: the model image is read-only from here on
  }

  const int* mi = reinterpret_cast<const int*>(smem);
  const int* parent = mi + MI.parent;
  const int* jtype = mi + MI.jtype;
  const int* idx_q = mi + MI.idx_q;
  const int* idx_v = mi + MI.idx_v;
  const int* depth = mi + MI.depth;
  const int* chain_len = mi + MI.chain_len;
  const int* chain = mi + MI.chain;
  const int* anc = mi + MI.anc;
  const int* dof_joint = mi + MI.dof_joint;
  const int* dof_k = mi + MI.dof_k;
  const int* cjoint = mi + MI.cjoint;
  const unsigned long long* csupp = reinterpret_cast<const unsigned long long*>(mi + MI.csupp);
  const double* axis = smem + MI.axis;
  const double* R0 = smem + MI.R0;
  const double* t0 = smem + MI.t0;
  const double* ct = smem + MI.ct;

  const int nv = NVC > 0 ? NVC : kp.nv;
  // the quadruped kernel carries no full-force mode (the engine runs that mode on the K1_C4 instantiation): its dead
  // paths cost the kernel registers (SGPR spills) and code
  const int kfull = NVC == 18 ? 0 : kp.full;
  const int nq = kp.nq, nc = kp.nc, NJ = kp.NJ, bd = kp.bd, nja = kp.nj, IN = kp.in_rows;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  static_assert(SPW == 1 || SPW == 2, "1 or 2 samples per wave (4 measured 34% slower)");
  constexpr bool OPQ = true;               // opaque per-sample lane index / LDS pointers (top of the loop)
  constexpr bool CHAIN_UNCOND = NVC == 18;  // unconditional chain loads in the column phase
  constexpr int HW = 64 / SPW;                       // lanes per sample
  const int half = lane / HW, hl = lane % HW;         // sample slot within the wave, lane within it
  static_assert(POV == 0 || NVC == 0, "the P overlay is a runtime-nv layout");
  const WLay L = wave_layout(kp.in_lds, nv, NJ, nc, NVC > 0 ? HW : 0, POV, QF);
  double* wr = smem + kp.mimg_dbl + (wave * SPW + half) * kp.wave_dbl;
  double* body = wr + L.body;
  double* Ws = wr + L.W;
  double* Pts = wr + L.Pt;
  double* Jws = wr + L.Jw;
  double* pfs = wr + L.pf;
  double* Jc = wr + L.Jc;
  double* Ms = wr + L.M;
  double* Ps = wr + L.P;
  double* H1 = wr + L.H1;
  double* Qt = wr + L.Z;  // Q-form: Q transposed, K1_QF_KMAX entries per row (over W / Pt / pf)
  double* tps = wr + L.tp;
  double* dqs = wr + L.dqs;

  // Samples are handed out SPW at a time from device counters, so a workgroup that becomes resident late,
  // or a slow CU, only ever costs its own last samples.  The next ones are claimed one step ahead and their
  // inputs prefetched into registers (channel c -> lane c, c+HW, ...) while the current ones run.  The
  // counters live in the launch's workspace and are zeroed on the launch stream right before the launch
  // (host side), so no state carries over from one launch to the next.
  // Sharded: one returning atomic on a single word serialises at ~88 per microsecond chip-wide (Spot 20k
  // = 10,000 claims ~ 114 us: most of K1's time; measured with every phase compiled out, 0.155 of 0.236 ms).
  // The samples are split into K1_SHARDS contiguous ranges with a counter each (128 B apart); a wave claims
  // from the range of its own XCD first (HW_REG_XCC_ID: speed only, never correctness), then from the others
  // in turn, skipping an exhausted range after one plain (relaxed, agent-scope) read of its counter.
  // The prefetch and the claim are issued at the top of a step and consumed in its middle (after the
  // projector): vmcnt retires in issue order, so consuming them at the top of the next step would first
  // wait for all of this step's panel stores.
  const int home = (int)(__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & (K1_SHARDS - 1));  // XCC_ID
  auto shard_begin = [&](int x) -> int64_t { return k1_shard_begin(N, x); };
  int sh = 0;  // shards (counted from home) found exhausted by this wave
  auto claim_issue = [&]() -> unsigned long long {
    unsigned long long v = 0;
    if (lane == 0) {
      // an opaque (per-lane) offset keeps the atomic optimizer from rewriting the claim as a wave scan,
      // which reads the returned value (and waits for it) right at the atomic
      int z = 16 * ((home + sh) & (K1_SHARDS - 1));
      asm volatile("" : "+v"(z));
      v = atomicAdd(work + z, (unsigned long long)SPW);
    }
    return v;
  };
  auto uniform64 = [&](unsigned long long v) -> unsigned long long {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
  };
  // the sample of a claim issued on the current shard, or (that shard exhausted) the next claim that succeeds
  // on the following shards, or N when every shard is exhausted
  auto claim_value = [&](unsigned long long raw) -> int64_t {
    unsigned long long v = uniform64(raw);
    bool have = true;  // v is a claim on shard (home + sh)
    while (sh < K1_SHARDS) {
      const int x = (home + sh) & (K1_SHARDS - 1);
      const int64_t b = shard_begin(x), e = shard_begin(x + 1);
      if (have && b + (int64_t)v < e) return b + (int64_t)v;
      ++sh;
      if (sh >= K1_SHARDS) break;
      const int y = (home + sh) & (K1_SHARDS - 1);
      unsigned long long seen = 0;
      if (lane == 0) seen = __hip_atomic_load(work + 16 * y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      have = (int64_t)uniform64(seen) < shard_begin(y + 1) - shard_begin(y);  // else exhausted: no claim
      if (have) v = uniform64(claim_issue());
    }
    return N;
  };
  // input registers per lane: <= 192 channels, the quadruped kernel <= K1_QUAD_IN_MAX (host-checked, k1_variant:
  // its 6 prefetch registers for 192 had held 6 dead VGPRs across every step of a 71-channel Spot sample)
  constexpr int NXR = ((NVC == 18 && HW == 32 ? K1_QUAD_IN_MAX : 192) + HW - 1) / HW;
  double xr[NXR];
#pragma unroll
  for (int u = 0; u < NXR; ++u) xr[u] = 0.0;
  auto fetch = [&](int64_t s) {  // s = the step's first sample; this half's is s + half
    const int64_t sh = s + half;
    // channel c of the sample at in[ib + c·is] (the row-major block: ib = sh, is = ld)
    const int64_t ib = sh, is = ld;
    // the lane's channel offsets are recomputed per step (opaque lane index): hoisted out of the sample loop they are
    // NXR 64-bit addresses live across every phase, and at the register limit the allocator spilled them (a scratch
    // reload and its vmcnt(0) wait for every earlier store, once per step)
    int hc = hl;
    asm volatile("" : "+v"(hc));
#pragma unroll
    for (int u = 0; u < NXR; ++u)
      if (hc + HW * u < IN && sh < N) xr[u] = in[(int64_t)(hc + HW * u) * is + ib];
  };
  double* sin_ = wr + L.in;
  const double* q = sin_;
  const double* dq = sin_ + nq;
  const double* ddq = dq + nv;
  const double* tau = ddq + nv;
  const double* cnt = tau + nja;

  auto commit = [&]() {
#pragma unroll
    for (int u = 0; u < NXR; ++u)
      if (hl + HW * u < IN) sin_[hl + HW * u] = xr[u];
  };

  int64_t s = claim_value(claim_issue());
  if (s < N) {
    fetch(s);
    commit();
  }
  int64_t s1 = s < N ? claim_value(claim_issue()) : N;
  // issue priority: the column phase runs at 0, everything else at 2, so a wave in a latency-bound phase
  // issues first when its operands arrive (K1 -1 to -2%, Spot and G1)
  __builtin_amdgcn_s_setprio(2);
  const int hl_outer = hl;
  while (s < N) {
    // Quadruped variant (OPQ): the lane index and the per-sample LDS region are re-derived opaquely every
    // step, so the per-lane index arithmetic of the phase loops (nv is a compile-time constant) and the
    // pointers into the region are recomputed per step instead of being hoisted out of the sample loop
    // into hundreds of live registers (Spot K1 -3%).  Elsewhere these are plain loop invariants.
    int hl = hl_outer;
    int woff = (wave * SPW + half) * kp.wave_dbl;
    if constexpr (OPQ) {
      asm volatile("" : "+v"(hl));
      asm volatile("" : "+v"(woff));
    }
    double* wr = smem + kp.mimg_dbl + woff;
    double* body = wr + L.body;
    double* Ws = wr + L.W;
    double* Pts = wr + L.Pt;
    double* Jws = wr + L.Jw;
    double* pfs = wr + L.pf;
    double* Jc = wr + L.Jc;
    double* Ms = wr + L.M;
    double* Ps = wr + L.P;
    double* H1 = wr + L.H1;
    double* Qt = wr + L.Z;
    double* tps = wr + L.tp;
    double* dqs = wr + L.dqs;
    const double* q = wr + L.in;
    const double* dq = q + nq;
    const double* ddq = dq + nv;
    const double* tau = ddq + nv;
    const double* cnt = tau + nja;
    const bool valid = s + half < N;  // the step's last samples may not exist
    wsync();
    if (s1 < N) fetch(s1);
    const unsigned long long pend = s1 < N ? claim_issue() : 0ull;  // the step after s1, read mid-step
    for (int x = hl; x < 24; x += HW) {
      double v = 0.0;
      if (x == 0 || x == 4 || x == 8) v = 1.0;   // oR_0 = I
      if (x >= 18 && x < 21) v = -(x == 18 ? kp.g0 : (x == 19 ? kp.g1 : kp.g2));
      body[x] = v;
    }
    wsync();

    // ---- forward pass (computeJointTorqueRegressor forward step), in two parts ----
    // (1) here: joint placements liMi = jointPlacement * M_J(q) of every joint at once (one lane per joint:
    //     the sincos / quaternion work is off the depth-serial path), parked in the joint's own pose slot,
    //     then the poses level by level, oR_j = oR_p liR_j, ot_j = oR_p lit_j + ot_p: the only depth-serial
    //     work, 36 FMAs per level;
    // (2) after the motion axes (below): every joint's velocity and acceleration at once, one lane per
    //     joint, as sums over its chain.
    // Poses are kept relative to the free-flyer (base) frame, not the world: the regressor rows of
    // pinocchio only see the base rotation through R_b^T g, and J_c's row space (hence P) is the same in
    // base-aligned and world-aligned axes because R_b is invertible.  This stays exact for the float32,
    // slightly non-unit quaternions of the reference's .dat logs.
    auto pose_step = [&](int j) {  // depth >= 2: a revolute joint (the free-flyer is on the first level)
      const double* bp = body + BODY_STRIDE * parent[j];
      double* bj = body + BODY_STRIDE * j;
      double liR[9], lit[3], oR[9], ot[3];
#pragma unroll
      for (int k = 0; k < 9; ++k) liR[k] = bj[k];
      lit[0] = bj[9]; lit[1] = bj[10]; lit[2] = bj[11];
      mat3mul(bp, liR, oR);
      mat3vec(bp, lit, ot);
      ot[0] += bp[9]; ot[1] += bp[10]; ot[2] += bp[11];
#pragma unroll
      for (int k = 0; k < 9; ++k) bj[k] = oR[k];
      bj[9] = ot[0]; bj[10] = ot[1]; bj[11] = ot[2];
    };
    for (int j = 1 + hl; j < NJ; j += HW) {
      double* bj = body + BODY_STRIDE * j;
      if (jtype[j] == JT_FREEFLYER) {
        // its pose in its own (base) frame: I, 0 (the quaternion only enters through R_b^T g, in part (2))
#pragma unroll
        for (int k = 0; k < 12; ++k) bj[k] = (k == 0 || k == 4 || k == 8) ? 1.0 : 0.0;
      } else {
        // liMi = (R0 R_axis(q), t0); on the first level (parent = the universe) that is the pose itself
        double RJ[9];
        axis_rotation(axis + 3 * j, q[idx_q[j]], RJ);
        mat3mul(R0 + 9 * j, RJ, bj);
        bj[9] = t0[3 * j]; bj[10] = t0[3 * j + 1]; bj[11] = t0[3 * j + 2];
      }
    }
    wsync();
    if constexpr (SPW == 1) {
      // One-sample waves (NJ <= 65: one lane per joint), poses by pointer jumping: lane j holds M_j, its pose in the
      // frame of joint p_j (initially its placement liMi, p_j its parent); each pass composes M_j <- M_{p_j} M_j and
      // jumps p_j <- p_{p_j}, every lane reading the values of the pass's start (LDS slots, pointers by ds_bpermute),
      // until p_j is the root (the universe, or the free-flyer whose frame the poses are in).  ceil(log2(depth))
      // passes of one 3x4 product instead of one per chain level (G1: 4 instead of up to 10); the products associate
      // differently from the level order (rounding-level differences).
      const int j = 1 + hl;
      const bool jv = j < NJ;
      auto is_root = [&](int p) { return p == 0 || jtype[p] == JT_FREEFLYER; };
      int pj = jv ? parent[j] : 0;
      bool done = !jv || jtype[j] == JT_FREEFLYER || is_root(pj);
      double* bj = body + BODY_STRIDE * (jv ? j : 1);
      double M[12];
#pragma unroll
      for (int x = 0; x < 12; ++x) M[x] = bj[x];
      for (int it = 0; (1 << it) < kp.maxdepth; ++it) {
        const double* bp = body + BODY_STRIDE * (done ? 1 : pj);
        double Mp[12];
#pragma unroll
        for (int x = 0; x < 12; ++x) Mp[x] = bp[x];
        const int pp = __shfl(pj, done ? hl : pj - 1, 64);
        wsync();  // every lane has read the pass's poses before any is overwritten
        if (!done) {
          double R[9], tt[3];
          mat3mul(Mp, M, R);
          mat3vec(Mp, M + 9, tt);
#pragma unroll
          for (int x = 0; x < 9; ++x) M[x] = R[x];
          M[9] = tt[0] + Mp[9]; M[10] = tt[1] + Mp[10]; M[11] = tt[2] + Mp[11];
#pragma unroll
          for (int x = 0; x < 12; ++x) bj[x] = M[x];
          pj = pp;
          done = is_root(pj);
        }
        wsync();
      }
    } else if constexpr (NVC == 18) {
      // Every joint has its own lane (one-sample waves: NJ <= 64; the quadruped kernel: nb <= 16 of 32 lanes): each
      // lane forms its joint's pose as the product
      // of the placements along its revolute chain, root first — the same products in the same order as the level
      // passes below, without their ordering point and LDS round trip per level (G1: 10 levels; Spot K1 -1.5%,
      // profiles/r05_s4).  The results are written after one ordering point (every lane has read the placements
      // it needs).
      static_assert(SPW == 1 || HW >= 17, "one lane per body of the quadruped kernel (nb <= 16)");
      const int j = 1 + hl;
      double M[12];
#pragma unroll
      for (int x = 0; x < 12; ++x) M[x] = 0.0;
      if (j < NJ && jtype[j] != JT_FREEFLYER) {
        const int cl = chain_len[j];
        // every placement's joint up front (entries past the chain are 0, a valid slot): no dependent index load
        // in front of each step's placement reads
        int aj[MAXCH];
#pragma unroll
        for (int t = 0; t < MAXCH; ++t) aj[t] = anc[j * kp.maxch + t];
        const double* b0 = body + BODY_STRIDE * aj[0];
#pragma unroll
        for (int x = 0; x < 12; ++x) M[x] = b0[x];
#pragma unroll
        for (int t = 1; t < MAXCH; ++t) {
          if (t >= kp.maxdepth) break;  // wave-uniform bound (chains are shorter than the tree is deep)
          if (t < cl) {
            const double* bl = body + BODY_STRIDE * aj[t];
            double liR[9], lit[3], R[9], tt[3];
#pragma unroll
            for (int x = 0; x < 9; ++x) liR[x] = bl[x];
            lit[0] = bl[9]; lit[1] = bl[10]; lit[2] = bl[11];
            mat3mul(M, liR, R);
            mat3vec(M, lit, tt);
#pragma unroll
            for (int x = 0; x < 9; ++x) M[x] = R[x];
            M[9] = tt[0] + M[9]; M[10] = tt[1] + M[10]; M[11] = tt[2] + M[11];
          }
        }
      }
      wsync();  // every placement read
      if (j < NJ && jtype[j] != JT_FREEFLYER) {
        double* bj = body + BODY_STRIDE * j;
#pragma unroll
        for (int x = 0; x < 12; ++x) bj[x] = M[x];
      }
      wsync();
    } else {
      // Poses level by level (a joint's parent is one level up); level 1 is final after the placement pass.
      for (int lvl = 2; lvl <= kp.maxdepth; ++lvl) {
        for (int j = 1 + hl; j < NJ; j += HW)
          if (depth[j] == lvl) pose_step(j);
        wsync();
      }
    }

    // ---- world motion axes of every dof; contact points ----
    for (int e = hl; e < nv + nc; e += HW) {
      if (e < nv) {
        const int r = e;
        const int j = dof_joint[r];
        const double* bj = body + BODY_STRIDE * j;
        double W[3], P[3] = {bj[9], bj[10], bj[11]};
        bool lin = false;
        if (jtype[j] == JT_FREEFLYER) {
          const int k = dof_k[r];
          const int col = k < 3 ? k : k - 3;
          W[0] = bj[col]; W[1] = bj[3 + col]; W[2] = bj[6 + col];
          lin = k < 3;
        } else {
          mat3vec(bj, axis + 3 * j, W);
        }
        Ws[3 * r] = W[0]; Ws[3 * r + 1] = W[1]; Ws[3 * r + 2] = W[2];
        Pts[3 * r] = P[0]; Pts[3 * r + 1] = P[1]; Pts[3 * r + 2] = P[2];
        double* jw = Jws + 6 * r;
        if (lin) {
          jw[0] = W[0]; jw[1] = W[1]; jw[2] = W[2]; jw[3] = 0.0; jw[4] = 0.0; jw[5] = 0.0;
        } else {
          double pw[3];
          cross3(P, W, pw);
          jw[0] = pw[0]; jw[1] = pw[1]; jw[2] = pw[2]; jw[3] = W[0]; jw[4] = W[1]; jw[5] = W[2];
        }
      } else {
        const int c = e - nv;
        const double* bj = body + BODY_STRIDE * cjoint[c];
        double x[3];
        mat3vec(bj, ct + 3 * c, x);
        pfs[3 * c] = x[0] + bj[9]; pfs[3 * c + 1] = x[1] + bj[10]; pfs[3 * c + 2] = x[2] + bj[11];
      }
    }
    // ---- forward pass, part (2): body velocities and accelerations ----
    // In base coordinates (the free-flyer frame) the recursion a_j = X_jp a_p + S_j ddq_j + v_j x S_j dq_j
    // reads A_j = A_p + S_d ddq_d + V_p x S_d dq_d (the adjoint commutes with the motion cross product, and
    // v_j x S_j dq_j = v_p x S_j dq_j), with S_d = Jws row d.  So per joint, over its revolute chain d (root
    // side first):  A += S_d ddq_d + V x S_d dq_d,  V += S_d dq_d,  from V_0 / A_0 = the free-flyer's
    // dq / ddq + R_b^T (-g) (its own frame: pinocchio's local free-flyer velocity), or (0, -g) for a joint
    // under the fixed base; then v_j = V.actInv(oM_j), a_gf_j = A.actInv(oM_j).  One lane per joint, no
    // depth-serial passes.  (A joint hangs under the free-flyer iff its depth exceeds its revolute chain.)
    wsync();  // Jws rows of other lanes
    for (int j = 1 + hl; j < NJ; j += HW) {
      double V[6], A[6];
      const int cl = chain_len[j];
      if (kp.has_ff && depth[j] > cl) {
        const int jf = dof_joint[kp.ff0], iq = idx_q[jf], iv = kp.ff0;
        double Rb[9], mg[3] = {-kp.g0, -kp.g1, -kp.g2}, gb[3];
        quat_to_matrix(q[iq + 3], q[iq + 4], q[iq + 5], q[iq + 6], Rb);
        mat3tvec(Rb, mg, gb);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          V[k] = dq[iv + k];
          V[3 + k] = dq[iv + 3 + k];
          A[k] = ddq[iv + k] + gb[k];
          A[3 + k] = ddq[iv + 3 + k];
        }
      } else {
        A[0] = -kp.g0; A[1] = -kp.g1; A[2] = -kp.g2;
        V[0] = V[1] = V[2] = V[3] = V[4] = V[5] = A[3] = A[4] = A[5] = 0.0;
      }
      const int* ch = chain + j * kp.maxch;
      int dch[MAXCH];  // the chain's dofs up front (unconditional: entries past the chain are 0, a valid dof)
#pragma unroll
      for (int t = 0; t < MAXCH; ++t) dch[t] = ch[t];
#pragma unroll
      for (int t = 0; t < MAXCH; ++t) {  // unrolled to the compile-time chain slots (K1 -1.3%)
        if (t >= cl) break;
        const int d = dch[t];
        const double* S = Jws + 6 * d;
        const double qd = dq[d], qdd = ddq[d];
        double Sd[6], sv[6], c1[3], c2[3], c3[3];
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          Sd[k] = S[k];
          sv[k] = Sd[k] * qd;
        }
        cross3(V + 3, sv, c1);      // w x s_lin
        cross3(V, sv + 3, c2);      // v x s_ang
        cross3(V + 3, sv + 3, c3);  // w x s_ang
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          A[k] += Sd[k] * qdd + (c1[k] + c2[k]);
          A[3 + k] += Sd[3 + k] * qdd + c3[k];
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) V[k] += sv[k];
      }
      double* bj = body + BODY_STRIDE * j;
      double vb[6], ab[6];
      act_inv_motion(bj, bj + 9, V, vb);
      act_inv_motion(bj, bj + 9, A, ab);
#pragma unroll
      for (int k = 0; k < 6; ++k) { bj[12 + k] = vb[k]; bj[18 + k] = ab[k]; }
    }
    // contacts with a non-zero value as a bit mask (independent loads, no search loop per entry below)
    unsigned long long amask = 0ull;
    for (int c = 0; c < nc; ++c) amask |= (cnt[c] != 0.0 ? 1ull : 0ull) << c;
    const int na = __popcll(amask);
    const int k = 3 * na;
    wsync();

    // ---- contact Jacobian (LOCAL_WORLD_ALIGNED, linear rows) ----
    // lane = (contact in contact, dof): the three rows of the contact at once (one cross product)
    for (int e = hl; e < na * nv; e += HW) {
      const int ci = e / nv, r = e - ci * nv;
      unsigned long long m = amask;  // the ci-th contact with a non-zero value
      for (int t = ci; t > 0; --t) m &= m - 1ull;
      const int c = __ffsll((long long)m) - 1;
      double x[3] = {0.0, 0.0, 0.0};
      if ((csupp[c] >> r) & 1ull) {
        const double* W = Ws + 3 * r;
        if (jtype[dof_joint[r]] == JT_FREEFLYER && dof_k[r] < 3) {
          x[0] = W[0]; x[1] = W[1]; x[2] = W[2];
        } else {
          double d[3];
          d[0] = pfs[3 * c] - Pts[3 * r];
          d[1] = pfs[3 * c + 1] - Pts[3 * r + 1];
          d[2] = pfs[3 * c + 2] - Pts[3 * r + 2];
          cross3(W, d, x);
        }
      }
      double* jr = Jc + 3 * ci * nv + r;
      jr[0] = x[0];
      jr[nv] = x[1];
      jr[2 * nv] = x[2];
    }
    wsync();

    // H1 = P[:, ff] J_w[:, ff]^T is P's free-flyer columns: in base coordinates the free-flyer's motion axes
    // are the unit vectors (oR = I, ot = 0), J_w[:, ff] = I exactly.  The column phase reads those P entries
    // in place (an even ff0 keeps the rows' 16-byte alignment); otherwise H1 is copied out below.
    const bool h1_in_p = kp.has_ff && (kp.ff0 & 1) == 0;
    int nrows = nv;  // output rows of the sample: nv, or nv - rank(J_c) in the nullspace mode (CMP)
    if (kfull) {
      // get_full_regressor_force (src/sys_identification.py:391-399): no projection.  With the overlay P = I
      // is written after the tau column below (which reads J_c, under P's slot there).
      if constexpr (!POV && !QF) {
        for (int e = hl; e < nv * nv; e += HW) {
          const int a = e / nv;
          Ps[e] = e - a * nv == a ? 1.0 : 0.0;
        }
        wsync();
      }
    } else {
      // ---- orthonormal basis of J_c's row space by modified Gram-Schmidt ----
      // P = I - pinv(J_c) J_c is the projector onto null(J_c) = I - Q^T Q for any orthonormal basis Q of
      // the row space.  Row p in turn, if its remaining norm is > thr_rel * the largest row norm, gives
      // q = x_p / |x_p|, whose direction is removed from every later row (lanes = later rows, one
      // wave-synchronous pass per row); otherwise it depends on the rows before it and is dropped, as
      // pinv drops singular values <= 1e-15 sigma_max.  Error ~eps * cond(J_c), pinv's own order (the
      // normal-equations inverse it replaces was eps * cond^2: 1e-5 at cond 1e6); choosing the largest
      // remaining row as the next pivot measured no more accurate (tests/test_projector.py) and costs a
      // k-way argmax per step.  q of slot j ends in J_c row j (in place) and, transposed, in column j of
      // Zt (stride 3 nc); dropped slots are zero in Zt, so P below sums over all k slots.
      double* nrm = Ms;  // squared remaining norm of each row slot; -1/|x_p| once taken
      double* Zt = wr + L.Z;
      const int K = 3 * nc;
      // Generic form: rows in LDS, lane groups per row, the norms through LDS.
      auto mgs_lds = [&]() {
        for (int j = hl; j < k; j += HW) nrm[j] = mgs_sqnorm<NVC>(Jc + j * nv, nv);
        wsync();
        {
          double nmax = 0.0;
          for (int j = 0; j < k; ++j) nmax = fmax(nmax, nrm[j]);
          const double thr = kp.thr_rel2 * nmax;
          // lane pairs per row for the compile-time-nv kernel when the rows fit (uniform per sample)
          const bool pairs = NVC > 0 && NVC % 2 == 0 && 2 * k <= HW;
          // otherwise lane groups of lpr = 8, 4, 2 or 1 lanes per row, the widest whose rows fit
          const int lpr = 8 * k <= HW ? 8 : (4 * k <= HW ? 4 : (2 * k <= HW ? 2 : 1));
          for (int p = 0; p < k; ++p) {
            const double best = nrm[p];
            if (!(best > thr)) continue;  // dependent on the rows before it: dropped (uniform per sample)
            const double inv = rsqrt_f64(best);
            const double inv2 = inv * inv;
            const double* xp = Jc + p * nv;
            if constexpr (NVC > 0 && NVC % 2 == 0) {
              if (pairs) {
                const int j = hl >> 1;
                // a taken slot keeps its scale as -1/|x_p| (its row is final: scaled below)
                if (j == p) {
                  if ((hl & 1) == 0) nrm[p] = -inv;
                } else if (j > p && j < k) {
                  const double a = mgs_step_pair<NVC>(xp, Jc + j * NVC, inv2, hl & 1);
                  if ((hl & 1) == 0) nrm[j] = a;
                }
              }
            }
            if (!pairs) {
              if (k * lpr <= HW) {
                const int j = hl / lpr, h = hl - j * lpr;
                if (j == p) {
                  if (h == 0) nrm[p] = -inv;
                } else if (j > p && j < k) {
                  const double a = mgs_step_group(xp, Jc + j * nv, inv2, nv, h, lpr);
                  if (h == 0) nrm[j] = a;
                }
              } else {
                for (int j = hl; j < k; j += HW) {
                  if (j == p) {
                    nrm[p] = -inv;
                  } else if (j > p) {
                    nrm[j] = mgs_step_group(xp, Jc + j * nv, inv2, nv, 0, 1);
                  }
                }
              }
            }
            wsync();
          }
          // q of each taken slot = its row x 1/|x_p| (in place, and transposed into Zt); dropped slots: 0
          for (int e = hl; e < k * nv; e += HW) {
            const int j = e / nv, r = e - j * nv;
            const double sc = nrm[j] < 0.0 ? -nrm[j] : 0.0;
            const double qv = Jc[e] * sc;
            Jc[e] = qv;
            Zt[r * K + j] = qv;
          }
          wsync();
        }
      };
      if constexpr (NVC == 18 && HW == 32) {
        {  // 2k <= HW: the engine picks this kernel for at most 5 contact frames (k <= 15)
          // Quadruped form: lane pair (2j, 2j+1) keeps its half-row of row j in registers through every
          // step; the pivot's norm comes from its lanes by readlane (no LDS round trip per step) and only
          // the pivot's half-row is read from LDS; an updated row is written back for its own turn.
          constexpr int H = ((NVC + 1) / 2 + 1) & ~1, H2 = H / 2;
          const int j = hl >> 1, h = hl & 1;
          const int n2 = h == 0 ? H2 : (NVC - H) / 2;
          const bool row = j < k;
          double2* xrow = reinterpret_cast<double2*>(Jc + (row ? j : 0) * NVC + h * H);
          double2 xv[H2];
          double a0 = 0.0, a1 = 0.0;
#pragma unroll
          for (int u = 0; u < H2; ++u) {
            xv[u] = (row && u < n2) ? xrow[u] : make_double2(0.0, 0.0);
            a0 += xv[u].x * xv[u].x;
            a1 += xv[u].y * xv[u].y;
          }
          double myn = pair_sum(a0 + a1);
          if (row && h == 0) nrm[j] = myn;
          wsync();
          double nmax = 0.0;
          for (int jj = 0; jj < k; ++jj) nmax = fmax(nmax, nrm[jj]);
          const double thr = kp.thr_rel2 * nmax;
          double sc = 0.0;  // 1/|x_j| once row j is taken; 0 if it is dropped
          for (int p = 0; p < k; ++p) {
            const double n0 = readlane_f64(myn, 2 * p), n1 = readlane_f64(myn, HW + 2 * p);
            const double best = half ? n1 : n0;
            if (!(best > thr)) continue;  // dependent on the rows before it: dropped
            const double inv = rsqrt_f64(best);
            if (j == p) sc = inv;
            if (row && j > p) {
              const double2* xp = reinterpret_cast<const double2*>(Jc + p * NVC + h * H);
              double2 pv[H2];
              double c0 = 0.0, c1 = 0.0;
#pragma unroll
              for (int u = 0; u < H2; ++u) {
                pv[u] = u < n2 ? xp[u] : make_double2(0.0, 0.0);
                c0 += pv[u].x * xv[u].x;
                c1 += pv[u].y * xv[u].y;
              }
              const double c = pair_sum(c0 + c1) * (inv * inv);
              double b0 = 0.0, b1 = 0.0;
#pragma unroll
              for (int u = 0; u < H2; ++u) {
                xv[u].x -= c * pv[u].x;
                xv[u].y -= c * pv[u].y;
                b0 += xv[u].x * xv[u].x;
                b1 += xv[u].y * xv[u].y;
                if (u < n2) xrow[u] = xv[u];
              }
              myn = pair_sum(b0 + b1);
            }
            wsync();
          }
          // Q rows = x_j / |x_j| (taken) or 0 (dropped), in place: P below reads Q from J_c
          if (row) {
#pragma unroll
            for (int u = 0; u < H2; ++u)
              if (u < n2) xrow[u] = make_double2(xv[u].x * sc, xv[u].y * sc);
            if (CMP && h == 0) nrm[j] = -sc;  // taken rows < 0, as in mgs_lds (read by the nullspace phase)
          }
          wsync();
        }
      } else if (8 * k <= HW && nv <= 8 * K1_MGS_NU) {
        // Runtime-nv form for at most HW / 8 rows and nv <= 40 (G1: k <= 6, nv = 35): lane group j (8 lanes) keeps row
        // j in registers,
        // lane h of it the entries h, h + 8, ...; the pivot row's entries come from its group by ds_bpermute, dot
        // products and norms are completed across the group by DPP, the norms read by readlane: no LDS round trip
        // and no ordering point per pivot (mgs_lds keeps the rows in LDS and passes each pivot through it).
        const int j = hl >> 3, h = hl & 7;
        const bool row = j < k;
        constexpr int NU = K1_MGS_NU;
        const int nu = __builtin_amdgcn_readfirstlane((nv + 7) >> 3);  // entries per lane (<= NU)
        double xv[NU];
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int r = h + 8 * u;
          xv[u] = u < nu && row && r < nv ? Jc[j * nv + r] : 0.0;
        }
        auto sqn = [&]() {
          double a0 = 0.0, a1 = 0.0;
#pragma unroll
          for (int u = 0; u < NU; ++u) {
            if (u < nu) {
              if (u & 1) a1 += xv[u] * xv[u];
              else a0 += xv[u] * xv[u];
            }
          }
          return group_sum(a0 + a1, 8);
        };
        double myn = sqn();  // row j's squared norm in every lane of group j
        double nmax = 0.0;
        for (int jj = 0; jj < k; ++jj) nmax = fmax(nmax, readlane_f64(myn, 8 * jj));
        const double thr = kp.thr_rel2 * nmax;
        double sc = 0.0;  // 1/|x_j| once row j is taken; 0 if it is dropped
        bool taken = false;
        for (int p = 0; p < k; ++p) {
          const double best = readlane_f64(myn, 8 * p);
          if (!(best > thr)) continue;  // dependent on the rows before it: dropped
          const double inv = rsqrt_f64(best);
          if (j == p) {
            sc = inv;
            taken = true;
          }
          double pv[NU];
#pragma unroll
          for (int u = 0; u < NU; ++u)
            if (u < nu) pv[u] = __shfl(xv[u], 8 * p + h, 64);
          if (row && j > p) {
            double c0 = 0.0, c1 = 0.0;
#pragma unroll
            for (int u = 0; u < NU; ++u) {
              if (u < nu) {
                if (u & 1) c1 += pv[u] * xv[u];
                else c0 += pv[u] * xv[u];
              }
            }
            const double c = group_sum(c0 + c1, 8) * (inv * inv);
#pragma unroll
            for (int u = 0; u < NU; ++u)
              if (u < nu) xv[u] -= c * pv[u];
            myn = sqn();
          }
        }
        wsync();  // every J_c read precedes the stores
        double* Zt = wr + L.Z;
        const int K = 3 * nc;
        if (row) {
#pragma unroll
          for (int u = 0; u < NU; ++u) {
            const int r = h + 8 * u;
            if (u < nu && r < nv) {
              const double qv = xv[u] * sc;
              Jc[j * nv + r] = qv;
              Zt[r * K + j] = qv;
            }
          }
          if (h == 0) Ms[j] = taken ? -sc : myn;  // as mgs_lds: taken slots < 0, dropped ones their squared norm
        }
        wsync();
      } else {
        mgs_lds();
      }

      if constexpr (CMP) {
        // ---- nullspace rows Zᵀ (m x nv, m = nv - r) in P's slot, row t at Ps + t nv ----
        // (a) Householder vectors of the QR of Qᵀ (nv x r, orthonormal columns = the r taken rows of J_c, in
        //     row order) by the unpivoted LU of Qᵀ - diag(s), s_a = -sign(d_a): every pivot d_a + sign(d_a) has
        //     modulus >= 1, so no pivoting is needed (Householder reconstruction).  In registers: lane = column i
        //     of Qᵀ (coordinate i), x[b] = entry i of taken row b; the pivot row's entries come by readlane.  Then
        //     v_a (0 before a, 1 at a, x_{i,a}/piv past it: whole rows, so the products below need no masks) is
        //     stored as J_c row a and tau_a = |d_a| + 1 = 2 / v_aᵀv_a as nrm[a].
        unsigned long long tm = 0ull;
        for (int j = 0; j < k; ++j) tm |= (nrm[j] < 0.0 ? 1ull : 0ull) << j;
        const int rk = __popcll(tm);
        {
          double x[K1_CMP_KMAX];
          {
            unsigned long long rb = tm;
#pragma unroll
            for (int u = 0; u < K1_CMP_KMAX; ++u) {
              const int pb = rb ? __ffsll((long long)rb) - 1 : 0;
              rb &= rb - 1ull;
              x[u] = u < rk && hl < nv ? Jc[pb * nv + hl] : 0.0;
            }
          }
          // the value of lane `src` of this sample's lanes (two samples per wave: either half)
          auto bcast = [&](double v, int src) -> double {
            if constexpr (SPW == 1) return readlane_f64(v, src);
            else return __shfl(v, half * HW + src, 64);  // each half its own source lane (ds_bpermute)
          };
          // tau_a = |d_a| + 1 goes straight to nrm[a] (the taken-row flags were read into tm above, and this wave's
          // LDS operations execute in order): no register array held across the factorisation
#pragma unroll
          for (int a = 0; a < K1_CMP_KMAX; ++a) {
            if (a < rk) {
              const double d = bcast(x[a], a);
              const double rp = 1.0 / (d + (d >= 0.0 ? 1.0 : -1.0));
              if (hl == 0) nrm[a] = fabs(d) + 1.0;
              const double l = x[a] * rp;
#pragma unroll
              for (int b2 = a + 1; b2 < K1_CMP_KMAX; ++b2) {
                const double xab = bcast(x[b2], a);
                if (hl > a) x[b2] -= l * xab;
              }
              x[a] = hl > a ? l : (hl == a ? 1.0 : 0.0);
            }
          }
          wsync();  // every J_c / nrm read above precedes the stores
          if (hl < nv) {
#pragma unroll
            for (int a = 0; a < K1_CMP_KMAX; ++a)
              if (a < rk) Jc[a * nv + hl] = x[a];
          }
          wsync();
        }
        // (b) row t of Zᵀ = (H_1 ... H_r e_{r+t})ᵀ, H_a = I - tau_a v_a v_aᵀ applied from a = r-1 down
        const int m = nv - rk;
        nrows = m;
        if constexpr (NVC == 18 && HW == 32) {
          if (hl < m) {  // lane = row, the row in registers
            double y[NVC];
#pragma unroll
            for (int i = 0; i < NVC; ++i) y[i] = i == rk + hl ? 1.0 : 0.0;
            for (int a = rk - 1; a >= 0; --a) {
              const double2* qa = reinterpret_cast<const double2*>(Jc + a * NVC);
              // v_a read twice from LDS (a register copy of it spilled): dot product, then the update
              double d0 = 0.0, d1 = 0.0;
#pragma unroll
              for (int u = 0; u < NVC / 2; ++u) {
                const double2 x = qa[u];
                d0 += x.x * y[2 * u];
                d1 += x.y * y[2 * u + 1];
              }
              const double c = nrm[a] * (d0 + d1);
#pragma unroll
              for (int u = 0; u < NVC / 2; ++u) {
                const double2 x = qa[u];
                y[2 * u] -= c * x.x;
                y[2 * u + 1] -= c * x.y;
              }
            }
            double2* zr = reinterpret_cast<double2*>(Ps + hl * NVC);
#pragma unroll
            for (int u = 0; u < NVC / 2; ++u) zr[u] = make_double2(y[2 * u], y[2 * u + 1]);
          }
        } else {
          // lpr lanes per row (entries i = h mod lpr), the row in place at its output position
          const int lpr = 2 * m <= HW ? 2 : 1;
          for (int it = hl; it < m * lpr; it += HW) {
            const int t = it / lpr, h = it - t * lpr;
            double* y = Ps + t * nv;
            for (int i = h; i < nv; i += lpr) y[i] = i == rk + t ? 1.0 : 0.0;
            for (int a = rk - 1; a >= 0; --a) {
              const double* qa = Jc + a * nv;  // the whole v_a (zeros before a)
              double dot = 0.0;
              for (int i = h; i < nv; i += lpr) dot += qa[i] * y[i];
              const double c = nrm[a] * group_sum(dot, lpr);
              for (int i = h; i < nv; i += lpr) y[i] -= c * qa[i];
            }
          }
        }
        wsync();
      } else if constexpr (!QF) {  // (the Q-form never forms P: its phases below read Q from J_c)
      // ---- P = I - Q^T Q  (Zt row a = column a of Q; J_c rows = rows of Q) ----
      if constexpr (NVC == 18 && HW == 32) {
        // Register-blocked: lane = (row pair, 6-column group), 27 lanes x 12 entries, every load before
        // any store, so P may overwrite Zt freely and no ordering point is needed between entries.
        const int rp = hl / 3, cg = hl - 3 * rp;
        if (hl < 27) {
          const int a0 = 2 * rp, b0 = 6 * cg;
          double acc[2][6];
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int c = 0; c < 6; ++c) acc[i][c] = 0.0;
#pragma unroll 4
          for (int j = 0; j < k; ++j) {
            const double2 zz = *reinterpret_cast<const double2*>(Jc + j * 18 + a0);  // Q[j][a0], Q[j][a0+1]
            const double z0 = zz.x, z1 = zz.y;
            const double2* qr = reinterpret_cast<const double2*>(Jc + j * 18 + b0);
            const double2 q0 = qr[0], q1 = qr[1], q2 = qr[2];
            const double qv[6] = {q0.x, q0.y, q1.x, q1.y, q2.x, q2.y};
#pragma unroll
            for (int c = 0; c < 6; ++c) {
              acc[0][c] += z0 * qv[c];
              acc[1][c] += z1 * qv[c];
            }
          }
          double pv[2][6];
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int c = 0; c < 6; ++c) pv[i][c] = (a0 + i == b0 + c ? 1.0 : 0.0) - acc[i][c];
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            double2* pr = reinterpret_cast<double2*>(Ps + (a0 + i) * 18 + b0);
#pragma unroll
            for (int c = 0; c < 3; ++c) pr[c] = make_double2(pv[i][2 * c], pv[i][2 * c + 1]);
          }
        }
        wsync();
      } else {
        // Runtime-nv kernels: P has its own region (wave_layout with hw = 0), so its passes need no
        // ordering point between them; with the overlay (POV) the passes whose entries land on J_c / Z
        // (the slot's tail, from entry L.Jc - L.P on) are held in registers until every entry is computed.
        if constexpr (POV) {
          auto p_entry = [&](int e) -> double {
            const int a = e / nv, b = e - a * nv;
            const double* za = Zt + a * K;
            double acc = 0.0;
#pragma unroll 4
            for (int j = 0; j < k; ++j) acc += za[j] * Jc[j * nv + b];
            return (a == b ? 1.0 : 0.0) - acc;
          };
          const int t0 = (L.Jc - L.P) / HW;  // first buffered pass
          for (int t = 0; t < t0; ++t) {
            const int e = hl + HW * t;
            if (e < nv * nv) Ps[e] = p_entry(e);
          }
          double pb[K1_POV_BUF];
#pragma unroll
          for (int u = 0; u < K1_POV_BUF; ++u) {
            const int e = hl + HW * (t0 + u);
            pb[u] = e < nv * nv ? p_entry(e) : 0.0;
          }
          wsync();  // every entry computed: the overlaid J_c / Z are dead
#pragma unroll
          for (int u = 0; u < K1_POV_BUF; ++u) {
            const int e = hl + HW * (t0 + u);
            if (e < nv * nv) Ps[e] = pb[u];
          }
        } else {
          for (int e = hl; e < nv * nv; e += HW) {
            const int a = e / nv, b = e - a * nv;
            const double* za = Zt + a * K;
            double acc = 0.0;
#pragma unroll 4
            for (int j = 0; j < k; ++j) acc += za[j] * Jc[j * nv + b];
            Ps[e] = (a == b ? 1.0 : 0.0) - acc;
          }
        }
        wsync();
      }
      }
    }

    // ---- tp = P S^T tau  (+ J_c^T lambda in the full mode) ;  H1 = P[:, ff] J_w[:, ff]^T ----
    // tp first: in the full mode H1 may be stored over J_c (overlay layout), which the tau column reads.
    // Q-form: tp = S^T tau - Qᵀ u, u_j = Q_j · S^T tau (u in the dead row-norm slots)
    if constexpr (QF) {
      if (!kfull) {
        // u_j = Q_j . S^T tau: eight lanes per row j (k <= K1_QF_KMAX <= 8 rows, whole 8-lane groups active), each
        // summing every eighth joint, then a DPP sum over the group — not one lane per row walking all nj joints
        // (a 29-long chain of dependent LDS reads on G1)
        static_assert(K1_QF_KMAX <= 8, "one 8-lane group per Q row");
        const int j = hl >> 3, part = hl & 7;
        if (j < k) {
          double acc = 0.0;
          for (int jj = part; jj < nja; jj += 8) acc += Jc[j * nv + bd + jj] * tau[jj];
          acc = group_sum(acc, 8);
          if (part == 0) Ms[j] = acc;
        }
        wsync();
      }
    }
    for (int r = hl; r < nrows; r += HW) {
      double acc = 0.0;
      if ((POV || QF) && kfull) {
        acc = r >= bd && r < bd + nja ? tau[r - bd] : 0.0;  // P = I (not yet written)
      } else if constexpr (QF) {
        acc = r >= bd && r < bd + nja ? tau[r - bd] : 0.0;
        for (int j = 0; j < k; ++j) acc -= Jc[j * nv + r] * Ms[j];
      } else {
#pragma unroll 4
        for (int jj = 0; jj < nja; ++jj) acc += Ps[r * nv + bd + jj] * tau[jj];
      }
      if (kfull) {
        // + J_c^T lambda, lambda = the measured forces of the feet in contact in foot order, world axes
        // (LOCAL_WORLD_ALIGNED).  J_c here is in base axes, J_c,world = R_b J_c, so lambda is moved to
        // base axes with R_b^T (R_b = the base quaternion's matrix, unnormalised like pinocchio's).
        double Rb[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        if (kp.has_ff && jtype[1] == JT_FREEFLYER) {
          const int iq = idx_q[1];
          quat_to_matrix(q[iq + 3], q[iq + 4], q[iq + 5], q[iq + 6], Rb);
        }
        const double* lam = cnt + nc;
        for (int rho = 0, c = -1; rho < k; ++rho) {
          const int comp = rho % 3;
          if (comp == 0)
            for (++c; c < nc && cnt[c] == 0.0; ++c) {}
          const double* lw = lam + 3 * c;
          // column `comp` of R_b by selects (a dynamic index would put Rb in scratch memory)
          const double c0 = comp == 0 ? Rb[0] : (comp == 1 ? Rb[1] : Rb[2]);
          const double c1 = comp == 0 ? Rb[3] : (comp == 1 ? Rb[4] : Rb[5]);
          const double c2 = comp == 0 ? Rb[6] : (comp == 1 ? Rb[7] : Rb[8]);
          const double lb = c0 * lw[0] + c1 * lw[1] + c2 * lw[2];
          acc += Jc[rho * nv + r] * lb;
        }
      }
      tps[r] = acc;
    }
    if (kfull && !POV) wsync();
    if (POV && kfull) {
      wsync();  // J_c read: P = I may overwrite it now
      for (int e = hl; e < nv * nv; e += HW) {
        const int a = e / nv;
        Ps[e] = e - a * nv == a ? 1.0 : 0.0;
      }
      wsync();
    }
    for (int e = hl; e < nrows * 6 && !h1_in_p && !QF; e += HW) {
      const int r = e / 6, c = e - 6 * r;
      H1[e] = kp.has_ff ? Ps[r * nv + kp.ff0 + c] : 0.0;  // J_w[:, ff] = I (see h1_in_p)
    }
    if constexpr (QF) {
      // Qt[r][j] = Q_j[r] (zero past the sample's k rows; in the full mode P = I: no rows), over the dead
      // W / Pt / contact-point slot: a row's K1_QF_KMAX entries are three 16-byte reads from one address
      const int kq = kfull ? 0 : k;
      for (int e = hl; e < nv * K1_QF_KMAX; e += HW) {
        const int r = e / K1_QF_KMAX, j = e - K1_QF_KMAX * r;
        Qt[e] = j < kq ? Jc[j * nv + r] : 0.0;
      }
    }
    wsync();
    if (dbg != nullptr && s + half == 0)  // sysid_debug_lds: the LDS image of sample 0
      for (int x = hl; x < L.total; x += HW) dbg[x] = wr[x];
    if constexpr (CMP) {
      if (hl == 0 && valid) rcount[s + half] = nrows;
    }
    // mid-step: the next inputs go to `in` (the friction columns keep this sample's dq in dqs)
    for (int x = hl; x < nv; x += HW) dqs[x] = dq[x];
    unsigned long long pv = pend;
    asm volatile("" : "+v"(pv));  // keeps the read of the claim (and its vmcnt wait) here
    const int64_t s2 = s1 < N ? claim_value(pv) : N;
    wsync();
    if (s1 < N) commit();
    wsync();
    __builtin_amdgcn_s_setprio(0);
    // ---- projected regressor Y_proj: lane = (body i, row group g), all ten columns of body i ----
    // Y_proj[r, block i] = G_i[r, :] F_i with G_i = P[:, ff] J_w[:, ff]^T + sum over the revolute
    // chain of i of P[:, d] J_w[:, d]^T (= H1 + ...), F_i the body's world-frame regressor block.
    // One G row (6 + 6*chain FMAs) feeds 42 FMAs.
    OutT* out = panel + ((s + half) * nv) * ldp;
    const int nbody = NJ - 1, nyi = nbody * kp.rg;
    auto block_row = [&](int r, const double* F, const int* dof, int cl, double* y) {
      const double* h = h1_in_p ? Ps + r * nv + kp.ff0 : H1 + 6 * r;
      const double* pr = Ps + r * nv;
      double G[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) G[k] = h[k];
      if constexpr (CHAIN_UNCOND) {
        // unconditional loads (dof[t] = 0 past the chain is a valid slot), masked products
#pragma unroll
        for (int t = 0; t < MAXCH; ++t) {
          const double pl = pr[dof[t]];
          const double pv = t < cl ? pl : 0.0;
          const double* jw = Jws + 6 * dof[t];
#pragma unroll
          for (int k = 0; k < 6; ++k) G[k] += pv * jw[k];
        }
      } else {
#pragma unroll
        for (int t = 0; t < MAXCH; ++t) {
          if (t < cl) {
            const double pv = pr[dof[t]];
            const double* jw = Jws + 6 * dof[t];
#pragma unroll
            for (int k = 0; k < 6; ++k) G[k] += pv * jw[k];
          }
        }
      }
#pragma unroll
      for (int c = 0; c < 4; ++c)
        y[c] = G[0] * F[6 * c] + G[1] * F[6 * c + 1] + G[2] * F[6 * c + 2] + G[3] * F[6 * c + 3] +
               G[4] * F[6 * c + 4] + G[5] * F[6 * c + 5];
#pragma unroll
      for (int c = 0; c < 6; ++c)
        y[4 + c] = G[3] * F[24 + 3 * c] + G[4] * F[24 + 3 * c + 1] + G[5] * F[24 + 3 * c + 2];
    };
    auto block_setup = [&](int i, double* F, int* dof) {
      body_regressor_block(body + BODY_STRIDE * i, F);
      const int cl = chain_len[i];
#pragma unroll
      for (int t = 0; t < MAXCH; ++t) dof[t] = t < cl ? chain[i * kp.maxch + t] : 0;
      return cl;
    };
    // Quadrupeds: the rg = 2 row groups' current rows are staged in LDS over the joint records (dead
    // once every lane holds its block F) and written out as whole contiguous panel rows: one 16-byte
    // store per lane per 512 contiguous bytes instead of 16-byte pieces 80 bytes apart.
    // (The host picks this kernel only for 11..16 bodies: rg = 2 row groups, nyi <= 32 lanes, and the two
    // staged rows fit in the joint records.)  Group g takes rows [g rh, g rh + rh) of the sample's nrows.
    if constexpr (NVC == 18 && HW == 32) {
      // rows per row group; the nullspace mode rounds it to even (row pairs, no odd tail: fewer registers) and
      // skips the stores of rows >= nrows
      const int rh = CMP ? ((nrows + 3) >> 2) << 1 : NVC / 2;
      const bool act = hl < nyi && valid;
      const int g = hl / nbody, i = hl - g * nbody + 1;  // lanes past nyi compute a real body's block
      double F[FBLK];
      int dof[MAXCH];
      const int cl = block_setup(i, F, dof);
      // The chain's motion axes are the same for every row: read once into registers (masked past the
      // chain), and each row's H1 / P entries are loaded one row ahead, so a row's LDS reads are in flight
      // while the previous row is multiplied and staged.
      double jw[MAXCH][6];
#pragma unroll
      for (int t = 0; t < MAXCH; ++t)
#pragma unroll
        for (int k = 0; k < 6; ++k) jw[t][k] = t < cl ? Jws[6 * dof[t] + k] : 0.0;
      double hn[6], pn[MAXCH];
      auto row_load = [&](int r, double* h, double* pp) {  // rows >= nrows: unused values from P's slot
        if constexpr (CMP) r = r < NVC ? r : NVC - 1;
        const double2* h2 = reinterpret_cast<const double2*>(h1_in_p ? Ps + r * NVC + kp.ff0 : H1 + 6 * r);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const double2 v = h2[k];
          h[2 * k] = v.x;
          h[2 * k + 1] = v.y;
        }
#pragma unroll
        for (int t = 0; t < MAXCH; ++t) pp[t] = Ps[r * NVC + dof[t]];
      };
      row_load(g * rh, hn, pn);
      wsync();  // every read of the joint records precedes the first staging store
      double* stg = body;  // [row group][wy]
      const int wy2 = kp.wy >> 1, n2 = kp.rg * wy2;
      // pair x of row group gg lands at row gg*rh + rho, column 2*(x - gg*wy2): from this row's start that is
      // 2x, plus dg for the second group.  The row start of the wave's first sample is wave-uniform (scalar
      // registers); the second sample's rows and the column go into a 32-bit lane byte offset, so each store is
      // a scalar-base + lane-offset store with no 64-bit address math.
      char* ybase = reinterpret_cast<char*>(panel + (s * NVC) * ldp);
      const uint32_t yhoff = (uint32_t)(half * NVC * (int)ldp * (int)sizeof(OutT));
      const int dg = rh * (int)ldp - kp.wy;
      // Rows in pairs with two explicit H1 / P register sets (no copies between them): row rho + 1's LDS reads
      // are in flight while row rho is multiplied, staged and stored.  The P entries past the body's chain
      // (dof slot 0, a finite entry of P) meet zero motion axes (jw), so they add exact zeros: no mask.
      double hB[6], pB[MAXCH];
      auto yrow = [&](int rho, const double* hc, const double* pc) {
        if (act) {
          double y[10], G[6];
#pragma unroll
          for (int k = 0; k < 6; ++k) G[k] = hc[k];
#pragma unroll
          for (int t = 0; t < MAXCH; ++t)
#pragma unroll
            for (int k = 0; k < 6; ++k) G[k] += pc[t] * jw[t][k];
#pragma unroll
          for (int c = 0; c < 4; ++c)
            y[c] = G[0] * F[6 * c] + G[1] * F[6 * c + 1] + G[2] * F[6 * c + 2] + G[3] * F[6 * c + 3] +
                   G[4] * F[6 * c + 4] + G[5] * F[6 * c + 5];
#pragma unroll
          for (int c = 0; c < 6; ++c)
            y[4 + c] = G[3] * F[24 + 3 * c] + G[4] * F[24 + 3 * c + 1] + G[5] * F[24 + 3 * c + 2];
          double2* sp = reinterpret_cast<double2*>(stg + g * kp.wy + 10 * (i - 1));
#pragma unroll
          for (int c = 0; c < 5; ++c) sp[c] = make_double2(y[2 * c], y[2 * c + 1]);
        }
        wsync();
        if (valid) {
          const double2* s2 = reinterpret_cast<const double2*>(stg);
          char* rb = ybase + (int64_t)rho * ldp * (int64_t)sizeof(OutT);
          // nullspace mode: the rows past nrows of either group are not stored
          const int n2v = !CMP ? n2 : rh + rho < nrows ? n2 : rho < nrows ? wy2 : 0;
          for (int x = hl; x < n2v; x += HW) {
            const uint32_t off = yhoff + (uint32_t)((2 * x + (x >= wy2 ? dg : 0)) * (int)sizeof(OutT));
            panel_store(reinterpret_cast<OutT*>(rb + off), s2[x].x, s2[x].y);
          }
        }
        wsync();
      };
      if constexpr (CMP) {
#pragma unroll 1
        for (int rho = 0; rho < rh; rho += 2) {
          row_load(g * rh + rho + 1, hB, pB);
          yrow(rho, hn, pn);
          row_load(g * rh + rho + 2, hn, pn);
          yrow(rho + 1, hB, pB);
        }
      } else {
        int rho = 0;
#pragma unroll 1
        for (; rho + 1 < rh; rho += 2) {
          row_load(g * rh + rho + 1, hB, pB);
          yrow(rho, hn, pn);
          if (rho + 2 < rh) row_load(g * rh + rho + 2, hn, pn);
          yrow(rho + 1, hB, pB);
        }
        if (rho < rh) yrow(rho, hn, pn);
      }
    } else if constexpr (QF) {
      // Q-form: G_i[r] = [r in S_i] J_r - Σ_j Q_j[r] K_ij, K_ij = Σ_{d in S_i} Q_j[d] J_d, S_i = the free-flyer
      // dofs (J = unit vectors in base coordinates: Q_j[ff0 + c]) and body i's chain; full mode: no Q (P = I).
      // Lane = (body i, block half h), every row: h = 0 the mass / first-moment columns 0..3, h = 1 the inertia
      // columns 4..9, both as one 6 x 6 matrix F6 (zero-padded) times G, so the two lanes of a body run the same
      // code and write their 32 + 48 bytes of the row's 80-byte block with the same store instructions (lanes
      // 2m, 2m + 1: a row of the panel per store set).  The pair shares G: lane h forms components 3h..3h+2
      // (its three columns of K) and takes the other three from its partner by DPP; F6's columns are permuted
      // per lane to [own three | partner's three].  k is wave-uniform (one sample per wave): the row loop is
      // specialised for k <= 3 and k <= 6.
      const int kq = __builtin_amdgcn_readfirstlane(kfull ? 0 : k);
      const int nyh = 2 * nbody;  // even: both lanes of a pair are always active together
      if constexpr (std::is_same_v<OutT, __bf16>) {
        float* q32w = reinterpret_cast<float*>(wr + L.q32);
        for (int e2 = hl; e2 < k1q32_pairs(nv) * 28; e2 += HW) {
          const int pr = e2 / 28, x = e2 - 28 * pr;
          int row, c;
          if (x < 16) {
            row = 2 * pr + (x & 1);
            c = x >> 1;
          } else if (x < 24) {
            const int y = x - 16;
            row = 2 * pr + ((y >> 1) & 1);
            c = 3 * (y >> 2) + (y & 1);
          } else {
            const int y = x - 24;
            row = 2 * pr + (y & 1);
            c = 2 + 3 * (y >> 1);
          }
          float v = 0.0f;
          if (row < nv) v = x < 16 ? (c < K1_QF_KMAX ? (float)Qt[row * K1_QF_KMAX + c] : 0.0f) : (float)Jws[6 * row + c];
          q32w[e2] = v;
        }
        wsync();
      }
      for (int it = hl; it < nyh && valid; it += HW) {
        const int i = (it >> 1) + 1, h = it & 1, c3 = 3 * h;
        // K (this lane's three columns) first, F is not live yet; the chain in a rolled loop
        const int cl = chain_len[i];
        unsigned long long smask = kp.has_ff ? (0x3Full << kp.ff0) : 0ull;
        // Qt is zero past the sample's k rows, so every slot runs unconditionally
        double Kq[K1_QF_KMAX][3];
        const int ffo = kp.has_ff ? kp.ff0 : 0;
        const double fff = kp.has_ff ? 1.0 : 0.0;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const double* qf = Qt + (ffo + c3 + c) * K1_QF_KMAX;
#pragma unroll
          for (int j = 0; j < K1_QF_KMAX; ++j) Kq[j][c] = fff * qf[j];
        }
#pragma unroll 1
        for (int t = 0; t < cl; ++t) {
          const int d = chain[i * kp.maxch + t];
          smask |= 1ull << d;
          const double* jw = Jws + 6 * d + c3;
          const double* qd = Qt + d * K1_QF_KMAX;
          double a3[3];
#pragma unroll
          for (int c = 0; c < 3; ++c) a3[c] = jw[c];
#pragma unroll
          for (int j = 0; j < K1_QF_KMAX; ++j) {
            const double qv = qd[j];
#pragma unroll
            for (int c = 0; c < 3; ++c) Kq[j][c] += qv * a3[c];
          }
        }
        if constexpr (std::is_same_v<OutT, __bf16>) {
          // bf16 chunk panels (the Gram-only bf16 Gram, config 5): a 6 x 6 form in packed f32.  F6[c] . [own G |
          // partner's G] = output c of this lane's half (an h = 1 lane's mass slots and the h = 0 lane's inertia
          // slots are zeros: in packed f32 two columns cost one instruction, and the even split of the f64 / f32 form
          // below measured more instructions per row here, 75 vs 69, and K1 +1.7%)
          const double* bi = body + BODY_STRIDE * i;
          double F6[6][6];
          {
            double FA[24], FB[18];
            if (h == 0) body_block_mass(bi, FA);
            else body_block_inertia(bi, FB);
#pragma unroll
            for (int c = 0; c < 6; ++c)
#pragma unroll
              for (int q = 0; q < 6; ++q) {
                const int qb = (q + 3) % 6;  // the G component in slot q of an h = 1 lane (compile-time indices)
                F6[c][q] = h == 0 ? (c < 4 ? FA[6 * c + q] : 0.0) : (qb < 3 ? 0.0 : FB[3 * c + qb - 3]);
              }
          }
          OutT* oi = out + 10 * (i - 1) + 4 * h;
          // The row loop reads row r + 1's Q entries and motion-axis components while row r is multiplied, and
          // stores through the same three instructions in both lanes of a pair (an h = 0 lane rewrites its columns
          // 2, 3 with the third store: no exec-masked branch per row).  Packed FMAs (v_pk_fma_f32: two FMAs per
          // instruction at the cost of one f64 FMA); G and the block's outputs carry
          // ~1e-7 relative error, far below the bf16 rounding (2^-9) the panel gets anyway; K and F6 are formed in
          // f64 and rounded once.
          const float* q32 = reinterpret_cast<const float*>(wr + L.q32);  // row pairs (k1q32_pairs)
          // Rows in pairs: the pair's two third components of G share packed FMAs, and the loop body takes two pairs
          // with two operand sets (pair p + 1's LDS reads in flight while pair p is multiplied, no register copies
          // between iterations).  Stores: the wave-uniform row base (one sample per wave) plus this lane's 32-bit byte
          // offset (no 64-bit address per row).
          const uint32_t sb0 = (uint32_t)((10 * (i - 1) + 4 * h) * (int)sizeof(OutT));
          const uint32_t sb2 = sb0 + (uint32_t)((h ? 4 : 2) * (int)sizeof(OutT));
          char* obase = reinterpret_cast<char*>(out);
          auto rows_f32 = [&](auto kqc) {
            constexpr int KQ = decltype(kqc)::value;
            f32x2_t K01[KQ], K22[KQ];
#pragma unroll
            for (int j = 0; j < KQ; ++j) {
              K01[j] = f32x2_t{(float)Kq[j][0], (float)Kq[j][1]};
              const float k2 = (float)Kq[j][2];
              K22[j] = f32x2_t{k2, k2};
            }
            f32x2_t Fp[3][6];  // Fp[p][q] = (F6[2p][q], F6[2p + 1][q])
#pragma unroll
            for (int pp = 0; pp < 3; ++pp)
#pragma unroll
              for (int q = 0; q < 6; ++q) Fp[pp][q] = f32x2_t{(float)F6[2 * pp][q], (float)F6[2 * pp + 1][q]};
            // a pair's operands (k1q32_pairs layout): qp[j] = (Q_j of row r, of row r + 1), jq = (J_r[c3], J_r[c3 + 1],
            // J_r1[c3], J_r1[c3 + 1]), j2 = (J_r[c3 + 2], J_r1[c3 + 2])
            struct PairOps {
              f32x2_t qp[KQ];
              flt4 jq;
              f32x2_t j2;
            };
            auto pair_ld = [&](int pr, PairOps& o) {
              const float* b = q32 + 28 * pr;
#pragma unroll
              for (int j = 0; j < KQ; ++j) o.qp[j] = *reinterpret_cast<const f32x2_t*>(b + 2 * j);
              o.jq = *reinterpret_cast<const flt4*>(b + 16 + 4 * h);
              o.j2 = *reinterpret_cast<const f32x2_t*>(b + 24 + 2 * h);
            };
            auto emit = [&](int r, float g0, float g1, float g2) {
              const float G[6] = {g0, g1, g2, pair_swap_f32(g0), pair_swap_f32(g1), pair_swap_f32(g2)};
              f32x2_t y01 = f32x2_t{0.0f, 0.0f}, y23 = y01, y45 = y01;
#pragma unroll
              for (int q = 0; q < 6; ++q) {
                y01 += G[q] * Fp[0][q];
                y23 += G[q] * Fp[1][q];
              }
              // outputs 4, 5: h = 1 lanes only, whose slots 3..5 are zero
#pragma unroll
              for (int q = 0; q < 3; ++q) y45 += G[q] * Fp[2][q];
              char* rb = obase + (int64_t)r * ldp * (int64_t)sizeof(OutT);  // wave-uniform
              uint32_t o0 = sb0, o2 = sb2;
              asm volatile("" : "+v"(o0), "+v"(o2));
              panel_store_f32(reinterpret_cast<__bf16*>(rb + o0), y01.x, y01.y);
              panel_store_f32(reinterpret_cast<__bf16*>(rb + o0 + 2 * sizeof(OutT)), y23.x, y23.y);
              panel_store_f32(reinterpret_cast<__bf16*>(rb + o2), h ? y45.x : y23.x, h ? y45.y : y23.y);
            };
            auto pair_do = [&](int r, const PairOps& o) {  // rows r (even) and r + 1 (< nrows only)
              const unsigned long long sm = smask >> r;
              const f32x2_t sf = f32x2_t{(sm & 1ull) ? 1.0f : 0.0f, (sm & 2ull) ? 1.0f : 0.0f};
              f32x2_t ga = sf.x * f32x2_t{o.jq.x, o.jq.y}, gb = sf.y * f32x2_t{o.jq.z, o.jq.w};
              f32x2_t g2 = sf * o.j2;
#pragma unroll
              for (int j = 0; j < KQ; ++j) {
                ga -= o.qp[j].x * K01[j];
                gb -= o.qp[j].y * K01[j];
                g2 -= o.qp[j] * K22[j];
              }
              emit(r, ga.x, ga.y, g2.x);
              if (r + 1 < nrows) emit(r + 1, gb.x, gb.y, g2.y);
            };
            PairOps A, B;  // two operand sets: pair p + 1's reads are in flight while pair p is multiplied
            pair_ld(0, A);
            int r = 0;
#pragma unroll 1
            for (; r + 4 <= nrows; r += 4) {
              pair_ld((r >> 1) + 1, B);
              pair_do(r, A);
              pair_ld((r >> 1) + 2, A);
              pair_do(r + 2, B);
            }
            if (r < nrows) {  // 1..3 rows left, rows r, r + 1 in set A
              pair_ld((r >> 1) + 1, B);
              pair_do(r, A);
              if (r + 2 < nrows) pair_do(r + 2, B);
            }
          };
          if (kq <= 3) rows_f32(std::integral_constant<int, 3>{});
          else rows_f32(std::integral_constant<int, K1_QF_KMAX>{});
        } else {
          // The block's ten columns split evenly between the pair: lane h takes two first-moment / mass columns (2h,
          // 2h + 1: six-term dot products with [own | partner's] G) and three inertia columns (h = 0: 6, 7 and 4;
          // h = 1: 8, 9 and 5: three-term products with G's angular half, which is the partner's half for h = 0 and
          // its own for h = 1), 21 FMAs per row and lane where the 6 x 6 form took 30 (an h = 1 lane's mass slots and
          // the h = 0 lane's inertia slots were zeros).  Both lanes store with the same instructions: the pair at 2h,
          // the single column at 4 + h and the inertia pair at 6 + 2h.
          const double* bi = body + BODY_STRIDE * i;
          double F6a[2][6], F3[3][3];
          {  // one block at a time (both live at once push the kernel over the register limit)
            double FA[24];
            body_block_mass(bi, FA);
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
              for (int q = 0; q < 6; ++q)  // slot q: G component q (h = 0) or (q + 3) % 6 (h = 1): compile-time indices
                F6a[a][q] = h ? FA[6 * (2 + a) + (q + 3) % 6] : FA[6 * a + q];
          }
          {
            double FB[18];
            body_block_inertia(bi, FB);
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
              for (int j = 0; j < 3; ++j) F3[a][j] = h ? FB[3 * (a == 2 ? 1 : 4 + a) + j] : FB[3 * (a == 2 ? 0 : 2 + a) + j];
          }
          OutT* oi = out + 10 * (i - 1);
          const int o6 = 2 * h, o3 = 6 + 2 * h, o1 = 4 + h;  // column offsets of the lane's stores
          const double* jrs = Jws + c3;
          // The row loops read row r + 1's Q entries and motion-axis components while row r is multiplied (one LDS
          // wait per row, behind a row of arithmetic, instead of two waits up front).
          auto rows = [&](auto kqc) {
            constexpr int KQ = decltype(kqc)::value;
            constexpr int KQ2 = (KQ + 1) / 2;
            double qn[2 * KQ2], jn[3];
            auto row_ld = [&](int r, double* qv, double* jv) {
              const double2* q2 = reinterpret_cast<const double2*>(Qt + r * K1_QF_KMAX);
#pragma unroll
              for (int j = 0; j < KQ2; ++j) {
                const double2 v = q2[j];
                qv[2 * j] = v.x;
                qv[2 * j + 1] = v.y;
              }
              const double* jr = jrs + 6 * r;
#pragma unroll
              for (int c = 0; c < 3; ++c) jv[c] = jr[c];
            };
            row_ld(0, qn, jn);
#pragma unroll 1
            for (int r = 0; r < nrows; ++r) {
              const double sf = ((smask >> r) & 1ull) ? 1.0 : 0.0;
              double qr[2 * KQ2], jr[3];
#pragma unroll
              for (int j = 0; j < 2 * KQ2; ++j) qr[j] = qn[j];
#pragma unroll
              for (int c = 0; c < 3; ++c) jr[c] = jn[c];
              row_ld(r + 1 < nrows ? r + 1 : r, qn, jn);
              double G[6];
#pragma unroll
              for (int c = 0; c < 3; ++c) G[c] = sf * jr[c];
#pragma unroll
              for (int j = 0; j < KQ; ++j)
#pragma unroll
                for (int c = 0; c < 3; ++c) G[c] -= qr[j] * Kq[j][c];
#pragma unroll
              for (int c = 0; c < 3; ++c) G[3 + c] = pair_swap(G[c]);
              double ga[3];  // G's angular half
#pragma unroll
              for (int c = 0; c < 3; ++c) ga[c] = h ? G[c] : G[3 + c];
              double y6[2], y3[3];
#pragma unroll
              for (int a = 0; a < 2; ++a)
                y6[a] = G[0] * F6a[a][0] + G[1] * F6a[a][1] + G[2] * F6a[a][2] + G[3] * F6a[a][3] +
                        G[4] * F6a[a][4] + G[5] * F6a[a][5];
#pragma unroll
              for (int a = 0; a < 3; ++a) y3[a] = ga[0] * F3[a][0] + ga[1] * F3[a][1] + ga[2] * F3[a][2];
              OutT* o2 = oi + (int64_t)r * ldp;
              panel_store(o2 + o6, y6[0], y6[1]);
              panel_store(o2 + o3, y3[0], y3[1]);
              panel_store1(o2 + o1, y3[2]);
            }
          };
          if (kq <= 3) rows(std::integral_constant<int, 3>{});
          else rows(std::integral_constant<int, K1_QF_KMAX>{});
        }
      }
    } else {
      for (int it = hl; it < nyi && valid; it += HW) {
        const int g = it / nbody, i = it - g * nbody + 1;
        const int r0 = g * nrows / kp.rg, r1 = (g + 1) * nrows / kp.rg;
        double F[FBLK];
        int dof[MAXCH];  // the chain's dofs, read once: no dependent index load per row
        const int cl = block_setup(i, F, dof);
        OutT* oi = out + 10 * (i - 1);
        for (int r = r0; r < r1; ++r) {
          double y[10];
          block_row(r, F, dof, cl, y);
          OutT* o2 = oi + (int64_t)r * ldp;
#pragma unroll
          for (int c = 0; c < 5; ++c) panel_store(o2 + 2 * c, y[2 * c], y[2 * c + 1]);
        }
      }
    }
    // ---- [B_v | B_c | tau_proj | pad]: 16-byte stores of column pairs ----
    // Up to 32 pairs (nj <= 31): lane = column pair m within a group of gs = 8, 16 or 32 lanes (the
    // narrowest that holds the pairs), the HW/gs groups taking every (HW/gs)-th row, so a lane's dq / sign(dq)
    // factors and column selects are fixed over its rows (Spot: 15 pairs, two 16-lane groups, 9 rows each);
    // otherwise lane = (row, column pair) with a division per item.
    const int npair = (kp.out_cols - kp.wy) >> 1;  // out_cols and wy are even
    if (NVC == 18 || npair <= 32) {
      const int lg = npair <= 8 ? 3 : (npair <= 16 ? 4 : 5);  // log2 of the group width
      const int NG = HW >> lg;
      const int fg = hl >> lg, m = hl & ((1 << lg) - 1);
      if (m < npair && valid) {
        int jc[2];
        double sc[2];
        bool tcol[2], fcol[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int jj = 2 * m + u;  // column - wy
          const bool coul = jj >= nja;
          const int j = coul ? jj - nja : jj;
          jc[u] = j < nja ? j : nja - 1;  // clamp for the tau/pad columns
          const double x = dqs[bd + jc[u]];
          sc[u] = coul ? sign_of(x) : x;
          fcol[u] = jj < 2 * nja;
          tcol[u] = kp.wy + jj == kp.w;
        }
        OutT* po = out + (int64_t)fg * ldp + kp.wy + 2 * m;  // advanced by NG rows per pass
        const int64_t pstep = (int64_t)NG * ldp;
        if constexpr (QF) {
          // P[r, bd + j] = δ - Σ_i Q_i[r] Q_i[bd + j]: the lane's two columns of Q in registers
          const int kq = __builtin_amdgcn_readfirstlane(kfull ? 0 : k);  // wave-uniform (one sample per wave)
          (void)kq;
          double qc[K1_QF_KMAX][2];
#pragma unroll
          for (int j = 0; j < K1_QF_KMAX; ++j)
#pragma unroll
            for (int u = 0; u < 2; ++u) qc[j][u] = Qt[(bd + jc[u]) * K1_QF_KMAX + j];  // zero past k
          if constexpr (std::is_same_v<OutT, __bf16>) {
            // bf16 chunk panels: the same in packed f32 from the per-sample f32 rows (q32, made by the Y phase)
            const float* q32 = reinterpret_cast<const float*>(wr + L.q32);
            f32x2_t qc2[K1_QF_KMAX];
#pragma unroll
            for (int j = 0; j < K1_QF_KMAX; ++j) qc2[j] = f32x2_t{(float)qc[j][0], (float)qc[j][1]};
            const f32x2_t sc2 = f32x2_t{fcol[0] ? (float)sc[0] : 0.0f, fcol[1] ? (float)sc[1] : 0.0f};
            // row pairs (the k1q32_pairs layout: a pair's Q entries in three 16-byte reads), group fg taking every NG-th
            // pair; stores from the sample's wave-uniform base (one sample per wave) plus the lane's 32-bit offset
            char* fbase = reinterpret_cast<char*>(out);
            const uint32_t frow = (uint32_t)ldp * (uint32_t)sizeof(OutT), fstep = 2 * (uint32_t)NG * frow;
            uint32_t fo = (uint32_t)((2 * fg * (int)ldp + kp.wy + 2 * m) * (int)sizeof(OutT));  // pair fg's first row
            const int npr = (nrows + 1) >> 1;
            for (int pr = fg; pr < npr; pr += NG, fo += fstep) {
              const float* b = q32 + 28 * pr;
              f32x2_t qp[K1_QF_KMAX];
#pragma unroll
              for (int j = 0; j < K1_QF_KMAX; ++j) qp[j] = *reinterpret_cast<const f32x2_t*>(b + 2 * j);
              const int r0 = 2 * pr, r1 = r0 + 1;
              f32x2_t pa = f32x2_t{r0 == bd + jc[0] ? 1.0f : 0.0f, r0 == bd + jc[1] ? 1.0f : 0.0f};
              f32x2_t pb = f32x2_t{r1 == bd + jc[0] ? 1.0f : 0.0f, r1 == bd + jc[1] ? 1.0f : 0.0f};
#pragma unroll
              for (int j = 0; j < K1_QF_KMAX; ++j) {
                pa -= qp[j].x * qc2[j];
                pb -= qp[j].y * qc2[j];
              }
              pa *= sc2;
              pb *= sc2;
              asm volatile("" : "+v"(pb));  // formed beside pa (interleaved packed FMAs), not sunk into the odd-row branch
              const float ta = (float)tps[r0], tb = (float)tps[r1 < nrows ? r1 : r0];
              uint32_t o = fo, o1 = fo + frow;
              asm volatile("" : "+v"(o), "+v"(o1));
              panel_store_f32(reinterpret_cast<__bf16*>(fbase + o), tcol[0] ? ta : pa.x, tcol[1] ? ta : pa.y);
              if (r1 < nrows) panel_store_f32(reinterpret_cast<__bf16*>(fbase + o1), tcol[0] ? tb : pb.x, tcol[1] ? tb : pb.y);
            }
          } else {
          double qn[K1_QF_KMAX], tn = 0.0;  // row r + NG's Q entries and torque, read while row r is formed
          auto fr_ld = [&](int r) {
            const double2* q2 = reinterpret_cast<const double2*>(Qt + r * K1_QF_KMAX);
#pragma unroll
            for (int j = 0; j < K1_QF_KMAX / 2; ++j) {
              const double2 v = q2[j];
              qn[2 * j] = v.x;
              qn[2 * j + 1] = v.y;
            }
            tn = tps[r];
          };
          if (fg < nrows) fr_ld(fg);
          for (int r = fg; r < nrows; r += NG, po += pstep) {
            double qv[K1_QF_KMAX];
#pragma unroll
            for (int j = 0; j < K1_QF_KMAX; ++j) qv[j] = qn[j];
            const double t = tn;
            fr_ld(r + NG < nrows ? r + NG : r);
            double pe[2] = {r == bd + jc[0] ? 1.0 : 0.0, r == bd + jc[1] ? 1.0 : 0.0};
#pragma unroll
            for (int j = 0; j < K1_QF_KMAX; ++j) {
              pe[0] -= qv[j] * qc[j][0];
              pe[1] -= qv[j] * qc[j][1];
            }
            double v2[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) v2[u] = fcol[u] ? pe[u] * sc[u] : (tcol[u] ? t : 0.0);
            panel_store(po, v2[0], v2[1]);
          }
          }
        } else if constexpr (NVC == 18 && HW == 32 && !CMP) {
          // Spot / Solo (13 column pairs: two 16-lane groups, 9 rows each): every row's LDS reads issued up front
          // instead of one wait per row of the rolled loop (Spot K1 -4%, profiles/r05_s4)
          constexpr int NR = NVC > 0 ? NVC / 2 : 1;
          double pv[NR][2], tv[NR];
#pragma unroll
          for (int i = 0; i < NR; ++i) {
            const int r = fg + 2 * i;
            const double* pr = Ps + r * NVC + bd;
            pv[i][0] = pr[jc[0]];
            pv[i][1] = pr[jc[1]];
            tv[i] = tps[r];
          }
#pragma unroll
          for (int i = 0; i < NR; ++i) {
            double v2[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) v2[u] = fcol[u] ? pv[i][u] * sc[u] : (tcol[u] ? tv[i] : 0.0);
            panel_store(po + i * pstep, v2[0], v2[1]);
          }
        } else {
          for (int r = fg; r < nrows; r += NG, po += pstep) {
            const double* pr = Ps + r * nv + bd;
            const double t = tps[r];
            double v2[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) v2[u] = fcol[u] ? pr[jc[u]] * sc[u] : (tcol[u] ? t : 0.0);  // pad: whole lines
            panel_store(po, v2[0], v2[1]);
          }
        }
      }
    } else {
      for (int it = hl; it < nrows * npair && valid; it += HW) {
        const int r = it / npair, m = it - r * npair;
        const double* pr = Ps + r * nv + bd;
        double v2[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int jj = 2 * m + u;                      // column - wy
          const bool coul = jj >= nja;
          const int j = coul ? jj - nja : jj;
          const int jc = j < nja ? j : nja - 1;          // clamp for the tau/pad columns
          const double x = dqs[bd + jc];
          const double sc = coul ? sign_of(x) : x;
          const double fr = pr[jc] * sc;
          v2[u] = jj < 2 * nja ? fr : (kp.wy + jj == kp.w ? tps[r] : 0.0);  // pad: keep lines whole
        }
        panel_store(out + (int64_t)r * ldp + kp.wy + 2 * m, v2[0], v2[1]);
      }
    }
    __builtin_amdgcn_s_setprio(2);
    s = s1;
    s1 = s2;
  }
}

template <int MAXCH, int NVC, int SPW, typename OutT, int POV = 0, int CMP = 0, int QF = 0>
// Two-sample waves are held to 256 registers (2 waves per SIMD, which the LDS budget allows there).
// The P overlay's instantiations run 8 one-sample waves per workgroup (one 8-wave workgroup per CU).
__global__ void __launch_bounds__(POV ? 512 : 64 * K1_WAVES, SPW == 2 || QF ? 2 : 1)
k1_regressor_panel(const K1Params kp, const uint32_t* __restrict__ mimg_g, const double* __restrict__ in,
                   int64_t N, int64_t ld, OutT* __restrict__ panel, int64_t ldp,
                   unsigned long long* __restrict__ work, double* __restrict__ dbg,
                   int* __restrict__ rcount) {
  k1_body<MAXCH, NVC, SPW, OutT, POV, CMP, QF>(kp, mimg_g, in, N, ld, panel, ldp, work, dbg, rcount);
}

// ------------------------------------------------------------------------------------------------
// K1s (nullspace mode): the list of live chunk-panel rows, in sample order, for the Gram kernels to gather.
// k1s_seg_sums: rseg[b] = the rows of the 1024 samples of segment b.  k1s_row_list: block b's first list
// position is the sum of the earlier segments' rows (from rseg, or, rseg = nullptr, summed from rcount itself: one
// launch instead of two for chunks of at most K1S_ONEPASS_SEGS segments), then a block scan of its own samples'
// counts; sample s with m rows lists s·nv, ..., s·nv + m - 1.  The last block writes the total.  Plain stores and integer
// arithmetic only (no atomics, nothing to zero beforehand): deterministic, and graph replays start clean.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int k1s_wave_incl(int v, int lane) {  // inclusive scan over the 64 lanes
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int u = __shfl_up(v, d, 64);
    if (lane >= d) v += u;
  }
  return v;
}

#ifndef SYSID_TEMPLATE_TU  // the non-template kernels live in sysid_engine.hip's translation unit only
// Zeroing on the device entry points' streams is done by kernels, never hipMemsetAsync: captured into a HIP graph,
// a memset became a node that a replay did not order after the default-stream writes just before it (measured:
// a 0xFF-filled workspace replayed into claim counters still at 0xFF..., so K1 claimed no samples and the Gram
// came back NaN or empty; tools/dbg_ns_graph.py, profiles/r04_dbg).  Kernel nodes are ordered.
__global__ void __launch_bounds__(256) k0_zero_u64(unsigned long long* __restrict__ p, int64_t n) {
  for (int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x; x < n; x += (int64_t)gridDim.x * 256) p[x] = 0ull;
}

// Host entry points' wire format (sysid_engine.hip, wire_layout): one block per staged chunk of n samples — q rows
// (nq x n, float32 when the caller's q is float32 as read_data returns it, else float64), the dq / ddq / tau rows
// (nd x n float64) and the contact rows (nc x n bytes: 1 where the value is non-zero, the only property the
// projector reads) — sent as one DMA (the first chunk: read by K0W from the mapped page-locked staging block
// itself, sysid_engine.hip Stager::stage).  K0W widens chunk [c0, c0 + n) into the row-major float64 input block K1
// reads (rows x ld) and zeroes K1's claim counters (`work`, nwork words) on the way: one launch per chunk, exact
// (float32 -> float64 and the 0 / 1 contacts).  Block (x, y): samples of row y.
__global__ void __launch_bounds__(256) k0_widen(const unsigned char* __restrict__ wire, int64_t n, int nq, int nd,
                                                int qsz, int64_t offd, int64_t offc, double* __restrict__ dst,
                                                int64_t ld, unsigned long long* __restrict__ work, int nwork) {
  if (work != nullptr && blockIdx.x == 0 && blockIdx.y == 0)
    for (int x = threadIdx.x; x < nwork; x += 256) work[x] = 0ull;
  const int r = blockIdx.y;
  double* out = dst + (int64_t)r * ld;
  for (int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x; s < n; s += (int64_t)gridDim.x * 256) {
    double v;
    if (r < nq)
      v = qsz == 4 ? (double)reinterpret_cast<const float*>(wire)[(int64_t)r * n + s]
                   : reinterpret_cast<const double*>(wire)[(int64_t)r * n + s];
    else if (r < nq + nd)
      v = reinterpret_cast<const double*>(wire + offd)[(int64_t)(r - nq) * n + s];
    else
      v = wire[offc + (int64_t)(r - nq - nd) * n + s] ? 1.0 : 0.0;
    out[s] = v;
  }
}

__global__ void __launch_bounds__(256)
k1s_seg_sums(const int* __restrict__ rcount, int n, int* __restrict__ rseg) {
  __shared__ int wsum[4];
  const int b = (int)blockIdx.x, t = (int)threadIdx.x, lane = t & 63, w = t >> 6;
  const int s0 = (b << K1_SEG_LOG) + 4 * t;
  int loc = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) loc += s0 + u < n ? rcount[s0 + u] : 0;
  loc = __shfl(k1s_wave_incl(loc, lane), 63, 64);
  if (lane == 0) wsum[w] = loc;
  __syncthreads();
  if (t == 0) rseg[b] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

__global__ void __launch_bounds__(256)
k1s_row_list(const int* __restrict__ rcount, const int* __restrict__ rseg, int n, int nv, int* __restrict__ rowlist,
             int* __restrict__ total) {
  __shared__ int wsum[4];
  const int b = (int)blockIdx.x, t = (int)threadIdx.x, lane = t & 63, w = t >> 6;
  auto wave_incl = [&](int v) { return k1s_wave_incl(v, lane); };
  int pre = 0;
  if (rseg != nullptr) {
    for (int x = t; x < b; x += 256) pre += rseg[x];
  } else {  // short chunks: the earlier (whole) segments' counts summed here, no k1s_seg_sums launch
    const int4* r4 = reinterpret_cast<const int4*>(rcount);
    for (int x = t; x < (b << (K1_SEG_LOG - 2)); x += 256) {
      const int4 v = r4[x];
      pre += (v.x + v.y) + (v.z + v.w);
    }
  }
  pre = __shfl(wave_incl(pre), 63, 64);
  if (lane == 0) wsum[w] = pre;
  __syncthreads();
  const int base = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  int c[4], loc = 0;
  const int s0 = (b << K1_SEG_LOG) + 4 * t;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    c[u] = s0 + u < n ? rcount[s0 + u] : 0;
    loc += c[u];
  }
  const int incl = wave_incl(loc);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int o = base + incl - loc;
  for (int x = 0; x < w; ++x) o += wsum[x];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r0 = (s0 + u) * nv;
    for (int j = 0; j < c[u]; ++j) rowlist[o + j] = r0 + j;
    o += c[u];
  }
  if (b == (int)gridDim.x - 1 && t == 255) *total = o;
}

#endif  // SYSID_TEMPLATE_TU

// ------------------------------------------------------------------------------------------------
// K2: G_partial[ks] = panel[rows of ks]^T panel[rows of ks]   (fp64 MFMA 16x16x4, upper tiles)
//
// Each workgroup (k2_waves(NTC) waves) walks a contiguous row range in chunks of KC rows.  A chunk of the
// panel is one contiguous byte range in HBM; every thread copies fixed double2 slots of it (offsets
// computed once, no divisions in the loop) through registers into an LDS buffer with a padded row
// stride (STRIDE ≡ 16 mod 32 doubles, so the 2 rows x 16 doubles of a 32-lane ds_read_b64 group hit
// disjoint banks).  Two LDS buffers and two staging register sets: chunk c+2's global loads are in flight
// while chunk c is multiplied and chunk c+1 is written to LDS.
// Each wave owns k2_spw(NTC) "super-tiles" (2x2 blocks of 16x16 output tiles): 4 fragment reads feed 4 MFMAs.
// The k-loop over a chunk is fully unrolled, so fragment reads use immediate LDS offsets.
// Fragment = 16 consecutive doubles of 4 consecutive rows: lane l holds row (l>>4), col (l&15), which is
// both the A layout (A[i=l&15][k=l>>4]) and the B layout (B[k=l>>4][j=l&15]) of v_mfma_f64_16x16x4_f64.
// ------------------------------------------------------------------------------------------------
// Waves per K2 workgroup and super-tile slots per wave, by Gram width: narrow Grams (one workgroup holds every
// super-tile, Spot: 16 pieces) run 16 waves of one slot each -- four waves per SIMD hide the per-chunk barrier
// and fragment-read latency better than two waves of two slots (Spot K2 -3.9%, profiles/r02_ab2/k2_waves16_ab.txt);
// wide ones 8 waves of two slots (the LDS-DMA kernel deals its chunk rows to 8 waves).
__host__ __device__ constexpr int k2_waves(int ntc) { return ntc < 16 ? 16 : 8; }
__host__ __device__ constexpr int k2_spw(int ntc) { return ntc < 16 ? 1 : 2; }
constexpr int K2_BF16_WAVES = 8;  // the bf16 kernel's waves
// Super-tile slots per wave of the f64 / f32 kernels (f32 keeps 2 for wide Grams: 4 measured 1.5% faster,
// 5 cost a workgroup per CU, profiles/r02_ab3/k2_f32_slots_per_wave_g1_125k.txt).
template <typename T>
__host__ __device__ constexpr int k2_slots(int ntc) { return k2_spw(ntc); }
// Super-tile slots per wave of the bf16 kernels.  A bf16 k-step is only 16 MFMA cycles per tile, so the kernel
// is fed, not MFMA, bound: every super-tile group re-reads (and re-stages) the whole panel, and with the f64
// kernels' 16 slots per group G1 (78 super-tiles) took 5 groups = 5 panel reads (G1 125k K2 3.1 ms).  Wide
// Grams run k2_gram_syrk_bf16_tr with 10 slots per wave (all of G1's super-tiles in one workgroup: the panel is
// read once; 5 slots: 1.64 vs 1.49 ms); narrow ones the f64 kernels' deal.
__host__ __device__ constexpr int k2_bf16_spw(int ntc) {
  return ntc >= 16 ? 10 : k2_waves(ntc) * k2_spw(ntc) / K2_BF16_WAVES;
}
// Measured and not kept: readfirstlane'd descriptors in the f64 kernels (G1 K2 1.80 -> 2.26 ms, Spot +3%);
// computing the redundant lower tiles of diagonal super-tiles too (Spot +6%, G1 +9%).

// Reduced-precision Gram (error reported, not gated): T = float runs the same
// kernel on v_mfma_f32_16x16x4_f32 (panel rounded to f32 while staged, f32 accumulation per workgroup,
// f64 across workgroups in K3); bf16 is k2_gram_syrk_bf16 below.
template <typename T> struct K2Acc;
template <> struct K2Acc<double> { typedef dbl4 type; };
template <> struct K2Acc<float> { typedef flt4 type; };

// Super-tile slot descriptor {I0, J0 | skip << 8}: skip bit t drops tile t = 2a + b (a super-tile split into
// row halves over two slots by the host's balancing; 0 otherwise).
__device__ __forceinline__ bool k2_tile_skip(int2 sp, int t) { return sp.x >= 0 && ((sp.y >> (8 + t)) & 1); }

// Workgroup -> (split-K slice ks, super-tile group).  Every group of a slice reads the same panel rows, so
// with several groups (wide Grams: G1 has 5) the rows are re-read once per group.  Blocks are dealt
// round-robin over the 8 XCDs (b and b + 8 share one, MI355X_MICROARCH.md §Workgroup dispatch), so the
// plain ks = b / ngroups put a slice's groups on different XCDs and every re-read went to HBM / MALL
// (G1 K2 at ~6 TB/s of re-reads).  Here the blocks of one XCD take consecutive (ks, group) pairs, so a
// slice's groups share an L2 and run side by side: one HBM read, the others L2 hits.  A bijection for any
// grid; speed only (any placement is correct).
__device__ __forceinline__ void k2_block_coords(int ngroups, int& group, int& ks) {
  int L = (int)blockIdx.x;
  if (ngroups > 1) {
    const int nb = (int)gridDim.x, x = L & 7, i = L >> 3;
    const int q = nb >> 3, r = nb & 7;  // XCD y holds q + (y < r) blocks
    L = x * q + (x < r ? x : r) + i;
  }
  group = L % ngroups;
  ks = L / ngroups;
}

__host__ __device__ constexpr int k2_stride(int ntc) { return ((ntc * 16 + 31) / 32) * 32 + 16; }

// Rows per staged chunk of the bf16 kernel: as many whole 32-row k-steps as two column-major LDS buffers of
// NTC*16 columns x (KC + 8) bf16 fit in ~150 KB, at most 128.  Each chunk is one global-load latency of the
// staging loop, and one bf16 k-step is only 16 cycles of MFMA per tile: small chunks left the kernel
// latency-bound (KC = 32: G1 125k K2 4.4 ms, 0.7 TB/s of staged panel).
__host__ __device__ constexpr int k2_bf16_kc(int ntc) {
  return ((150 * 1024 / (64 * ntc)) - 8) / 32 * 32 > 128 ? 128
         : ((150 * 1024 / (64 * ntc)) - 8) / 32 * 32 < 32 ? 32
                                                          : ((150 * 1024 / (64 * ntc)) - 8) / 32 * 32;
}

// GATHER (nullspace mode): the rows are those listed in rowlist (k1s_row_list), *d_rows of them.  A staging slot's
// row of the chunk after next is looked up one chunk ahead of its load (one list entry per slot and chunk, two
// register sets), so the gather adds a 4-byte load per slot and no latency to the staging pipeline.
template <typename T, int NTC, int KC, bool GATHER>
__device__ __forceinline__ void k2_syrk_body(const T* __restrict__ panel, int64_t rows, int64_t ldp,
                                             const int2* __restrict__ supers, int ngroups, int ksplit, int nslots,
                                             int accumulate, double* __restrict__ slab,
                                             const int* __restrict__ rowlist, const int* __restrict__ d_rows) {
  typedef typename K2Acc<T>::type accT;
  constexpr int K2W = k2_waves(NTC), K2S = k2_slots<T>(NTC);
  constexpr int STRIDE = k2_stride(NTC);
  constexpr int BUF = KC * STRIDE;                       // elements per LDS buffer
  constexpr int NT = 64 * K2W;
  __shared__ T lds[2 * BUF];
  int group, ks;
  k2_block_coords(ngroups, group, ks);
  const int64_t prows = rows;  // GATHER: the panel's rows (the list holds at most these)
  if constexpr (GATHER) rows = min((int64_t)__builtin_amdgcn_readfirstlane(*d_rows), prows);
  // whole chunks per workgroup: only the panel's last chunk may be partial
  const int64_t nck = (rows + KC - 1) / KC;
  const int64_t r0 = (nck * ks / ksplit) * KC;
  const int64_t r1 = ks + 1 == ksplit ? rows : (nck * (ks + 1) / ksplit) * KC;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int sbase = (group * K2W + wave) * K2S;

  // zero both buffers once: columns >= ldp (up to NTC*16) are never staged and must read as 0
  for (int x = threadIdx.x; x < 2 * BUF; x += NT) lds[x] = 0.0;

  // staging slots: the chunk is KC*ldp contiguous elements; thread slot u copies the 16 bytes [EP x, EP x + EP)
  // (EP = 2 doubles or 4 floats; the panel's ld is a multiple of EP, so a slot never straddles two rows)
  constexpr int EP = 16 / (int)sizeof(T);
  const int chunk_s = (int)((KC * ldp) / EP);
  constexpr int PER = (KC * NTC * 16 / EP + NT - 1) / NT;  // >= ceil(KC*ldp/EP / NT)
  int loff[PER];
  bool used[PER];
  int srow[PER], scol[PER];  // GATHER: the slot's row in the chunk and element offset in the row
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int x = threadIdx.x + u * NT;
    used[u] = x < chunk_s;
    const int e = EP * x;
    const int row = used[u] ? e / (int)ldp : 0;
    loff[u] = used[u] ? row * STRIDE + (e - row * (int)ldp) : 0;
    if constexpr (GATHER) {
      srow[u] = row;
      scol[u] = used[u] ? e - row * (int)ldp : 0;
    }
  }
  auto list_row = [&](int64_t x) -> int64_t {  // a list entry, clamped into the panel
    const int v = rowlist[x];
    return v >= 0 && v < prows ? v : 0;
  };
  uint4 st[PER];
  auto load_chunk = [&](int64_t c0) {
    const uint4* src = reinterpret_cast<const uint4*>(panel + c0 * ldp);
    const int64_t lim = (r1 - c0) * ldp / EP;  // 16-byte slots inside [c0, r1)
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int x = threadIdx.x + u * NT;
      if constexpr (GATHER) {
        const bool live = used[u] && c0 + srow[u] < r1;
        st[u] = live ? *reinterpret_cast<const uint4*>(panel + list_row(c0 + srow[u]) * ldp + scol[u])
                     : make_uint4(0u, 0u, 0u, 0u);
      } else {
        st[u] = (used[u] && x < lim) ? src[x] : make_uint4(0u, 0u, 0u, 0u);
      }
    }
  };
  auto store_chunk = [&](T* b) {
#pragma unroll
    for (int u = 0; u < PER; ++u)
      if (used[u]) *reinterpret_cast<uint4*>(b + loff[u]) = st[u];
  };

  // One super-tile slot per wave (K2S = 1: this kernel serves the narrow Grams, < 16 tile columns).  Its
  // fragment columns are {I0, I0+1, J0, J0+1} (16-column blocks) and its tile mask (tile t = 2a + b is (I0 + a,
  // J0 + b); a diagonal super-tile skips its lower tile, tiles past NTC and a split super-tile's other half are
  // skipped) is wave-uniform.  The chunk loop below is instantiated once per mask and selected by one scalar
  // switch, so the k-loop is straight-line MFMAs: a per-tile `if (need)` on a value the compiler could not prove
  // uniform had wrapped every MFMA in an exec-mask save / branch / restore (3.4 SALU + 1.4 branches per MFMA,
  // profiles/r03_pmc) with an lgkmcnt(0) in front of it, and serialised the fragment reads of consecutive k-steps.
  static_assert(K2S == 1, "one super-tile slot per wave");
  const int2 sp = supers[sbase];
  int foff[4];
  int mask = 0;
  {
    const bool live = sp.x >= 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int I = 2 * sp.x + (t >> 1), J = 2 * (sp.y & 0xFF) + (t & 1);
      mask |= (live && I <= J && J < NTC && !k2_tile_skip(sp, t)) ? 1 << t : 0;
    }
    const int blk[4] = {2 * sp.x, 2 * sp.x + 1, 2 * (sp.y & 0xFF), 2 * (sp.y & 0xFF) + 1};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int b = live && blk[u] < NTC ? blk[u] : 0;
      foff[u] = (lane >> 4) * STRIDE + 16 * b + (lane & 15);
    }
  }
  mask = __builtin_amdgcn_readfirstlane(mask);
  const bool live = sp.x >= 0;

  const int64_t nfull = (r1 - r0) / KC;
  uint4 sa[PER], sb[PER];  // the two staging register sets (selected at compile time)
  int64_t la[PER], lb[PER];  // GATHER: the slots' panel rows of the chunk set A / B loads next
  // GATHER: the list entries of chunk c into set S (clamped like load_full: past the last full chunk, its rows again)
  auto list_full = [&](int64_t c, auto set) {
    if constexpr (GATHER) {
      constexpr int S = decltype(set)::value;
      const int64_t cc = c < nfull ? c : nfull - 1;
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int64_t v = list_row(r0 + cc * KC + srow[u]);
        if constexpr (S == 0) la[u] = v; else lb[u] = v;
      }
    }
  };
  auto load_full = [&](int64_t c, auto set) {
    constexpr int S = decltype(set)::value;
    const int64_t cc = c < nfull ? c : nfull - 1;
    const uint4* src = reinterpret_cast<const uint4*>(panel + (r0 + cc * KC) * ldp);
#pragma unroll
    for (int u = 0; u < PER; ++u) {  // unconditional (an unused slot re-reads the chunk's last 16 bytes)
      const int x = (int)threadIdx.x + u * NT;
      if constexpr (GATHER) {
        const uint4 v = *reinterpret_cast<const uint4*>(panel + (S == 0 ? la[u] : lb[u]) * ldp + scol[u]);
        if constexpr (S == 0) sa[u] = v; else sb[u] = v;
      } else {
        const uint4 v = src[x < chunk_s ? x : chunk_s - 1];
        if constexpr (S == 0) sa[u] = v; else sb[u] = v;
      }
    }
  };
  auto store_set = [&](auto set, T* b) {
    constexpr int S = decltype(set)::value;
#pragma unroll
    for (int u = 0; u < PER; ++u)
      if (used[u]) *reinterpret_cast<uint4*>(b + loff[u]) = S == 0 ? sa[u] : sb[u];
  };

  // Loads run two chunks ahead through two register sets: chunk c + 2 is requested while chunk c is
  // multiplied and chunk c + 1 (requested one chunk earlier) is written to the other LDS buffer, so each
  // load has about two chunks of MFMA time to land.  Every load is unconditional (past the last full chunk
  // the index is clamped: a reload of a chunk just read, from L2), so the compiler's vmcnt bookkeeping
  // waits only for the set being stored.  The partial tail chunk of the panel's last workgroup runs last,
  // zero-filled.
  auto run = [&](auto mc) {
    constexpr int M = decltype(mc)::value;
    // fragments the mask reads: A0 = I0 (tiles 0, 1), A1 = I0 + 1 (2, 3), B0 = J0 (0, 2), B1 = J0 + 1 (1, 3)
    constexpr bool uA0 = M & 3, uA1 = M & 12, uB0 = M & 5, uB1 = M & 10;
    accT acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = accT{0, 0, 0, 0};
    auto mfma_chunk = [&](const T* cur) {
#pragma unroll
      for (int kk = 0; kk < KC; kk += 4) {
        T x[4] = {0, 0, 0, 0};
        if constexpr (uA0) x[0] = cur[foff[0] + kk * STRIDE];
        if constexpr (uA1) x[1] = cur[foff[1] + kk * STRIDE];
        if constexpr (uB0) x[2] = cur[foff[2] + kk * STRIDE];
        if constexpr (uB1) x[3] = cur[foff[3] + kk * STRIDE];
        auto tile = [&](auto tc) {  // tile t = 2a + b: A fragment a, B fragment 2 + b
          constexpr int t = decltype(tc)::value;
          if constexpr (((M >> t) & 1) != 0) {
            if constexpr (sizeof(T) == 8)
              acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(x[t >> 1], x[2 + (t & 1)], acc[t], 0, 0, 0);
            else
              acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[t >> 1], x[2 + (t & 1)], acc[t], 0, 0, 0);
          }
        };
        tile(std::integral_constant<int, 0>{});
        tile(std::integral_constant<int, 1>{});
        tile(std::integral_constant<int, 2>{});
        tile(std::integral_constant<int, 3>{});
      }
    };
    constexpr std::integral_constant<int, 0> A{};
    constexpr std::integral_constant<int, 1> B{};
    __syncthreads();  // LDS zeroed
    if (nfull > 0) {
      if constexpr (GATHER) list_full(0, A);
      if constexpr (GATHER) list_full(1, B);
      load_full(0, A);
      load_full(1, B);
      if constexpr (GATHER) list_full(2, A);
      store_set(A, lds);
    }
    __syncthreads();
    int64_t c = 0;
    for (; c + 1 < nfull; c += 2) {  // chunks c (buffer 0, set A) and c + 1 (buffer 1, set B)
      if constexpr (GATHER) list_full(c + 3, B);
      load_full(c + 2, A);
      mfma_chunk(lds);
      store_set(B, lds + BUF);
      __syncthreads();
      if constexpr (GATHER) list_full(c + 4, A);
      load_full(c + 3, B);
      mfma_chunk(lds + BUF);
      if (c + 2 < nfull) store_set(A, lds);
      __syncthreads();
    }
    if (c < nfull) {  // an odd last full chunk, already in buffer 0
      mfma_chunk(lds);
      __syncthreads();
    }
    if (r0 + nfull * KC < r1) {  // the panel's partial last chunk
      load_chunk(r0 + nfull * KC);
      store_chunk(lds);
      __syncthreads();
      mfma_chunk(lds);
    }
    // D layout: col = lane & 15; row = (lane >> 4) + 4 * reg for f64, 4 * (lane >> 4) + reg for f32.  Only the
    // mask's tiles are written: K3 reads the tile slots the deal lists, never a skipped one.
    if (!live) return;
    auto put = [&](auto tc) {
      constexpr int t = decltype(tc)::value;
      if constexpr (((M >> t) & 1) != 0) {
        double* o = slab + ((size_t)ks * nslots + (size_t)sbase * 4 + t) * 256;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = sizeof(T) == 8 ? (lane >> 4) + 4 * j : 4 * (lane >> 4) + j;
          double* x = o + row * 16 + (lane & 15);
          const double v = (double)acc[t][j];
          *x = accumulate ? *x + v : v;  // chunked Gram: slabs carry over chunks
        }
      }
    };
    put(std::integral_constant<int, 0>{});
    put(std::integral_constant<int, 1>{});
    put(std::integral_constant<int, 2>{});
    put(std::integral_constant<int, 3>{});
  };
  switch (mask) {
#define SYSID_K2_MASK(m) \
  case m:                \
    run(std::integral_constant<int, m>{}); \
    break;
    SYSID_K2_MASK(0) SYSID_K2_MASK(1) SYSID_K2_MASK(2) SYSID_K2_MASK(3) SYSID_K2_MASK(4) SYSID_K2_MASK(5)
    SYSID_K2_MASK(6) SYSID_K2_MASK(7) SYSID_K2_MASK(8) SYSID_K2_MASK(9) SYSID_K2_MASK(10) SYSID_K2_MASK(11)
    SYSID_K2_MASK(12) SYSID_K2_MASK(13) SYSID_K2_MASK(14) SYSID_K2_MASK(15)
#undef SYSID_K2_MASK
  }
}

template <typename T, int NTC, int KC>
__global__ void __launch_bounds__(64 * k2_waves(NTC))
k2_gram_syrk(const T* __restrict__ panel, int64_t rows, int64_t ldp, const int2* __restrict__ supers, int ngroups,
             int ksplit, int nslots, int accumulate, double* __restrict__ slab) {
  k2_syrk_body<T, NTC, KC, false>(panel, rows, ldp, supers, ngroups, ksplit, nslots, accumulate, slab, nullptr,
                                  nullptr);
}
// the gathered rows of the nullspace mode (rowlist / d_rows as in k2_gram_syrk_dma)
template <typename T, int NTC, int KC>
__global__ void __launch_bounds__(64 * k2_waves(NTC))
k2_gram_syrk_gather(const T* __restrict__ panel, int64_t rows, int64_t ldp, const int2* __restrict__ supers,
                    int ngroups, int ksplit, int nslots, int accumulate, double* __restrict__ slab,
                    const int* __restrict__ rowlist, const int* __restrict__ d_rows) {
  k2_syrk_body<T, NTC, KC, true>(panel, rows, ldp, supers, ngroups, ksplit, nslots, accumulate, slab, rowlist,
                                 d_rows);
}

// ------------------------------------------------------------------------------------------------
// K2, LDS-DMA form (the default for the f64 / f32 Gram): the same super-tiles, k-loop and slab epilogue as
// k2_gram_syrk above, but the panel chunks go HBM -> LDS by global_load_lds_dwordx4 (no staging registers, no
// ds_write pass) into THREE LDS buffers, so chunk c + 2 streams in while chunk c is multiplied and chunk c + 1
// waits complete.  Row rr of a chunk is copied by wave rr % 8 as NP pieces of <= 1 KiB (64 lanes x 16 B; the
// destination of one instruction is lane-linear, and a row's pieces never cross into the padded stride).  The
// pipeline spans the per-chunk barrier: a counted `s_waitcnt vmcnt(G)` (G = this wave's DMA instructions per
// chunk) retires chunk c + 1 and leaves chunk c + 2 in flight, then `lgkmcnt(0)` (this chunk's fragment
// reads, so its buffer may be refilled) and a raw s_barrier -- never __syncthreads(), whose fence would drain
// every DMA in flight (cdna_hip_programming.md, "Pipelining across barriers").  All LDS is one __shared__
// array (a second object made hipcc wait vmcnt(0) before fragment reads, same guide).  The partial last chunk
// of a row range runs after the pipelined loop: its rows past the range are zero-filled by ds_write.
// Measured against the register-staged kernel: profiles/r02_*.
// ------------------------------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void k2_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// vmcnt(G) for G = RPW * np DMA instructions per chunk (np: pieces per row, 1..3)
template <int RPW>
__device__ __forceinline__ void k2_wait_chunk(int np) {
  if (np == 1) k2_wait_vm<RPW>();
  else if (np == 2) k2_wait_vm<2 * RPW>();
  else k2_wait_vm<3 * RPW>();
}
__device__ __forceinline__ void k2_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Rows per chunk of the DMA kernel: three buffers of KC x k2_stride(NTC) elements in the CU's 160 KB (one
// workgroup per CU, NTC < 16) or in half of it (two, NTC >= 16); a multiple of 8 (rows are dealt to the 8 waves).
__host__ __device__ constexpr int k2_dma_kc(int ntc) { return ntc <= 10 ? 32 : ntc < 16 ? 16 : 8; }

// GATHER (nullspace mode): the rows are those listed in rowlist (k1s_row_list), *d_rows of them; every wave
// reads its rows' list entries for the chunk after next by scalar loads, one chunk ahead of their DMA.
template <typename T, int NTC, int KC, bool GATHER = false>
__global__ void __launch_bounds__(64 * k2_waves(NTC))
k2_gram_syrk_dma(const T* __restrict__ panel, int64_t rows, int64_t ldp, const int2* __restrict__ supers,
                 int ngroups, int ksplit, int nslots, int accumulate, double* __restrict__ slab,
                 const int* __restrict__ rowlist, const int* __restrict__ d_rows) {
  typedef typename K2Acc<T>::type accT;
  constexpr int K2W = k2_waves(NTC), K2S = k2_slots<T>(NTC);
  static_assert(KC % K2W == 0 && KC % 4 == 0, "chunk rows are dealt to the waves, k-steps of 4");
  constexpr int STRIDE = k2_stride(NTC);
  constexpr int BUF = KC * STRIDE;  // elements per LDS buffer
  constexpr int NT = 64 * K2W;
  constexpr int RPW = KC / K2W;  // rows per wave per chunk
  constexpr int EB = (int)sizeof(T);
  static_assert(3 * BUF * EB <= 160 * 1024, "three LDS buffers");
  __shared__ __attribute__((aligned(16))) T lds[3 * BUF];
  int group, ks;
  k2_block_coords(ngroups, group, ks);
  const int64_t prows = rows;  // GATHER: the panel's rows (the list holds at most these)
  if constexpr (GATHER) rows = min((int64_t)__builtin_amdgcn_readfirstlane(*d_rows), prows);
  const int64_t q4 = rows / 4;
  const int64_t r0 = 4 * (q4 * ks / ksplit);
  const int64_t r1 = ks + 1 == ksplit ? rows : 4 * (q4 * (ks + 1) / ksplit);
  // the wave index in a scalar register for the row list's scalar loads; the super-tile descriptors stay per
  // lane (uniform ones measured slower, see above)
  const int wave = GATHER ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int sbase = (group * K2W + (int)(threadIdx.x >> 6)) * K2S;

  // zero the three buffers once: columns >= ldp (up to NTC*16) are never written by the DMA and must read as 0
  for (int x = threadIdx.x; x < 3 * BUF; x += NT) lds[x] = (T)0;

  const int rowbytes = (int)ldp * EB;             // <= STRIDE * EB
  const int np = (rowbytes + 1023) >> 10;         // 1 KiB pieces per row (wave-uniform, 1..3)
  constexpr int NPMAX = (16 * NTC * EB + 1023) / 1024;
  auto dma_row = [&](const T* src_row, T* dst_row) {
    const char* src = reinterpret_cast<const char*>(src_row);
    char* dst = reinterpret_cast<char*>(dst_row);
#pragma unroll
    for (int p = 0; p < NPMAX; ++p) {
      if (p < np) {  // wave-uniform; every piece below np has >= 1 live lane: exactly np instructions per row
        const int off = (p << 10) + 16 * lane;
        if (off < rowbytes)
          __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + off),
                                           reinterpret_cast<void*>(dst + (p << 10)), 16, 0, 0);
      }
    }
  };
  // GATHER: the list entries of the wave's rows of the next chunk to DMA, loaded one chunk ahead (SGPRs)
  int gidx[RPW];
  auto list_load = [&](int64_t c0) {
    if constexpr (GATHER) {
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        const int64_t x = c0 + wave + K2W * q;
        const int v = x < r1 ? rowlist[x] : 0;
        gidx[q] = v >= 0 && v < prows ? v : 0;
      }
    }
  };
  auto dma_chunk = [&](int64_t c0, T* buf) {  // RPW * np instructions per wave
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int rr = wave + K2W * q;
      dma_row(panel + (GATHER ? (int64_t)gidx[q] : c0 + rr) * ldp, buf + rr * STRIDE);
    }
  };

  int foff[4 * K2S];
  bool live[K2S];
  bool need[K2S][4];
#pragma unroll
  for (int s = 0; s < K2S; ++s) {
    int2 sp = supers[sbase + s];
    live[s] = sp.x >= 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int I = 2 * sp.x + (t >> 1), J = 2 * (sp.y & 0xFF) + (t & 1);
      need[s][t] = live[s] && I <= J && J < NTC && !k2_tile_skip(sp, t);
    }
    const int blk[4] = {2 * sp.x, 2 * sp.x + 1, 2 * (sp.y & 0xFF), 2 * (sp.y & 0xFF) + 1};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int b = live[s] && blk[u] < NTC ? blk[u] : 0;
      foff[4 * s + u] = (lane >> 4) * STRIDE + 16 * b + (lane & 15);
    }
  }
  accT acc[K2S][4];
#pragma unroll
  for (int s = 0; s < K2S; ++s)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[s][t] = accT{0, 0, 0, 0};
  auto mfma_chunk = [&](const T* cur) {
#pragma unroll
    for (int kk = 0; kk < KC; kk += 4) {
      T x[4 * K2S];
#pragma unroll
      for (int u = 0; u < 4 * K2S; ++u) x[u] = cur[foff[u] + kk * STRIDE];
#pragma unroll
      for (int s = 0; s < K2S; ++s) {
        constexpr int AB[4][2] = {{0, 2}, {0, 3}, {1, 2}, {1, 3}};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (!need[s][t]) continue;
          if constexpr (sizeof(T) == 8)
            acc[s][t] = __builtin_amdgcn_mfma_f64_16x16x4f64(x[4 * s + AB[t][0]], x[4 * s + AB[t][1]], acc[s][t], 0, 0, 0);
          else
            acc[s][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[4 * s + AB[t][0]], x[4 * s + AB[t][1]], acc[s][t], 0, 0, 0);
        }
      }
    }
  };

  const int64_t nfull = (r1 - r0) / KC;  // whole chunks; then one partial chunk if rows remain
  __syncthreads();                        // LDS zeroed (no DMA in flight yet)
  T* b0 = lds;                            // chunk c
  T* b1 = lds + BUF;                      // chunk c + 1
  T* b2 = lds + 2 * BUF;                  // chunk c + 2
  list_load(r0);
  if (nfull > 0) dma_chunk(r0, b0);
  list_load(r0 + KC);
  if (nfull > 1) {
    dma_chunk(r0 + KC, b1);
    list_load(r0 + 2 * KC);
    k2_wait_chunk<RPW>(np);  // chunk 0 landed (chunk 1 in flight)
  } else {
    k2_wait_vm<0>();
  }
  k2_barrier();
  for (int64_t c = 0; c < nfull; ++c) {
    const bool pre = c + 2 < nfull;
    if (pre) {
      dma_chunk(r0 + (c + 2) * KC, b2);
      list_load(r0 + (c + 3) * KC);
    }
    mfma_chunk(b0);
    if (pre) k2_wait_chunk<RPW>(np);  // chunk c + 1 landed, chunk c + 2 stays in flight
    else k2_wait_vm<0>();
    k2_barrier();                     // ... for every wave; b0's fragment reads retired (it is refilled next)
    T* t = b0;
    b0 = b1;
    b1 = b2;
    b2 = t;
  }
  if (r0 + nfull * KC < r1) {  // the partial last chunk, into b0 (free: its last chunk finished two barriers ago)
    const int64_t c0 = r0 + nfull * KC;
    const int valid = (int)(r1 - c0);
    list_load(c0);
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int rr = wave + K2W * q;
      T* dst = b0 + rr * STRIDE;
      if (rr < valid) {
        dma_row(panel + (GATHER ? (int64_t)gidx[q] : c0 + rr) * ldp, dst);
      } else {
        for (int x = 16 * lane; x < rowbytes; x += 16 * 64) *reinterpret_cast<uint4*>(reinterpret_cast<char*>(dst) + x) = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    k2_wait_vm<0>();
    k2_barrier();
    mfma_chunk(b0);
  }
  // D layout: col = lane & 15; row = (lane >> 4) + 4 * reg for f64, 4 * (lane >> 4) + reg for f32
#pragma unroll
  for (int s = 0; s < K2S; ++s) {
    if (!live[s]) continue;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      double* o = slab + ((size_t)ks * nslots + (size_t)(sbase + s) * 4 + t) * 256;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = sizeof(T) == 8 ? (lane >> 4) + 4 * j : 4 * (lane >> 4) + j;
        double* x = o + row * 16 + (lane & 15);
        const double v = (double)acc[s][t][j];
        *x = accumulate ? *x + v : v;  // chunked Gram: slabs carry over chunks
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// K2 bf16: the same super-tile decomposition on v_mfma_f32_16x16x32_bf16, from a bf16 panel (K1 rounds the
// Gram-only chunk panel to bf16 as it writes it; ld a multiple of 8).  A chunk of KC (a multiple of 32) rows is
// staged column-major in LDS (column stride CS = KC + 8 bf16), so the fragment of lane l — 8 consecutive rows
// 8(l>>4).. of column (l & 15) of a 16-column block, which is both the A layout A[i = l&15][k = 8(l>>4) + j] and
// the B layout B[k][j = l&15] — is one 16-byte ds_read.  Staging item = (8-column group, 8-row group): eight
// 16-byte global loads (one row's 8 columns each), an 8x8 transpose of 16-bit elements in registers
// (v_perm_b32), eight 16-byte LDS stores (one column's 8 rows each).  f32 accumulation per workgroup, f64
// across workgroups (K3).
// ------------------------------------------------------------------------------------------------
// out[j] = column j of the 8x8 block whose row t is in[t] (8 bf16 per uint4, element j in the 16-bit half
// (j & 1) of word (j >> 1)).
__device__ __forceinline__ void transpose8x8_b16(const uint4 (&in)[8], uint4 (&out)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const unsigned sel = (j & 1) ? 0x07060302u : 0x05040100u;  // hi halves / lo halves of (b, a) -> a | b << 16
    unsigned w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4& a = in[2 * q];
      const uint4& b = in[2 * q + 1];
      const unsigned wa = (j >> 1) == 0 ? a.x : (j >> 1) == 1 ? a.y : (j >> 1) == 2 ? a.z : a.w;
      const unsigned wb = (j >> 1) == 0 ? b.x : (j >> 1) == 1 ? b.y : (j >> 1) == 2 ? b.z : b.w;
      w[q] = __builtin_amdgcn_perm(wb, wa, sel);
    }
    out[j] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

template <int NTC, int KC>
__global__ void __launch_bounds__(64 * K2_BF16_WAVES)
k2_gram_syrk_bf16(const __bf16* __restrict__ panel, int64_t rows, int64_t ldp, const int2* __restrict__ supers,
                  int ngroups, int ksplit, int nslots, int accumulate, double* __restrict__ slab) {
  static_assert(KC % 32 == 0, "bf16 K2 chunks are whole 32-row k-steps");
  // always 8 waves (16 spill its transposes at 128 VGPRs), k2_bf16_spw(NTC) super-tile slots each
  constexpr int K2W = K2_BF16_WAVES, K2S = k2_bf16_spw(NTC);
  constexpr int NCOL = NTC * 16;
  constexpr int CS = KC + 8;
  constexpr int BUF = NCOL * CS;
  constexpr int NT = 64 * K2W;
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * BUF];
  int group, ks;
  k2_block_coords(ngroups, group, ks);
  const int64_t q4 = rows / 4;
  const int64_t r0 = 4 * (q4 * ks / ksplit);
  const int64_t r1 = ks + 1 == ksplit ? rows : 4 * (q4 * (ks + 1) / ksplit);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int sbase = (group * K2W + wave) * K2S;

  // zero both buffers once: columns >= ldp are never staged and must read as 0
  for (int x = threadIdx.x; x < 2 * BUF; x += NT) lds[x] = (__bf16)0.0f;

  const int ncg = (int)(ldp >> 3);  // 8-column groups per row
  constexpr int PER = (NTC * 2 * (KC / 8) + NT - 1) / NT;
  int cg[PER], ro[PER];
  bool used[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int it = threadIdx.x + u * NT;
    used[u] = it < ncg * (KC / 8);
    ro[u] = used[u] ? it / ncg : 0;
    cg[u] = used[u] ? it - ro[u] * ncg : 0;
  }
  uint4 st[PER][8];
  auto load_chunk = [&](int64_t c0) {
#pragma unroll
    for (int u = 0; u < PER; ++u)
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int64_t r = c0 + 8 * ro[u] + t;
        st[u][t] = (used[u] && r < r1) ? reinterpret_cast<const uint4*>(panel + r * ldp)[cg[u]]
                                       : make_uint4(0u, 0u, 0u, 0u);
      }
  };
  auto store_chunk = [&](__bf16* b) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      if (!used[u]) continue;
      uint4 col[8];
      transpose8x8_b16(st[u], col);
#pragma unroll
      for (int j = 0; j < 8; ++j) *reinterpret_cast<uint4*>(b + (8 * cg[u] + j) * CS + 8 * ro[u]) = col[j];
    }
  };

  int foff[4 * K2S];
  bool live[K2S];
  bool need[K2S][4];
#pragma unroll
  for (int s = 0; s < K2S; ++s) {
    int2 sp = supers[sbase + s];
    live[s] = sp.x >= 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int I = 2 * sp.x + (t >> 1), J = 2 * (sp.y & 0xFF) + (t & 1);
      need[s][t] = live[s] && I <= J && J < NTC && !k2_tile_skip(sp, t);
    }
    const int blk[4] = {2 * sp.x, 2 * sp.x + 1, 2 * (sp.y & 0xFF), 2 * (sp.y & 0xFF) + 1};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int b = live[s] && blk[u] < NTC ? blk[u] : 0;
      foff[4 * s + u] = (16 * b + (lane & 15)) * CS + 8 * (lane >> 4);
    }
  }
  flt4 acc[K2S][4];
#pragma unroll
  for (int s = 0; s < K2S; ++s)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[s][t] = flt4{0.f, 0.f, 0.f, 0.f};

  const int64_t nchunks = (r1 - r0 + KC - 1) / KC;
  __syncthreads();  // LDS zeroed
  if (nchunks > 0) {
    load_chunk(r0);
    store_chunk(lds);
  }
  __syncthreads();
  for (int64_t c = 0; c < nchunks; ++c) {
    const __bf16* cur = lds + (c & 1) * BUF;
    if (c + 1 < nchunks) load_chunk(r0 + (c + 1) * KC);
#pragma unroll
    for (int kk = 0; kk < KC; kk += 32) {
#pragma unroll
      for (int s = 0; s < K2S; ++s) {
        // one slot's four fragments at a time (all of them at once would hold 4 K2S x 4 VGPRs)
        bf16x8 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = *reinterpret_cast<const bf16x8*>(cur + foff[4 * s + u] + kk);
        constexpr int AB[4][2] = {{0, 2}, {0, 3}, {1, 2}, {1, 3}};
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (need[s][t])
            acc[s][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[AB[t][0]], x[AB[t][1]], acc[s][t], 0, 0, 0);
      }
    }
    if (c + 1 < nchunks) store_chunk(lds + ((c + 1) & 1) * BUF);
    __syncthreads();
  }
#pragma unroll
  for (int s = 0; s < K2S; ++s) {
    if (!live[s]) continue;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      double* o = slab + ((size_t)ks * nslots + (size_t)(sbase + s) * 4 + t) * 256;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        double* x = o + (4 * (lane >> 4) + j) * 16 + (lane & 15);
        const double v = (double)acc[s][t][j];
        *x = accumulate ? *x + v : v;
      }
    }
  }
}

// K2 bf16, wide Grams: the panel is staged by LDS-DMA into three row-major buffers (no staging registers, no
// transpose pass, two chunks in flight) and every MFMA fragment is read transposed by two ds_read_b64_tr_b16
// (lane 4q+p of a 16-lane group addresses row q, columns 4p..4p+3 of a 4 x 16 block; lane i receives column i
// of the 4 rows), so one workgroup holds all super-tiles of G1 (10 slots per wave, 160 f32 accumulator VGPRs)
// and the panel is read once.  Reads are issued by every lane (EXEC all ones: the gather crosses lanes).
typedef short s16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ bf16x8 k2_frag_tr(const __bf16* p, int stride) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p + 4 * stride));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Rows per chunk of the transposed-read kernel: three row-major buffers of NTC*16 + 8 bf16 per row in 160 KB.
__host__ __device__ constexpr int k2_bf16_tr_kc(int ntc) {
  return (160 * 1024 / (3 * (ntc * 16 + 8) * 2)) / 32 * 32 > 128 ? 128 : (160 * 1024 / (3 * (ntc * 16 + 8) * 2)) / 32 * 32;
}

template <int NTC, int KC, bool GATHER = false>
__global__ void __launch_bounds__(64 * K2_BF16_WAVES)
k2_gram_syrk_bf16_tr(const __bf16* __restrict__ panel, int64_t rows, int64_t ldp, const int2* __restrict__ supers,
                     int ngroups, int ksplit, int nslots, int accumulate, double* __restrict__ slab,
                     const int* __restrict__ rowlist, const int* __restrict__ d_rows) {
  static_assert(KC % 32 == 0 && KC % K2_BF16_WAVES == 0, "whole 32-row k-steps, rows dealt to the waves");
  constexpr int K2W = K2_BF16_WAVES, K2S = k2_bf16_spw(NTC);
  constexpr int STRIDE = NTC * 16 + 8;  // elements per LDS row (16-byte multiple)
  constexpr int BUF = KC * STRIDE;
  constexpr int NT = 64 * K2W;
  constexpr int RPW = KC / K2W;
  static_assert(3 * BUF * 2 <= 160 * 1024, "three LDS buffers");
  __shared__ __attribute__((aligned(16))) __bf16 lds[3 * BUF];
  int group, ks;
  k2_block_coords(ngroups, group, ks);
  const int64_t prows = rows;  // GATHER: the panel's rows (the list holds at most these)
  if constexpr (GATHER) rows = min((int64_t)__builtin_amdgcn_readfirstlane(*d_rows), prows);
  const int64_t q4 = rows / 4;
  const int64_t r0 = 4 * (q4 * ks / ksplit);
  const int64_t r1 = ks + 1 == ksplit ? rows : 4 * (q4 * (ks + 1) / ksplit);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int sbase = (group * K2W + wave) * K2S;

  for (int x = threadIdx.x; x < 3 * BUF; x += NT) lds[x] = (__bf16)0.0f;  // columns >= ldp read as 0

  const int rowbytes = (int)ldp * 2;  // <= 1 KiB for NTC <= 32: one DMA piece per row
  auto dma_row = [&](const __bf16* src_row, __bf16* dst_row) {
    const int off = 16 * lane;
    if (off < rowbytes)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(reinterpret_cast<const char*>(src_row) + off),
                                       reinterpret_cast<void*>(dst_row), 16, 0, 0);
  };
  int gidx[RPW];  // GATHER: list entries of the wave's rows of the next chunk to DMA (as k2_gram_syrk_dma)
  auto list_load = [&](int64_t c0) {
    if constexpr (GATHER) {
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        const int64_t x = c0 + wave + K2W * q;
        const int v = x < r1 ? rowlist[x] : 0;
        gidx[q] = v >= 0 && v < prows ? v : 0;
      }
    }
  };
  auto dma_chunk = [&](int64_t c0, __bf16* buf) {  // RPW instructions per wave
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int rr = wave + K2W * q;
      dma_row(panel + (GATHER ? (int64_t)gidx[q] : c0 + rr) * ldp, buf + rr * STRIDE);
    }
  };

  // fragment base of this lane: rows 8g + q (and + 4), columns 4p..4p+3 of each 16-column block
  const int lb = (8 * (lane >> 4) + ((lane & 15) >> 2)) * STRIDE + 4 * (lane & 3);
  // slot descriptors are wave-uniform (sbase depends on the wave only): SGPRs, and the needed tiles as one
  // scalar bit mask, so the 160 accumulator VGPRs keep the vector file to themselves
  int2 spv[K2S];
  unsigned long long needm = 0;  // 4 K2S <= 64 bits
#pragma unroll
  for (int s = 0; s < K2S; ++s) {
    int2 sp = supers[sbase + s];
    sp.x = __builtin_amdgcn_readfirstlane(sp.x);
    sp.y = __builtin_amdgcn_readfirstlane(sp.y);
    spv[s] = sp;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int I = 2 * sp.x + (t >> 1), J = 2 * (sp.y & 0xFF) + (t & 1);
      if (sp.x >= 0 && I <= J && J < NTC && !k2_tile_skip(sp, t)) needm |= 1ull << (4 * s + t);
    }
  }
  flt4 acc[K2S][4];
#pragma unroll
  for (int s = 0; s < K2S; ++s)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[s][t] = flt4{0.f, 0.f, 0.f, 0.f};

  auto mfma_chunk = [&](const __bf16* cur) {
#pragma unroll
    for (int kk = 0; kk < KC; kk += 32) {
#pragma unroll
      for (int s = 0; s < K2S; ++s) {
        const int2 sp = spv[s];
        const bool live = sp.x >= 0;
        const int blk[4] = {2 * sp.x, 2 * sp.x + 1, 2 * (sp.y & 0xFF), 2 * (sp.y & 0xFF) + 1};
        bf16x8 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int b = live && blk[u] < NTC ? blk[u] : 0;  // every lane reads (EXEC all ones)
          x[u] = k2_frag_tr(cur + kk * STRIDE + lb + 16 * b, STRIDE);
        }
        constexpr int AB[4][2] = {{0, 2}, {0, 3}, {1, 2}, {1, 3}};
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if ((needm >> (4 * s + t)) & 1ull)
            acc[s][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[AB[t][0]], x[AB[t][1]], acc[s][t], 0, 0, 0);
      }
    }
  };

  const int64_t nfull = (r1 - r0) / KC;
  __syncthreads();  // LDS zeroed (no DMA in flight yet)
  __bf16* b0 = lds;
  __bf16* b1 = lds + BUF;
  __bf16* b2 = lds + 2 * BUF;
  list_load(r0);
  if (nfull > 0) dma_chunk(r0, b0);
  list_load(r0 + KC);
  if (nfull > 1) {
    dma_chunk(r0 + KC, b1);
    list_load(r0 + 2 * KC);
    k2_wait_vm<RPW>();  // chunk 0 landed (chunk 1 in flight)
  } else {
    k2_wait_vm<0>();
  }
  k2_barrier();
  for (int64_t c = 0; c < nfull; ++c) {
    const bool pre = c + 2 < nfull;
    if (pre) {
      dma_chunk(r0 + (c + 2) * KC, b2);
      list_load(r0 + (c + 3) * KC);
    }
    mfma_chunk(b0);
    if (pre) k2_wait_vm<RPW>();  // chunk c + 1 landed, chunk c + 2 stays in flight
    else k2_wait_vm<0>();
    k2_barrier();
    __bf16* t = b0;
    b0 = b1;
    b1 = b2;
    b2 = t;
  }
  if (r0 + nfull * KC < r1) {  // the partial last chunk into b0 (its last reads retired at the barrier above)
    const int64_t c0 = r0 + nfull * KC;
    const int valid = (int)(r1 - c0);
    list_load(c0);
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int rr = wave + K2W * q;
      __bf16* dst = b0 + rr * STRIDE;
      if (rr < valid) {
        dma_row(panel + (GATHER ? (int64_t)gidx[q] : c0 + rr) * ldp, dst);
      } else {
        for (int x = 16 * lane; x < rowbytes; x += 16 * 64)
          *reinterpret_cast<uint4*>(reinterpret_cast<char*>(dst) + x) = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    k2_wait_vm<0>();
    k2_barrier();
    mfma_chunk(b0);
  }
#pragma unroll
  for (int s = 0; s < K2S; ++s) {
    if (spv[s].x < 0) continue;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      double* o = slab + ((size_t)ks * nslots + (size_t)(sbase + s) * 4 + t) * 256;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        double* x = o + (4 * (lane >> 4) + j) * 16 + (lane & 15);
        const double v = (double)acc[s][t][j];
        *x = accumulate ? *x + v : v;
      }
    }
  }
}

// K2 bf16, wide Grams of 16..23 tile columns: register-blocked tiles.  The super-tile kernel above reads two
// A and two B fragments for every 2x2 super-tile and k-step: 1 fragment read per MFMA, and a
// ds_read_b64_tr_b16 pair moves 1 KiB while the MFMA it feeds takes 16 cycles, so 8 waves of 10 super-tiles
// asked 2.5k LDS cycles per 32-row k-step of a CU (conflicts included) for 1.25k cycles of MFMA per SIMD.  A
// Gram's A and B fragments of one column block are the same registers (the MFMA takes both operands K-major),
// so here every wave owns a block of tiles and reads each of its column blocks' fragments once per k-step:
// three waves own the diagonal triangles of a three-way split of the columns (s = ceil(NTC/3) blocks: s
// fragments feed s(s+1)/2 tiles), five the rectangles above them (nr + nc fragments feed nr x nc tiles).  G1
// (23 tile columns): 84 fragment reads per CU and k-step instead of 312, per-SIMD MFMA loads 70/71/71/64
// tiles (waves w and w + 4 share a SIMD).  The LDS image is row-major with a stride of 8 (mod 64) dwords, the
// rows whose bit 3 is set in a second set of row slots 32 dwords further round the banks (k2b_row_off), so the
// eight 32-byte row segments one 32-lane half of a transposed read touches fall on disjoint banks.
struct K2BRole {
  int diag, nr, nc, ra, ca;
};
__host__ __device__ constexpr K2BRole k2b_role(int ntc, int w) {
  const int s = (ntc + 2) / 3, t = ntc - 2 * s;  // diagonal blocks [0,s) [s,2s) [2s,ntc)
  const int h0 = (2 * s + 2) / 3, h1 = (2 * s - h0 + 1) / 2, h2 = 2 * s - h0 - h1;  // rows of [0,2s) x [2s,ntc)
  const int b0 = (s + 1) / 2;                                                        // rows of [0,s) x [s,2s)
  return w == 0   ? K2BRole{1, t, t, 2 * s, 2 * s}
         : w == 1 ? K2BRole{1, s, s, 0, 0}
         : w == 2 ? K2BRole{1, s, s, s, s}
         : w == 3 ? K2BRole{0, b0, s, 0, s}
         : w == 4 ? K2BRole{0, h0, t, 0, 2 * s}
         : w == 5 ? K2BRole{0, h1, t, h0, 2 * s}
         : w == 6 ? K2BRole{0, h2, t, h0 + h1, 2 * s}
                  : K2BRole{0, s - b0, s, b0, s};
}
__host__ __device__ constexpr int k2b_ntiles(int ntc, int w) {
  return k2b_role(ntc, w).diag ? k2b_role(ntc, w).nr * (k2b_role(ntc, w).nr + 1) / 2
                               : k2b_role(ntc, w).nr * k2b_role(ntc, w).nc;
}
__host__ __device__ constexpr int k2b_base(int ntc, int w) { return w == 0 ? 0 : k2b_base(ntc, w - 1) + k2b_ntiles(ntc, w - 1); }
__host__ __device__ constexpr int k2b_maxtiles(int ntc) {
  int m = 0;
  for (int w = 0; w < 8; ++w) m = k2b_ntiles(ntc, w) > m ? k2b_ntiles(ntc, w) : m;
  return m;
}
__host__ __device__ constexpr bool k2b_supported(int ntc) { return ntc >= 16 && ntc <= 23; }
// local tile index -> (I, J) of wave w (the slab / K3 tile order: wave by wave, row by row)
__host__ __device__ constexpr int k2b_tile_index(int ntc, int w, int i, int j) {
  return k2b_role(ntc, w).diag ? i * k2b_role(ntc, w).nr - i * (i - 1) / 2 + (j - i) : i * k2b_role(ntc, w).nc + j;
}
// LDS row stride of the block kernel in bytes: >= 16 NTC bf16, = 8 (mod 64) dwords
__host__ __device__ constexpr int k2b_stride_bytes(int ntc) { return 4 * (((8 * ntc - 8 + 63) / 64) * 64 + 8); }
// row r of a 64-row chunk: rows with bit 3 clear fill the first 32 row slots, rows with it set the next 32,
// 128 bytes further on (so the two sets' banks differ by 32 dwords without a row running into the next)
__host__ __device__ constexpr int k2b_row_off(int ntc, int r) {
  return ((r >> 3) & 1) * (32 * k2b_stride_bytes(ntc) + 128) + ((r >> 4) * 8 + (r & 7)) * k2b_stride_bytes(ntc);
}
constexpr int K2B_KC = 64;  // rows per staged chunk (three buffers of 64 rows: G1 3 x 51.3 KB)

template <int NTC, int W>
__device__ __forceinline__ void k2b_mfma(const __bf16* cur, int lb, flt4 (&acc)[k2b_ntiles(NTC, W)]) {
  constexpr K2BRole R = k2b_role(NTC, W);
  constexpr int SE = k2b_stride_bytes(NTC) / 2;  // elements per LDS row
#pragma unroll
  for (int kk = 0; kk < K2B_KC; kk += 32) {
    const __bf16* base = cur + (kk / 2) * SE + lb;  // k-step rows kk.. sit kk / 2 row slots on in both sets
    if constexpr (R.diag) {
      bf16x8 f[R.nr];
#pragma unroll
      for (int i = 0; i < R.nr; ++i) f[i] = k2_frag_tr(base + 16 * (R.ra + i), SE);
#pragma unroll
      for (int i = 0; i < R.nr; ++i)
#pragma unroll
        for (int j = i; j < R.nr; ++j) {
          const int x = k2b_tile_index(NTC, W, i, j);
          acc[x] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[i], f[j], acc[x], 0, 0, 0);
        }
    } else {
      bf16x8 a[R.nr];
#pragma unroll
      for (int i = 0; i < R.nr; ++i) a[i] = k2_frag_tr(base + 16 * (R.ra + i), SE);
#pragma unroll
      for (int j = 0; j < R.nc; ++j) {
        const bf16x8 b = k2_frag_tr(base + 16 * (R.ca + j), SE);
#pragma unroll
        for (int i = 0; i < R.nr; ++i) {
          const int x = i * R.nc + j;
          acc[x] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b, acc[x], 0, 0, 0);
        }
      }
    }
  }
}

// One wave's whole pass (its role W fixed at compile time, so its accumulators are exactly its tiles): the
// three-buffer LDS-DMA pipeline of k2_gram_syrk_bf16_tr, every wave staging KC / 8 rows of each chunk.
template <int NTC, bool GATHER, int W>
__device__ __forceinline__ void k2b_wave(char* lds, const __bf16* __restrict__ panel, int64_t r0, int64_t r1,
                                         int64_t prows, int64_t ldp, int ks, int nslots, int accumulate,
                                         double* __restrict__ slab, const int* __restrict__ rowlist, int lane) {
  constexpr int K2W = K2_BF16_WAVES, KC = K2B_KC;
  constexpr int BUFB = KC * k2b_stride_bytes(NTC) + 128;
  constexpr int RPW = KC / K2W;
  constexpr int NTW = k2b_ntiles(NTC, W);
  const int rowbytes = (int)ldp * 2;  // <= 1 KiB: one DMA piece per row
  auto dma_row = [&](const __bf16* src_row, char* dst_row) {
    const int off = 16 * lane;
    if (off < rowbytes)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(reinterpret_cast<const char*>(src_row) + off),
                                       reinterpret_cast<void*>(dst_row), 16, 0, 0);
  };
  int gidx[RPW];
  auto list_load = [&](int64_t c0) {
    if constexpr (GATHER) {
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        const int64_t x = c0 + W + K2W * q;
        const int v = x < r1 ? rowlist[x] : 0;
        gidx[q] = v >= 0 && v < prows ? v : 0;
      }
    }
  };
  auto dma_chunk = [&](int64_t c0, char* buf) {
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int rr = W + K2W * q;
      dma_row(panel + (GATHER ? (int64_t)gidx[q] : c0 + rr) * ldp, buf + k2b_row_off(NTC, rr));
    }
  };
  // this lane's fragment base (elements): row 8g + q of the k-step, columns 4p..4p+3 of a 16-column block
  const int lb = k2b_row_off(NTC, 8 * (lane >> 4) + ((lane & 15) >> 2)) / 2 + 4 * (lane & 3);
  flt4 acc[NTW];
#pragma unroll
  for (int x = 0; x < NTW; ++x) acc[x] = flt4{0.f, 0.f, 0.f, 0.f};

  const int64_t nfull = (r1 - r0) / KC;
  char* b0 = lds;
  char* b1 = lds + BUFB;
  char* b2 = lds + 2 * BUFB;
  list_load(r0);
  if (nfull > 0) dma_chunk(r0, b0);
  list_load(r0 + KC);
  if (nfull > 1) {
    dma_chunk(r0 + KC, b1);
    list_load(r0 + 2 * KC);
    k2_wait_vm<RPW>();  // chunk 0 landed (chunk 1 in flight)
  } else {
    k2_wait_vm<0>();
  }
  k2_barrier();
  for (int64_t c = 0; c < nfull; ++c) {
    const bool pre = c + 2 < nfull;
    if (pre) {
      dma_chunk(r0 + (c + 2) * KC, b2);
      list_load(r0 + (c + 3) * KC);
    }
    k2b_mfma<NTC, W>(reinterpret_cast<const __bf16*>(b0), lb, acc);
    if (pre) k2_wait_vm<RPW>();  // chunk c + 1 landed, chunk c + 2 stays in flight
    else k2_wait_vm<0>();
    k2_barrier();
    char* t = b0;
    b0 = b1;
    b1 = b2;
    b2 = t;
  }
  if (r0 + nfull * KC < r1) {  // the partial last chunk into b0 (its last reads retired at the barrier above)
    const int64_t c0 = r0 + nfull * KC;
    const int valid = (int)(r1 - c0);
    list_load(c0);
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int rr = W + K2W * q;
      char* dst = b0 + k2b_row_off(NTC, rr);
      if (rr < valid) {
        dma_row(panel + (GATHER ? (int64_t)gidx[q] : c0 + rr) * ldp, dst);
      } else {
        for (int x = 16 * lane; x < rowbytes; x += 16 * 64)
          *reinterpret_cast<uint4*>(dst + x) = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    k2_wait_vm<0>();
    k2_barrier();
    k2b_mfma<NTC, W>(reinterpret_cast<const __bf16*>(b0), lb, acc);
  }
  constexpr int B = k2b_base(NTC, W);
#pragma unroll
  for (int x = 0; x < NTW; ++x) {
    double* o = slab + ((size_t)ks * nslots + B + x) * 256;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      double* y = o + (4 * (lane >> 4) + j) * 16 + (lane & 15);
      const double v = (double)acc[x][j];
      *y = accumulate ? *y + v : v;
    }
  }
}

template <int NTC, bool GATHER = false>
__global__ void __launch_bounds__(64 * K2_BF16_WAVES)
k2_gram_syrk_bf16_blk(const __bf16* __restrict__ panel, int64_t rows, int64_t ldp, int ksplit, int nslots,
                      int accumulate, double* __restrict__ slab, const int* __restrict__ rowlist,
                      const int* __restrict__ d_rows) {
  static_assert(k2b_supported(NTC), "16..23 tile columns");
  constexpr int BUFB = K2B_KC * k2b_stride_bytes(NTC) + 128;  // bytes per LDS buffer
  static_assert(3 * BUFB <= 160 * 1024, "three LDS buffers");
  __shared__ __attribute__((aligned(16))) char lds[3 * BUFB];
  const int ks = (int)blockIdx.x;
  const int64_t prows = rows;
  if constexpr (GATHER) rows = min((int64_t)__builtin_amdgcn_readfirstlane(*d_rows), prows);
  const int64_t q4 = rows / 4;
  const int64_t r0 = 4 * (q4 * ks / ksplit);
  const int64_t r1 = ks + 1 == ksplit ? rows : 4 * (q4 * (ks + 1) / ksplit);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  for (int x = 16 * threadIdx.x; x < 3 * BUFB; x += 16 * 64 * K2_BF16_WAVES)
    *reinterpret_cast<uint4*>(lds + x) = make_uint4(0u, 0u, 0u, 0u);  // pads and columns >= ldp read as 0
  __syncthreads();  // LDS zeroed (no DMA in flight yet)
#define SYSID_K2B_WAVE(W) \
  k2b_wave<NTC, GATHER, W>(lds, panel, r0, r1, prows, ldp, ks, nslots, accumulate, slab, rowlist, lane)
  switch (wave) {  // every wave runs the same chunk loop and barriers with its own tiles
    case 0: SYSID_K2B_WAVE(0); break;
    case 1: SYSID_K2B_WAVE(1); break;
    case 2: SYSID_K2B_WAVE(2); break;
    case 3: SYSID_K2B_WAVE(3); break;
    case 4: SYSID_K2B_WAVE(4); break;
    case 5: SYSID_K2B_WAVE(5); break;
    case 6: SYSID_K2B_WAVE(6); break;
    default: SYSID_K2B_WAVE(7); break;
  }
#undef SYSID_K2B_WAVE
}

// K2 f32 / f64, wide Grams of 16..23 tile columns: the same register blocking on v_mfma_f32_16x16x4_f32 /
// v_mfma_f64_16x16x4_f64 (4-row k-steps, one element per lane and fragment).  The super-tile kernels hold 16
// super-tiles per workgroup, so G1's 78 took 5 groups and every panel row was staged 5 times (G1 20k f64 K2: 10
// GB of staged rows in 1.67 ms).  f32 keeps its 276 tiles in one group (the bf16 roles: 4 accumulator VGPRs per
// tile); an f64 tile takes 8, so f64 splits the Gram over two groups of 8 waves: four diagonal triangles of a
// four-way split of the columns and the six rectangles above them cut in row halves (G1: per-SIMD loads
// 36/36/36/33 and 33/33/33/36 tiles, 168 accumulator VGPRs at most).  LDS image: the f64 / f32 kernels' padded
// row stride (k2_stride: the two rows of a 32-lane half of a fragment read on disjoint banks).
__host__ __device__ constexpr int k2d_bstart(int ntc, int i) { return i * (ntc / 4) + (i < ntc % 4 ? i : ntc % 4); }
__host__ __device__ constexpr int k2d_bsize(int ntc, int i) { return ntc / 4 + (i < ntc % 4 ? 1 : 0); }
// rectangle (x, y) of the four-way split, row half h
__host__ __device__ constexpr K2BRole k2d_rect(int ntc, int x, int y, int h) {
  return K2BRole{0, h == 0 ? (k2d_bsize(ntc, x) + 1) / 2 : k2d_bsize(ntc, x) / 2, k2d_bsize(ntc, y),
                 k2d_bstart(ntc, x) + (h == 0 ? 0 : (k2d_bsize(ntc, x) + 1) / 2), k2d_bstart(ntc, y)};
}
__host__ __device__ constexpr K2BRole k2d_role(int ntc, int w) {  // w = 8 group + wave; waves w, w + 4 share a SIMD
  return w < 4     ? K2BRole{1, k2d_bsize(ntc, w), k2d_bsize(ntc, w), k2d_bstart(ntc, w), k2d_bstart(ntc, w)}
         : w == 4  ? k2d_rect(ntc, 0, 3, 0)
         : w == 5  ? k2d_rect(ntc, 0, 3, 1)
         : w == 6  ? k2d_rect(ntc, 1, 3, 0)
         : w == 7  ? k2d_rect(ntc, 0, 1, 0)
         : w == 8  ? k2d_rect(ntc, 0, 1, 1)
         : w == 9  ? k2d_rect(ntc, 0, 2, 0)
         : w == 10 ? k2d_rect(ntc, 0, 2, 1)
         : w == 11 ? k2d_rect(ntc, 1, 2, 0)
         : w == 12 ? k2d_rect(ntc, 1, 3, 1)
         : w == 13 ? k2d_rect(ntc, 2, 3, 0)
         : w == 14 ? k2d_rect(ntc, 2, 3, 1)
                   : k2d_rect(ntc, 1, 2, 1);
}
// per element type: roles (8 per group), groups, rows per staged chunk
template <typename T> __host__ __device__ constexpr int k2x_groups() { return sizeof(T) == 8 ? 2 : 1; }
template <typename T> __host__ __device__ constexpr K2BRole k2x_role(int ntc, int w) {
  return sizeof(T) == 8 ? k2d_role(ntc, w) : k2b_role(ntc, w);
}
template <typename T> __host__ __device__ constexpr int k2x_ntiles(int ntc, int w) {
  return k2x_role<T>(ntc, w).diag ? k2x_role<T>(ntc, w).nr * (k2x_role<T>(ntc, w).nr + 1) / 2
                                  : k2x_role<T>(ntc, w).nr * k2x_role<T>(ntc, w).nc;
}
template <typename T> __host__ __device__ constexpr int k2x_base(int ntc, int w) {
  return w == 0 ? 0 : k2x_base<T>(ntc, w - 1) + k2x_ntiles<T>(ntc, w - 1);
}
template <typename T> __host__ __device__ constexpr int k2x_kc(int ntc) {  // three buffers in 160 KB, 8 | KC
  return (160 * 1024 / (3 * k2_stride(ntc) * (int)sizeof(T))) / 8 * 8 > 32 ? 32
                                                                           : (160 * 1024 / (3 * k2_stride(ntc) * (int)sizeof(T))) / 8 * 8;
}

template <typename T, int NTC, int W>
__device__ __forceinline__ void k2x_mfma(const T* cur, int lb, typename K2Acc<T>::type (&acc)[k2x_ntiles<T>(NTC, W)]) {
  constexpr K2BRole R = k2x_role<T>(NTC, W);
  constexpr int STRIDE = k2_stride(NTC), KC = k2x_kc<T>(NTC);
  auto mm = [](T a, T b, typename K2Acc<T>::type c) {
    if constexpr (sizeof(T) == 8) return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  };
  if constexpr (sizeof(T) == 8) {
    // f64: fragments read next to their MFMAs (the 64-cycle MFMAs cover the reads; the f32 form below measured
    // 1.1% slower here, profiles/r03_n)
#pragma unroll
    for (int kk = 0; kk < KC; kk += 4) {
      const T* base = cur + kk * STRIDE + lb;
      if constexpr (R.diag) {
        T f[R.nr];
#pragma unroll
        for (int i = 0; i < R.nr; ++i) f[i] = base[16 * (R.ra + i)];
#pragma unroll
        for (int i = 0; i < R.nr; ++i)
#pragma unroll
          for (int j = i; j < R.nr; ++j) {
            const int x = i * R.nr - i * (i - 1) / 2 + (j - i);
            acc[x] = mm(f[i], f[j], acc[x]);
          }
      } else {
        T a[R.nr];
#pragma unroll
        for (int i = 0; i < R.nr; ++i) a[i] = base[16 * (R.ra + i)];
#pragma unroll
        for (int j = 0; j < R.nc; ++j) {
          const T b = base[16 * (R.ca + j)];
#pragma unroll
          for (int i = 0; i < R.nr; ++i) acc[i * R.nc + j] = mm(a[i], b, acc[i * R.nc + j]);
        }
      }
    }
    return;
  }
  // f32: every fragment of k-step kk + 4 is read before k-step kk's MFMAs issue (two register sets, renamed by the
  // unrolled loop): the reads of one k-step land while the previous one multiplies.  Reading each column block's
  // fragment just before its MFMAs (the compiler's own schedule) left an lgkmcnt(0) wait in front of every group
  // of nr MFMAs (361 in the G1 kernel, 90 after), with only two waves per SIMD to hide it: G1 125k f32 K2 -3.4%.
  constexpr int NF = R.diag ? R.nr : R.nr + R.nc;
  auto load = [&](int kk, T (&f)[NF]) {
    const T* base = cur + kk * STRIDE + lb;
#pragma unroll
    for (int i = 0; i < R.nr; ++i) f[i] = base[16 * (R.ra + i)];
    if constexpr (!R.diag) {
#pragma unroll
      for (int j = 0; j < R.nc; ++j) f[R.nr + j] = base[16 * (R.ca + j)];
    }
  };
  T f[NF];
  load(0, f);
#pragma unroll
  for (int kk = 0; kk < KC; kk += 4) {
    T g[NF];
    if (kk + 4 < KC) load(kk + 4, g);
    __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of this k-step's MFMAs (the scheduler sinks them)
    if constexpr (R.diag) {
#pragma unroll
      for (int i = 0; i < R.nr; ++i)
#pragma unroll
        for (int j = i; j < R.nr; ++j) {
          const int x = i * R.nr - i * (i - 1) / 2 + (j - i);
          acc[x] = mm(f[i], f[j], acc[x]);
        }
    } else {
#pragma unroll
      for (int j = 0; j < R.nc; ++j)
#pragma unroll
        for (int i = 0; i < R.nr; ++i) acc[i * R.nc + j] = mm(f[i], f[R.nr + j], acc[i * R.nc + j]);
    }
    if (kk + 4 < KC) {
#pragma unroll
      for (int i = 0; i < NF; ++i) f[i] = g[i];
    }
  }
}

template <typename T, int NTC, bool GATHER, int W>
__device__ __forceinline__ void k2x_wave(T* lds, const T* __restrict__ panel, int64_t r0, int64_t r1, int64_t prows,
                                         int64_t ldp, int ks, int nslots, int accumulate, double* __restrict__ slab,
                                         const int* __restrict__ rowlist, int wave, int lane) {
  typedef typename K2Acc<T>::type accT;
  constexpr int K2W = 8, KC = k2x_kc<T>(NTC), STRIDE = k2_stride(NTC);
  constexpr int BUF = KC * STRIDE;
  constexpr int RPW = KC / K2W;
  constexpr int EB = (int)sizeof(T);
  constexpr int NTW = k2x_ntiles<T>(NTC, W);
  const int rowbytes = (int)ldp * EB;
  const int np = (rowbytes + 1023) >> 10;  // 1 KiB pieces per row (wave-uniform, 1..3)
  constexpr int NPMAX = (16 * NTC * EB + 1023) / 1024;
  auto dma_row = [&](const T* src_row, T* dst_row) {
    const char* src = reinterpret_cast<const char*>(src_row);
    char* dst = reinterpret_cast<char*>(dst_row);
#pragma unroll
    for (int p = 0; p < NPMAX; ++p) {
      if (p < np) {
        const int off = (p << 10) + 16 * lane;
        if (off < rowbytes)
          __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + off),
                                           reinterpret_cast<void*>(dst + (p << 10)), 16, 0, 0);
      }
    }
  };
  int gidx[RPW];
  auto list_load = [&](int64_t c0) {
    if constexpr (GATHER) {
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        const int64_t x = c0 + wave + K2W * q;
        const int v = x < r1 ? rowlist[x] : 0;
        gidx[q] = v >= 0 && v < prows ? v : 0;
      }
    }
  };
  auto dma_chunk = [&](int64_t c0, T* buf) {
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int rr = wave + K2W * q;
      dma_row(panel + (GATHER ? (int64_t)gidx[q] : c0 + rr) * ldp, buf + rr * STRIDE);
    }
  };
  const int lb = (lane >> 4) * STRIDE + (lane & 15);  // A/B fragment: k = lane >> 4, column lane & 15
  accT acc[NTW];
#pragma unroll
  for (int x = 0; x < NTW; ++x) acc[x] = accT{0, 0, 0, 0};

  const int64_t nfull = (r1 - r0) / KC;
  T* b0 = lds;
  T* b1 = lds + BUF;
  T* b2 = lds + 2 * BUF;
  list_load(r0);
  if (nfull > 0) dma_chunk(r0, b0);
  list_load(r0 + KC);
  if (nfull > 1) {
    dma_chunk(r0 + KC, b1);
    list_load(r0 + 2 * KC);
    k2_wait_chunk<RPW>(np);  // chunk 0 landed (chunk 1 in flight)
  } else {
    k2_wait_vm<0>();
  }
  k2_barrier();
  for (int64_t c = 0; c < nfull; ++c) {
    const bool pre = c + 2 < nfull;
    if (pre) {
      dma_chunk(r0 + (c + 2) * KC, b2);
      list_load(r0 + (c + 3) * KC);
    }
    k2x_mfma<T, NTC, W>(b0, lb, acc);
    if (pre) k2_wait_chunk<RPW>(np);  // chunk c + 1 landed, chunk c + 2 stays in flight
    else k2_wait_vm<0>();
    k2_barrier();
    T* t = b0;
    b0 = b1;
    b1 = b2;
    b2 = t;
  }
  if (r0 + nfull * KC < r1) {  // the partial last chunk into b0
    const int64_t c0 = r0 + nfull * KC;
    const int valid = (int)(r1 - c0);
    list_load(c0);
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int rr = wave + K2W * q;
      T* dst = b0 + rr * STRIDE;
      if (rr < valid) {
        dma_row(panel + (GATHER ? (int64_t)gidx[q] : c0 + rr) * ldp, dst);
      } else {
        for (int x = 16 * lane; x < rowbytes; x += 16 * 64)
          *reinterpret_cast<uint4*>(reinterpret_cast<char*>(dst) + x) = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    k2_wait_vm<0>();
    k2_barrier();
    k2x_mfma<T, NTC, W>(b0, lb, acc);
  }
  constexpr int B = k2x_base<T>(NTC, W);
  // D layout: col = lane & 15; row = (lane >> 4) + 4 * reg for f64, 4 * (lane >> 4) + reg for f32
#pragma unroll
  for (int x = 0; x < NTW; ++x) {
    double* o = slab + ((size_t)ks * nslots + B + x) * 256;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = EB == 8 ? (lane >> 4) + 4 * j : 4 * (lane >> 4) + j;
      double* y = o + row * 16 + (lane & 15);
      const double v = (double)acc[x][j];
      *y = accumulate ? *y + v : v;
    }
  }
}

template <typename T, int NTC, bool GATHER = false>
__global__ void __launch_bounds__(512)
k2_gram_syrk_blk(const T* __restrict__ panel, int64_t rows, int64_t ldp, int ksplit, int nslots, int accumulate,
                 double* __restrict__ slab, const int* __restrict__ rowlist, const int* __restrict__ d_rows) {
  static_assert(k2b_supported(NTC), "16..23 tile columns");
  constexpr int KC = k2x_kc<T>(NTC), BUF = KC * k2_stride(NTC);
  static_assert(KC % 8 == 0 && KC >= 8 && 3 * BUF * (int)sizeof(T) <= 160 * 1024, "three LDS buffers");
  __shared__ __attribute__((aligned(16))) T lds[3 * BUF];
  int group, ks;
  k2_block_coords(k2x_groups<T>(), group, ks);
  const int64_t prows = rows;
  if constexpr (GATHER) rows = min((int64_t)__builtin_amdgcn_readfirstlane(*d_rows), prows);
  const int64_t q4 = rows / 4;
  const int64_t r0 = 4 * (q4 * ks / ksplit);
  const int64_t r1 = ks + 1 == ksplit ? rows : 4 * (q4 * (ks + 1) / ksplit);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  for (int x = threadIdx.x; x < 3 * BUF; x += 512) lds[x] = (T)0;  // columns >= ldp read as 0
  __syncthreads();
#define SYSID_K2X_WAVE(W)                                                                                        \
  case W:                                                                                                        \
    k2x_wave<T, NTC, GATHER, W>(lds, panel, r0, r1, prows, ldp, ks, nslots, accumulate, slab, rowlist, wave, lane); \
    break;
  switch (8 * group + wave) {
    SYSID_K2X_WAVE(0) SYSID_K2X_WAVE(1) SYSID_K2X_WAVE(2) SYSID_K2X_WAVE(3)
    SYSID_K2X_WAVE(4) SYSID_K2X_WAVE(5) SYSID_K2X_WAVE(6) SYSID_K2X_WAVE(7)
    default:
      if constexpr (k2x_groups<T>() == 2) {
        switch (8 * group + wave) {
          SYSID_K2X_WAVE(8) SYSID_K2X_WAVE(9) SYSID_K2X_WAVE(10) SYSID_K2X_WAVE(11)
          SYSID_K2X_WAVE(12) SYSID_K2X_WAVE(13) SYSID_K2X_WAVE(14)
          default: k2x_wave<T, NTC, GATHER, 15>(lds, panel, r0, r1, prows, ldp, ks, nslots, accumulate, slab, rowlist, wave, lane);
        }
      }
      break;
  }
#undef SYSID_K2X_WAVE
}

#ifndef SYSID_TEMPLATE_TU
// K3, one pass: G = the sum of the ksplit slabs, in a fixed order, mirrored.  A workgroup of 16 waves owns 64
// consecutive entries of one tile slot (so a dead slot drops the whole workgroup); wave w sums slabs w, w + 16,
// ... with eight loads in flight per lane, and the 16 wave sums are added in LDS as a fixed pairwise tree.
// Every slab byte is requested by a quarter of a million lanes at once: the pass is one HBM read of the
// slabs, with no partial-sum round trip and no second launch.
__global__ void __launch_bounds__(1024)
k3_gram_reduce(const double* __restrict__ slab, const int2* __restrict__ tiles, int64_t nx, int ksplit, int ncol,
               double* __restrict__ G) {
  __shared__ double red[16][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t e = (int64_t)blockIdx.x * 64 + lane;
  const int2 ij = tiles[(int)(e >> 8)];
  if (ij.x < 0) return;  // workgroup-uniform: the 64 entries share one slot
  double a[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  int ks = wave;
  for (; ks + 7 * 16 < ksplit; ks += 8 * 16) {
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] += slab[(size_t)(ks + 16 * u) * nx + e];
  }
  for (; ks < ksplit; ks += 16) a[0] += slab[(size_t)ks * nx + e];
  red[wave][lane] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
#pragma unroll
  for (int h = 8; h >= 1; h >>= 1) {
    if (wave < h) red[wave][lane] += red[wave + h][lane];
    __syncthreads();
  }
  if (wave == 0) {
    const int x = (int)(e & 255);
    const int gi = ij.x * 16 + (x >> 4), gj = ij.y * 16 + (x & 15);
    // a diagonal tile's upper half only, each entry written to both mirrored positions: the Gram is bitwise
    // symmetric whatever order the MFMA summed a diagonal tile's two halves in
    if (gi < ncol && gj < ncol && (ij.x != ij.y || (x >> 4) <= (x & 15))) {
      const double acc = red[0][lane];
      G[(int64_t)gi * ncol + gj] = acc;
      G[(int64_t)gj * ncol + gi] = acc;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// K4: torque-prediction errors of the stacked system (print_tau_prediction_rmse,
// src/sys_identification.py:421-437, without its second pass over the samples):
//   e[s, d] = Y_proj[s*nv + d, :] . phi - tau_proj[s*nv + d];   part[block][d] = sum over its samples e^2.
// Thread t of a block owns dof d = t % nv of samples t / nv, t / nv + spb, ... (spb = 256 / nv), so
// every thread accumulates one dof and the block sum per dof runs in a fixed order: deterministic.
// HBM-bound (reads the Y_proj and tau columns once).
// ------------------------------------------------------------------------------------------------
constexpr int K4_MAXWY = 640;

__global__ void __launch_bounds__(256)
k4_tau_error(const double* __restrict__ panel, int64_t ldp, int64_t N, int nv, int wy, int w,
             const double* __restrict__ phi, double* __restrict__ part) {
  __shared__ double sphi[K4_MAXWY];
  __shared__ double red[256];
  for (int c = threadIdx.x; c < wy; c += 256) sphi[c] = phi[c];
  __syncthreads();
  const int spb = 256 / nv, t = threadIdx.x, so = t / nv, d = t - so * nv;
  const int64_t s0 = (int64_t)blockIdx.x * N / gridDim.x, s1 = (int64_t)(blockIdx.x + 1) * N / gridDim.x;
  double acc = 0.0;
  if (so < spb) {
    for (int64_t s = s0 + so; s < s1; s += spb) {
      const double* row = panel + (s * nv + d) * ldp;
      const double2* row2 = reinterpret_cast<const double2*>(row);
      double a0 = 0.0, a1 = 0.0;
      for (int c = 0; c < (wy >> 1); ++c) {
        const double2 v = row2[c];
        a0 += v.x * sphi[2 * c];
        a1 += v.y * sphi[2 * c + 1];
      }
      const double e = (a0 + a1) - row[w];
      acc += e * e;
    }
  }
  red[t] = acc;
  __syncthreads();
  if (t < nv) {
    double sum = 0.0;
    for (int u = 0; u < spb; ++u) sum += red[u * nv + t];
    part[(int64_t)blockIdx.x * nv + t] = sum;
  }
}

__global__ void __launch_bounds__(64)
k4_tau_error_final(const double* __restrict__ part, int nblocks, int nv, double* __restrict__ err_sq) {
  for (int d = threadIdx.x; d < nv; d += 64) {
    double sum = 0.0;
    for (int b = 0; b < nblocks; ++b) sum += part[(int64_t)b * nv + d];
    err_sq[d] = sum;
  }
}

// ------------------------------------------------------------------------------------------------
// K5: the host entry point's de-interleave.  The panel's row r = [Y_proj | B_v | B_c | tau_proj | pad] is
// split into the reference's separate stacked arrays (demo/spot_identification.py:84-87), each contiguous in
// one device staging buffer, so every output leaves the device as ONE contiguous copy (instead of a 2-D copy
// of rows x 8..1040 bytes).  One wave per row (grid-stride): the Y block as 16-byte pairs, the friction and
// torque columns as 8-byte elements (nj may be odd).  A null output pointer skips that output.  HBM-bound.
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
k5_unstack(const double* __restrict__ panel, int64_t rows, int64_t ldp, int wy, int nj,
           double* __restrict__ Y, double* __restrict__ tau, double* __restrict__ Bv, double* __restrict__ Bc) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int y2 = wy >> 1, nf = 2 * nj + 1;
  for (int64_t r = wave; r < rows; r += nwaves) {
    const double* pr = panel + r * ldp;
    if (Y != nullptr) {
      const double2* src = reinterpret_cast<const double2*>(pr);
      double2* dst = reinterpret_cast<double2*>(Y + r * wy);
      for (int c = lane; c < y2; c += 64) dst[c] = src[c];
    }
    for (int c = lane; c < nf; c += 64) {
      const double v = pr[wy + c];
      if (c < nj) {
        if (Bv != nullptr) Bv[r * nj + c] = v;
      } else if (c < 2 * nj) {
        if (Bc != nullptr) Bc[r * nj + (c - nj)] = v;
      } else if (tau != nullptr) {
        tau[r] = v;
      }
    }
  }
}

// Diagnostics kernel: lane l computes column (l % 10) of the body regressor in world frame.
__global__ void debug_body_column_kernel(const double* __restrict__ body24, double* __restrict__ out) {
  __shared__ double b[24];
  if (threadIdx.x < 24) b[threadIdx.x] = body24[threadIdx.x];
  __syncthreads();
  double fw[6];
  double F[FBLK];
  body_regressor_block(b, F);
  block_column(F, threadIdx.x % 10, fw);
  for (int k = 0; k < 6; ++k) out[threadIdx.x * 6 + k] = fw[k];
}
#endif  // SYSID_TEMPLATE_TU

}  // namespace sysid_dev
