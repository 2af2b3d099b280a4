// sysid_engine.hip — MI355X (gfx950) identification-regressor engine: kernels + C ABI (include/sysid.h).
//
// Hot path: per sample, the inverse-dynamics regressor Y(q, dq, ddq) (pinocchio
// computeJointTorqueRegressor, called at src/sys_identification.py:406), the contact-nullspace projector
// P = I - pinv(J_c) J_c (:119-135), the projected regressor / torque / friction regressors (:401-418),
// stacked sample-major (demo/spot_identification.py:37-56, 84-87), and the Gram of the stacked system
// the Solver's objective implies (src/solver.py:186-190).
//
// Kernels
//   K1 regressor_panel_kernel  one workgroup per sample (grid-stride).  fp64 VALU, LDS-resident
//      kinematics.  Formulation (validated in tests/alg_mirror.py against the oracle):
//        - world motion axes of every dof from forward kinematics;
//        - J_c from those axes; P = I - Q^T Q with Q = L^-1 J_c, L L^T = J_c J_c^T (Cholesky-QR);
//        - H_i = P M_i J_w^T (nv x 6) by one rank-1 update per body from its parent (M_i: the dofs
//          supporting body i);  column (i, p) of P·Y = H_i · (world-frame body-regressor column);
//        - friction / torque columns straight from P.
//      Writes the panel [Y_proj | B_v | B_c | tau_proj] row-major, coalesced across columns.
//   K2 gram_syrk_kernel        split-K SYRK of the panel on v_mfma_f64_16x16x4_f64, upper 16x16 tiles,
//      rows staged through LDS, per-block partial tiles written to a slab.
//   K3 gram_reduce_kernel      deterministic sum of the slabs -> full symmetric Gram.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "sysid.h"

namespace {

constexpr int NJ_MAX = 64;   // joints incl. universe
constexpr int NC_MAX = 8;    // contact frames
constexpr int NV_MAX = 64;   // velocity dimension (support masks are 64-bit)
constexpr int K1_MAX_THREADS = 256;
constexpr int K2_THREADS = 256;
constexpr int K2_TPW = 14;   // Gram tiles per wave (4 waves -> 56 tiles per workgroup)

constexpr int JT_FREEFLYER = 1;
constexpr int JT_REVOLUTE = 2;

struct DevModel {
  int nq, nv, njoints, nc, base_dof, nj, maxdepth, wy;
  int w, ncol, in_rows, pad0;
  int parent[NJ_MAX], jtype[NJ_MAX], idx_q[NJ_MAX], idx_v[NJ_MAX], depth[NJ_MAX];
  int dof_joint[NV_MAX], dof_k[NV_MAX];
  int cjoint[NC_MAX];
  unsigned long long csupp[NC_MAX];
  double axis[NJ_MAX][3];
  double R0[NJ_MAX][9];
  double t0[NJ_MAX][3];
  double cR[NC_MAX][9];
  double ct[NC_MAX][3];
  double g[3];
};

// LDS layout of K1 (offsets in doubles).  Shared by host (sizing) and device.
struct K1Layout {
  int in, body, W, Pt, Jw, pf, Jc, L, M, P, H, total;
};

__host__ __device__ inline K1Layout k1_layout(int in_rows, int nv, int njoints, int nc) {
  K1Layout l;
  const int kmax = 3 * nc;
  int o = 0;
  l.in = o;   o += (in_rows + 1) & ~1;
  l.body = o; o += njoints * 24;              // oR(9) ot(3) v(6) a_gf(6)
  l.W = o;    o += nv * 3;
  l.Pt = o;   o += nv * 3;
  l.Jw = o;   o += nv * 6;                    // world spatial axis [lin at origin; ang]
  l.pf = o;   o += ((nc * 3) + 1) & ~1;
  l.Jc = o;   o += kmax * nv;                 // J_c, then Q in place
  l.L = o;    o += kmax * kmax;
  l.M = o;    o += kmax * kmax;
  l.P = o;    o += nv * nv;
  o = (o + 1) & ~1;
  l.H = o;    o += njoints * nv * 6;
  l.total = o;
  return l;
}

// ---- small device helpers ----------------------------------------------------------------------

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

// SE3(R, t).actInv(motion m) -> out   (motion = [v; w])
__device__ inline void act_inv_motion(const double* R, const double* t, const double* m, double* out) {
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

// a x e_k for the unit vector e_k
__host__ __device__ inline void cross_unit(const double* a, int k, double* c) {
  if (k == 0) { c[0] = 0.0; c[1] = a[2]; c[2] = -a[1]; }
  else if (k == 1) { c[0] = -a[2]; c[1] = 0.0; c[2] = a[0]; }
  else { c[0] = a[1]; c[1] = -a[0]; c[2] = 0.0; }
}

__device__ inline double sign_of(double x) {
  return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : (x == x ? 0.0 : x));
}

// Column p of the body regressor of body i (local frame, pinocchio bodyRegressor with parameters
// [m, mc, Ixx, Ixy, Iyy, Ixz, Iyz, Izz]) moved to the world frame: fw = oX_i^* f.
// bi = per-body LDS record: oR(9) ot(3) v(6) a_gf(6).
__host__ __device__ inline void body_regressor_world_column(const double* bi, int p, double* fw) {
  // Branch-free: every lane of a wave evaluates the same instructions whatever its column p.
  const double* v = bi + 12;
  const double* a = bi + 18;
  const double* w = v + 3;
  const double* dw = a + 3;
  double ac[3], tmp[3];
  cross3(w, v, tmp);
  ac[0] = a[0] + tmp[0]; ac[1] = a[1] + tmp[1]; ac[2] = a[2] + tmp[2];
  // column selectors: mass (p = 0), first moment e_k (p = 1..3), inertia [xx xy yy xz yz zz] (p = 4..9)
  const double sm = p == 0 ? 1.0 : 0.0;
  const double e[3] = {p == 1 ? 1.0 : 0.0, p == 2 ? 1.0 : 0.0, p == 3 ? 1.0 : 0.0};
  const double s0 = p == 4 ? 1.0 : 0.0, s1 = p == 5 ? 1.0 : 0.0, s2 = p == 6 ? 1.0 : 0.0;
  const double s3 = p == 7 ? 1.0 : 0.0, s4 = p == 8 ? 1.0 : 0.0, s5 = p == 9 ? 1.0 : 0.0;
  // f = m ac + (dw x + w x w x) h ;  n = h x ac + I dw + w x (I w)
  double x1[3], x2[3], x3[3], n[3], f[3];
  cross3(dw, e, x1);
  cross3(w, e, x2);
  cross3(w, x2, x3);
  f[0] = sm * ac[0] + x1[0] + x3[0];
  f[1] = sm * ac[1] + x1[1] + x3[1];
  f[2] = sm * ac[2] + x1[2] + x3[2];
  cross3(e, ac, n);
  double bdw[3], bw[3];
  bdw[0] = s0 * dw[0] + s1 * dw[1] + s3 * dw[2];
  bdw[1] = s1 * dw[0] + s2 * dw[1] + s4 * dw[2];
  bdw[2] = s3 * dw[0] + s4 * dw[1] + s5 * dw[2];
  bw[0] = s0 * w[0] + s1 * w[1] + s3 * w[2];
  bw[1] = s1 * w[0] + s2 * w[1] + s4 * w[2];
  bw[2] = s3 * w[0] + s4 * w[1] + s5 * w[2];
  cross3(w, bw, x2);
  n[0] += bdw[0] + x2[0];
  n[1] += bdw[1] + x2[1];
  n[2] += bdw[2] + x2[2];
  // to world: f_w = oR f, n_w = oR n + ot x f_w
  double nl[3];
  mat3vec(bi, f, fw);
  mat3vec(bi, n, nl);
  cross3(bi + 9, fw, tmp);
  fw[3] = nl[0] + tmp[0]; fw[4] = nl[1] + tmp[1]; fw[5] = nl[2] + tmp[2];
}

// index of the a-th contact frame whose contact value is non-zero
__device__ inline int active_contact(const double* cnt, int nc, int a) {
  int seen = 0;
  for (int c = 0; c < nc; ++c) {
    if (cnt[c] != 0.0) {
      if (seen == a) return c;
      ++seen;
    }
  }
  return 0;
}

// ------------------------------------------------------------------------------------------------
// K1: regressor + projector -> panel
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(K1_MAX_THREADS)
regressor_panel_kernel(const DevModel* __restrict__ mdl, const double* __restrict__ in, int64_t N,
                       int64_t ld, double* __restrict__ panel, int64_t ldp, double* __restrict__ lds_dump) {
  extern __shared__ double sm[];
  const DevModel& m = *mdl;
  const int nv = m.nv, nq = m.nq, nc = m.nc, NJ = m.njoints, bd = m.base_dof, nja = m.nj;
  const K1Layout L = k1_layout(m.in_rows, nv, NJ, nc);
  const int tid = threadIdx.x, nt = blockDim.x;
  double* sin_ = sm + L.in;
  const double* q = sin_;
  const double* dq = sin_ + nq;
  const double* ddq = dq + nv;
  const double* tau = ddq + nv;
  const double* cnt = tau + nja;
  double* body = sm + L.body;
  double* Ws = sm + L.W;
  double* Pts = sm + L.Pt;
  double* Jws = sm + L.Jw;
  double* pfs = sm + L.pf;
  double* Jc = sm + L.Jc;
  double* Ls = sm + L.L;
  double* Ms = sm + L.M;
  double* Ps = sm + L.P;
  double* Hs = sm + L.H;

  for (int64_t s = blockIdx.x; s < N; s += gridDim.x) {
    // ---- phase 0: inputs (channel-major) + universe body ----
    for (int c = tid; c < m.in_rows; c += nt) sin_[c] = in[(int64_t)c * ld + s];
    if (tid < 24) {
      double v = 0.0;
      if (tid == 0 || tid == 4 || tid == 8) v = 1.0;        // oR = I
      if (tid >= 18 && tid < 21) v = -m.g[tid - 18];        // a_gf[0] = -gravity (linear)
      body[tid] = v;
    }
    __syncthreads();

    // ---- phase 1: forward pass (computeJointTorqueRegressor forward step + world placements) ----
    for (int lvl = 1; lvl <= m.maxdepth; ++lvl) {
      for (int j = 1 + tid; j < NJ; j += nt) {
        if (m.depth[j] != lvl) continue;
        const int p = m.parent[j];
        const int iq = m.idx_q[j], iv = m.idx_v[j];
        const double* bp = body + 24 * p;
        double* bj = body + 24 * j;
        double RJ[9], tJ[3], vJ[6], Sa[6];
        const bool ff = m.jtype[j] == JT_FREEFLYER;
        if (ff) {
          quat_to_matrix(q[iq + 3], q[iq + 4], q[iq + 5], q[iq + 6], RJ);
          tJ[0] = q[iq]; tJ[1] = q[iq + 1]; tJ[2] = q[iq + 2];
#pragma unroll
          for (int k = 0; k < 6; ++k) { vJ[k] = dq[iv + k]; Sa[k] = ddq[iv + k]; }
        } else {
          const double* ax = m.axis[j];
          axis_rotation(ax, q[iq], RJ);
          tJ[0] = tJ[1] = tJ[2] = 0.0;
          const double w = dq[iv], aa = ddq[iv];
          vJ[0] = vJ[1] = vJ[2] = 0.0; Sa[0] = Sa[1] = Sa[2] = 0.0;
          vJ[3] = ax[0] * w; vJ[4] = ax[1] * w; vJ[5] = ax[2] * w;
          Sa[3] = ax[0] * aa; Sa[4] = ax[1] * aa; Sa[5] = ax[2] * aa;
        }
        double liR[9], lit[3], tmp[3];
        mat3mul(m.R0[j], RJ, liR);
        mat3vec(m.R0[j], tJ, tmp);
        lit[0] = tmp[0] + m.t0[j][0]; lit[1] = tmp[1] + m.t0[j][1]; lit[2] = tmp[2] + m.t0[j][2];
        double vp[6], ap[6], vi[6], ai[6], c1[3], c2[3];
        act_inv_motion(liR, lit, bp + 12, vp);
        act_inv_motion(liR, lit, bp + 18, ap);
#pragma unroll
        for (int k = 0; k < 6; ++k) vi[k] = vJ[k] + vp[k];
        if (ff) {
#pragma unroll
          for (int k = 0; k < 6; ++k) ai[k] = Sa[k] + ap[k];   // v x v = 0
        } else {
          // motion cross v_i x vJ with vJ = (0, wJ): (v x wJ, w x wJ)
          cross3(vi, vJ + 3, c1);
          cross3(vi + 3, vJ + 3, c2);
          ai[0] = c1[0] + Sa[0] + ap[0]; ai[1] = c1[1] + Sa[1] + ap[1]; ai[2] = c1[2] + Sa[2] + ap[2];
          ai[3] = c2[0] + Sa[3] + ap[3]; ai[4] = c2[1] + Sa[4] + ap[4]; ai[5] = c2[2] + Sa[5] + ap[5];
        }
        double oR[9], ot[3];
        mat3mul(bp, liR, oR);
        mat3vec(bp, lit, ot);
        ot[0] += bp[9]; ot[1] += bp[10]; ot[2] += bp[11];
#pragma unroll
        for (int k = 0; k < 9; ++k) bj[k] = oR[k];
        bj[9] = ot[0]; bj[10] = ot[1]; bj[11] = ot[2];
#pragma unroll
        for (int k = 0; k < 6; ++k) { bj[12 + k] = vi[k]; bj[18 + k] = ai[k]; }
      }
      __syncthreads();
    }

    // ---- phase 2: world motion axes of every dof, contact points ----
    for (int e = tid; e < nv + nc; e += nt) {
      if (e < nv) {
        const int r = e;
        const int j = m.dof_joint[r];
        const double* bj = body + 24 * j;
        double W[3], P[3] = {bj[9], bj[10], bj[11]};
        bool lin = false;
        if (m.jtype[j] == JT_FREEFLYER) {
          const int k = m.dof_k[r];
          const int col = k < 3 ? k : k - 3;
          W[0] = bj[col]; W[1] = bj[3 + col]; W[2] = bj[6 + col];
          lin = k < 3;
        } else {
          mat3vec(bj, m.axis[j], W);
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
        const double* bj = body + 24 * m.cjoint[c];
        double x[3];
        mat3vec(bj, m.ct[c], x);
        pfs[3 * c] = x[0] + bj[9]; pfs[3 * c + 1] = x[1] + bj[10]; pfs[3 * c + 2] = x[2] + bj[11];
      }
    }
    int na = 0;
    for (int c = 0; c < nc; ++c) na += cnt[c] != 0.0 ? 1 : 0;
    const int k = 3 * na;
    __syncthreads();

    // ---- phase 3: contact Jacobian (LOCAL_WORLD_ALIGNED, linear rows) ----
    for (int e = tid; e < k * nv; e += nt) {
      const int rho = e / nv, r = e - rho * nv;
      const int c = active_contact(cnt, nc, rho / 3), comp = rho % 3;
      double val = 0.0;
      if ((m.csupp[c] >> r) & 1ull) {
        const double* W = Ws + 3 * r;
        if (m.jtype[m.dof_joint[r]] == JT_FREEFLYER && m.dof_k[r] < 3) {
          val = W[comp];
        } else {
          double d[3], x[3];
          d[0] = pfs[3 * c] - Pts[3 * r];
          d[1] = pfs[3 * c + 1] - Pts[3 * r + 1];
          d[2] = pfs[3 * c + 2] - Pts[3 * r + 2];
          cross3(W, d, x);
          val = x[comp];
        }
      }
      Jc[rho * nv + r] = val;
    }
    __syncthreads();

    // ---- phase 4: M = J_c J_c^T ----
    for (int e = tid; e < k * k; e += nt) {
      const int a = e / k, b = e - a * k;
      double acc = 0.0;
      for (int r = 0; r < nv; ++r) acc += Jc[a * nv + r] * Jc[b * nv + r];
      Ms[e] = acc;
    }
    __syncthreads();

    // ---- phase 5: Cholesky M = L L^T (right-looking, rank-deficient pivots dropped) ----
    double dmax = 0.0;
    for (int a = 0; a < k; ++a) dmax = fmax(dmax, Ms[a * k + a]);
    const double thr = 1e-13 * dmax;
    for (int j = 0; j < k; ++j) {
      const double djj = Ms[j * k + j];
      const bool keep = djj > thr;
      const double ljj = keep ? sqrt(djj) : 0.0;
      for (int i = j + tid; i < k; i += nt) Ls[i * k + j] = !keep ? 0.0 : (i == j ? ljj : Ms[i * k + j] / ljj);
      __syncthreads();
      const int rem = k - j - 1;
      for (int e = tid; e < rem * rem; e += nt) {
        const int i = j + 1 + e / rem, l = j + 1 + e % rem;
        if (l <= i) Ms[i * k + l] -= Ls[i * k + j] * Ls[l * k + j];
      }
      __syncthreads();
    }

    // ---- phase 6: Q = L^-1 J_c (in place over J_c, one column per thread) ----
    for (int r = tid; r < nv; r += nt) {
      for (int j = 0; j < k; ++j) {
        const double ljj = Ls[j * k + j];
        double x = Jc[j * nv + r];
        for (int l = 0; l < j; ++l) x -= Ls[j * k + l] * Jc[l * nv + r];
        Jc[j * nv + r] = ljj != 0.0 ? x / ljj : 0.0;
      }
    }
    __syncthreads();

    // ---- phase 7: P = I - Q^T Q ----
    for (int e = tid; e < nv * nv; e += nt) {
      const int a = e / nv, b = e - a * nv;
      double acc = 0.0;
      for (int j = 0; j < k; ++j) acc += Jc[j * nv + a] * Jc[j * nv + b];
      Ps[e] = (a == b ? 1.0 : 0.0) - acc;
    }
    __syncthreads();

    // ---- phase 8: H_i = P M_i J_w^T, one rank-1 update per dof along the DFS order ----
    for (int e = tid; e < nv * 6; e += nt) {
      const int r = e / 6, c = e - r * 6;
      for (int j = 1; j < NJ; ++j) {
        const int p = m.parent[j];
        double h = p > 0 ? Hs[(p * nv + r) * 6 + c] : 0.0;
        const int iv = m.idx_v[j];
        const int nd = m.jtype[j] == JT_FREEFLYER ? 6 : 1;
        for (int d = 0; d < nd; ++d) h += Ps[r * nv + iv + d] * Jws[6 * (iv + d) + c];
        Hs[(j * nv + r) * 6 + c] = h;
      }
    }
    __syncthreads();

    if (lds_dump != nullptr && s == 0) {  // diagnostics: LDS image of sample 0 after phase 8
      for (int x = tid; x < L.total; x += nt) lds_dump[x] = sm[x];
    }

    // ---- phase 9: panel columns ----
    double* out = panel + (s * nv) * ldp;
    for (int col = tid; col < m.ncol; col += nt) {
      if (col < m.wy) {
        const int i = col / 10 + 1, p = col - 10 * (col / 10);
        const double* bi = body + 24 * i;
        const double* v = bi + 12;
        const double* a = bi + 18;
        double fw[6];
        body_regressor_world_column(bi, p, fw);
        const double* Hi = Hs + (size_t)i * nv * 6;
        for (int r = 0; r < nv; ++r) {
          const double* h = Hi + 6 * r;
          out[(int64_t)r * ldp + col] =
              h[0] * fw[0] + h[1] * fw[1] + h[2] * fw[2] + h[3] * fw[3] + h[4] * fw[4] + h[5] * fw[5];
        }
      } else if (col < m.wy + 2 * nja) {
        const bool coul = col >= m.wy + nja;
        const int jj = col - m.wy - (coul ? nja : 0);
        const double x = dq[bd + jj];
        const double sc = coul ? sign_of(x) : x;
        for (int r = 0; r < nv; ++r) out[(int64_t)r * ldp + col] = Ps[r * nv + bd + jj] * sc;
      } else {
        for (int r = 0; r < nv; ++r) {
          double acc = 0.0;
          for (int jj = 0; jj < nja; ++jj) acc += Ps[r * nv + bd + jj] * tau[jj];
          out[(int64_t)r * ldp + col] = acc;
        }
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// K2: split-K SYRK of the panel on fp64 MFMA (16x16x4), upper-triangular 16x16 tiles.
// ------------------------------------------------------------------------------------------------
typedef double dbl4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(K2_THREADS)
gram_syrk_kernel(const double* __restrict__ panel, int64_t rows, int64_t ldp, int ncol, int ntc,
                 int lds_stride, int kc, const int2* __restrict__ tiles, int ngroups, int ksplit,
                 int ntiles_total, double* __restrict__ slab) {
  extern __shared__ double chunk[];
  const int group = blockIdx.x % ngroups;
  const int ks = blockIdx.x / ngroups;
  const int64_t r0 = rows * ks / ksplit, r1 = rows * (ks + 1) / ksplit;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int2* wt = tiles + (group * 4 + wave) * K2_TPW;
  int tI[K2_TPW], tJ[K2_TPW];
#pragma unroll
  for (int t = 0; t < K2_TPW; ++t) {
    const int2 ij = wt[t];
    tI[t] = ij.x;
    tJ[t] = ij.y;
  }
  dbl4 acc[K2_TPW];
#pragma unroll
  for (int t = 0; t < K2_TPW; ++t) acc[t] = dbl4{0.0, 0.0, 0.0, 0.0};

  const int cols_p = ntc * 16;
  const int kr = lane >> 4, kc16 = lane & 15;
  for (int64_t c0 = r0; c0 < r1; c0 += kc) {
    const int pairs = kc * (cols_p / 2);
    for (int e = threadIdx.x; e < pairs; e += K2_THREADS) {
      const int rr = e / (cols_p / 2);
      const int col = 2 * (e - rr * (cols_p / 2));
      const int64_t grow = c0 + rr;
      double x = 0.0, y = 0.0;
      if (grow < r1 && col < ncol) {
        const double* src = panel + grow * ldp + col;
        if (col + 1 < ldp) {
          const double2 v = *reinterpret_cast<const double2*>(src);
          x = v.x;
          y = (col + 1 < ncol) ? v.y : 0.0;
        } else {
          x = src[0];
        }
      }
      chunk[rr * lds_stride + col] = x;
      chunk[rr * lds_stride + col + 1] = y;
    }
    __syncthreads();
    for (int kk = 0; kk < kc; kk += 4) {
      const double* rowp = chunk + (kk + kr) * lds_stride + kc16;
#pragma unroll
      for (int t = 0; t < K2_TPW; ++t) {
        if (tI[t] >= 0) {
          const double a = rowp[tI[t] * 16];
          const double b = rowp[tJ[t] * 16];
          acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[t], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  // epilogue: D layout of v_mfma_f64_16x16x4: col = lane & 15, row = (lane >> 4) + 4 * reg
  const int tbase = (group * 4 + wave) * K2_TPW;
#pragma unroll
  for (int t = 0; t < K2_TPW; ++t) {
    if (tI[t] < 0) continue;
    const int tid_global = tbase + t;  // tile slot == global tile index (host lays tiles out densely)
    double* o = slab + ((size_t)ks * ntiles_total + tid_global) * 256;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[((lane >> 4) + 4 * j) * 16 + (lane & 15)] = acc[t][j];
  }
}

// K3: G[I*16+r][J*16+c] = sum_ks slab[ks][tile][r*16+c], mirrored to the lower triangle.
__global__ void __launch_bounds__(256)
gram_reduce_kernel(const double* __restrict__ slab, const int2* __restrict__ tiles, int ntiles_total,
                   int ksplit, int ncol, double* __restrict__ G) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)ntiles_total * 256) return;
  const int t = (int)(e >> 8), x = (int)(e & 255);
  const int2 ij = tiles[t];
  if (ij.x < 0) return;
  double acc = 0.0;
  for (int ks = 0; ks < ksplit; ++ks) acc += slab[((size_t)ks * ntiles_total + t) * 256 + x];
  const int gi = ij.x * 16 + (x >> 4), gj = ij.y * 16 + (x & 15);
  if (gi < ncol && gj < ncol) {
    G[(int64_t)gi * ncol + gj] = acc;
    G[(int64_t)gj * ncol + gi] = acc;
  }
}

// Diagnostics kernel: lane l computes column (l % 10) of the body regressor in world frame.
__global__ void debug_body_column_kernel(const double* __restrict__ body24, double* __restrict__ out) {
  __shared__ double b[24];
  if (threadIdx.x < 24) b[threadIdx.x] = body24[threadIdx.x];
  __syncthreads();
  double fw[6];
  body_regressor_world_column(b, threadIdx.x % 10, fw);
  for (int k = 0; k < 6; ++k) out[threadIdx.x * 6 + k] = fw[k];
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
thread_local std::string g_thread_error = "";

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

}  // namespace

struct sysid_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  DevModel hm{};
  DevModel* d_model = nullptr;
  int nq = 0, nv = 0, nj = 0, nb = 0, nc = 0, wy = 0, w = 0, ncol = 0, ldp = 0, in_rows = 0;
  // Gram tiling
  int ntc = 0, ntiles = 0, ngroups = 0, lds_stride = 0, kc = 0;
  int2* d_tiles = nullptr;
  // K1 launch shape
  int k1_threads = 128;
  size_t k1_lds = 0;
  // host-API buffers (grow-only)
  double* d_in = nullptr;
  size_t in_cap = 0;
  double* d_panel = nullptr;
  size_t panel_cap = 0;
  double* d_gram = nullptr;
  void* d_ws = nullptr;
  size_t ws_cap = 0;
  double* d_dump = nullptr;  // diagnostics only (sysid_debug_lds)
  std::string err;
};

namespace {

int set_err(sysid_engine* e, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (e) e->err = buf;
  g_thread_error = buf;
  return code;
}

#define HIP_TRY(e, expr)                                                                       \
  do {                                                                                         \
    hipError_t _st = (expr);                                                                   \
    if (_st != hipSuccess)                                                                     \
      return set_err((e), SYSID_E_DEVICE, "%s failed: %s", #expr, hipGetErrorString(_st));     \
  } while (0)

int ksplit_for(const sysid_engine* e, int64_t rows) {
  int ks = 256 / (e->ngroups > 0 ? e->ngroups : 1);
  if (ks < 1) ks = 1;
  const int64_t cap = (rows + 255) / 256;
  if (cap < ks) ks = (int)(cap < 1 ? 1 : cap);
  return ks;
}

size_t slab_bytes(const sysid_engine* e, int64_t rows) {
  return align256((size_t)ksplit_for(e, rows) * e->ntiles * 256 * sizeof(double));
}

int grow(sysid_engine* e, void** p, size_t* cap, size_t need) {
  if (need <= *cap) return SYSID_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  HIP_TRY(e, hipMalloc(p, need));
  *cap = need;
  return SYSID_OK;
}

int launch_stages(sysid_engine* e, const double* d_in, int64_t N, int64_t ld, uint32_t flags,
                  double* d_panel, int64_t ld_panel, double* d_gram, void* d_ws, size_t ws_bytes,
                  hipStream_t st, hipEvent_t* ev /* 4 events or null */) {
  if (N <= 0) return SYSID_OK;
  const int64_t rows = N * e->nv;
  int grid1 = (int)(N < (int64_t)(1 << 30) ? N : (1 << 30));
  if (ev) HIP_TRY(e, hipEventRecord(ev[0], st));
  hipLaunchKernelGGL(regressor_panel_kernel, dim3(grid1), dim3(e->k1_threads), e->k1_lds, st,
                     e->d_model, d_in, N, ld, d_panel, ld_panel, e->d_dump);
  HIP_TRY(e, hipGetLastError());
  if (ev) HIP_TRY(e, hipEventRecord(ev[1], st));
  if (flags & SYSID_EMIT_GRAM) {
    const int ks = ksplit_for(e, rows);
    const size_t need = slab_bytes(e, rows);
    if (d_ws == nullptr || ws_bytes < need)
      return set_err(e, SYSID_E_INVALID, "workspace too small: %zu < %zu bytes", ws_bytes, need);
    double* slab = static_cast<double*>(d_ws);
    const size_t lds2 = (size_t)e->kc * e->lds_stride * sizeof(double);
    hipLaunchKernelGGL(gram_syrk_kernel, dim3(e->ngroups * ks), dim3(K2_THREADS), lds2, st, d_panel,
                       rows, ld_panel, e->ncol, e->ntc, e->lds_stride, e->kc, e->d_tiles, e->ngroups,
                       ks, e->ngroups * 4 * K2_TPW, slab);
    HIP_TRY(e, hipGetLastError());
    if (ev) HIP_TRY(e, hipEventRecord(ev[2], st));
    const int tot = e->ngroups * 4 * K2_TPW;
    const int64_t elems = (int64_t)tot * 256;
    hipLaunchKernelGGL(gram_reduce_kernel, dim3((unsigned)((elems + 255) / 256)), dim3(256), 0, st, slab,
                       e->d_tiles, tot, ks, e->ncol, d_gram);
    HIP_TRY(e, hipGetLastError());
    if (ev) HIP_TRY(e, hipEventRecord(ev[3], st));
  } else if (ev) {
    HIP_TRY(e, hipEventRecord(ev[2], st));
    HIP_TRY(e, hipEventRecord(ev[3], st));
  }
  return SYSID_OK;
}

}  // namespace

extern "C" {

int32_t sysid_abi_version(void) { return 1; }

int32_t sysid_debug_body_column_device(const double* body24, double* fw_64x6) {
  double *d_b = nullptr, *d_o = nullptr;
  HIP_TRY(nullptr, hipMalloc(&d_b, 24 * sizeof(double)));
  HIP_TRY(nullptr, hipMalloc(&d_o, 64 * 6 * sizeof(double)));
  HIP_TRY(nullptr, hipMemcpy(d_b, body24, 24 * sizeof(double), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(debug_body_column_kernel, dim3(1), dim3(64), 0, 0, d_b, d_o);
  HIP_TRY(nullptr, hipGetLastError());
  HIP_TRY(nullptr, hipMemcpy(fw_64x6, d_o, 64 * 6 * sizeof(double), hipMemcpyDeviceToHost));
  (void)hipFree(d_b);
  (void)hipFree(d_o);
  return SYSID_OK;
}

int32_t sysid_debug_lds(sysid_engine* e, const double* q, const double* dq, const double* ddq, const double* tau,
                        const double* cnt, double* lds_image, int64_t image_doubles) {
  if (!e || !lds_image) return set_err(e, SYSID_E_INVALID, "null argument");
  const K1Layout L = k1_layout(e->in_rows, e->nv, e->nb + 1, e->nc);
  if (image_doubles < L.total) return set_err(e, SYSID_E_INVALID, "image needs %d doubles", L.total);
  HIP_TRY(e, hipSetDevice(e->device));
  HIP_TRY(e, hipMalloc(&e->d_dump, (size_t)L.total * sizeof(double)));
  double* tmp[4] = {nullptr, nullptr, nullptr, nullptr};
  tmp[0] = e->d_dump;
  const uint32_t flags = SYSID_EMIT_Y | SYSID_EMIT_TAU | SYSID_EMIT_FRICTION;
  int rc = sysid_build(e, q, dq, ddq, tau, cnt, 1, 1, flags, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                       nullptr);
  if (rc == SYSID_OK) {
    if (hipMemcpy(lds_image, e->d_dump, (size_t)L.total * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
      rc = set_err(e, SYSID_E_DEVICE, "dump copy failed");
  }
  (void)hipFree(e->d_dump);
  e->d_dump = nullptr;
  (void)tmp;
  return rc;
}

int32_t sysid_debug_layout(const sysid_engine* e, int32_t* offsets12) {
  if (!e || !offsets12) return SYSID_E_INVALID;
  const K1Layout L = k1_layout(e->in_rows, e->nv, e->nb + 1, e->nc);
  const int o[12] = {L.in, L.body, L.W, L.Pt, L.Jw, L.pf, L.Jc, L.L, L.M, L.P, L.H, L.total};
  for (int k = 0; k < 12; ++k) offsets12[k] = o[k];
  return SYSID_OK;
}

int32_t sysid_debug_body_column(const double* body24, int32_t p, double* fw6) {
  if (!body24 || !fw6 || p < 0 || p > 9) return SYSID_E_INVALID;
  body_regressor_world_column(body24, p, fw6);
  return SYSID_OK;
}

const char* sysid_last_error(const sysid_engine* e) {
  return e ? e->err.c_str() : g_thread_error.c_str();
}

int32_t sysid_model_create(const void* packed, size_t nbytes, int32_t device, sysid_engine** out) {
  if (!out || !packed) return set_err(nullptr, SYSID_E_INVALID, "null argument");
  *out = nullptr;
  if (nbytes < 64) return set_err(nullptr, SYSID_E_MODEL, "packed model too small");
  const int32_t* h = static_cast<const int32_t*>(packed);
  if (h[0] != 0x44495953 || h[1] != 1) return set_err(nullptr, SYSID_E_MODEL, "bad packed-model magic/version");
  const int nq = h[2], nv = h[3], NJ = h[4], nc = h[5], bd = h[6], nja = h[7];
  if (NJ < 2 || NJ > NJ_MAX || nv < 1 || nv > NV_MAX || nc < 0 || nc > NC_MAX || nq < nv ||
      (bd != 0 && bd != 6) || nja != nv - bd)
    return set_err(nullptr, SYSID_E_MODEL, "unsupported model dims nq=%d nv=%d njoints=%d nc=%d (max %d/%d/%d)",
                   nq, nv, NJ, nc, NV_MAX, NJ_MAX, NC_MAX);
  const int nints = 4 * NJ + nc;
  const size_t ioff = 64, doff = ioff + (size_t)((nints + 1) & ~1) * 4;
  const size_t need = doff + (size_t)(NJ * 15 + nc * 12 + 3) * 8;
  if (nbytes < need) return set_err(nullptr, SYSID_E_MODEL, "packed model truncated (%zu < %zu)", nbytes, need);
  const int32_t* I = reinterpret_cast<const int32_t*>(static_cast<const char*>(packed) + ioff);
  std::vector<double> D((need - doff) / 8);
  std::memcpy(D.data(), static_cast<const char*>(packed) + doff, need - doff);

  sysid_engine* e = new sysid_engine();
  e->device = device;
  DevModel& m = e->hm;
  m.nq = nq; m.nv = nv; m.njoints = NJ; m.nc = nc; m.base_dof = bd; m.nj = nja;
  int qcount = 0, vcount = 0, maxdepth = 0;
  for (int j = 0; j < NJ; ++j) {
    m.parent[j] = I[j];
    m.jtype[j] = I[NJ + j];
    m.idx_q[j] = I[2 * NJ + j];
    m.idx_v[j] = I[3 * NJ + j];
    if (j == 0) { m.depth[0] = 0; continue; }
    const int jt = m.jtype[j];
    if ((jt != JT_FREEFLYER && jt != JT_REVOLUTE) || m.parent[j] < 0 || m.parent[j] >= j ||
        (jt == JT_FREEFLYER && m.parent[j] != 0) || m.idx_q[j] != qcount || m.idx_v[j] != vcount) {
      delete e;
      return set_err(nullptr, SYSID_E_MODEL, "joint %d: unsupported type/parent/index layout", j);
    }
    qcount += jt == JT_FREEFLYER ? 7 : 1;
    const int nd = jt == JT_FREEFLYER ? 6 : 1;
    for (int d = 0; d < nd; ++d) { m.dof_joint[vcount + d] = j; m.dof_k[vcount + d] = d; }
    vcount += nd;
    m.depth[j] = m.depth[m.parent[j]] + 1;
    if (m.depth[j] > maxdepth) maxdepth = m.depth[j];
  }
  if (qcount != nq || vcount != nv) {
    delete e;
    return set_err(nullptr, SYSID_E_MODEL, "joint dims do not add up (nq %d/%d, nv %d/%d)", qcount, nq, vcount, nv);
  }
  m.maxdepth = maxdepth;
  const double* ax = D.data();
  const double* R0 = ax + 3 * NJ;
  const double* t0 = R0 + 9 * NJ;
  const double* cR = t0 + 3 * NJ;
  const double* ct = cR + 9 * nc;
  const double* g = ct + 3 * nc;
  for (int j = 0; j < NJ; ++j) {
    for (int k = 0; k < 3; ++k) { m.axis[j][k] = ax[3 * j + k]; m.t0[j][k] = t0[3 * j + k]; }
    for (int k = 0; k < 9; ++k) m.R0[j][k] = R0[9 * j + k];
  }
  for (int c = 0; c < nc; ++c) {
    const int cj = I[4 * NJ + c];
    if (cj < 0 || cj >= NJ) { delete e; return set_err(nullptr, SYSID_E_MODEL, "contact %d: bad joint", c); }
    m.cjoint[c] = cj;
    unsigned long long mask = 0;
    for (int j = cj; j > 0; j = m.parent[j]) {
      const int nd = m.jtype[j] == JT_FREEFLYER ? 6 : 1;
      for (int d = 0; d < nd; ++d) mask |= 1ull << (m.idx_v[j] + d);
    }
    m.csupp[c] = mask;
    for (int k = 0; k < 9; ++k) m.cR[c][k] = cR[9 * c + k];
    for (int k = 0; k < 3; ++k) m.ct[c][k] = ct[3 * c + k];
  }
  for (int k = 0; k < 3; ++k) m.g[k] = g[k];
  m.wy = 10 * (NJ - 1);
  m.w = m.wy + 2 * nja;
  m.ncol = m.w + 1;
  m.in_rows = nq + 2 * nv + nja + nc;

  e->nq = nq; e->nv = nv; e->nj = nja; e->nb = NJ - 1; e->nc = nc;
  e->wy = m.wy; e->w = m.w; e->ncol = m.ncol; e->in_rows = m.in_rows;
  e->ldp = (m.ncol + 1) & ~1;

  // K1 shape
  e->k1_threads = m.ncol <= 128 ? 128 : (m.ncol <= 192 ? 192 : 256);
  const K1Layout L = k1_layout(m.in_rows, nv, NJ, nc);
  e->k1_lds = (size_t)L.total * sizeof(double);
  if (e->k1_lds > 160 * 1024) {
    delete e;
    return set_err(nullptr, SYSID_E_MODEL, "model needs %zu B of LDS per sample (max 160 KiB)", e->k1_lds);
  }

  // Gram tiling: upper-triangular tiles of 16 columns, groups of 4 waves x K2_TPW tiles
  e->ntc = (m.ncol + 15) / 16;
  std::vector<int2> tl;
  for (int I0 = 0; I0 < e->ntc; ++I0)
    for (int J0 = I0; J0 < e->ntc; ++J0) tl.push_back(int2{I0, J0});
  e->ntiles = (int)tl.size();
  const int per_group = 4 * K2_TPW;
  e->ngroups = (e->ntiles + per_group - 1) / per_group;
  tl.resize((size_t)e->ngroups * per_group, int2{-1, -1});
  e->ntiles = (int)tl.size();  // padded slots (reduction skips the -1 ones)
  e->lds_stride = ((e->ntc * 16 + 31) / 32) * 32 + 16;
  int kc = (48 * 1024) / (e->lds_stride * 8);
  kc = (kc / 4) * 4;
  if (kc < 4) kc = 4;
  e->kc = kc;

  hipError_t st = hipSetDevice(device);
  if (st == hipSuccess) st = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
  if (st == hipSuccess) st = hipMalloc(&e->d_model, sizeof(DevModel));
  if (st == hipSuccess) st = hipMemcpy(e->d_model, &m, sizeof(DevModel), hipMemcpyHostToDevice);
  if (st == hipSuccess) st = hipMalloc(&e->d_tiles, tl.size() * sizeof(int2));
  if (st == hipSuccess) st = hipMemcpy(e->d_tiles, tl.data(), tl.size() * sizeof(int2), hipMemcpyHostToDevice);
  if (st == hipSuccess && e->k1_lds > 64 * 1024)
    st = hipFuncSetAttribute(reinterpret_cast<const void*>(regressor_panel_kernel),
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)e->k1_lds);
  if (st != hipSuccess) {
    set_err(nullptr, SYSID_E_DEVICE, "device setup failed: %s", hipGetErrorString(st));
    sysid_destroy(e);
    return SYSID_E_DEVICE;
  }
  *out = e;
  return SYSID_OK;
}

void sysid_destroy(sysid_engine* e) {
  if (!e) return;
  (void)hipSetDevice(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  if (e->d_model) (void)hipFree(e->d_model);
  if (e->d_tiles) (void)hipFree(e->d_tiles);
  if (e->d_in) (void)hipFree(e->d_in);
  if (e->d_panel) (void)hipFree(e->d_panel);
  if (e->d_gram) (void)hipFree(e->d_gram);
  if (e->d_ws) (void)hipFree(e->d_ws);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
}

int32_t sysid_dims(const sysid_engine* e, int32_t* nq, int32_t* nv, int32_t* nj, int32_t* nb, int32_t* n_contact,
                   int32_t* panel_cols, int32_t* panel_ld) {
  if (!e) return set_err(nullptr, SYSID_E_INVALID, "null engine");
  if (nq) *nq = e->nq;
  if (nv) *nv = e->nv;
  if (nj) *nj = e->nj;
  if (nb) *nb = e->nb;
  if (n_contact) *n_contact = e->nc;
  if (panel_cols) *panel_cols = e->ncol;
  if (panel_ld) *panel_ld = e->ldp;
  return SYSID_OK;
}

size_t sysid_workspace_bytes(const sysid_engine* e, int64_t N, uint32_t flags) {
  if (!e || N <= 0 || !(flags & SYSID_EMIT_GRAM)) return 0;
  return slab_bytes(e, N * e->nv);
}

int32_t sysid_check_contacts(const sysid_engine* e, const double* cnt, int64_t N, int64_t ld, int64_t* bad) {
  if (!e) return set_err(nullptr, SYSID_E_INVALID, "null engine");
  if (e->nc == 0 || N <= 0) return SYSID_OK;
  if (!cnt || ld < N) return set_err(const_cast<sysid_engine*>(e), SYSID_E_INVALID, "bad contact buffer");
  for (int64_t s = 0; s < N; ++s) {
    double sum = 0.0;
    int64_t nz = 0;
    for (int c = 0; c < e->nc; ++c) {
      const double v = cnt[(int64_t)c * ld + s];
      sum += v;
      nz += v != 0.0;
    }
    // reference: m = int(np.sum(cnt)) rows of three are allocated, one block per truthy foot
    const double tr = std::trunc(sum);
    if (!(tr >= (double)nz)) {
      if (bad) *bad = s;
      return set_err(const_cast<sysid_engine*>(e), SYSID_E_CONTACT,
                     "sample %lld: int(sum(contact)) = %g is smaller than the %lld feet in contact",
                     (long long)s, tr, (long long)nz);
    }
  }
  return SYSID_OK;
}

int32_t sysid_build_device(sysid_engine* e, const double* d_in, int64_t N, int64_t ld, uint32_t flags,
                           double* d_panel, int64_t ld_panel, double* d_gram, void* d_ws, size_t ws_bytes,
                           void* stream) {
  if (!e) return set_err(nullptr, SYSID_E_INVALID, "null engine");
  if (N < 0 || ld < N || (N > 0 && (!d_in || !d_panel)) || ld_panel < e->ncol || (ld_panel & 1))
    return set_err(e, SYSID_E_INVALID, "bad arguments (N=%lld ld=%lld ld_panel=%lld, need an even ld_panel >= %d)",
                   (long long)N, (long long)ld, (long long)ld_panel, e->ncol);
  if ((flags & SYSID_EMIT_GRAM) && !d_gram) return set_err(e, SYSID_E_INVALID, "EMIT_GRAM without gram buffer");
  if (N == 0) {
    if (flags & SYSID_EMIT_GRAM) {
      HIP_TRY(e, hipMemsetAsync(d_gram, 0, (size_t)e->ncol * e->ncol * sizeof(double),
                                stream ? (hipStream_t)stream : e->stream));
    }
    return SYSID_OK;
  }
  HIP_TRY(e, hipSetDevice(e->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : e->stream;
  return launch_stages(e, d_in, N, ld, flags, d_panel, ld_panel, d_gram, d_ws, ws_bytes, st, nullptr);
}

int32_t sysid_time_stages(sysid_engine* e, const double* d_in, int64_t N, int64_t ld, uint32_t flags,
                          double* d_panel, int64_t ld_panel, double* d_gram, void* d_ws, size_t ws_bytes,
                          int32_t iters, double* ms) {
  if (!e || !ms || iters <= 0) return set_err(e, SYSID_E_INVALID, "bad arguments");
  HIP_TRY(e, hipSetDevice(e->device));
  hipEvent_t ev[4];
  for (auto& x : ev) HIP_TRY(e, hipEventCreate(&x));
  double acc[3] = {0, 0, 0};
  int rc = SYSID_OK;
  for (int it = 0; it < iters && rc == SYSID_OK; ++it) {
    rc = launch_stages(e, d_in, N, ld, flags, d_panel, ld_panel, d_gram, d_ws, ws_bytes, e->stream, ev);
    if (rc != SYSID_OK) break;
    if (hipEventSynchronize(ev[3]) != hipSuccess) { rc = set_err(e, SYSID_E_DEVICE, "event sync failed"); break; }
    for (int k = 0; k < 3; ++k) {
      float t = 0.f;
      (void)hipEventElapsedTime(&t, ev[k], ev[k + 1]);
      acc[k] += t;
    }
  }
  for (auto& x : ev) (void)hipEventDestroy(x);
  for (int k = 0; k < 3; ++k) ms[k] = acc[k] / iters;
  return rc;
}

int32_t sysid_build(sysid_engine* e, const double* q, const double* dq, const double* ddq, const double* tau,
                    const double* cnt, int64_t N, int64_t ld, uint32_t flags, double* Y_proj, double* tau_proj,
                    double* B_v, double* B_c, double* gram, double* Atb, double* btb) {
  if (!e) return set_err(nullptr, SYSID_E_INVALID, "null engine");
  if (N < 0 || ld < N) return set_err(e, SYSID_E_INVALID, "bad N/ld (%lld/%lld)", (long long)N, (long long)ld);
  if (N > 0 && (!q || !dq || !ddq || (!tau && e->nj) || (!cnt && e->nc)))
    return set_err(e, SYSID_E_INVALID, "null input buffer");
  if (N > 0 && e->nc) {
    const int rc = sysid_check_contacts(e, cnt, N, ld, nullptr);
    if (rc != SYSID_OK) return rc;
  }
  const bool want_gram = (flags & SYSID_EMIT_GRAM) && (gram || Atb || btb);
  if (want_gram) flags |= SYSID_EMIT_GRAM; else flags &= ~SYSID_EMIT_GRAM;
  HIP_TRY(e, hipSetDevice(e->device));
  if (N == 0) {
    const size_t W = (size_t)e->w;
    if (gram) std::memset(gram, 0, W * W * sizeof(double));
    if (Atb) std::memset(Atb, 0, W * sizeof(double));
    if (btb) *btb = 0.0;
    return SYSID_OK;
  }
  const int64_t rows = N * e->nv;
  int rc;
  if ((rc = grow(e, reinterpret_cast<void**>(&e->d_in), &e->in_cap, (size_t)e->in_rows * N * sizeof(double)))) return rc;
  if ((rc = grow(e, reinterpret_cast<void**>(&e->d_panel), &e->panel_cap, (size_t)rows * e->ldp * sizeof(double)))) return rc;
  if (!e->d_gram) HIP_TRY(e, hipMalloc(&e->d_gram, (size_t)e->ncol * e->ncol * sizeof(double)));
  const size_t wsb = sysid_workspace_bytes(e, N, flags);
  if ((rc = grow(e, &e->d_ws, &e->ws_cap, wsb ? wsb : 256))) return rc;
  hipStream_t st = e->stream;
  const size_t rowb = (size_t)N * sizeof(double);
  const double* srcs[5] = {q, dq, ddq, tau, cnt};
  const int nrows[5] = {e->nq, e->nv, e->nv, e->nj, e->nc};
  int64_t r0 = 0;
  for (int k = 0; k < 5; ++k) {
    if (nrows[k] > 0)
      HIP_TRY(e, hipMemcpy2DAsync(e->d_in + r0 * N, rowb, srcs[k], (size_t)ld * sizeof(double), rowb, nrows[k],
                                  hipMemcpyHostToDevice, st));
    r0 += nrows[k];
  }
  rc = launch_stages(e, e->d_in, N, N, flags, e->d_panel, e->ldp, e->d_gram, e->d_ws, e->ws_cap, st, nullptr);
  if (rc != SYSID_OK) return rc;
  const size_t pitch = (size_t)e->ldp * sizeof(double);
  if (Y_proj && (flags & SYSID_EMIT_Y))
    HIP_TRY(e, hipMemcpy2DAsync(Y_proj, (size_t)e->wy * sizeof(double), e->d_panel, pitch,
                                (size_t)e->wy * sizeof(double), rows, hipMemcpyDeviceToHost, st));
  if (tau_proj && (flags & SYSID_EMIT_TAU))
    HIP_TRY(e, hipMemcpy2DAsync(tau_proj, sizeof(double), e->d_panel + e->w, pitch, sizeof(double), rows,
                                hipMemcpyDeviceToHost, st));
  if (flags & SYSID_EMIT_FRICTION) {
    if (B_v && e->nj)
      HIP_TRY(e, hipMemcpy2DAsync(B_v, (size_t)e->nj * sizeof(double), e->d_panel + e->wy, pitch,
                                  (size_t)e->nj * sizeof(double), rows, hipMemcpyDeviceToHost, st));
    if (B_c && e->nj)
      HIP_TRY(e, hipMemcpy2DAsync(B_c, (size_t)e->nj * sizeof(double), e->d_panel + e->wy + e->nj, pitch,
                                  (size_t)e->nj * sizeof(double), rows, hipMemcpyDeviceToHost, st));
  }
  if (want_gram) {
    const size_t W = (size_t)e->w;
    if (gram)
      HIP_TRY(e, hipMemcpy2DAsync(gram, W * sizeof(double), e->d_gram, (size_t)e->ncol * sizeof(double),
                                  W * sizeof(double), W, hipMemcpyDeviceToHost, st));
    if (Atb)
      HIP_TRY(e, hipMemcpyAsync(Atb, e->d_gram + W * e->ncol, W * sizeof(double), hipMemcpyDeviceToHost, st));
    if (btb)
      HIP_TRY(e, hipMemcpyAsync(btb, e->d_gram + W * e->ncol + W, sizeof(double), hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(e, hipStreamSynchronize(st));
  return SYSID_OK;
}

}  // extern "C"
