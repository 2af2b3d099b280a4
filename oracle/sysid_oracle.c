/*
 * sysid_oracle.c — CPU ORACLE (test infrastructure only; never linked into the product).
 *
 * Plain-C restatement of the reference hot path, used by tests/ as a second checker and by
 * bench.py's cpu_baseline leg as the timed CPU path ("kind": "port").  It keeps the reference's
 * structure:
 *   - per sample, get_proj_regressor_torque (src/sys_identification.py:401-410) and, in a second
 *     pass, get_proj_friction_regressors (:412-418), each recomputing forward kinematics (:113-117)
 *     and the projector P = I - pinv(J_c) J_c (:119-135);
 *   - pinocchio's computeJointTorqueRegressor restated as its forward pass (liMi, v, a_gf) and
 *     backward pass (bodyRegressor pushed to every ancestor through liMi force transforms);
 *   - pinv by SVD with numpy's cut-off sigma > 1e-15 * sigma_max (one-sided Jacobi on J_c^T: the
 *     orthogonalised columns are the right singular vectors of J_c, so P = I - sum u u^T);
 *   - stacking sample-major (demo/spot_identification.py:84-87) and G = A^T A, g = A^T b, b^T b.
 * Parity status as for oracle/ref_numpy.py: pinned by identities, unpinned against pinocchio.
 *
 * Model input: the packed model of include/sysid.h.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MAXJ 64
#define MAXV 64
#define MAXC 8

typedef struct {
  int nq, nv, nj_total, nc, bd, na;
  int parent[MAXJ], type[MAXJ], iq[MAXJ], iv[MAXJ], cj[MAXC];
  double axis[MAXJ][3], R0[MAXJ][9], t0[MAXJ][3], cR[MAXC][9], ct[MAXC][3], g[3];
} omodel;

typedef struct {
  double liR[MAXJ][9], lit[MAXJ][3], oR[MAXJ][9], ot[MAXJ][3], v[MAXJ][6], a[MAXJ][6];
} odata;

static int parse_model(const void* blob, size_t n, omodel* m) {
  const int32_t* h = (const int32_t*)blob;
  if (n < 64 || h[0] != 0x44495953 || h[1] != 1) return -2;
  m->nq = h[2]; m->nv = h[3]; m->nj_total = h[4]; m->nc = h[5]; m->bd = h[6]; m->na = h[7];
  const int NJ = m->nj_total, nc = m->nc;
  if (NJ > MAXJ || m->nv > MAXV || nc > MAXC) return -2;
  const int32_t* I = (const int32_t*)((const char*)blob + 64);
  const int nints = 4 * NJ + nc;
  const double* D = (const double*)((const char*)blob + 64 + ((nints + 1) & ~1) * 4);
  for (int j = 0; j < NJ; ++j) {
    m->parent[j] = I[j]; m->type[j] = I[NJ + j]; m->iq[j] = I[2 * NJ + j]; m->iv[j] = I[3 * NJ + j];
  }
  for (int c = 0; c < nc; ++c) m->cj[c] = I[4 * NJ + c];
  const double* ax = D; const double* R0 = ax + 3 * NJ; const double* t0 = R0 + 9 * NJ;
  const double* cR = t0 + 3 * NJ; const double* ct = cR + 9 * nc; const double* g = ct + 3 * nc;
  for (int j = 0; j < NJ; ++j) {
    for (int k = 0; k < 3; ++k) { m->axis[j][k] = ax[3 * j + k]; m->t0[j][k] = t0[3 * j + k]; }
    for (int k = 0; k < 9; ++k) m->R0[j][k] = R0[9 * j + k];
  }
  for (int c = 0; c < nc; ++c) {
    for (int k = 0; k < 9; ++k) m->cR[c][k] = cR[9 * c + k];
    for (int k = 0; k < 3; ++k) m->ct[c][k] = ct[3 * c + k];
  }
  for (int k = 0; k < 3; ++k) m->g[k] = g[k];
  return 0;
}

static void mm3(const double* A, const double* B, double* C) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}
static void mv3(const double* A, const double* x, double* y) {
  for (int i = 0; i < 3; ++i) y[i] = A[3 * i] * x[0] + A[3 * i + 1] * x[1] + A[3 * i + 2] * x[2];
}
static void mtv3(const double* A, const double* x, double* y) {
  for (int i = 0; i < 3; ++i) y[i] = A[i] * x[0] + A[3 + i] * x[1] + A[6 + i] * x[2];
}
static void cr3(const double* a, const double* b, double* c) {
  c[0] = a[1] * b[2] - a[2] * b[1]; c[1] = a[2] * b[0] - a[0] * b[2]; c[2] = a[0] * b[1] - a[1] * b[0];
}
static void act_inv(const double* R, const double* t, const double* m, double* o) {
  double tw[3], d[3];
  cr3(t, m + 3, tw);
  for (int k = 0; k < 3; ++k) d[k] = m[k] - tw[k];
  mtv3(R, d, o);
  mtv3(R, m + 3, o + 3);
}

/* pinocchio forward pass (computeJointTorqueRegressor) + world placements */
static void forward(const omodel* m, const double* q, const double* v, const double* a, odata* d) {
  memset(d->oR[0], 0, sizeof d->oR[0]);
  d->oR[0][0] = d->oR[0][4] = d->oR[0][8] = 1.0;
  memset(d->ot[0], 0, sizeof d->ot[0]);
  memset(d->v[0], 0, sizeof d->v[0]);
  for (int k = 0; k < 3; ++k) { d->a[0][k] = -m->g[k]; d->a[0][3 + k] = 0.0; }
  for (int j = 1; j < m->nj_total; ++j) {
    const int p = m->parent[j], iq = m->iq[j], iv = m->iv[j];
    double RJ[9], tJ[3] = {0, 0, 0}, vJ[6] = {0}, Sa[6] = {0};
    if (m->type[j] == 1) {
      const double x = q[iq + 3], y = q[iq + 4], z = q[iq + 5], w = q[iq + 6];
      const double tx = 2 * x, ty = 2 * y, tz = 2 * z, twx = tx * w, twy = ty * w, twz = tz * w;
      const double txx = tx * x, txy = ty * x, txz = tz * x, tyy = ty * y, tyz = tz * y, tzz = tz * z;
      RJ[0] = 1 - (tyy + tzz); RJ[1] = txy - twz; RJ[2] = txz + twy;
      RJ[3] = txy + twz; RJ[4] = 1 - (txx + tzz); RJ[5] = tyz - twx;
      RJ[6] = txz - twy; RJ[7] = tyz + twx; RJ[8] = 1 - (txx + tyy);
      for (int k = 0; k < 3; ++k) tJ[k] = q[iq + k];
      for (int k = 0; k < 6; ++k) { vJ[k] = v[iv + k]; Sa[k] = a[iv + k]; }
    } else {
      const double* u = m->axis[j];
      const double s = sin(q[iq]), c = cos(q[iq]);
      if (u[0] == 1 && u[1] == 0 && u[2] == 0) {
        double R[9] = {1, 0, 0, 0, c, -s, 0, s, c}; memcpy(RJ, R, sizeof R);
      } else if (u[0] == 0 && u[1] == 1 && u[2] == 0) {
        double R[9] = {c, 0, s, 0, 1, 0, -s, 0, c}; memcpy(RJ, R, sizeof R);
      } else if (u[0] == 0 && u[1] == 0 && u[2] == 1) {
        double R[9] = {c, -s, 0, s, c, 0, 0, 0, 1}; memcpy(RJ, R, sizeof R);
      } else {
        const double C = 1 - c, x = u[0], y = u[1], z = u[2];
        double R[9] = {1 + C * (x * x - 1), -s * z + C * x * y, s * y + C * x * z,
                       s * z + C * x * y, 1 + C * (y * y - 1), -s * x + C * y * z,
                       -s * y + C * x * z, s * x + C * y * z, 1 + C * (z * z - 1)};
        memcpy(RJ, R, sizeof R);
      }
      for (int k = 0; k < 3; ++k) { vJ[3 + k] = u[k] * v[iv]; Sa[3 + k] = u[k] * a[iv]; }
    }
    double tmp[3], vp[6], ap[6];
    mm3(m->R0[j], RJ, d->liR[j]);
    mv3(m->R0[j], tJ, tmp);
    for (int k = 0; k < 3; ++k) d->lit[j][k] = tmp[k] + m->t0[j][k];
    act_inv(d->liR[j], d->lit[j], d->v[p], vp);
    act_inv(d->liR[j], d->lit[j], d->a[p], ap);
    for (int k = 0; k < 6; ++k) d->v[j][k] = vJ[k] + (p > 0 ? vp[k] : 0.0);
    double c1[3], c2[3];
    cr3(d->v[j] + 3, vJ, c1);   /* w x vJ_lin */
    {
      double c3[3];
      cr3(d->v[j], vJ + 3, c3); /* v x wJ */
      for (int k = 0; k < 3; ++k) c1[k] += c3[k];
    }
    cr3(d->v[j] + 3, vJ + 3, c2);
    for (int k = 0; k < 3; ++k) {
      d->a[j][k] = c1[k] + Sa[k] + ap[k];
      d->a[j][3 + k] = c2[k] + Sa[3 + k] + ap[3 + k];
    }
    mm3(d->oR[p], d->liR[j], d->oR[j]);
    mv3(d->oR[p], d->lit[j], tmp);
    for (int k = 0; k < 3; ++k) d->ot[j][k] = tmp[k] + d->ot[p][k];
  }
}

/* pinocchio bodyRegressor(v, a): 6x10, row-major */
static void body_regressor(const double* v, const double* a, double Y[6][10]) {
  const double *vl = v, *w = v + 3, *al = a, *dw = a + 3;
  double ac[3], t[3];
  cr3(w, vl, t);
  for (int k = 0; k < 3; ++k) ac[k] = al[k] + t[k];
  memset(Y, 0, sizeof(double) * 60);
  for (int k = 0; k < 3; ++k) Y[k][0] = ac[k];
  for (int c = 0; c < 3; ++c) {
    double e[3] = {0, 0, 0}, x1[3], x2[3], x3[3], n[3];
    e[c] = 1.0;
    cr3(dw, e, x1); cr3(w, e, x2); cr3(w, x2, x3); cr3(e, ac, n);
    for (int k = 0; k < 3; ++k) { Y[k][1 + c] = x1[k] + x3[k]; Y[3 + k][1 + c] = n[k]; }
  }
  /* I x = B(x) [xx xy yy xz yz zz] */
  const double Bsel[6][3][3] = {
      {{1, 0, 0}, {0, 0, 0}, {0, 0, 0}}, {{0, 1, 0}, {1, 0, 0}, {0, 0, 0}}, {{0, 0, 0}, {0, 1, 0}, {0, 0, 0}},
      {{0, 0, 1}, {0, 0, 0}, {1, 0, 0}}, {{0, 0, 0}, {0, 0, 1}, {0, 1, 0}}, {{0, 0, 0}, {0, 0, 0}, {0, 0, 1}}};
  for (int c = 0; c < 6; ++c) {
    double bdw[3], bw[3], x[3];
    for (int r = 0; r < 3; ++r) {
      bdw[r] = Bsel[c][r][0] * dw[0] + Bsel[c][r][1] * dw[1] + Bsel[c][r][2] * dw[2];
      bw[r] = Bsel[c][r][0] * w[0] + Bsel[c][r][1] * w[1] + Bsel[c][r][2] * w[2];
    }
    cr3(w, bw, x);
    for (int k = 0; k < 3; ++k) Y[3 + k][4 + c] = bdw[k] + x[k];
  }
}

/* pinocchio computeJointTorqueRegressor backward pass: Y (nv x 10 nb), row-major, ld = 10 nb */
static void joint_torque_regressor(const omodel* m, const odata* d, double* Y) {
  const int nv = m->nv, nb = m->nj_total - 1, ldy = 10 * nb;
  memset(Y, 0, sizeof(double) * nv * ldy);
  for (int i = nb; i >= 1; --i) {
    double B[6][10];
    body_regressor(d->v[i], d->a[i], B);
    for (int j = i; j > 0; j = m->parent[j]) {
      const int iv = m->iv[j];
      if (m->type[j] == 1) {
        for (int r = 0; r < 6; ++r)
          for (int c = 0; c < 10; ++c) Y[(iv + r) * ldy + 10 * (i - 1) + c] = B[r][c];
      } else {
        const double* u = m->axis[j];
        for (int c = 0; c < 10; ++c) Y[iv * ldy + 10 * (i - 1) + c] = u[0] * B[3][c] + u[1] * B[4][c] + u[2] * B[5][c];
      }
      if (m->parent[j] > 0) { /* force act with liMi[j]: f' = R f, n' = R n + t x f' */
        const double *R = d->liR[j], *t = d->lit[j];
        for (int c = 0; c < 10; ++c) {
          double f[3] = {B[0][c], B[1][c], B[2][c]}, n[3] = {B[3][c], B[4][c], B[5][c]}, fr[3], nr[3], tx[3];
          mv3(R, f, fr); mv3(R, n, nr); cr3(t, fr, tx);
          for (int k = 0; k < 3; ++k) { B[k][c] = fr[k]; B[3 + k][c] = nr[k] + tx[k]; }
        }
      }
    }
  }
}

/* P = I - pinv(J_c) J_c, J_c stacked for every truthy contact (LOCAL_WORLD_ALIGNED, linear rows) */
static void projector(const omodel* m, const odata* d, const double* cnt, double* P) {
  const int nv = m->nv;
  double JT[MAXV][3 * MAXC]; /* J_c^T: nv x k */
  int k = 0;
  for (int c = 0; c < m->nc; ++c) {
    if (cnt[c] == 0.0) continue;
    const int fj = m->cj[c];
    double pf[3], tmp[3];
    mv3(d->oR[fj], m->ct[c], tmp);
    for (int x = 0; x < 3; ++x) pf[x] = tmp[x] + d->ot[fj][x];
    for (int r = 0; r < nv; ++r) JT[r][k] = JT[r][k + 1] = JT[r][k + 2] = 0.0;
    for (int j = fj; j > 0; j = m->parent[j]) {
      const int iv = m->iv[j];
      if (m->type[j] == 1) {
        for (int x = 0; x < 3; ++x) {
          double Wc[3] = {d->oR[j][x], d->oR[j][3 + x], d->oR[j][6 + x]}, dd[3], cc[3];
          for (int y = 0; y < 3; ++y) { JT[iv + x][k + y] = Wc[y]; dd[y] = pf[y] - d->ot[j][y]; }
          cr3(Wc, dd, cc);
          for (int y = 0; y < 3; ++y) JT[iv + 3 + x][k + y] = cc[y];
        }
      } else {
        double Wv[3], dd[3], cc[3];
        mv3(d->oR[j], m->axis[j], Wv);
        for (int y = 0; y < 3; ++y) dd[y] = pf[y] - d->ot[j][y];
        cr3(Wv, dd, cc);
        for (int y = 0; y < 3; ++y) JT[iv][k + y] = cc[y];
      }
    }
    k += 3;
  }
  for (int a = 0; a < nv; ++a)
    for (int b = 0; b < nv; ++b) P[a * nv + b] = a == b ? 1.0 : 0.0;
  if (k == 0) return;
  /* one-sided Jacobi on the k columns of J_c^T */
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0.0;
    for (int i = 0; i < k - 1; ++i)
      for (int j = i + 1; j < k; ++j) {
        double alpha = 0, beta = 0, gamma = 0;
        for (int r = 0; r < nv; ++r) { alpha += JT[r][i] * JT[r][i]; beta += JT[r][j] * JT[r][j]; gamma += JT[r][i] * JT[r][j]; }
        if (fabs(gamma) <= 1e-300 || fabs(gamma) <= 1e-17 * sqrt(alpha * beta)) continue;
        off = fmax(off, fabs(gamma) / sqrt(alpha * beta));
        const double zeta = (beta - alpha) / (2 * gamma);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1 + zeta * zeta));
        const double c = 1 / sqrt(1 + t * t), s = c * t;
        for (int r = 0; r < nv; ++r) {
          const double x = JT[r][i], y = JT[r][j];
          JT[r][i] = c * x - s * y;
          JT[r][j] = s * x + c * y;
        }
      }
    if (off < 1e-16) break;
  }
  double sig[3 * MAXC], smax = 0;
  for (int i = 0; i < k; ++i) {
    double s2 = 0;
    for (int r = 0; r < nv; ++r) s2 += JT[r][i] * JT[r][i];
    sig[i] = sqrt(s2);
    smax = fmax(smax, sig[i]);
  }
  for (int i = 0; i < k; ++i) {
    if (!(sig[i] > 1e-15 * smax)) continue;
    for (int a = 0; a < nv; ++a)
      for (int b = 0; b < nv; ++b) P[a * nv + b] -= (JT[a][i] / sig[i]) * (JT[b][i] / sig[i]);
  }
}

typedef struct {
  omodel m;
} oracle_t;

void* oracle_create(const void* blob, size_t n) {
  oracle_t* o = (oracle_t*)calloc(1, sizeof(oracle_t));
  if (!o) return NULL;
  if (parse_model(blob, n, &o->m) != 0) { free(o); return NULL; }
  return o;
}
void oracle_destroy(void* o) { free(o); }

/* Inputs channel-major (channels x ld).  Outputs (row-major, stacked): Y (N nv x 10 nb), tau (N nv),
 * Bv, Bc (N nv x na), G (W x W), g (W), btb.  Any output may be NULL.  nthreads <= 0: all cores. */
int oracle_build(void* h, const double* q, const double* dq, const double* ddq, const double* tau,
                 const double* cnt, int64_t N, int64_t ld, double* Y, double* tp, double* Bv, double* Bc,
                 double* G, double* g, double* btb, double* ymax, int nthreads) {
  const omodel* m = &((oracle_t*)h)->m;
  const int nv = m->nv, nb = m->nj_total - 1, na = m->na, bd = m->bd, wy = 10 * nb, W = wy + 2 * na;
  if (G) memset(G, 0, sizeof(double) * W * W);
  if (g) memset(g, 0, sizeof(double) * W);
  double bb = 0.0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
#pragma omp parallel
  {
    double* Gl = G ? (double*)calloc((size_t)W * W, sizeof(double)) : NULL;
    double* gl = g ? (double*)calloc((size_t)W, sizeof(double)) : NULL;
    double bbl = 0.0;
    double* Ys = (double*)malloc(sizeof(double) * nv * wy);
    double* A = (double*)malloc(sizeof(double) * nv * (W + 1));
    odata* d = (odata*)malloc(sizeof(odata));
    double P[MAXV * MAXV];
    double qs[2 * MAXV], vs[MAXV], as[MAXV], ts[MAXV], cs[MAXC];
#pragma omp for schedule(static)
    for (int64_t s = 0; s < N; ++s) {
      for (int k = 0; k < m->nq; ++k) qs[k] = q[k * ld + s];
      for (int k = 0; k < nv; ++k) { vs[k] = dq[k * ld + s]; as[k] = ddq[k * ld + s]; }
      for (int k = 0; k < na; ++k) ts[k] = tau[k * ld + s];
      for (int k = 0; k < m->nc; ++k) cs[k] = cnt[k * ld + s];
      /* pass 1: get_proj_regressor_torque (src/sys_identification.py:401-410) */
      forward(m, qs, vs, as, d);
      joint_torque_regressor(m, d, Ys);
      if (ymax) { /* the sample's unprojected scale: the floor of the per-sample Y_proj parity metric */
        double mx = 0.0;
        for (int x = 0; x < nv * wy; ++x) mx = fabs(Ys[x]) > mx ? fabs(Ys[x]) : mx;
        ymax[s] = mx;
      }
      projector(m, d, cs, P);
      for (int r = 0; r < nv; ++r) {
        for (int c = 0; c < wy; ++c) {
          double acc = 0.0;
          for (int x = 0; x < nv; ++x) acc += P[r * nv + x] * Ys[x * wy + c];
          A[r * (W + 1) + c] = acc;
        }
        double acc = 0.0;
        for (int j = 0; j < na; ++j) acc += P[r * nv + bd + j] * ts[j];
        A[r * (W + 1) + W] = acc;
      }
      /* pass 2: get_proj_friction_regressors (:412-418) recomputes FK and P, as the reference does */
      forward(m, qs, vs, as, d);
      projector(m, d, cs, P);
      for (int r = 0; r < nv; ++r)
        for (int j = 0; j < na; ++j) {
          const double x = vs[bd + j];
          const double sg = x > 0 ? 1.0 : (x < 0 ? -1.0 : 0.0);
          A[r * (W + 1) + wy + j] = P[r * nv + bd + j] * x;
          A[r * (W + 1) + wy + na + j] = P[r * nv + bd + j] * sg;
        }
      for (int r = 0; r < nv; ++r) {
        const int64_t row = s * nv + r;
        const double* ar = A + r * (W + 1);
        if (Y) memcpy(Y + row * wy, ar, sizeof(double) * wy);
        if (Bv) memcpy(Bv + row * na, ar + wy, sizeof(double) * na);
        if (Bc) memcpy(Bc + row * na, ar + wy + na, sizeof(double) * na);
        if (tp) tp[row] = ar[W];
        if (gl)
          for (int a = 0; a < W; ++a) gl[a] += ar[a] * ar[W];
        bbl += ar[W] * ar[W];
      }
      /* the sample's nv rows into the upper triangle, Gram row by Gram row (each Gram row read once per sample,
       * not once per panel row: the thread's W x W partial stays in its cache) */
      if (Gl) {
        for (int a = 0; a < W; ++a) {
          double* Gr = Gl + (size_t)a * W;
          for (int r = 0; r < nv; ++r) {
            const double* ar = A + r * (W + 1);
            const double x = ar[a];
            if (x == 0.0) continue;
            for (int b = a; b < W; ++b) Gr[b] += x * ar[b];
          }
        }
      }
    }
#pragma omp critical
    {
      if (G)
        for (int a = 0; a < W; ++a)
          for (int b = a; b < W; ++b) G[a * W + b] += Gl[(size_t)a * W + b];
      if (g)
        for (int a = 0; a < W; ++a) g[a] += gl[a];
      bb += bbl;
    }
    free(Gl); free(gl); free(Ys); free(A); free(d);
  }
  if (G)
    for (int a = 0; a < W; ++a)
      for (int b = 0; b < a; ++b) G[a * W + b] = G[b * W + a];
  if (btb) *btb = bb;
  return 0;
}
