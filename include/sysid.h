/*
 * sysid.h — C ABI of the MI355X identification-regressor engine (libsysid.so, gfx950).
 *
 * Hot path replaced (reference @ xiaohu97/system_identification):
 *   per sample i:  Y_proj_i = P_i · Y(q_i, dq_i, ddq_i)           src/sys_identification.py:401-410
 *                  tau_proj_i = P_i · Sᵀ · tau_i                  src/sys_identification.py:409
 *                  B_v_i = P_i Sᵀ diag(dq_i[6:]), B_c_i = P_i Sᵀ diag(sign(dq_i[6:]))
 *                                                                  src/sys_identification.py:412-418
 *                  P_i = I − pinv(J_c,i) J_c,i                     src/sys_identification.py:119-135
 *   stacked over samples (row block i = rows [i·nv, (i+1)·nv))     demo/spot_identification.py:37-56, 84-87
 *   plus the normal equations the Solver objective implies        src/solver.py:186-190
 *        G = Aᵀ A, g = Aᵀ b, bᵀ b  with A = [Y_proj | B_v | B_c], b = tau_proj.
 *
 * The reference has no FFI layer; its boundary is the Python method surface.  The Python package
 * system_identification_amd (ctypes, engine.py) binds exactly these entry points.
 *
 * Conventions
 *   - Inputs are float64, channel-major ("SoA", the reference's .dat layout: one channel per row,
 *     one sample per column, demo/spot_identification.py:10-14) with leading dimension ld >= N.
 *   - Contact values: a foot is in contact when its value is non-zero (CONTACT_LOST = 2 counts, as in
 *     the reference's truthiness test, src/sys_identification.py:125).  Host entry points reject a
 *     sample whose int(sum(cnt)) is smaller than its number of non-zero feet (the reference raises a
 *     numpy broadcast error there) with SYSID_E_CONTACT.
 *   - Return codes: 0 = OK, < 0 = error; nothing is thrown across the ABI.  sysid_last_error() gives
 *     a message.  Python maps E_INVALID/E_MODEL/E_CONTACT to ValueError, E_DEVICE/E_NOMEM to RuntimeError.
 *   - A handle is bound to one device and owns one HIP stream.  The host-buffer entry points (sysid_build,
 *     sysid_build_full, sysid_tau_error) use buffers owned by the handle: they are synchronous and not
 *     re-entrant (one thread at a time per handle).  The device entry points enqueue on the stream they are
 *     given, NULL being the device's null stream (the engine's own stream is not ordered with the caller's
 *     writes of the buffers; round 3's illegal access and round 4's NaN panel were launches left on it while
 *     PyTorch freed or refilled the buffers on the default stream).  They keep every piece of per-launch
 *     state in the caller's workspace (K1's sample counters, one per XCD shard of the samples, are its first
 *     1 KiB, zeroed by a kernel on the launch stream before each launch; no hipMemsetAsync, whose graph node a
 *     replay did not order after the stream's earlier writes): launches of one handle on different streams
 *     with different workspaces may run concurrently, and an aborted launch leaves nothing behind.
 *   - Every argument check of an entry point happens before its first enqueue: an error return means that
 *     nothing was enqueued (also under graph capture).
 *
 * Packed model (produced by system_identification_amd.model.Model.pack()), little endian:
 *   int32  header[16] = {0x44495953 'SYID', version 1, nq, nv, njoints, n_contact, base_dof, nj, 0...}
 *   int32  parent[njoints], jtype[njoints] (0 universe, 1 free-flyer, 2 revolute),
 *          idx_q[njoints], idx_v[njoints], contact_joint[n_contact], (one int32 pad if the count is odd)
 *   double axis[njoints][3], placement_R[njoints][9] (row-major), placement_t[njoints][3],
 *          contact_R[n_contact][9], contact_t[n_contact][3], gravity[3]
 *
 * Device panel layout (one row per generalized coordinate of every sample, row-major, ld >= W+1):
 *   columns [0, Wy)            Y_proj        (Wy = 10·nb, pinocchio body order)
 *           [Wy, Wy+nj)        B_v
 *           [Wy+nj, W)         B_c            (W = Wy + 2·nj)
 *           W                  tau_proj
 *   The Gram buffer is the full symmetric (W+1)x(W+1) matrix panelᵀ·panel (row-major):
 *   G[:W,:W] = AᵀA, G[:W,W] = Aᵀb, G[W,W] = bᵀb.
 */
#ifndef SYSID_H
#define SYSID_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SYSID_OK           0
#define SYSID_E_INVALID   -1
#define SYSID_E_MODEL     -2
#define SYSID_E_DEVICE    -3
#define SYSID_E_NOMEM     -4
#define SYSID_E_CONTACT   -5

#define SYSID_EMIT_Y        1u  /* stacked Y_proj                   */
#define SYSID_EMIT_TAU      2u  /* stacked tau_proj                 */
#define SYSID_EMIT_FRICTION 4u  /* stacked B_v and B_c              */
#define SYSID_EMIT_GRAM     8u  /* G = panelᵀ panel (AᵀA, Aᵀb, bᵀb) */
#define SYSID_EMIT_ALL     15u
/* Gram arithmetic (default fp64, the parity path).  Reduced precision for the Gram-only throughput config
 * (its error is reported, not gated): the panel is rounded to f32 / bf16 as it is
 * staged into the MFMA tiles, accumulated in f32 per workgroup and in f64 across workgroups. */
#define SYSID_GRAM_F32     16u
#define SYSID_GRAM_BF16    32u
/* Rows of the Gram-only paths.  NULLSPACE: every sample contributes Zᵀ·A, the nv - rank(J_c) rows of its
 * system in an orthonormal basis Z of null(J_c) (ZᵀZ = P, so Σ (ZᵀA)ᵀ(ZᵀA) = Σ (PA)ᵀ(PA): the same Gram from
 * fewer rows; north_star's "batched QR/nullspace"; models with at most 4 contact frames).  PROJECTOR: the
 * reference's own P·A rows, nv per sample.  Neither flag: nullspace rows for the f64 / f32 Grams of models
 * whose K1 is not the Q-form (Spot: step -7%, 10.4 of 18 rows), projector rows otherwise (G1: the Q-form K1
 * costs far less than the basis saves) and for bf16, whose Gram is too cheap to repay the per-sample basis
 * (measured in DESIGN.md). */
#define SYSID_GRAM_PROJECTOR 64u
#define SYSID_GRAM_NULLSPACE 128u

typedef struct sysid_engine sysid_engine;

/* ABI version (bumped on any signature or layout change). */
int32_t sysid_abi_version(void);  /* 8 */

/* Create an engine for one device from a packed model.  Replaces the model construction of
 * SystemIdentification.__init__ (src/sys_identification.py:11-73; pin.buildModelFromUrdf at :16). */
int32_t sysid_model_create(const void* packed_model, size_t nbytes, int32_t device, sysid_engine** out);
void sysid_destroy(sysid_engine* e);

/* Last error message of an engine, or of the calling thread when e == NULL. Never NULL. */
const char* sysid_last_error(const sysid_engine* e);

/* Model dimensions. panel_cols = W+1; panel_ld = default row stride of the device panel. */
int32_t sysid_dims(const sysid_engine* e, int32_t* nq, int32_t* nv, int32_t* nj, int32_t* nb,
                   int32_t* n_contact, int32_t* panel_cols, int32_t* panel_ld);

/* Host-buffer entry point: the batched get_projected_y_tau + get_projected_friction_regressors
 * (demo/spot_identification.py:37-56) followed by the stacking at :84-87 and the Gram.
 *   q (nq x ld), dq/ddq (nv x ld), tau (nj x ld), cnt (n_contact x ld): float64, channel-major.
 *   Y_proj (N·nv x 10·nb), tau_proj (N·nv), B_v/B_c (N·nv x nj): row-major, caller-allocated;
 *   gram (W x W), Atb (W), btb (1).  Any output may be NULL ("don't emit"); flags select work.
 * Synchronous: returns after all outputs are in host memory.  With SYSID_EMIT_GRAM and no stacked output
 * requested the panel is never materialised in full (the Gram-only path of sysid_build_gram_device). */
int32_t sysid_build(sysid_engine* e, const double* q, const double* dq, const double* ddq,
                    const double* tau, const double* cnt, int64_t N, int64_t ld, uint32_t flags,
                    double* Y_proj, double* tau_proj, double* B_v, double* B_c,
                    double* gram, double* Atb, double* btb);

/* sysid_build with q and cnt in float32, the dtypes read_data returns them in (demo/spot_identification.py:10-14:
 * np.loadtxt(..., dtype=np.float32); the Butterworth filter at :20-25 makes dq, ddq and tau float64).  Same outputs
 * and behaviour; the inputs cross PCIe as q float32 and one byte per contact value (the non-zero test is all the
 * projector reads: `if contact_scedule[index]`, src/sys_identification.py:125), 464 instead of 568 bytes per Spot
 * sample, and are widened exactly on the device.  Replaces the same reference interface as sysid_build. */
int32_t sysid_build_f32qc(sysid_engine* e, const float* q, const double* dq, const double* ddq,
                          const double* tau, const float* cnt, int64_t N, int64_t ld, uint32_t flags,
                          double* Y_proj, double* tau_proj, double* B_v, double* B_c,
                          double* gram, double* Atb, double* btb);

/* get_full_regressor_force (src/sys_identification.py:391-399), batched: the unprojected joint-torque
 * regressor Y (N·nv x 10·nb) and F = Sᵀ tau + J_cᵀ lambda (N·nv), lambda = the measured forces
 * ee_force (3·n_contact x ld, channel-major, foot k in rows 3k..3k+2) of the feet in contact, in foot
 * order (:137-146).  A sample whose int(sum(cnt)) differs from its number of non-zero feet is rejected with
 * SYSID_E_CONTACT (the reference's J_cᵀ @ lambda has mismatched shapes there).  Y or F may be NULL. */
int32_t sysid_build_full(sysid_engine* e, const double* q, const double* dq, const double* ddq,
                         const double* tau, const double* ee_force, const double* cnt, int64_t N, int64_t ld,
                         double* Y, double* F);

/* Device workspace needed by sysid_build_device for N samples (bytes; > 0 for every N > 0): the K1 sample
 * counter, plus the Gram split-K slabs with SYSID_EMIT_GRAM.  The workspace must be 256-byte aligned. */
size_t sysid_workspace_bytes(const sysid_engine* e, int64_t N, uint32_t flags);

/* Device-buffer entry point (stream-ordered, no host synchronisation, no allocation: graph-capturable).
 *   d_in     : (nq + 2nv + nj + n_contact) x ld channel block [q; dq; ddq; tau; cnt], float64
 *   d_panel  : (N·nv) x ld_panel panel (see layout above); always written
 *   d_gram   : (W+1) x (W+1) Gram, written when flags & SYSID_EMIT_GRAM
 *   stream   : hipStream_t; NULL is the device's null stream (ordered with PyTorch's default stream), never
 *              the engine's own stream, which is not ordered with the caller's work on the buffers.
 * Inputs are not validated on the device (see sysid_check_contacts). */
int32_t sysid_build_device(sysid_engine* e, const double* d_in, int64_t N, int64_t ld, uint32_t flags,
                           double* d_panel, int64_t ld_panel, double* d_gram,
                           void* d_workspace, size_t workspace_bytes, void* stream);

/* Gram-only device entry point ("K1 fused with K2"): normal equations of N samples
 * without the N·nv-row panel.  The panel is produced in chunks (4 GiB by default) inside the workspace
 * and folded into the same Gram accumulators chunk after chunk; d_gram as in sysid_build_device.
 * flags may select a reduced-precision Gram (SYSID_GRAM_F32 / SYSID_GRAM_BF16, config 5): K1 then writes
 * the chunk panel already rounded to f32 / bf16, and the Gram kernel runs on f32 / bf16 MFMA (f32
 * accumulation per workgroup, f64 across workgroups).  The stacked-output entry points reject these flags.
 * Replaces what Solver.__init__ (src/solver.py:6-29) needs from the stacked arrays: G, g, bᵀb and
 * num_rows = N·nv (the objective scale of :190).  Stream-ordered, no allocation. */
size_t sysid_gram_workspace_bytes(const sysid_engine* e, int64_t N);
int32_t sysid_build_gram_device(sysid_engine* e, const double* d_in, int64_t N, int64_t ld, uint32_t flags,
                                double* d_gram, void* d_workspace, size_t workspace_bytes, void* stream);
/* Chunk panel size of the Gram-only path (bytes, >= 1 MiB; 0 restores the 4 GiB default): the workspace that
 * sysid_gram_workspace_bytes reports follows it.  That workspace is exactly: 1 KiB of K1 sample counters, the
 * chunk panel (min(chunk bytes, N·nv rows of the Gram's element type)), the split-K slabs (K2 workgroups x
 * Gram tile slots x 2 KiB: Spot <= 29 MB, G1 <= 141 MB) and, for the nullspace rows, 4·(nv + 1) bytes per
 * chunk sample of row counts and row list plus 4 bytes per 1024 samples of segment sums.  A workspace sized before a change
 * of these settings is checked again at launch (SYSID_E_INVALID when short, never overrun).  Fewer, larger chunks
 * are faster (each costs a K1 launch tail and a pass over the split-K slabs: 16 GiB is 2-3% faster than 4 GiB
 * on G1 1M); a smaller chunk bounds the device memory of very large N. */
int32_t sysid_set_gram_chunk_bytes(sysid_engine* e, uint64_t bytes);
/* The rows sysid_build_gram_device uses for these flags: 1 = nullspace (Zᵀ·A), 0 = projector (P·A), < 0 error. */
int32_t sysid_gram_rows(const sysid_engine* e, uint32_t flags);

/* Torque-prediction errors: print_tau_prediction_rmse
 * (src/sys_identification.py:421-437) as one reduction over the stacked panel instead of a second
 * per-sample pass.  err_sq[d] = sum over samples of (Y_proj[s·nv+d, :]·phi − tau_proj[s·nv+d])², for all nv
 * rows d (the reference reports d >= 6: total = sum(err_sq[6:]) / N, per joint sqrt(err_sq[6+j] / N)).
 * phi: 10·nb inertial parameters (pinocchio order).  Deterministic (fixed reduction order).
 * Host form: builds the panel on the device (never copied back) and returns err_sq (nv doubles).
 * Device form: d_panel as written by sysid_build_device, d_phi/d_err_sq device buffers. */
int32_t sysid_tau_error(sysid_engine* e, const double* q, const double* dq, const double* ddq,
                        const double* tau, const double* cnt, int64_t N, int64_t ld, const double* phi,
                        double* err_sq);
size_t sysid_tau_error_workspace_bytes(const sysid_engine* e, int64_t N);
int32_t sysid_tau_error_device(sysid_engine* e, const double* d_panel, int64_t ld_panel, int64_t N,
                               const double* d_phi, double* d_err_sq, void* d_workspace,
                               size_t workspace_bytes, void* stream);

/* Host-side check of the contact contract for n_contact x ld contact values (SYSID_E_CONTACT on the
 * first offending sample, whose index is written to *bad_sample when non-NULL). */
int32_t sysid_check_contacts(const sysid_engine* e, const double* cnt, int64_t N, int64_t ld,
                             int64_t* bad_sample);

/* Multi-GPU exchange: one process per GPU, samples sharded, each rank builds its
 * partial Gram, then one in-place sum all-reduce of the (W+1)x(W+1) fp64 Gram over RCCL/xGMI.
 * RCCL is loaded at run time (the copy already in the process if any).  sysid_rccl_unique_id fills a
 * 128-byte ncclUniqueId on one rank (distribute it out of band), sysid_rccl_comm_init creates the
 * communicator of `rank` on `device`, sysid_allreduce_gram enqueues the reduction on `stream` (NULL = the
 * device's null stream).  Errors: SYSID_E_DEVICE with sysid_rccl_last_error() (per thread). */
int32_t sysid_rccl_unique_id(void* id128);
int32_t sysid_rccl_comm_init(void** comm, int32_t nranks, const void* id128, int32_t rank, int32_t device);
int32_t sysid_rccl_comm_destroy(void* comm);
int32_t sysid_allreduce_gram(const sysid_engine* e, double* d_gram, void* comm, void* stream);
const char* sysid_rccl_last_error(void);
/* The packed exchange: the upper triangle of the (W+1)x(W+1) device Gram (G, Aᵀb and bᵀb,
 * row by row) plus the rank's row count, (W+1)(W+2)/2 + 1 doubles (Spot W+1 = 155: 12,091, G1 W+1 = 359: 64,621 — half the
 * bytes of sysid_allreduce_gram), summed by one RCCL all-reduce and unpacked into both triangles of d_gram
 * (bitwise symmetric).  d_xbuf: a device buffer of sysid_exchange_bytes(e) bytes, 8-byte aligned; after the
 * call its last element holds the summed row count (num_rows of the whole job).  Stream-ordered. */
size_t sysid_exchange_bytes(const sysid_engine* e);
int32_t sysid_allreduce_normal_equations(const sysid_engine* e, double* d_gram, double* d_xbuf, double rows,
                                         void* comm, void* stream);

/* Ingest: native reader of the reference's .dat logs (read_data,
 * demo/spot_identification.py:9-14): tab-delimited text, one channel per line, parsed like
 * np.loadtxt(path, delimiter='\t', dtype=np.float32) (field -> double, correctly rounded -> float32),
 * in parallel over spans of each line.  Host-only; no device needed.  Errors: SYSID_E_INVALID with
 * sysid_io_last_error() (per thread). */
int32_t sysid_dat_shape(const char* path, int64_t* rows, int64_t* cols);
int32_t sysid_dat_read(const char* path, float* out, int64_t rows, int64_t cols, int32_t nthreads);
const char* sysid_io_last_error(void);

/* Kernel-only timing helper for bench.py: runs sysid_build_device (or, with d_panel == NULL, the Gram-only
 * path of sysid_build_gram_device, workspace sized by sysid_gram_workspace_bytes) `iters` times on the
 * engine's stream bracketed by HIP events and returns the mean milliseconds per step spent in each stage:
 * ms[0] = regressor/projector kernel(s), ms[1] = Gram kernel(s), ms[2] = Gram reduction kernels.  The
 * Gram-only path sums its chunks' K1 and K2 launches. */
int32_t sysid_time_stages(sysid_engine* e, const double* d_in, int64_t N, int64_t ld, uint32_t flags,
                          double* d_panel, int64_t ld_panel, double* d_gram,
                          void* d_workspace, size_t workspace_bytes, int32_t iters, double* ms);

/* Diagnostics: the host instantiation of the kernel's body-regressor column helper.
 * body24 = {oR (9, row-major), ot (3), v (6, local [lin; ang]), a_gf (6, local)}; fw6 = column p (0..9)
 * of pinocchio's bodyRegressor(v, a_gf) moved to the world frame.  Used by the CPU test-suite. */
int32_t sysid_debug_body_column(const double* body24, int32_t p, double* fw6);
/* LDS image of K1 for one sample (inputs as in sysid_build with N = ld = 1) after the projector / H1
 * phases; sysid_debug_layout gives the offsets {in, body, W, Pt, Jw, pf, Jc, M(=X, two buffers), P, H1, tp,
 * total} (W/Pt/pf share their space with Z = X J_c). */
int32_t sysid_debug_lds(sysid_engine* e, const double* q, const double* dq, const double* ddq,
                        const double* tau, const double* cnt, double* lds_image, int64_t image_doubles);
int32_t sysid_debug_layout(const sysid_engine* e, int32_t* offsets12);
/* K1 launch shape chosen at model creation: {waves per workgroup, workgroups per CU, LDS bytes, chain tpl}. */
int32_t sysid_debug_k1_config(const sysid_engine* e, int32_t* cfg4);
/* K2 Gram deal chosen at model creation: {tile columns, tile slots of the f64, f32 and bf16 deals}. */
int32_t sysid_debug_k2_config(const sysid_engine* e, int32_t* cfg4);
/* Tests: the host entry points stage their inputs in `chunks` equal chunks (1..64; 0 restores the default: a first
 * chunk of ~30% of N, then the rest) — exercises the multi-chunk staging pipeline. */
int32_t sysid_debug_set_stage_chunks(sysid_engine* e, int32_t chunks);

/* Same helper run on the device: lane l (0..63) computes column l % 10 into fw_64x6[l*6 .. l*6+5]. */
int32_t sysid_debug_body_column_device(const double* body24, double* fw_64x6);

#ifdef __cplusplus
}
#endif

#endif /* SYSID_H */
