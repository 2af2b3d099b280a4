// sysid_engine.hip — MI355X (gfx950) identification-regressor engine: host side + C ABI (include/sysid.h).
//
// Hot path: per sample, the inverse-dynamics regressor Y(q, dq, ddq) (pinocchio
// computeJointTorqueRegressor, called at src/sys_identification.py:406), the contact-nullspace projector
// P = I - pinv(J_c) J_c (:119-135), the projected regressor / torque / friction regressors (:401-418),
// stacked sample-major (demo/spot_identification.py:37-56, 84-87), and the Gram of the stacked system
// that the Solver's objective implies (src/solver.py:186-190).  Device code: sysid_kernels.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "sysid.h"
#include "sysid_kernels.h"
#include "sysid_launch.h"

using namespace sysid_dev;

namespace {

constexpr int NJ_MAX = 64;   // joints incl. universe
constexpr int NC_MAX = 8;    // contact frames
constexpr int NV_MAX = 64;   // velocity dimension (support masks are 64-bit)
constexpr int IN_MAX = 192;  // input channels per sample (3 prefetch registers per lane)

thread_local std::string g_thread_error = "";

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Every device workspace starts with K1's sample counter (one 256-byte piece).  It is zeroed on the launch
// stream right before each K1 launch, so launches are independent of each other: an aborted launch leaves
// nothing behind, and launches on different streams with different workspaces may run concurrently.
constexpr size_t WORK_BYTES = 128 * K1_SHARDS;  // one 128-byte line per claim counter

// A persistent pool of host threads for the host entry points' input packing (Stager): started on first use, joined
// by sysid_destroy.  start(f) calls f(t) on every worker t; wait() returns when all have finished.  A worker that
// has finished a job spins for SPIN_US before it blocks on the condition variable: a call that follows within that
// window (back-to-back host calls) starts packing at once instead of paying a thread wake-up (~20-40 us, on the
// critical path of the first chunk's DMA).
class HostPool {
 public:
  explicit HostPool(int n) : n_(n) {
    for (int t = 0; t < n_; ++t) th_.emplace_back([this, t] { loop(t); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& x : th_) x.join();
  }
  int size() const { return n_; }
  // starts f on every worker and returns at once; wait() blocks until all have finished
  void start(std::function<void(int)> f) {
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = std::move(f);
      pending_ = n_;
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> g(m_);
    done_cv_.wait(g, [this] { return pending_ == 0; });
  }

 private:
  // After a job a worker polls for the next one for SPIN_US before it blocks: back-to-back host calls (~0.5 ms
  // apart) then skip the condition-variable wake-up.  The poll pauses between reads (no clock read per iteration),
  // so an idle engine costs at most ~1 ms of mostly paused core time per worker and call.
  static constexpr int SPIN_US = 1000;
  void loop(int t) {
    uint64_t seen = 0;
    for (;;) {
      std::function<void(int)> f;
      const auto spin_end = std::chrono::steady_clock::now() + std::chrono::microseconds(SPIN_US);
      for (int it = 0; gen_.load(std::memory_order_acquire) == seen && !stop_.load(std::memory_order_relaxed); ++it) {
        __builtin_ia32_pause();
        if ((it & 63) == 63 && std::chrono::steady_clock::now() >= spin_end) break;
      }
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_.load() || gen_.load() != seen; });
        if (stop_) return;
        seen = gen_.load();
        f = job_;
      }
      f(t);
      {
        std::lock_guard<std::mutex> g(m_);
        if (--pending_ == 0) done_cv_.notify_all();
      }
    }
  }
  int n_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  std::function<void(int)> job_;
  int pending_ = 0;
  std::atomic<uint64_t> gen_{0};
  std::atomic<bool> stop_{false};
};

}  // namespace

struct sysid_engine {
  int device = 0;
  size_t gram_chunk = (size_t)4 << 30;  // Gram-only chunk panel bytes (sysid_set_gram_chunk_bytes)
  int cus = 256;
  hipStream_t stream = nullptr;
  int nq = 0, nv = 0, nj = 0, nb = 0, nc = 0, wy = 0, w = 0, ncol = 0, ldp = 0, in_rows = 0, in_lds = 0;
  // K1
  K1Params kp{};
  uint32_t* d_mimg = nullptr;
  unsigned long long* d_work = nullptr;  // K1 sample counter of the host-API paths (engine-owned buffers)
  // a K1 launch shape: the instantiation (variant), its workgroup (waves), resident workgroups per CU, dynamic
  // LDS, per-sample LDS doubles and layout switches (pov: P overlay, qf: Q-form without a P slot)
  struct K1Shape {
    int variant = 0, waves = 4, bpc = 1, wave_dbl = 0, pov = 0, qf = 0;
    size_t lds = 0;
  };
  K1Shape k1m[3];  // projector rows, per panel element type (0 f64 / every stacked output, 1 f32, 2 bf16)
  K1Shape k1c[3];  // the Gram-only nullspace mode (CMP instantiations of the plain layout), per element type
  K1Shape k1f;     // the full-force mode (sysid_build_full): k1m[0], or K1_C4 where k1m[0] is the quadruped kernel
  int k1_maxch_tpl = 4;
  // K2/K3 Gram tiling
  int ntc = 0;
  // super-tile deal per Gram arithmetic (0 f64, 1 f32, 2 bf16): each kernel's waves x slots per wave
  struct Deal {
    int ngroups = 0, nsuper = 0, nslots = 0;
    int blk = 0;  // the register-blocked kernel (k2_gram_syrk_blk / _bf16_blk): one workgroup per CU
    int2* d_tiles = nullptr;  // [super slots | tile slots]
  } k2d[3];
  // host-API buffers (grow-only)
  double* d_in = nullptr;
  size_t in_cap = 0;
  double* d_panel = nullptr;
  size_t panel_cap = 0;
  double* d_gram = nullptr;
  void* d_ws = nullptr;
  size_t ws_cap = 0;
  double* d_out = nullptr;   // host API: de-interleaved stacked outputs (grow-only)
  size_t out_cap = 0;
  int host_register = -1;    // host API copies: 1 page-lock the caller's arrays, 0 pageable, -1 by size
  int stage_chunks = 0;      // host API staging: k > 0 forces k equal staged chunks (sysid_debug_set_stage_chunks)
  double* d_dump = nullptr;  // diagnostics only
  double* h_stage = nullptr;  // host API: page-locked staging of the inputs' wire blocks (grow-only)
  size_t h_stage_cap = 0;
  unsigned char* d_wire = nullptr;  // host API: the wire blocks on the device (K0W widens them into d_in)
  size_t wire_cap = 0;
  double* h_gram = nullptr;   // host API: page-locked copy of the (W+1)^2 Gram, one DMA back (grow-only)
  HostPool* pool = nullptr;   // host API: packing threads (stage_inputs), started on first use
  hipStream_t copy_stream = nullptr;     // host API: the staged input chunks' DMA (created on first use)
  std::vector<hipEvent_t> stage_ev;      // host API: one event per staged chunk (grow-only)
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

// The engine's device for the duration of one entry point, the caller's current device restored on return: a C-ABI
// call must not change the calling thread's device (PyTorch reads it for its own allocations).
struct DevScope {
  int prev = -1;
  hipError_t st = hipSuccess;
  explicit DevScope(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != d) st = hipSetDevice(d);
  }
  ~DevScope() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
  DevScope(const DevScope&) = delete;
  DevScope& operator=(const DevScope&) = delete;
};

#define HIP_TRY(e, expr)                                                                       \
  do {                                                                                         \
    hipError_t _st = (expr);                                                                   \
    if (_st != hipSuccess)                                                                     \
      return set_err((e), SYSID_E_DEVICE, "%s failed: %s", #expr, hipGetErrorString(_st));     \
  } while (0)

// K2 split-K: one workgroup per CU and super-tile group; wide Grams (>= 16 tile columns, small row
// chunks) run two workgroups per CU (measured: G1 K2 -11%, Spot unchanged net of the larger K3).
int ksplit_for(const sysid_engine* e, int64_t rows, int prec = 0) {
  // the bf16 kernel's large chunks take most of a CU's LDS: one workgroup per CU
  const int mult = e->ntc >= 16 && prec != 2 && !e->k2d[prec].blk ? 2 : 1;
  int ks = std::max(1, mult * e->cus / std::max(1, e->k2d[prec].ngroups));
  const int64_t cap = std::max<int64_t>(1, rows / 64);  // >= 16 k-steps per workgroup
  return (int)std::min<int64_t>(ks, cap);
}

size_t slab_bytes(const sysid_engine* e, int64_t rows, int prec = 0) {
  return align256((size_t)ksplit_for(e, rows, prec) * e->k2d[prec].nslots * 256 * sizeof(double));
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

// K1 variants and their instantiations: sysid_launch.h / sysid_k1_inst.hip.
using sysid_launch::K1_C4_NV18;
using sysid_launch::K1_C4;
using sysid_launch::K1_C12;
using sysid_launch::K1_C16;
using sysid_launch::K1_C12P;
using sysid_launch::K1_C16P;
using sysid_launch::K1_C4Q;
using sysid_launch::K1_C12Q;
using sysid_launch::K1_C16Q;
constexpr int SYSID_K1_SPW_QUAD = sysid_launch::SPW_QUAD, SYSID_K1_SPW_GEN = sysid_launch::SPW_GEN;
constexpr int SYSID_K1_QCH = sysid_launch::QCH;
int k1_qf_variant(int variant) {
  return variant == K1_C4 ? K1_C4Q : variant == K1_C12 ? K1_C12Q : variant == K1_C16 ? K1_C16Q : -1;
}
bool k1_is_qf(int variant) { return variant == K1_C4Q || variant == K1_C12Q || variant == K1_C16Q; }
int k1_pov_variant(int variant) { return variant == K1_C12 ? K1_C12P : variant == K1_C16 ? K1_C16P : -1; }
bool k1_is_pov(int variant) { return variant == K1_C12P || variant == K1_C16P; }
// a 12-slot instantiation for chains of 5..12 revolute joints (G1: 10; -2.8% against 16 slots)
int k1_chain_slots(int maxch) { return maxch <= 4 ? 4 : maxch <= 12 ? 12 : 16; }

// maxch: the longest revolute chain.  The nv = 18 kernel unrolls SYSID_K1_QCH chain slots.
int k1_variant(int maxch, int nv, int nbody, int in_lds, int nc) {
  // the nv = 18 kernel stages two panel rows of all bodies (lane = body x row group: 11..16 bodies), prefetches at
  // most K1_QUAD_IN_MAX input channels (its registers are sized for them) and keeps J_c's rows in lane pairs (3 nc
  // rows in 32 lanes: at most 5 contact frames)
  if (maxch <= SYSID_K1_QCH && nv == 18 && nbody >= 11 && nbody <= 16 && in_lds <= K1_QUAD_IN_MAX && 6 * nc <= 32)
    return K1_C4_NV18;
  return maxch <= 4 ? K1_C4 : k1_chain_slots(maxch) == 12 ? K1_C12 : K1_C16;
}

int k1_spw(int variant) { return variant == K1_C4_NV18 ? SYSID_K1_SPW_QUAD : SYSID_K1_SPW_GEN; }

// wave_layout's `hw`: lanes per sample of the compile-time-nv kernel (P over Z), 0 for the others.
int k1_layout_hw(int variant) { return variant == K1_C4_NV18 ? 64 / k1_spw(variant) : 0; }

// The kernel of a variant for a panel element type (prec: 0 f64, 1 f32, 2 bf16), for occupancy queries.
const void* k1_fn(int variant, int prec = 0) {
  return prec == 0 ? sysid_launch::k1_fn<0, 0>(variant)
         : prec == 1 ? sysid_launch::k1_fn<1, 0>(variant)
                     : sysid_launch::k1_fn<2, 0>(variant);
}
// The nullspace-mode instantiation of a variant (OutT of the Gram arithmetic).
const void* k1_fn_cmp(int variant, int prec) {
  return prec == 0 ? sysid_launch::k1_fn<0, 1>(variant)
         : prec == 1 ? sysid_launch::k1_fn<1, 1>(variant)
                     : sysid_launch::k1_fn<2, 1>(variant);
}

// Panel element of each Gram arithmetic: 0 = f64 (parity; every stacked output), 1 = f32, 2 = bf16 (the
// Gram-only chunk panel of a reduced-precision Gram, rounded once by K1).
size_t prec_bytes(int prec) { return prec == 0 ? 8 : prec == 1 ? 4 : 2; }

// Gram arithmetic selected by the flags: 0 = f64 (parity), 1 = f32 MFMA, 2 = bf16 MFMA (error reported).
int gram_prec(uint32_t flags) { return (flags & SYSID_GRAM_BF16) ? 2 : (flags & SYSID_GRAM_F32) ? 1 : 0; }

// zero `bytes` (a multiple of 8) on `st` with a kernel (see k0_zero_u64: graph-safe, unlike hipMemsetAsync)
hipError_t zero_async(void* p, size_t bytes, hipStream_t st) {
  const int64_t n = (int64_t)(bytes / sizeof(unsigned long long));
  const unsigned g = (unsigned)std::min<int64_t>(1024, std::max<int64_t>(1, (n + 255) / 256));
  hipLaunchKernelGGL(k0_zero_u64, dim3(g), dim3(256), 0, st, static_cast<unsigned long long*>(p), n);
  return hipGetLastError();
}

// cmp: the Gram-only nullspace mode (rcount: its per-sample row counts).
int launch_k1(sysid_engine* e, const double* d_in, int64_t N, int64_t ld, void* d_panel, int64_t ld_panel,
              unsigned long long* work, hipStream_t st, double* dbg, int full = 0, int prec = 0, int cmp = 0,
              int* rcount = nullptr, bool zeroed = false) {
  K1Params kp = e->kp;
  // the claim counters start at 0 (zeroed = true: the host path's K0W of this chunk has just zeroed them)
  if (!zeroed) HIP_TRY(e, zero_async(work, WORK_BYTES, st));
  if (full) {
    kp.full = 1;
    kp.in_rows = e->in_lds;
  }
  const sysid_engine::K1Shape& K = cmp ? e->k1c[prec] : full ? e->k1f : e->k1m[prec];
  const int variant = K.variant, waves = K.waves, bpc = K.bpc;
  const size_t lds = K.lds;
  kp.pov = K.pov;
  kp.wave_dbl = K.wave_dbl;
  const int spw = k1_spw(variant);
  kp.rg = k1_row_groups(kp.NJ, 64 / spw);
  kp.out_cols = (int)std::min<int64_t>(ld_panel, prec == 0 ? e->ldp : ld_panel);
  const int64_t waves_needed = (N + spw - 1) / spw;
  const int64_t cap = (int64_t)e->cus * bpc;
  const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(cap, (waves_needed + waves - 1) / waves));
  const dim3 g1((unsigned)grid), b1(64 * waves);
  // the instantiation unit of (panel type, row mode)
  using K1L = void (*)(int, dim3, dim3, size_t, hipStream_t, const K1Params&, const uint32_t*, const double*, int64_t,
                       int64_t, void*, int64_t, unsigned long long*, double*, int*);
  static constexpr K1L k1l[6] = {sysid_launch::k1_launch<0, 0>, sysid_launch::k1_launch<0, 1>,
                                 sysid_launch::k1_launch<1, 0>, sysid_launch::k1_launch<1, 1>,
                                 sysid_launch::k1_launch<2, 0>, sysid_launch::k1_launch<2, 1>};
  k1l[prec * 2 + (cmp ? 1 : 0)](variant, g1, b1, lds, st, kp, e->d_mimg, d_in, N, ld, d_panel, ld_panel, work, dbg,
                                rcount);
  HIP_TRY(e, hipGetLastError());
  return SYSID_OK;
}

// rowlist / d_rows: the nullspace mode's gathered rows (k1s_row_list; `rows` is then only the bound the split
// was sized for): the LDS-DMA / blocked kernels for every width and arithmetic (sysid_k2_inst.hip).
int launch_k2(sysid_engine* e, const void* d_panel, int64_t rows, int64_t ld_panel, int ks, int accumulate,
              double* slab, hipStream_t st, int prec, const int* rowlist = nullptr, const int* d_rows = nullptr) {
  if (ld_panel > 16 * e->ntc)
    return set_err(e, SYSID_E_INVALID, "Gram path needs ld_panel <= %d (16-column tiles)", 16 * e->ntc);
  const sysid_engine::Deal& D = e->k2d[prec];
  const sysid_launch::K2Args a{e->ntc, D.d_tiles, D.ngroups, D.nslots, D.blk, d_panel, rows, ld_panel, ks,
                               accumulate, slab, st, rowlist, d_rows};
  // the instantiation unit of (Gram arithmetic, width class)
  static constexpr bool (*k2l[6])(const sysid_launch::K2Args&) = {
      sysid_launch::k2_launch<0, 0>, sysid_launch::k2_launch<0, 1>, sysid_launch::k2_launch<1, 0>,
      sysid_launch::k2_launch<1, 1>, sysid_launch::k2_launch<2, 0>, sysid_launch::k2_launch<2, 1>};
  const bool ok = k2l[prec * 2 + (e->ntc >= 16 ? 1 : 0)](a);
  if (!ok) return set_err(e, SYSID_E_MODEL, "Gram width %d columns is not supported (max 384)", e->ncol);
  HIP_TRY(e, hipGetLastError());
  return SYSID_OK;
}

int launch_k3(sysid_engine* e, int ks, const double* slab, double* d_gram, hipStream_t st, int prec = 0) {
  const sysid_engine::Deal& D = e->k2d[prec];  // the slabs follow the K2 kernel's own deal
  const int64_t nx = (int64_t)D.nslots * 256;
  const int2* tiles = D.d_tiles + D.nsuper;
  hipLaunchKernelGGL(k3_gram_reduce, dim3((unsigned)(nx / 64)), dim3(1024), 0, st, slab, tiles, nx, ks, e->ncol,
                     d_gram);
  HIP_TRY(e, hipGetLastError());
  return SYSID_OK;
}

// Workspace of sysid_build_device: [K1 counter | K2 slabs] (the slabs with EMIT_GRAM).
size_t stages_ws_bytes(const sysid_engine* e, int64_t N, uint32_t flags) {
  if (N <= 0) return 0;
  const int64_t rows = N * e->nv;
  size_t slabs = 0;
  if (flags & SYSID_EMIT_GRAM) slabs = slab_bytes(e, rows);
  return WORK_BYTES + slabs;
}

// Every check of a launch sequence happens before its first enqueue: an error return means nothing was
// enqueued (no half-written panel behind an error, no half-recorded graph under capture).
int check_stages(sysid_engine* e, int64_t N, int64_t ld_panel, uint32_t flags, const void* d_ws, size_t ws_bytes) {
  const size_t need = stages_ws_bytes(e, N, flags);
  if (need > 0 && (d_ws == nullptr || ws_bytes < need))
    return set_err(e, SYSID_E_INVALID, "workspace too small: %zu < %zu bytes", d_ws ? ws_bytes : 0, need);
  if ((flags & SYSID_EMIT_GRAM) && ld_panel > 16 * e->ntc)
    return set_err(e, SYSID_E_INVALID, "Gram path needs ld_panel <= %d (16-column tiles)", 16 * e->ntc);
  if (gram_prec(flags) != 0)
    return set_err(e, SYSID_E_INVALID, "a reduced-precision Gram (SYSID_GRAM_F32/BF16) is a Gram-only mode "
                   "(sysid_build_gram_device, or sysid_build without stacked outputs)");
  if (reinterpret_cast<uintptr_t>(d_ws) & 255)
    return set_err(e, SYSID_E_INVALID, "workspace must be 256-byte aligned");
  return SYSID_OK;
}

int launch_stages(sysid_engine* e, const double* d_in, int64_t N, int64_t ld, uint32_t flags, double* d_panel,
                  int64_t ld_panel, double* d_gram, void* d_ws, size_t ws_bytes, hipStream_t st,
                  hipEvent_t* ev /* 4 events or null */, bool zeroed = false) {
  if (N <= 0) return SYSID_OK;
  int rc = check_stages(e, N, ld_panel, flags, d_ws, ws_bytes);
  if (rc != SYSID_OK) return rc;
  const int64_t rows = N * e->nv;
  auto* work = static_cast<unsigned long long*>(d_ws);
  if (ev) HIP_TRY(e, hipEventRecord(ev[0], st));
  if ((rc = launch_k1(e, d_in, N, ld, d_panel, ld_panel, work, st, nullptr, 0, 0, 0, nullptr, zeroed)) != SYSID_OK)
    return rc;
  if (ev) HIP_TRY(e, hipEventRecord(ev[1], st));
  if (flags & SYSID_EMIT_GRAM) {
    const int ks = ksplit_for(e, rows);
    double* slab = reinterpret_cast<double*>(static_cast<char*>(d_ws) + WORK_BYTES);
    const int prec = gram_prec(flags);
    if ((rc = launch_k2(e, d_panel, rows, ld_panel, ks, 0, slab, st, prec)) != SYSID_OK) return rc;
    if (ev) HIP_TRY(e, hipEventRecord(ev[2], st));
    if ((rc = launch_k3(e, ks, slab, d_gram, st, prec)) != SYSID_OK) return rc;
    if (ev) HIP_TRY(e, hipEventRecord(ev[3], st));
  } else if (ev) {
    HIP_TRY(e, hipEventRecord(ev[2], st));
    HIP_TRY(e, hipEventRecord(ev[3], st));
  }
  return SYSID_OK;
}

// Gram-only: the panel never leaves the device and is produced chunk by chunk into the workspace; K2
// accumulates every chunk into the same slabs, K3 reduces once.  The chunk panel is in the Gram's arithmetic
// (f64, or f32 / bf16 rounded by K1) with ld a multiple of 16 bytes' worth of elements.
// Chunk panel of 4 GiB by default (sysid_set_gram_chunk_bytes; bench.py's config-5 lines set 16 GiB, 2-3% faster
// than 4 GiB): each chunk costs a K1 launch tail of partly idle
// CUs and a K2 pass that reads and rewrites the split-K slabs (G1: 256 x 276 tiles x 2 KiB = 141 MB each way), so
// few large chunks win and the MALL does not (G1 125k step, 128 MB / 256 MB / 1 GiB / 2 GiB / 4 GiB chunks: bf16
// 6.39 / 4.45 / 3.25 / 3.05 / 2.82 ms, f32 12.1 / 10.6 / 7.62 / 7.17 / 7.00 ms; f64 1 -> 4 GiB 13.73 -> 12.98 ms;
// 4 -> 16 GiB: f64 / f32 125k -2.0 / -2.5%, G1 1M bf16 / f32 -2.5 / -3.2%; profiles/r03_q).  288 GB of HBM holds it
// easily (5.6%); callers short of memory set a smaller chunk.

int64_t gram_ld(const sysid_engine* e, int prec) {
  const int64_t m = prec == 0 ? 2 : prec == 1 ? 4 : 8;
  return (e->ncol + m - 1) / m * m;
}

int64_t gram_chunk(const sysid_engine* e, int64_t N, int prec) {
  const int64_t per = (int64_t)e->nv * gram_ld(e, prec) * (int64_t)prec_bytes(prec);
  const int64_t c = std::max<int64_t>(4096, (int64_t)e->gram_chunk / per);
  return std::max<int64_t>(1, std::min(c, N));
}

// Nullspace mode extras: after the claim counters, the live-row total (one 256-byte line) and the segment sums;
// after the slabs, the per-sample row counts and the row list.
size_t cmp_head_bytes(int64_t C) { return 256 + align256((size_t)((C + (1 << K1_SEG_LOG) - 1) >> K1_SEG_LOG) * 4); }
size_t cmp_tail_bytes(const sysid_engine* e, int64_t C) {
  return align256((size_t)C * 4) + align256((size_t)C * e->nv * 4);
}

// [K1 counters | row total, segment sums | panel chunk | K2 slabs | row counts | row list]
size_t gram_ws_bytes_prec(const sysid_engine* e, int64_t N, int prec) {
  const int64_t C = gram_chunk(e, N, prec), rows = C * e->nv;
  const size_t chunked = WORK_BYTES + cmp_head_bytes(C) + align256((size_t)rows * gram_ld(e, prec) * prec_bytes(prec)) +
                         slab_bytes(e, rows, prec) + cmp_tail_bytes(e, C);
  return chunked;
}

size_t gram_ws_bytes(const sysid_engine* e, int64_t N) {  // enough for every precision
  return std::max({gram_ws_bytes_prec(e, N, 0), gram_ws_bytes_prec(e, N, 1), gram_ws_bytes_prec(e, N, 2)});
}

// ev (optional, diagnostics): 2 events per chunk + 2 for K3, recorded around each K1 (+ row list) / K2 / K3 launch.
// Nullspace mode: K1 emits Zᵀ·A, nv - rank(J_c) rows per sample, k1s_seg_sums / k1s_row_list list them and K2
// gathers them; projector mode: the reference's P·A rows (nv per sample), contiguous.
// The Gram-only rows for these flags: 1 = nullspace (needs K1's register LU: at most K1_CMP_KMAX contact rows),
// 0 = projector.  Neither flag: nullspace rows unless the projector rows come from the Q-form K1 (G1 125k f64
// 13.80 vs 14.95 ms, f32 7.81 vs 9.58, bf16 3.33 vs 5.23: its K1 is far cheaper than the nullspace K1, and G1 keeps
// 31 of 35 rows anyway) or are bf16 (narrow Grams: the gathered rows cost the bf16 K2 more than they save).
int gram_nullspace(const sysid_engine* e, uint32_t flags) {
  const int prec = gram_prec(flags);
  const bool want_ns = (flags & SYSID_GRAM_NULLSPACE)   ? true
                       : (flags & SYSID_GRAM_PROJECTOR) ? false
                                                        : prec != 2 && !e->k1m[prec].qf;
  return want_ns && 3 * e->nc <= K1_CMP_KMAX ? 1 : 0;
}

// samples one round of K1 takes: every resident wave one step (Spot: 256 CUs x 2 workgroups x 4 waves x 2 samples)
int64_t k1_round_samples(const sysid_engine* e, int prec, int cmp) {
  const sysid_engine::K1Shape& K = cmp ? e->k1c[prec] : e->k1m[prec];
  return (int64_t)e->cus * K.bpc * K.waves * k1_spw(K.variant);
}

// staged (host entry point): the staged chunks' bounds (staged chunk k = samples [b[k], b[k+1])), and
// (*stage_upto)(n) before the K1 of a chunk ending at sample n (it orders `st` after the DMA and the K0W widening of
// the inputs [0, n), returning > 0 when it staged a chunk, whose K0W has then zeroed K1's claim counters);
// nullptr: the workspace's chunk size, inputs already on the device.
int launch_gram_chunked(sysid_engine* e, const double* d_in, int64_t N, int64_t ld, uint32_t flags, double* d_gram,
                        void* d_ws, size_t ws_bytes, hipStream_t st, std::vector<hipEvent_t>* ev = nullptr,
                        const std::vector<int64_t>* staged = nullptr,
                        const std::function<int(int64_t)>* stage_upto = nullptr) {
  if (N <= 0) return SYSID_OK;
  const int prec = gram_prec(flags);
  const int cmp = gram_nullspace(e, flags);
  if (d_ws == nullptr || ws_bytes < gram_ws_bytes_prec(e, N, prec))
    return set_err(e, SYSID_E_INVALID, "workspace too small: %zu < %zu bytes", d_ws ? ws_bytes : 0,
                   gram_ws_bytes_prec(e, N, prec));
  if (reinterpret_cast<uintptr_t>(d_ws) & 255) return set_err(e, SYSID_E_INVALID, "workspace must be 256-byte aligned");
  const int64_t C = gram_chunk(e, N, prec), rows0 = C * e->nv, ldc = gram_ld(e, prec);
  if (rows0 >= ((int64_t)1 << 31)) return set_err(e, SYSID_E_INVALID, "Gram-only chunk of %lld rows", (long long)rows0);
  auto* work = static_cast<unsigned long long*>(d_ws);
  char* head = static_cast<char*>(d_ws) + WORK_BYTES;
  int* d_rows = reinterpret_cast<int*>(head);
  int* rseg = reinterpret_cast<int*>(head + 256);
  char* panel = head + cmp_head_bytes(C);
  double* slab = reinterpret_cast<double*>(panel + align256((size_t)rows0 * ldc * prec_bytes(prec)));
  int* rcount = reinterpret_cast<int*>(reinterpret_cast<char*>(slab) + slab_bytes(e, rows0, prec));
  int* rowlist = reinterpret_cast<int*>(reinterpret_cast<char*>(rcount) + align256((size_t)C * 4));
  const int ks0 = ksplit_for(e, rows0, prec);  // slab_bytes(e, rows0, prec): the slabs fit the workspace
  int rc;
  size_t k = 0;
  auto mark = [&]() -> int {
    if (ev && k < ev->size()) HIP_TRY(e, hipEventRecord((*ev)[k++], st));
    return SYSID_OK;
  };
  size_t sc = 0;  // the staged chunk holding c0
  for (int64_t c0 = 0, n = 0; c0 < N; c0 += n) {
    n = std::min(C, N - c0);
    // staged chunk [k0, k1): a launch never straddles two of them, so each chunk's kernels wait only for its own
    // DMA (a staged chunk larger than the workspace chunk runs as several launches)
    if (staged) {
      while (sc + 2 < staged->size() && (*staged)[sc + 1] <= c0) ++sc;
      n = std::min(n, (*staged)[sc + 1] - c0);
    }
    bool zeroed = false;  // a chunk staged just now: its K0W zeroed the claim counters
    if (stage_upto) {
      if ((rc = (*stage_upto)(c0 + n)) < 0) return rc;  // this chunk's inputs
      zeroed = rc > 0;
    }
    if ((rc = mark())) return rc;
    const double* cin = d_in + c0;
    const int64_t cld = ld;
    if (cmp) {
      if ((rc = launch_k1(e, cin, n, cld, panel, ldc, work, st, nullptr, 0, prec, 1, rcount, zeroed)))
        return rc;
      const unsigned nseg = (unsigned)((n + (1 << K1_SEG_LOG) - 1) >> K1_SEG_LOG);
      const bool onepass = nseg <= (unsigned)K1S_ONEPASS_SEGS;
      if (!onepass) hipLaunchKernelGGL(k1s_seg_sums, dim3(nseg), dim3(256), 0, st, rcount, (int)n, rseg);
      hipLaunchKernelGGL(k1s_row_list, dim3(nseg), dim3(256), 0, st, rcount, onepass ? nullptr : rseg, (int)n, e->nv,
                         rowlist, d_rows);
      HIP_TRY(e, hipGetLastError());
    } else if ((rc = launch_k1(e, cin, n, cld, panel, ldc, work, st, nullptr, 0, prec, 0, nullptr, zeroed))) {
      return rc;
    }
    if ((rc = mark())) return rc;
    const int ks = std::min(ks0, ksplit_for(e, n * e->nv, prec));
    if ((rc = launch_k2(e, panel, n * e->nv, ldc, ks, c0 > 0, slab, st, prec, cmp ? rowlist : nullptr,
                        cmp ? d_rows : nullptr)) != SYSID_OK)
      return rc;
  }
  if ((rc = mark())) return rc;
  if ((rc = launch_k3(e, ks0, slab, d_gram, st, prec))) return rc;
  return mark();
}

int k4_blocks(const sysid_engine* e, int64_t N) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)e->cus * 4, N));
}

int launch_k4(sysid_engine* e, const double* d_panel, int64_t ld_panel, int64_t N, const double* d_phi,
              double* d_err_sq, void* d_ws, size_t ws_bytes, hipStream_t st) {
  const int nb = k4_blocks(e, N);
  if (d_ws == nullptr || ws_bytes < (size_t)nb * e->nv * sizeof(double))
    return set_err(e, SYSID_E_INVALID, "workspace too small for the torque-error reduction");
  if (e->wy > K4_MAXWY) return set_err(e, SYSID_E_MODEL, "regressor width %d > %d", e->wy, K4_MAXWY);
  double* part = static_cast<double*>(d_ws);
  hipLaunchKernelGGL(k4_tau_error, dim3((unsigned)nb), dim3(256), 0, st, d_panel, ld_panel, N, e->nv, e->wy, e->w,
                     d_phi, part);
  HIP_TRY(e, hipGetLastError());
  hipLaunchKernelGGL(k4_tau_error_final, dim3(1), dim3(64), 0, st, part, nb, e->nv, d_err_sq);
  HIP_TRY(e, hipGetLastError());
  return SYSID_OK;
}

// Host <-> device copies of the host entry points.  The caller's numpy arrays are pageable; a large copy
// page-locks the destination in place for its duration (hipHostRegister), so the DMA engine writes it
// directly instead of bouncing through the runtime's pinned staging buffers.  Memory that is already
// pinned is copied as is.  Returns the host ranges registered here (unregistered after the stream sync).
constexpr size_t REGISTER_MIN_BYTES = 8u << 20;

int host_copy(sysid_engine* e, void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t st,
              std::vector<void*>* registered) {
  if (bytes == 0) return SYSID_OK;
  void* host = kind == hipMemcpyDeviceToHost ? dst : const_cast<void*>(src);
  const bool want = e->host_register > 0 || (e->host_register < 0 && bytes >= REGISTER_MIN_BYTES);
  if (want) {
    const hipError_t r = hipHostRegister(host, bytes, hipHostRegisterDefault);
    if (r == hipSuccess) registered->push_back(host);
    else (void)hipGetLastError();  // already pinned, or not registrable: the plain copy below still works
  }
  HIP_TRY(e, hipMemcpyAsync(dst, src, bytes, kind, st));
  return SYSID_OK;
}

// Host entry points: the caller's channel arrays (pageable numpy memory) -> the device input block, pipelined with
// the kernels.  Host threads (the engine's pool) pack the channels into the engine's page-locked staging block
// chunk by chunk (samples [c0, c1) of every channel); stage(c) waits until chunk c is packed, sends it as one 2-D
// DMA on the engine's copy stream and makes the launch stream wait for that DMA only — so the caller enqueues chunk
// c's kernels right away and they run while chunk c + 1 is packed and copied (the Gram-only path: K1 / K2 per
// chunk; the stacked-output path stages every chunk before its single K1).  Measured on Spot 20k Gram-only: the
// pack-everything-first form took 0.19 ms of packing before the first kernel (profiles/r04_g).  The staging block
// is reused by the next call only after this call's launch-stream synchronise, which follows every DMA.
// The host entry points' copy stream, created on first use and warmed by one small DMA: the runtime sets up the
// stream's copy queue lazily on its first copy, which under a resident full-chip K1 took milliseconds
// (profiles/r04_s3).
int warm_copy_stream(sysid_engine* e, hipStream_t* sp) {
  HIP_TRY(e, hipStreamCreateWithFlags(sp, hipStreamNonBlocking));
  double* h = nullptr;
  HIP_TRY(e, hipHostMalloc(reinterpret_cast<void**>(&h), 256, hipHostMallocDefault));
  double* d = nullptr;
  hipError_t r = hipMalloc(reinterpret_cast<void**>(&d), 256);
  if (r == hipSuccess) r = hipMemcpyAsync(d, h, 256, hipMemcpyHostToDevice, *sp);
  if (r == hipSuccess) r = hipStreamSynchronize(*sp);
  if (d) (void)hipFree(d);
  (void)hipHostFree(h);
  if (r != hipSuccess) return set_err(e, SYSID_E_DEVICE, "copy stream set-up failed: %s", hipGetErrorString(r));
  return SYSID_OK;
}
int ensure_copy_stream(sysid_engine* e) {
  if (e->copy_stream) return SYSID_OK;
  return warm_copy_stream(e, &e->copy_stream);
}

// Wire format of the host entry points' inputs (K0W, sysid_kernels.h): per staged chunk of n samples, the q rows in
// the caller's element type (float32 from read_data, demo/spot_identification.py:10, or float64), the dq / ddq / tau
// rows in float64 and the contact rows as one byte each (non-zero flag); sections 16-byte aligned.  Spot with float32
// q: 464 instead of 568 bytes per sample over PCIe (19·4 + 48·8 + 4).
struct Wire {
  int64_t d, c, bytes;  // byte offsets of the float64 rows and of the contact bytes; block size
};
Wire wire_layout(int nq, int nd, int nc, int64_t n, int qsz) {
  auto a16 = [](int64_t x) { return (x + 15) & ~(int64_t)15; };
  Wire w;
  w.d = a16((int64_t)nq * n * qsz);
  w.c = w.d + a16((int64_t)nd * n * 8);
  w.bytes = w.c + a16((int64_t)nc * n);
  return w;
}

// The caller's channel rows: q (element size qsz), dq, ddq, tau (float64), contact (element size csz), channel-major
// with leading dimension ld.
struct HostInputs {
  const void* q;
  int qsz;
  const double* dq;
  const double* ddq;
  const double* tau;
  const void* cnt;
  int csz;
  int64_t ld;
};

#ifndef SYSID_FIRST_TENTHS  // the Gram-only first staged chunk, tenths of N (rounded up to half K1 rounds); -D for A/B
#define SYSID_FIRST_TENTHS 3
#endif
#ifndef SYSID_ZC_FIRST  // 1: the first staged chunk is widened straight from the staging block (no DMA); -D for A/B
#define SYSID_ZC_FIRST 1
#endif

class Stager {
 public:
  Stager(sysid_engine* e, int64_t N) : e_(e), N_(N) {}
  ~Stager() { finish(); }
  const std::vector<int64_t>& bounds() const { return b_; }  // staged chunk c = samples [b_[c], b_[c + 1])
  int chunks() const { return nch_; }
  // Host threads (the engine's pool) pack chunk after chunk of the caller's rows into the engine's page-locked
  // staging block in the wire format; stage(c) waits until chunk c is packed, sends it as ONE DMA on the engine's
  // copy stream into the device wire buffer, makes `st` wait for that DMA and widens the chunk into the row-major
  // float64 input block e->d_in (ld = N) with K0W, which also zeroes K1's claim counters (`work`).  Chunk 0 has no
  // DMA: K0W reads it from the mapped staging block over PCIe, which takes the copy engine's time (~55-65 us for
  // Spot's 6,144-sample first chunk) without the copy-engine -> compute-stream hand-off after it (~17 us);
  // Spot 20k Gram-only e2e 0.507 -> 0.488 ms (median of per-run best, profiles/r06_s16).
  int begin(const HostInputs& in, const std::vector<int64_t>* bounds = nullptr) {
    sysid_engine* e = e_;
    in_ = in;
    // chunks: the first one's pack + DMA is the pipeline's fill, the kernels' efficiency wants few (Spot 20k
    // Gram-only e2e, 1 / 2 / 4 / 8 chunks: 0.74 / 0.67 / 0.75 / 1.05 ms; profiles/r04_h)
    const int parts = e->stage_chunks > 0 ? e->stage_chunks : 2;
    const int64_t CH = std::max<int64_t>(2048, (N_ + parts - 1) / parts);
    b_.clear();
    if (bounds && e->stage_chunks == 0) {
      b_ = *bounds;
    } else {
      for (int64_t c0 = 0; c0 < N_; c0 += CH) b_.push_back(c0);
      b_.push_back(N_);
    }
    nch_ = (int)b_.size() - 1;
    nd_ = 2 * e->nv + e->nj;
    off_.assign(nch_ + 1, 0);
    for (int c = 0; c < nch_; ++c)
      off_[c + 1] = off_[c] + wire_layout(e->nq, nd_, e->nc, b_[c + 1] - b_[c], in_.qsz).bytes;
    const size_t need = (size_t)off_[nch_];
    if (need > e->h_stage_cap) {
      if (e->h_stage) (void)hipHostFree(e->h_stage);
      e->h_stage = nullptr;
      e->h_stage_cap = 0;
      HIP_TRY(e, hipHostMalloc(reinterpret_cast<void**>(&e->h_stage), need, hipHostMallocDefault));
      e->h_stage_cap = need;
    }
    if (int rc = grow(e, reinterpret_cast<void**>(&e->d_wire), &e->wire_cap, need)) return rc;
    // below 1 MiB the calling thread packs everything at once (no pool hand-off)
    inline_ = need < ((size_t)1 << 20);
    if (!inline_ && !e->pool) {
      int T = 8;  // the GPU box grants a job 16 host threads (OMP_NUM_THREADS): half of them pack
      if (const char* v = std::getenv("OMP_NUM_THREADS")) T = std::max(1, std::min(8, std::atoi(v) / 2));
      e->pool = new HostPool(T);
    }
    if (int rc = ensure_copy_stream(e)) return rc;
    while ((int)e->stage_ev.size() < nch_) {
      hipEvent_t x;
      HIP_TRY(e, hipEventCreateWithFlags(&x, hipEventDisableTiming));
      e->stage_ev.push_back(x);
    }
    done_.reset(new std::atomic<int>[nch_]);
    for (int c = 0; c < nch_; ++c) done_[c].store(0);
    const int T = inline_ ? 1 : e->pool->size(), R = e->nq + nd_ + e->nc;
    packers_ = T;
    unsigned char* hs = reinterpret_cast<unsigned char*>(e->h_stage);
    auto pack = [this, T, R, hs](int t) {
      const int nq = e_->nq, nc = e_->nc;
      const int nv = e_->nv;
      for (int c = 0; c < nch_; ++c) {
        const int64_t c0 = b_[c], n = b_[c + 1] - c0;
        const Wire w = wire_layout(nq, nd_, nc, n, in_.qsz);
        unsigned char* blk = hs + off_[c];
        for (int r = t; r < R; r += T) {
          if (r < nq) {
            const char* src = static_cast<const char*>(in_.q) + ((int64_t)r * in_.ld + c0) * in_.qsz;
            std::memcpy(blk + (int64_t)r * n * in_.qsz, src, (size_t)n * in_.qsz);
          } else if (r < nq + nd_) {
            const int k = r - nq;  // dq rows, ddq rows, tau rows
            const double* src = k < nv ? in_.dq + (int64_t)k * in_.ld
                                : k < 2 * nv ? in_.ddq + (int64_t)(k - nv) * in_.ld
                                             : in_.tau + (int64_t)(k - 2 * nv) * in_.ld;
            std::memcpy(blk + w.d + (int64_t)k * n * 8, src + c0, (size_t)n * 8);
          } else {
            const int k = r - nq - nd_;
            if (k == 0) check(c0, n);  // the packer of a chunk's first contact row checks the chunk's contacts
            unsigned char* dst = blk + w.c + (int64_t)k * n;
            if (in_.csz == 4) {
              const float* src = static_cast<const float*>(in_.cnt) + (int64_t)k * in_.ld + c0;
              for (int64_t x = 0; x < n; ++x) dst[x] = src[x] != 0.0f;  // NaN counts as non-zero, as in K1
            } else {
              const double* src = static_cast<const double*>(in_.cnt) + (int64_t)k * in_.ld + c0;
              for (int64_t x = 0; x < n; ++x) dst[x] = src[x] != 0.0;
            }
          }
        }
        done_[c].fetch_add(1, std::memory_order_release);
      }
    };
    if (inline_) {
      pack(0);
    } else {
      e->pool->start(pack);
      started_ = true;
    }
    return SYSID_OK;
  }
  // chunk c: wait until packed, DMA it, order `st` after that DMA and widen it into e->d_in (zeroing `work`)
  int stage(int c, hipStream_t st, unsigned long long* work) {
    sysid_engine* e = e_;
    while (done_[c].load(std::memory_order_acquire) < packers_) std::this_thread::yield();
    if (bad_.load(std::memory_order_acquire) >= 0) return SYSID_E_CONTACT;  // the caller reports it (contact_error)
    stamp();  // SYSID_TRACE_HOST: chunk c packed
    const int64_t c0 = b_[c], n = b_[c + 1] - c0;
    const Wire w = wire_layout(e->nq, nd_, e->nc, n, in_.qsz);
    const unsigned char* hs = reinterpret_cast<const unsigned char*>(e->h_stage) + off_[c];
    const unsigned char* src = e->d_wire + off_[c];
    void* mapped = nullptr;
    if (c == 0 && SYSID_ZC_FIRST && hipHostGetDevicePointer(&mapped, e->h_stage, 0) != hipSuccess) {
      (void)hipGetLastError();  // not mapped into this device: chunk 0 takes the DMA like the others
      mapped = nullptr;
    }
    if (mapped != nullptr) {
      // chunk 0, the pipeline's fill: K0W reads the page-locked staging block over PCIe itself, so the compute
      // stream starts on it without a copy-engine -> compute hand-off
      src = static_cast<const unsigned char*>(mapped) + off_[c];
    } else {
      hipStream_t cs = e->copy_stream;
      if (hipMemcpyAsync(e->d_wire + off_[c], hs, (size_t)w.bytes, hipMemcpyHostToDevice, cs) != hipSuccess ||
          hipEventRecord(e->stage_ev[c], cs) != hipSuccess ||
          hipStreamWaitEvent(st, e->stage_ev[c], 0) != hipSuccess)
        return set_err(e, SYSID_E_DEVICE, "input copy failed");
    }
#ifndef SYSID_K0W_ITERS  // samples per K0W lane and row (grid-stride iterations); -D for A/B
#define SYSID_K0W_ITERS 4
#endif
    const int64_t per_block = 256 * SYSID_K0W_ITERS;
    const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(65536 / per_block, (n + per_block - 1) / per_block));
    hipLaunchKernelGGL(k0_widen, dim3(gx, (unsigned)(e->nq + nd_ + e->nc)), dim3(256), 0, st, src, n, e->nq, nd_,
                       in_.qsz, w.d, w.c, e->d_in + c0, N_, work, (int)(WORK_BYTES / 8));
    HIP_TRY(e, hipGetLastError());
    stamp();  // chunk c's DMA and widening enqueued
    return SYSID_OK;
  }
  // host-clock stamps (ms since t0) of the trace, two per chunk: packed, DMA enqueued
  void trace_from(std::chrono::steady_clock::time_point t0) {
    t0_ = t0;
    trace_ = true;
  }
  const std::vector<double>& stamps() const { return stamps_; }
  bool contacts_bad() const { return bad_.load(std::memory_order_acquire) >= 0; }
  void finish() {
    if (started_) e_->pool->wait();
    started_ = false;
  }

 private:
  sysid_engine* e_;
  int64_t N_;
  int nch_ = 0, nd_ = 0, packers_ = 1;
  bool inline_ = false;
  std::atomic<int64_t> bad_{-1};  // a sample that breaks the contact contract (check), -1: none found
  // The reference's contact contract (m = int(np.sum(cnt)) blocks of three rows, one per truthy foot,
  // src/sys_identification.py:121-128) on samples [c0, c0 + n): checked while the chunk is packed, off the call's
  // critical path; stage() refuses the chunk's DMA once a violation is found.
  void check(int64_t c0, int64_t n) {
    const int nc = e_->nc;
    for (int64_t s = c0; s < c0 + n; ++s) {
      double sum = 0.0;
      int nz = 0;
      for (int k = 0; k < nc; ++k) {
        const double v = in_.csz == 4 ? (double)static_cast<const float*>(in_.cnt)[(int64_t)k * in_.ld + s]
                                      : static_cast<const double*>(in_.cnt)[(int64_t)k * in_.ld + s];
        sum += v;
        nz += v != 0.0;
      }
      if (!(std::trunc(sum) >= (double)nz)) {
        int64_t cur = bad_.load();
        while ((cur < 0 || s < cur) && !bad_.compare_exchange_weak(cur, s)) {}
        return;
      }
    }
  }
  HostInputs in_{};
  std::vector<int64_t> b_;    // staged chunk bounds (begin())
  std::vector<int64_t> off_;  // byte offset of chunk c's wire block (staging and device)
  std::unique_ptr<std::atomic<int>[]> done_;
  bool started_ = false;
  bool trace_ = false;
  std::chrono::steady_clock::time_point t0_;
  std::vector<double> stamps_;
  void stamp() {
    if (trace_)
      stamps_.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0_).count());
  }
};

int host_unregister(sysid_engine* e, std::vector<void*>& registered) {
  for (void* p : registered) (void)hipHostUnregister(p);
  registered.clear();
  (void)e;
  return SYSID_OK;
}

int launch_k5(sysid_engine* e, const double* d_panel, int64_t rows, int64_t ld_panel, double* Y, double* tau,
              double* Bv, double* Bc, hipStream_t st) {
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((rows + 3) / 4, (int64_t)e->cus * 8));
  hipLaunchKernelGGL(k5_unstack, dim3((unsigned)blocks), dim3(256), 0, st, d_panel, rows, ld_panel, e->wy, e->nj, Y,
                     tau, Bv, Bc);
  HIP_TRY(e, hipGetLastError());
  return SYSID_OK;
}

}  // namespace

extern "C" {

int32_t sysid_abi_version(void) { return 8; }

const char* sysid_last_error(const sysid_engine* e) { return e ? e->err.c_str() : g_thread_error.c_str(); }

int32_t sysid_model_create(const void* packed, size_t nbytes, int32_t device, sysid_engine** out) {
  if (!out || !packed) return set_err(nullptr, SYSID_E_INVALID, "null argument");
  *out = nullptr;
  if (nbytes < 64) return set_err(nullptr, SYSID_E_MODEL, "packed model too small");
  const int32_t* h = static_cast<const int32_t*>(packed);
  if (h[0] != 0x44495953 || h[1] != 1) return set_err(nullptr, SYSID_E_MODEL, "bad packed-model magic/version");
  const int nq = h[2], nv = h[3], NJ = h[4], nc = h[5], bd = h[6], nja = h[7];
  if (NJ < 2 || NJ > NJ_MAX || nv < 1 || nv > NV_MAX || nc < 0 || nc > NC_MAX || nq < nv || (bd != 0 && bd != 6) ||
      nja != nv - bd)
    return set_err(nullptr, SYSID_E_MODEL, "unsupported model dims nq=%d nv=%d njoints=%d nc=%d (max %d/%d/%d)", nq,
                   nv, NJ, nc, NV_MAX, NJ_MAX, NC_MAX);
  const int nints = 4 * NJ + nc;
  const size_t ioff = 64, doff = ioff + (size_t)((nints + 1) & ~1) * 4;
  const size_t need = doff + (size_t)(NJ * 15 + nc * 12 + 3) * 8;
  if (nbytes < need) return set_err(nullptr, SYSID_E_MODEL, "packed model truncated (%zu < %zu)", nbytes, need);
  const int32_t* I = reinterpret_cast<const int32_t*>(static_cast<const char*>(packed) + ioff);
  std::vector<double> D((need - doff) / 8);
  std::memcpy(D.data(), static_cast<const char*>(packed) + doff, need - doff);
  const double* ax = D.data();
  const double* R0 = ax + 3 * NJ;
  const double* t0 = R0 + 9 * NJ;
  const double* ctr = t0 + 3 * NJ + 9 * nc;  // contact_R is not needed (LWA linear rows)
  const double* g = ctr + 3 * nc;

  std::vector<int> parent(NJ), jtype(NJ), idx_q(NJ), idx_v(NJ), depth(NJ, 0), dof_joint(nv), dof_k(nv), cjoint(nc);
  int qcount = 0, vcount = 0, maxdepth = 0, nff = 0, ff0 = 0;
  for (int j = 0; j < NJ; ++j) {
    parent[j] = I[j];
    jtype[j] = I[NJ + j];
    idx_q[j] = I[2 * NJ + j];
    idx_v[j] = I[3 * NJ + j];
    if (j == 0) continue;
    const int jt = jtype[j];
    if ((jt != JT_FREEFLYER && jt != JT_REVOLUTE) || parent[j] < 0 || parent[j] >= j ||
        (jt == JT_FREEFLYER && parent[j] != 0) || idx_q[j] != qcount || idx_v[j] != vcount)
      return set_err(nullptr, SYSID_E_MODEL, "joint %d: unsupported type/parent/index layout", j);
    const int nd = jt == JT_FREEFLYER ? 6 : 1;
    if (jt == JT_FREEFLYER) { ++nff; ff0 = vcount; }
    for (int d = 0; d < nd; ++d) { dof_joint[vcount + d] = j; dof_k[vcount + d] = d; }
    qcount += jt == JT_FREEFLYER ? 7 : 1;
    vcount += nd;
    depth[j] = depth[parent[j]] + 1;
    maxdepth = std::max(maxdepth, depth[j]);
  }
  if (qcount != nq || vcount != nv)
    return set_err(nullptr, SYSID_E_MODEL, "joint dims do not add up (nq %d/%d, nv %d/%d)", qcount, nq, vcount, nv);
  if (10 * (NJ - 1) + 2 * nja + 1 > 384)
    return set_err(nullptr, SYSID_E_MODEL, "regressor too wide for the Gram kernels (W+1 = %d > 384)",
                   10 * (NJ - 1) + 2 * nja + 1);
  if (nff > 1) return set_err(nullptr, SYSID_E_MODEL, "at most one free-flyer (the root) is supported");
  if (bd == 6 && !(nff == 1 && ff0 == 0))
    return set_err(nullptr, SYSID_E_MODEL, "floating base requires the free-flyer as the first joint");
  // revolute chains (root side first) and contact supports
  std::vector<std::vector<int>> chains(NJ);
  int maxch = 1;
  for (int j = 1; j < NJ; ++j) {
    std::vector<int> c;
    for (int x = j; x > 0; x = parent[x])
      if (jtype[x] == JT_REVOLUTE) c.push_back(idx_v[x]);
    std::reverse(c.begin(), c.end());
    chains[j] = c;
    maxch = std::max<int>(maxch, (int)c.size());
  }
  if (maxch > 16) return set_err(nullptr, SYSID_E_MODEL, "kinematic chains deeper than 16 revolute joints");
  std::vector<unsigned long long> csupp(nc);
  for (int c = 0; c < nc; ++c) {
    cjoint[c] = I[4 * NJ + c];
    if (cjoint[c] < 0 || cjoint[c] >= NJ) return set_err(nullptr, SYSID_E_MODEL, "contact %d: bad joint", c);
    unsigned long long mask = 0;
    for (int j = cjoint[c]; j > 0; j = parent[j]) {
      const int nd = jtype[j] == JT_FREEFLYER ? 6 : 1;
      for (int d = 0; d < nd; ++d) mask |= 1ull << (idx_v[j] + d);
    }
    csupp[c] = mask;
  }
  const int in_rows = nq + 2 * nv + nja + nc;
  const int in_lds = in_rows + 3 * nc;  // + measured foot forces in the full-force mode
  if (in_lds > IN_MAX) return set_err(nullptr, SYSID_E_MODEL, "too many input channels (%d > %d)", in_lds, IN_MAX);

  // model image (layout sysid_dev::mimg_layout)
  const int maxch_tpl = k1_chain_slots(maxch);
  const MImg MI = mimg_layout(NJ, nv, nc, maxch_tpl);
  std::vector<uint32_t> img((size_t)MI.ndbl * 2, 0u);
  int* ii = reinterpret_cast<int*>(img.data());
  double* dd = reinterpret_cast<double*>(img.data());
  for (int j = 0; j < NJ; ++j) {
    ii[MI.parent + j] = parent[j];
    ii[MI.jtype + j] = jtype[j];
    ii[MI.idx_q + j] = idx_q[j];
    ii[MI.idx_v + j] = idx_v[j];
    ii[MI.depth + j] = depth[j];
    ii[MI.chain_len + j] = (int)chains[j].size();
    for (size_t t = 0; t < chains[j].size(); ++t) {
      ii[MI.chain + j * maxch_tpl + (int)t] = chains[j][t];
      ii[MI.anc + j * maxch_tpl + (int)t] = dof_joint[chains[j][t]];
    }
    for (int k = 0; k < 3; ++k) { dd[MI.axis + 3 * j + k] = ax[3 * j + k]; dd[MI.t0 + 3 * j + k] = t0[3 * j + k]; }
    for (int k = 0; k < 9; ++k) dd[MI.R0 + 9 * j + k] = R0[9 * j + k];
  }
  for (int r = 0; r < nv; ++r) { ii[MI.dof_joint + r] = dof_joint[r]; ii[MI.dof_k + r] = dof_k[r]; }
  for (int c = 0; c < nc; ++c) {
    ii[MI.cjoint + c] = cjoint[c];
    std::memcpy(ii + MI.csupp + 2 * c, &csupp[c], 8);
    for (int k = 0; k < 3; ++k) dd[MI.ct + 3 * c + k] = ctr[3 * c + k];
  }

  sysid_engine* e = new sysid_engine();
  e->device = device;
  e->nq = nq; e->nv = nv; e->nj = nja; e->nb = NJ - 1; e->nc = nc;
  e->wy = 10 * (NJ - 1);
  e->w = e->wy + 2 * nja;
  e->ncol = e->w + 1;
  e->ldp = (e->ncol + 1) & ~1;
  e->in_rows = in_rows;
  e->in_lds = in_lds;
  const int v0 = k1_variant(maxch, nv, NJ - 1, in_lds, nc);
  const int lhw = k1_layout_hw(v0);
  const WLay WL0 = wave_layout(in_lds, nv, NJ, nc, lhw);
  // P overlay (wave_layout `pov`): runtime-nv kernels whose H1 is read from P (an even free-flyer offset), when
  // D's working set fits under P's slot and the passes landing on it fit the kernel's register buffer
  bool pov_ok = false;
  WLay WL1 = WL0;
  if (lhw == 0 && k1_pov_variant(v0) >= 0 && nff > 0 && (ff0 & 1) == 0) {
    const int pp = (nv * nv + 1) & ~1, qsize = WL0.P - WL0.Jc;
    if (qsize <= pp) {
      WL1 = wave_layout(in_lds, nv, NJ, nc, lhw, 1);
      const int passes = (nv * nv + 63) / 64, t0 = (WL1.Jc - WL1.P) / 64;
      pov_ok = passes - t0 <= K1_POV_BUF;
    }
  }
  // Q-form (no P): runtime-nv kernels with at most K1_QF_KMAX contact rows and <= 32 friction column pairs
  const bool qf_ok = lhw == 0 && k1_qf_variant(v0) >= 0 && nc > 0 && 3 * nc <= K1_QF_KMAX && nja <= 31;
  const WLay WLQ = wave_layout(in_lds, nv, NJ, nc, 0, 0, 1);
  K1Params& kp = e->kp;
  kp.nq = nq; kp.nv = nv; kp.NJ = NJ; kp.nc = nc; kp.bd = bd; kp.nj = nja; kp.maxdepth = maxdepth;
  kp.wy = e->wy; kp.w = e->w; kp.ncol = e->ncol; kp.in_rows = in_rows; kp.maxch = maxch_tpl;
  kp.in_lds = in_lds; kp.full = 0;
  kp.has_ff = nff; kp.ff0 = ff0; kp.mimg_dbl = MI.ndbl; kp.wave_dbl = WL0.total; kp.out_cols = e->ldp;
  kp.rg = k1_row_groups(NJ, 64);  // per launch: k1_row_groups(NJ, lanes per sample)
  kp.thr_rel = 1e-14;  // rank cut of the Gram-Schmidt projector (pinv: 1e-15 sigma_max)
  kp.thr_rel2 = kp.thr_rel * kp.thr_rel;
  kp.g0 = g[0]; kp.g1 = g[1]; kp.g2 = g[2];
  e->k1_maxch_tpl = maxch_tpl;

  // Gram tiling: 16x16 tiles grouped in 2x2 super-tiles (upper triangle of the super grid);
  // K2W x K2S super slots per workgroup group; 4 tile slots per super slot.
  e->ntc = (e->ncol + 15) / 16;
  // K2W waves x K2S super slots per workgroup group -> d_tiles = [super slots | tile slots]
  auto deal = [&](int K2W, int K2S, int& ngroups, int& nsuper, int& nslots, int ntx) -> std::vector<int2> {
    const int nsg = (ntx + 1) / 2;
    std::vector<int2> sl;
    for (int I0 = 0; I0 < nsg; ++I0)
      for (int J0 = I0; J0 < nsg; ++J0) sl.push_back(int2{I0, J0});
    const int per_group = K2W * K2S;
    ngroups = ((int)sl.size() + per_group - 1) / per_group;
    {
      // MFMA balance: super-tiles carry 1-4 tiles (diagonal ones skip their lower tile, edge ones the tiles
      // past the Gram).  The waves of a workgroup share 4 SIMDs (wave w on SIMD w % 4, two waves each), so
      // super-tiles are dealt largest first to the least loaded group, then SIMD, then wave with a free slot.
      auto ntiles = [&](int2 t) {
        int n = 0;
        for (int a = 0; a < 2; ++a)
          for (int b = 0; b < 2; ++b) {
            const int I0 = 2 * t.x + a, J0 = 2 * t.y + b;
            n += (I0 <= J0 && J0 < ntx) ? 1 : 0;
          }
        return n;
      };
      std::vector<int2> order(sl);
      std::stable_sort(order.begin(), order.end(), [&](int2 a, int2 b) { return ntiles(a) > ntiles(b); });
      const int nsimd = 4, wps = K2W / nsimd;  // waves per SIMD
      std::vector<int2> dealt((size_t)ngroups * per_group, int2{-1, -1});
      std::vector<int> gload(ngroups, 0), wload((size_t)ngroups * K2W, 0),
          wfill((size_t)ngroups * K2W, 0);
      for (int2 t : order) {
        const int n = ntiles(t);
        int g = -1;
        for (int x = 0; x < ngroups; ++x) {
          int free = 0;
          for (int w = 0; w < K2W; ++w) free += K2S - wfill[x * K2W + w];
          if (free > 0 && (g < 0 || gload[x] < gload[g])) g = x;
        }
        int bw = -1;
        for (int w = 0; w < K2W; ++w) {
          if (wfill[g * K2W + w] >= K2S) continue;
          const int sm = w % nsimd;
          int sl_load = 0;
          for (int k = 0; k < wps; ++k) sl_load += wload[g * K2W + sm + nsimd * k];
          int bl = 0;
          if (bw >= 0)
            for (int k = 0; k < wps; ++k) bl += wload[g * K2W + bw % nsimd + nsimd * k];
          if (bw < 0 || sl_load < bl || (sl_load == bl && wload[g * K2W + w] < wload[g * K2W + bw])) bw = w;
        }
        dealt[(size_t)(g * K2W + bw) * K2S + wfill[g * K2W + bw]] = t;
        ++wfill[g * K2W + bw];
        wload[g * K2W + bw] += n;
        gload[g] += n;
      }
      if (ngroups == 1) {
        // One workgroup holds every super-tile: split off-diagonal super-tiles into row halves (two tiles each,
        // sharing their A fragment; the skipped half rides in sp.y >> 8, k2_tile_skip) while free slots remain
        // and the busiest SIMD gets lighter.  Spot: 15 super-tiles of 3-4 tiles, busiest SIMD 15 -> 14 tiles.
        auto simd_max = [&](const std::vector<std::pair<int2, int>>& pcs, std::vector<int2>* out) {
          std::vector<std::pair<int2, int>> v(pcs);
          std::stable_sort(v.begin(), v.end(), [](const std::pair<int2, int>& a, const std::pair<int2, int>& b) {
            return a.second > b.second;
          });
          std::vector<int> load(nsimd, 0), fill(nsimd, 0);
          std::vector<int2> d((size_t)per_group, int2{-1, -1});
          for (auto& pc : v) {
            int b = -1;
            for (int m = 0; m < nsimd; ++m)
              if (fill[m] < wps * K2S && (b < 0 || load[m] < load[b])) b = m;
            if (b < 0) return 1 << 30;
            const int slot = fill[b]++;  // SIMD b's slots: wave b + nsimd * (slot % wps), super slot slot / wps
            d[(size_t)(b + nsimd * (slot % wps)) * K2S + slot / wps] = pc.first;
            load[b] += pc.second;
          }
          if (out) out->swap(d);
          return *std::max_element(load.begin(), load.end());
        };
        std::vector<int> sload(nsimd, 0);
        for (int w = 0; w < K2W; ++w) sload[w % nsimd] += wload[w];
        int cur = *std::max_element(sload.begin(), sload.end());
        std::vector<std::pair<int2, int>> pcs;
        for (int2 t : order) pcs.push_back({t, ntiles(t)});
        for (size_t x = 0; x < pcs.size() && (int)pcs.size() < per_group; ++x) {
          const int2 t = pcs[x].first;
          if (pcs[x].second != 4 || (t.y >> 8) != 0) continue;  // whole off-diagonal super-tiles only
          std::vector<std::pair<int2, int>> trial(pcs);
          trial[x] = {int2{t.x, t.y | (0xC << 8)}, 2};             // keep tiles 0, 1 (row 2 I0)
          trial.push_back({int2{t.x, t.y | (0x3 << 8)}, 2});       // keep tiles 2, 3 (row 2 I0 + 1)
          std::vector<int2> d;
          const int m = simd_max(trial, &d);
          if (m < cur) {
            cur = m;
            pcs.swap(trial);
            dealt.swap(d);
          }
        }
      }
      sl.swap(dealt);
    }
    std::vector<int2> tl(sl.size() * 4, int2{-1, -1});
    for (size_t k = 0; k < sl.size(); ++k) {
      if (sl[k].x < 0) continue;
      const int skip = sl[k].y >> 8, sy = sl[k].y & 0xFF;
      for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) {
          const int I0 = 2 * sl[k].x + a, J0 = 2 * sy + b;
          if (I0 <= J0 && I0 < ntx && J0 < ntx && !((skip >> (2 * a + b)) & 1)) tl[4 * k + 2 * a + b] = int2{I0, J0};
        }
    }
    nslots = (int)tl.size();
    std::vector<int2> both(sl);
    both.insert(both.end(), tl.begin(), tl.end());  // d_tiles = [super slots | tile slots]
    nsuper = (int)sl.size();
    return both;
  };
  // the f64 / f32 kernels' workgroup shape for this width, and the bf16 kernel's (more slots per wave)
  std::vector<int2> dealt[3];
  for (int p = 0; p < 3; ++p) {
    sysid_engine::Deal& D = e->k2d[p];
    const int w = p == 2 ? K2_BF16_WAVES : k2_waves(e->ntc);
    const int sp = p == 0 ? k2_slots<double>(e->ntc) : p == 1 ? k2_slots<float>(e->ntc) : k2_bf16_spw(e->ntc);
    dealt[p] = deal(w, sp, D.ngroups, D.nsuper, D.nslots, e->ntc);
    if (k2b_supported(e->ntc)) {
      // the register-blocked kernels: no super-tile slots, the roles' tiles in slab order (8 roles per group;
      // f64 two groups, f32 / bf16 one)
      const int ng = p == 0 ? k2x_groups<double>() : 1;
      std::vector<int2> tl;
      for (int w8 = 0; w8 < 8 * ng; ++w8) {
        const K2BRole R = p == 0 ? k2x_role<double>(e->ntc, w8) : k2b_role(e->ntc, w8);
        for (int i = 0; i < R.nr; ++i)
          for (int j = R.diag ? i : 0; j < R.nc; ++j) tl.push_back(int2{R.ra + i, R.ca + j});
      }
      D.blk = 1;
      D.ngroups = ng;
      D.nsuper = 0;
      D.nslots = (int)tl.size();
      dealt[p].swap(tl);
    }
  }

  DevScope dev_scope(device);
  hipError_t st = dev_scope.st;
  hipDeviceProp_t prop;
  if (st == hipSuccess) st = hipGetDeviceProperties(&prop, device);
  if (st == hipSuccess) e->cus = prop.multiProcessorCount;
  if (st == hipSuccess) st = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
  if (st == hipSuccess) st = hipMalloc(&e->d_mimg, img.size() * sizeof(uint32_t));
  if (st == hipSuccess) st = hipMemcpy(e->d_mimg, img.data(), img.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  if (st == hipSuccess) st = hipMalloc(&e->d_work, WORK_BYTES);
  if (st == hipSuccess) st = hipMemset(e->d_work, 0, WORK_BYTES);
  for (int p = 0; p < 3; ++p) {
    int2*& t = e->k2d[p].d_tiles;
    if (st == hipSuccess) st = hipMalloc(&t, dealt[p].size() * sizeof(int2));
    if (st == hipSuccess) st = hipMemcpy(t, dealt[p].data(), dealt[p].size() * sizeof(int2), hipMemcpyHostToDevice);
  }
  // K1 shapes: per instantiation, the waves per workgroup that maximise resident waves per CU under the LDS
  // budget.  Layout candidates of the projector rows: the Q-form when it applies (less arithmetic, no P slot),
  // else the plain layout (kept on ties) and the P overlay.  The nullspace mode: CMP of the plain layout.
  auto shape = [&](sysid_engine::K1Shape& K, int prec, int cmp, const int* vars, const WLay* wls, const int* povs,
                   const int* qfs, int ncand) -> bool {
    int best = -1;
    for (int c = 0; c < ncand; ++c) {
      const void* fn = cmp ? k1_fn_cmp(vars[c], prec) : k1_fn(vars[c], prec);
      for (int wv : {8, 4, 2, 1}) {
        if (wv > K1_WAVES && !k1_is_pov(vars[c])) continue;  // 8-wave workgroups: the overlay instantiations only
        const size_t lds = (size_t)(MI.ndbl + wv * k1_spw(vars[c]) * wls[c].total) * sizeof(double);
        if (lds > 160 * 1024) continue;
        (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, 64 * wv, lds) != hipSuccess) nb = 0;
        if (nb * wv > best) {
          best = nb * wv;
          K.variant = vars[c];
          K.waves = wv;
          K.bpc = std::max(1, nb);
          K.lds = lds;
          K.wave_dbl = wls[c].total;
          K.pov = povs[c];
          K.qf = qfs[c];
        }
      }
    }
    if (best <= 0) return false;
    return hipFuncSetAttribute(cmp ? k1_fn_cmp(K.variant, prec) : k1_fn(K.variant, prec),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)K.lds) == hipSuccess;
  };
  if (st == hipSuccess) {
    bool ok = true;
    for (int pr = 0; pr < 3 && ok; ++pr) {
      if (qf_ok) {
        const int vq[1] = {k1_qf_variant(v0)}, z[1] = {0}, one[1] = {1};
        ok = shape(e->k1m[pr], pr, 0, vq, &WLQ, z, one, 1);
      } else {
        const int vp[2] = {v0, pov_ok ? k1_pov_variant(v0) : v0}, pv[2] = {0, 1}, z[2] = {0, 0};
        const WLay wl[2] = {WL0, WL1};
        ok = shape(e->k1m[pr], pr, 0, vp, wl, pv, z, pov_ok ? 2 : 1);
      }
      const int z1[1] = {0};
      if (ok) ok = shape(e->k1c[pr], pr, 1, &v0, &WL0, z1, z1, 1);
    }
    // the full-force mode: the quadruped kernel has none (its instantiation drops the mode's paths), so those models
    // run it on the generic 4-slot kernel with the plain layout
    e->k1f = e->k1m[0];
    if (ok && v0 == K1_C4_NV18) {
      const int vf[1] = {sysid_launch::K1_C4}, z1[1] = {0};
      const WLay WLF = wave_layout(in_lds, nv, NJ, nc, 0);
      ok = shape(e->k1f, 0, 0, vf, &WLF, z1, z1, 1);
    }
    if (!ok) {
      set_err(nullptr, SYSID_E_MODEL, "model needs too much LDS per sample (%zu B)", (size_t)WL0.total * 8);
      sysid_destroy(e);
      return SYSID_E_MODEL;
    }
  }
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
  DevScope dev_scope(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  for (void* p : {(void*)e->d_mimg, (void*)e->d_work, (void*)e->k2d[0].d_tiles, (void*)e->k2d[1].d_tiles, (void*)e->k2d[2].d_tiles, (void*)e->d_in, (void*)e->d_panel,
                  (void*)e->d_gram, e->d_ws, (void*)e->d_out, (void*)e->d_dump})
    if (p) (void)hipFree(p);
  if (e->h_stage) (void)hipHostFree(e->h_stage);
  if (e->h_gram) (void)hipHostFree(e->h_gram);
  if (e->d_wire) (void)hipFree(e->d_wire);
  delete e->pool;
  for (hipEvent_t x : e->stage_ev) (void)hipEventDestroy(x);
  if (e->copy_stream) (void)hipStreamDestroy(e->copy_stream);
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
  if (!e) return 0;
  return stages_ws_bytes(e, N, flags);
}

int32_t sysid_check_contacts(const sysid_engine* e, const double* cnt, int64_t N, int64_t ld, int64_t* bad);

int32_t sysid_build_device(sysid_engine* e, const double* d_in, int64_t N, int64_t ld, uint32_t flags,
                           double* d_panel, int64_t ld_panel, double* d_gram, void* d_ws, size_t ws_bytes,
                           void* stream) {
  if (!e) return set_err(nullptr, SYSID_E_INVALID, "null engine");
  if (N < 0 || ld < N || (N > 0 && (!d_in || !d_panel)) || ld_panel < e->ncol || (ld_panel & 1))
    return set_err(e, SYSID_E_INVALID, "bad arguments (N=%lld ld=%lld ld_panel=%lld, need an even ld_panel >= %d)",
                   (long long)N, (long long)ld, (long long)ld_panel, e->ncol);
  if ((flags & SYSID_EMIT_GRAM) && !d_gram) return set_err(e, SYSID_E_INVALID, "EMIT_GRAM without gram buffer");
  if (reinterpret_cast<uintptr_t>(d_panel) & 15)
    return set_err(e, SYSID_E_INVALID, "d_panel must be 16-byte aligned (the panel is written with 16-byte stores)");
  DevScope dev_scope(e->device);
  HIP_TRY(e, dev_scope.st);
  hipStream_t st = static_cast<hipStream_t>(stream);  // NULL: the null stream (see sysid.h)
  if (N == 0) {
    if (flags & SYSID_EMIT_GRAM)
      HIP_TRY(e, zero_async(d_gram, (size_t)e->ncol * e->ncol * sizeof(double), st));
    return SYSID_OK;
  }
  return launch_stages(e, d_in, N, ld, flags, d_panel, ld_panel, d_gram, d_ws, ws_bytes, st, nullptr);
}

size_t sysid_gram_workspace_bytes(const sysid_engine* e, int64_t N) {
  if (!e || N <= 0) return 0;
  return gram_ws_bytes(e, N);
}

int32_t sysid_build_gram_device(sysid_engine* e, const double* d_in, int64_t N, int64_t ld, uint32_t flags,
                                double* d_gram, void* d_ws, size_t ws_bytes, void* stream) {
  if (!e) return set_err(nullptr, SYSID_E_INVALID, "null engine");
  if (N < 0 || ld < N || (N > 0 && !d_in) || !d_gram)
    return set_err(e, SYSID_E_INVALID, "bad arguments (N=%lld ld=%lld)", (long long)N, (long long)ld);
  DevScope dev_scope(e->device);
  HIP_TRY(e, dev_scope.st);
  hipStream_t st = static_cast<hipStream_t>(stream);  // NULL: the null stream (see sysid.h)
  if (N == 0) {
    HIP_TRY(e, zero_async(d_gram, (size_t)e->ncol * e->ncol * sizeof(double), st));
    return SYSID_OK;
  }
  return launch_gram_chunked(e, d_in, N, ld, flags, d_gram, d_ws, ws_bytes, st);
}

size_t sysid_tau_error_workspace_bytes(const sysid_engine* e, int64_t N) {
  if (!e) return 0;
  return align256((size_t)k4_blocks(e, N) * e->nv * sizeof(double));
}

int32_t sysid_tau_error_device(sysid_engine* e, const double* d_panel, int64_t ld_panel, int64_t N,
                               const double* d_phi, double* d_err_sq, void* d_ws, size_t ws_bytes, void* stream) {
  if (!e) return set_err(nullptr, SYSID_E_INVALID, "null engine");
  if (N < 0 || ld_panel < e->ncol || (ld_panel & 1) || !d_phi || !d_err_sq || (N > 0 && !d_panel) ||
      (reinterpret_cast<uintptr_t>(d_panel) & 15))
    return set_err(e, SYSID_E_INVALID, "bad arguments");
  DevScope dev_scope(e->device);
  HIP_TRY(e, dev_scope.st);
  hipStream_t st = static_cast<hipStream_t>(stream);  // NULL: the null stream (see sysid.h)
  if (N == 0) {
    HIP_TRY(e, zero_async(d_err_sq, (size_t)e->nv * sizeof(double), st));
    return SYSID_OK;
  }
  return launch_k4(e, d_panel, ld_panel, N, d_phi, d_err_sq, d_ws, ws_bytes, st);
}

int32_t sysid_tau_error(sysid_engine* e, const double* q, const double* dq, const double* ddq, const double* tau,
                        const double* cnt, int64_t N, int64_t ld, const double* phi, double* err_sq) {
  if (!e) return set_err(nullptr, SYSID_E_INVALID, "null engine");
  if (N < 0 || ld < N || !phi || !err_sq) return set_err(e, SYSID_E_INVALID, "bad arguments");
  if (N > 0 && (!q || !dq || !ddq || (!tau && e->nj) || (!cnt && e->nc)))
    return set_err(e, SYSID_E_INVALID, "null input buffer");
  if (N == 0) {
    std::memset(err_sq, 0, (size_t)e->nv * sizeof(double));
    return SYSID_OK;
  }
  if (e->nc) {
    const int rc = sysid_check_contacts(e, cnt, N, ld, nullptr);
    if (rc != SYSID_OK) return rc;
  }
  DevScope dev_scope(e->device);
  HIP_TRY(e, dev_scope.st);
  const int64_t rows = N * e->nv;
  int rc;
  if ((rc = grow(e, reinterpret_cast<void**>(&e->d_in), &e->in_cap, (size_t)e->in_rows * N * sizeof(double)))) return rc;
  if ((rc = grow(e, reinterpret_cast<void**>(&e->d_panel), &e->panel_cap, (size_t)rows * e->ldp * sizeof(double))))
    return rc;
  const size_t wsb = sysid_tau_error_workspace_bytes(e, N) + align256((size_t)(e->wy + e->nv) * sizeof(double));
  if ((rc = grow(e, &e->d_ws, &e->ws_cap, wsb))) return rc;
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
  double* d_phi = reinterpret_cast<double*>(static_cast<char*>(e->d_ws) + sysid_tau_error_workspace_bytes(e, N));
  double* d_err = d_phi + e->wy;
  HIP_TRY(e, hipMemcpyAsync(d_phi, phi, (size_t)e->wy * sizeof(double), hipMemcpyHostToDevice, st));
  if ((rc = launch_k1(e, e->d_in, N, N, e->d_panel, e->ldp, e->d_work, st, nullptr)) != SYSID_OK) return rc;
  if ((rc = launch_k4(e, e->d_panel, e->ldp, N, d_phi, d_err, e->d_ws, sysid_tau_error_workspace_bytes(e, N), st)))
    return rc;
  HIP_TRY(e, hipMemcpyAsync(err_sq, d_err, (size_t)e->nv * sizeof(double), hipMemcpyDeviceToHost, st));
  HIP_TRY(e, hipStreamSynchronize(st));
  return SYSID_OK;
}

int32_t sysid_build_full(sysid_engine* e, const double* q, const double* dq, const double* ddq, const double* tau,
                         const double* ee_force, const double* cnt, int64_t N, int64_t ld, double* Y, double* F) {
  if (!e) return set_err(nullptr, SYSID_E_INVALID, "null engine");
  if (N < 0 || ld < N) return set_err(e, SYSID_E_INVALID, "bad N/ld (%lld/%lld)", (long long)N, (long long)ld);
  if (N > 0 && (!q || !dq || !ddq || (!tau && e->nj) || (!cnt && e->nc) || (!ee_force && e->nc)))
    return set_err(e, SYSID_E_INVALID, "null input buffer");
  if (N == 0) return SYSID_OK;
  // reference: lambda has 3*int(sum(cnt)) entries and J_c one 3-row block per truthy foot; J_c^T lambda
  // is only defined when the two agree (otherwise numpy raises a shape error there)
  for (int64_t s = 0; s < N && e->nc; ++s) {
    double sum = 0.0;
    int64_t nz = 0;
    for (int c = 0; c < e->nc; ++c) {
      const double v = cnt[(int64_t)c * ld + s];
      sum += v;
      nz += v != 0.0;
    }
    if (std::trunc(sum) != (double)nz)
      return set_err(e, SYSID_E_CONTACT, "sample %lld: int(sum(contact)) = %g != %lld feet in contact (J_c^T lambda "
                     "has mismatched shapes in the reference)", (long long)s, std::trunc(sum), (long long)nz);
  }
  DevScope dev_scope(e->device);
  HIP_TRY(e, dev_scope.st);
  const int64_t rows = N * e->nv;
  int rc;
  if ((rc = grow(e, reinterpret_cast<void**>(&e->d_in), &e->in_cap, (size_t)e->in_lds * N * sizeof(double)))) return rc;
  if ((rc = grow(e, reinterpret_cast<void**>(&e->d_panel), &e->panel_cap, (size_t)rows * e->ldp * sizeof(double))))
    return rc;
  hipStream_t st = e->stream;
  const size_t rowb = (size_t)N * sizeof(double);
  const double* srcs[6] = {q, dq, ddq, tau, cnt, ee_force};
  const int nrows[6] = {e->nq, e->nv, e->nv, e->nj, e->nc, 3 * e->nc};
  int64_t r0 = 0;
  for (int k = 0; k < 6; ++k) {
    if (nrows[k] > 0)
      HIP_TRY(e, hipMemcpy2DAsync(e->d_in + r0 * N, rowb, srcs[k], (size_t)ld * sizeof(double), rowb, nrows[k],
                                  hipMemcpyHostToDevice, st));
    r0 += nrows[k];
  }
  if ((rc = launch_k1(e, e->d_in, N, N, e->d_panel, e->ldp, e->d_work, st, nullptr, 1)) != SYSID_OK) return rc;
  // de-interleave on the device (Y block, and the torque column that holds F), one contiguous copy each
  const size_t nY = Y ? (size_t)rows * e->wy : 0, nF = F ? (size_t)rows : 0;
  if ((rc = grow(e, reinterpret_cast<void**>(&e->d_out), &e->out_cap, (nY + nF) * sizeof(double) + 64))) return rc;
  if ((rc = launch_k5(e, e->d_panel, rows, e->ldp, Y ? e->d_out : nullptr, F ? e->d_out + nY : nullptr, nullptr,
                      nullptr, st)) != SYSID_OK)
    return rc;
  std::vector<void*> reg;
  if ((Y && (rc = host_copy(e, Y, e->d_out, nY * sizeof(double), hipMemcpyDeviceToHost, st, &reg))) ||
      (F && (rc = host_copy(e, F, e->d_out + nY, nF * sizeof(double), hipMemcpyDeviceToHost, st, &reg)))) {
    (void)hipStreamSynchronize(st);
    host_unregister(e, reg);
    return rc;
  }
  const hipError_t sst = hipStreamSynchronize(st);
  host_unregister(e, reg);
  if (sst != hipSuccess) return set_err(e, SYSID_E_DEVICE, "stream sync failed: %s", hipGetErrorString(sst));
  return SYSID_OK;
}

int32_t sysid_time_stages(sysid_engine* e, const double* d_in, int64_t N, int64_t ld, uint32_t flags, double* d_panel,
                          int64_t ld_panel, double* d_gram, void* d_ws, size_t ws_bytes, int32_t iters, double* ms) {
  if (!e || !ms || iters <= 0 || N <= 0) return set_err(e, SYSID_E_INVALID, "bad arguments");
  DevScope dev_scope(e->device);
  HIP_TRY(e, dev_scope.st);
  HIP_TRY(e, hipDeviceSynchronize());  // the caller's buffers, written on any stream, are complete
  double acc[3] = {0, 0, 0};
  int rc = SYSID_OK;
  if (d_panel == nullptr) {
    // Gram-only path: per chunk K1 and K2, then K3; events around each launch
    const int prec = gram_prec(flags);
    const int64_t nchunks = (N + gram_chunk(e, N, prec) - 1) / gram_chunk(e, N, prec);
    std::vector<hipEvent_t> ev((size_t)(2 * nchunks + 2));
    for (auto& x : ev) HIP_TRY(e, hipEventCreate(&x));
    for (int it = 0; it < iters && rc == SYSID_OK; ++it) {
      rc = launch_gram_chunked(e, d_in, N, ld, flags, d_gram, d_ws, ws_bytes, e->stream, &ev);
      if (rc != SYSID_OK) break;
      if (hipEventSynchronize(ev.back()) != hipSuccess) { rc = set_err(e, SYSID_E_DEVICE, "event sync failed"); break; }
      for (int64_t c = 0; c < nchunks; ++c) {
        float t1 = 0.f, t2 = 0.f;
        (void)hipEventElapsedTime(&t1, ev[2 * c], ev[2 * c + 1]);                        // K1 of chunk c
        (void)hipEventElapsedTime(&t2, ev[2 * c + 1], ev[2 * c + 2]);                    // K2 of chunk c
        acc[0] += t1;
        acc[1] += t2;
      }
      float t3 = 0.f;
      (void)hipEventElapsedTime(&t3, ev[2 * nchunks], ev[2 * nchunks + 1]);
      acc[2] += t3;
    }
    for (auto& x : ev) (void)hipEventDestroy(x);
  } else {
    hipEvent_t ev[4];
    for (auto& x : ev) HIP_TRY(e, hipEventCreate(&x));
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
  }
  for (int k = 0; k < 3; ++k) ms[k] = acc[k] / iters;
  return rc;
}

}  // extern "C"

namespace {

// The reference's contact contract (m = int(np.sum(cnt)) blocks of three rows, one per truthy foot) on the
// caller's contact rows (float32 from read_data, or float64).
template <typename T>
int check_contacts_t(sysid_engine* e, const T* cnt, int64_t N, int64_t ld, int64_t* bad) {
  for (int64_t s = 0; s < N; ++s) {
    double sum = 0.0;
    int64_t nz = 0;
    for (int c = 0; c < e->nc; ++c) {
      const T v = cnt[(int64_t)c * ld + s];
      sum += (double)v;
      nz += v != (T)0;
    }
    const double tr = std::trunc(sum);
    if (!(tr >= (double)nz)) {
      if (bad) *bad = s;
      return set_err(e, SYSID_E_CONTACT, "sample %lld: int(sum(contact)) = %g is smaller than the %lld feet in contact",
                     (long long)s, tr, (long long)nz);
    }
  }
  return SYSID_OK;
}

// The host entry points (sysid_build, sysid_build_f32qc): the caller's rows go to the device in the wire format
// (Stager, K0W), the kernels run on the engine's stream, the outputs come back in one copy each.
int build_host(sysid_engine* e, const HostInputs& in, int64_t N, uint32_t flags, double* Y_proj, double* tau_proj,
               double* B_v, double* B_c, double* gram, double* Atb, double* btb) {
  if (!e) return set_err(nullptr, SYSID_E_INVALID, "null engine");
  if (N < 0 || in.ld < N) return set_err(e, SYSID_E_INVALID, "bad N/ld (%lld/%lld)", (long long)N, (long long)in.ld);
  if (N > 0 && (!in.q || !in.dq || !in.ddq || (!in.tau && e->nj) || (!in.cnt && e->nc)))
    return set_err(e, SYSID_E_INVALID, "null input buffer");
  // SYSID_TRACE_HOST=1: host-clock phase times of this call on stderr (diagnostics of the e2e number)
  static const bool trace = std::getenv("SYSID_TRACE_HOST") != nullptr;
  using clk = std::chrono::steady_clock;
  const clk::time_point t0 = clk::now();
  double tph[4] = {0, 0, 0, 0};
  auto ms_since = [&](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
  // the contact contract is checked by the packing threads (Stager::check), chunk by chunk; a violation makes the
  // call return SYSID_E_CONTACT (message: the first offending sample) before any output is written
  auto contact_error = [&]() -> int {
    const int r = in.csz == 4 ? check_contacts_t(e, static_cast<const float*>(in.cnt), N, in.ld, nullptr)
                              : check_contacts_t(e, static_cast<const double*>(in.cnt), N, in.ld, nullptr);
    return r != SYSID_OK ? r : set_err(e, SYSID_E_CONTACT, "contact contract violated");
  };
  const bool want_gram = (flags & SYSID_EMIT_GRAM) && (gram || Atb || btb);
  if (want_gram) flags |= SYSID_EMIT_GRAM; else flags &= ~SYSID_EMIT_GRAM;
  tph[0] = ms_since(t0);  // contact check
  DevScope dev_scope(e->device);
  HIP_TRY(e, dev_scope.st);
  if (N == 0) {
    const size_t W = (size_t)e->w;
    if (gram) std::memset(gram, 0, W * W * sizeof(double));
    if (Atb) std::memset(Atb, 0, W * sizeof(double));
    if (btb) *btb = 0.0;
    return SYSID_OK;
  }
  const int64_t rows = N * e->nv;
  // no stacked output requested: Gram-only, the panel is produced chunk by chunk on the device
  const bool panel_out = ((flags & SYSID_EMIT_Y) && Y_proj) || ((flags & SYSID_EMIT_TAU) && tau_proj) ||
                         ((flags & SYSID_EMIT_FRICTION) && (B_v || B_c) && e->nj);
  const bool gram_only = want_gram && !panel_out;
  const int gp = gram_prec(flags);
  // Gram-only staged chunks.  Two staged chunks: a short first one,
  // whose DMA lands early so the kernels start while the second chunk's DMA runs, then the rest (against three or more
  // chunks, which each add a K1 tail, a row list and a K2 pass to the kernel chain: profiles/r05_s4).  The first chunk
  // is ~30% of N in half K1 rounds (a round = every resident wave one step), at least one round: Spot 20k Gram-only
  // e2e, float32 q, 5 interleaved rounds of 12 calls: first chunk 4,096 / 5,120 / 6,144 / 7,168 samples, median
  // 0.556 / 0.530 / 0.526 / 0.532 ms, best 0.530 / 0.514 / 0.499 / 0.509 (profiles/r05_s24); with the zero-copy first
  // chunk, 4,096 / 6,144 / 8,192: median of per-run best 0.514 / 0.486 / 0.512 ms (profiles/r06_s24).  The round-5 sweeps of
  // these bounds, of more chunks and of more copy streams ran on environment knobs that round 6 removed (git history).
  std::vector<int64_t> round_bounds;
  const bool big = (size_t)e->in_rows * N * sizeof(double) >= ((size_t)1 << 20);
  if (gram_only && big) {
    const int64_t R = k1_round_samples(e, gp, gram_nullspace(e, flags));
    if (R > 0 && N >= 2 * R) {
      const int64_t half = std::max<int64_t>(1, R / 2);
      const int64_t first = std::min(std::max((SYSID_FIRST_TENTHS * N / 10 + half - 1) / half * half, R), N - R);
      round_bounds = {0, first, N};
    } else {
      round_bounds = {0, (N + 1) / 2, N};
    }
  } else {
    round_bounds = {0, N};  // one chunk (stacked outputs read every sample in one K1; small inputs)
    if (big && !gram_only) round_bounds.clear();  // stacked outputs, large: the Stager's default chunks
  }
  int rc;
  if ((rc = grow(e, reinterpret_cast<void**>(&e->d_in), &e->in_cap, (size_t)e->in_rows * N * sizeof(double))))
    return rc;
  if (!gram_only &&
      (rc = grow(e, reinterpret_cast<void**>(&e->d_panel), &e->panel_cap, (size_t)rows * e->ldp * sizeof(double))))
    return rc;
  if (!e->d_gram) HIP_TRY(e, hipMalloc(&e->d_gram, (size_t)e->ncol * e->ncol * sizeof(double)));
  const size_t wsb = gram_only ? gram_ws_bytes(e, N) : sysid_workspace_bytes(e, N, flags);
  if ((rc = grow(e, &e->d_ws, &e->ws_cap, wsb ? wsb : 256))) return rc;
  hipStream_t st = e->stream;
  auto* work = static_cast<unsigned long long*>(e->d_ws);
  std::vector<void*> reg;
  Stager stager(e, N);
  auto fail = [&](int code) {
    (void)hipStreamSynchronize(st);
    if (e->copy_stream) (void)hipStreamSynchronize(e->copy_stream);
    host_unregister(e, reg);
    stager.finish();
    return code == SYSID_E_CONTACT && stager.contacts_bad() ? contact_error() : code;
  };
  if (trace) stager.trace_from(t0);
  int nstaged = 0;  // chunks sent so far
  // > 0: staged at least one chunk (its K0W zeroed K1's claim counters); < 0: error
  const std::function<int(int64_t)> stage_upto = [&](int64_t upto) -> int {
    int k = 0;
    for (; nstaged < stager.chunks() && stager.bounds()[nstaged] < upto; ++nstaged, ++k) {
      const int r = stager.stage(nstaged, st, work);
      if (r != SYSID_OK) return r;
    }
    return k;
  };
  if ((rc = stager.begin(in, round_bounds.empty() ? nullptr : &round_bounds)) != SYSID_OK) return fail(rc);
  // the stacked-output path reads every sample in one launch: all chunks first
  bool zeroed = false;
  if (!gram_only) {
    if ((rc = stage_upto(N)) < 0) return fail(rc);
    zeroed = true;
  }
  tph[1] = ms_since(t0);  // + buffers, packing started (stacked outputs: every chunk's DMA enqueued)
  rc = gram_only ? launch_gram_chunked(e, e->d_in, N, N, flags, e->d_gram, e->d_ws, e->ws_cap, st, nullptr,
                                       &stager.bounds(), &stage_upto)
                 : launch_stages(e, e->d_in, N, N, flags, e->d_panel, e->ldp, e->d_gram, e->d_ws, e->ws_cap, st, nullptr,
                                 zeroed);
  if (rc != SYSID_OK) return fail(rc);
  const double t_kern = ms_since(t0);  // + kernels enqueued (before the output copies)
  if (panel_out) {
    // de-interleave the requested outputs on the device, then one contiguous copy per output
    const bool wY = Y_proj && (flags & SYSID_EMIT_Y), wT = tau_proj && (flags & SYSID_EMIT_TAU);
    const bool wV = B_v && (flags & SYSID_EMIT_FRICTION) && e->nj, wC = B_c && (flags & SYSID_EMIT_FRICTION) && e->nj;
    const size_t nY = wY ? (size_t)rows * e->wy : 0, nT = wT ? (size_t)rows : 0;
    const size_t nV = wV ? (size_t)rows * e->nj : 0, nC = wC ? (size_t)rows * e->nj : 0;
    if ((rc = grow(e, reinterpret_cast<void**>(&e->d_out), &e->out_cap, (nY + nT + nV + nC) * sizeof(double) + 64)))
      return fail(rc);
    double* dY = e->d_out;
    double* dT = dY + nY;
    double* dV = dT + nT;
    double* dC = dV + nV;
    if ((rc = launch_k5(e, e->d_panel, rows, e->ldp, wY ? dY : nullptr, wT ? dT : nullptr, wV ? dV : nullptr,
                        wC ? dC : nullptr, st)) != SYSID_OK)
      return fail(rc);
    const struct { double* h; const double* d; size_t n; } outs[4] = {{Y_proj, dY, nY}, {tau_proj, dT, nT},
                                                                       {B_v, dV, nV}, {B_c, dC, nC}};
    for (const auto& o : outs)
      if (o.n && (rc = host_copy(e, o.h, o.d, o.n * sizeof(double), hipMemcpyDeviceToHost, st, &reg)) != SYSID_OK)
        return fail(rc);
  }
  if (want_gram) {
    // the whole (W+1)^2 buffer in ONE DMA into page-locked memory; gram / Atb / btb are split out on the host
    // after the synchronize (three copies into the caller's pageable arrays cost ~50 us of staged-copy overhead)
    // (errors past the first enqueue leave through fail(): the kernels may still be reading the staging block)
    if (!e->h_gram && hipHostMalloc(reinterpret_cast<void**>(&e->h_gram), (size_t)e->ncol * e->ncol * sizeof(double),
                                    hipHostMallocDefault) != hipSuccess) {
      e->h_gram = nullptr;
      return fail(set_err(e, SYSID_E_DEVICE, "page-locked Gram buffer: allocation failed"));
    }
    if (hipMemcpyAsync(e->h_gram, e->d_gram, (size_t)e->ncol * e->ncol * sizeof(double), hipMemcpyDeviceToHost, st) !=
        hipSuccess)
      return fail(set_err(e, SYSID_E_DEVICE, "Gram copy failed"));
  }
  tph[2] = ms_since(t0);  // + kernels and output copies enqueued
  const hipError_t sst = hipStreamSynchronize(st);
  host_unregister(e, reg);
  stager.finish();  // every chunk packed and checked
  if (stager.contacts_bad()) return contact_error();
  if (sst == hipSuccess && want_gram) {
    const size_t W = (size_t)e->w, n1 = (size_t)e->ncol;
    if (gram)
      for (size_t i = 0; i < W; ++i) std::memcpy(gram + i * W, e->h_gram + i * n1, W * sizeof(double));
    if (Atb) std::memcpy(Atb, e->h_gram + W * n1, W * sizeof(double));
    if (btb) *btb = e->h_gram[W * n1 + W];
  }
  tph[3] = ms_since(t0);  // + synchronised
  if (trace)
    std::fprintf(stderr, "sysid_build N=%lld flags=%u: contacts %.3f, staging started %.3f, kernels enqueued "
                 "%.3f, launched %.3f, done %.3f ms\n", (long long)N, flags, tph[0], tph[1], t_kern, tph[2], tph[3]);
  if (trace && !stager.stamps().empty()) {
    std::string line = "  chunk stamps (packed, DMA + K0W enqueued) ms:";
    char buf[32];
    for (double x : stager.stamps()) {
      std::snprintf(buf, sizeof buf, " %.3f", x);
      line += buf;
    }
    std::fprintf(stderr, "%s\n", line.c_str());
  }
  if (sst != hipSuccess) return set_err(e, SYSID_E_DEVICE, "stream sync failed: %s", hipGetErrorString(sst));
  return SYSID_OK;
}

}  // namespace

extern "C" {

int32_t sysid_build(sysid_engine* e, const double* q, const double* dq, const double* ddq, const double* tau,
                    const double* cnt, int64_t N, int64_t ld, uint32_t flags, double* Y_proj, double* tau_proj,
                    double* B_v, double* B_c, double* gram, double* Atb, double* btb) {
  const HostInputs in{q, 8, dq, ddq, tau, cnt, 8, ld};
  return build_host(e, in, N, flags, Y_proj, tau_proj, B_v, B_c, gram, Atb, btb);
}

int32_t sysid_check_contacts(const sysid_engine* e, const double* cnt, int64_t N, int64_t ld, int64_t* bad) {
  if (!e) return set_err(nullptr, SYSID_E_INVALID, "null engine");
  if (e->nc == 0 || N <= 0) return SYSID_OK;
  if (!cnt || ld < N) return set_err(const_cast<sysid_engine*>(e), SYSID_E_INVALID, "bad contact buffer");
  return check_contacts_t(const_cast<sysid_engine*>(e), cnt, N, ld, bad);
}

int32_t sysid_build_f32qc(sysid_engine* e, const float* q, const double* dq, const double* ddq, const double* tau,
                          const float* cnt, int64_t N, int64_t ld, uint32_t flags, double* Y_proj, double* tau_proj,
                          double* B_v, double* B_c, double* gram, double* Atb, double* btb) {
  const HostInputs in{q, 4, dq, ddq, tau, cnt, 4, ld};
  return build_host(e, in, N, flags, Y_proj, tau_proj, B_v, B_c, gram, Atb, btb);
}

// ---- diagnostics --------------------------------------------------------------------------------

int32_t sysid_debug_body_column(const double* body24, int32_t p, double* fw6) {
  if (!body24 || !fw6 || p < 0 || p > 9) return SYSID_E_INVALID;
  double F[FBLK];
  body_regressor_block(body24, F);
  block_column(F, p, fw6);
  return SYSID_OK;
}

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

int32_t sysid_debug_layout(const sysid_engine* e, int32_t* offsets12) {
  if (!e || !offsets12) return SYSID_E_INVALID;
  const WLay L = wave_layout(e->in_lds, e->nv, e->nb + 1, e->nc, k1_layout_hw(e->k1m[0].variant), e->k1m[0].pov, e->k1m[0].qf);
  const int o[12] = {L.in, L.body, L.W, L.Pt, L.Jw, L.pf, L.Jc, L.M, L.P, L.H1, L.tp, L.total};
  for (int k = 0; k < 12; ++k) offsets12[k] = o[k];
  return SYSID_OK;
}

int32_t sysid_debug_lds(sysid_engine* e, const double* q, const double* dq, const double* ddq, const double* tau,
                        const double* cnt, double* lds_image, int64_t image_doubles) {
  if (!e || !lds_image) return set_err(e, SYSID_E_INVALID, "null argument");
  const WLay L = wave_layout(e->in_lds, e->nv, e->nb + 1, e->nc, k1_layout_hw(e->k1m[0].variant), e->k1m[0].pov, e->k1m[0].qf);
  if (image_doubles < L.total) return set_err(e, SYSID_E_INVALID, "image needs %d doubles", L.total);
  DevScope dev_scope(e->device);
  HIP_TRY(e, dev_scope.st);
  int rc = sysid_build(e, q, dq, ddq, tau, cnt, 1, 1, SYSID_EMIT_Y, nullptr, nullptr, nullptr, nullptr, nullptr,
                       nullptr, nullptr);  // allocates the device buffers
  if (rc != SYSID_OK) return rc;
  HIP_TRY(e, hipMalloc(&e->d_dump, (size_t)L.total * sizeof(double)));
  rc = launch_k1(e, e->d_in, 1, 1, e->d_panel, e->ldp, e->d_work, e->stream, e->d_dump);
  if (rc == SYSID_OK && hipStreamSynchronize(e->stream) != hipSuccess) rc = set_err(e, SYSID_E_DEVICE, "sync failed");
  if (rc == SYSID_OK &&
      hipMemcpy(lds_image, e->d_dump, (size_t)L.total * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
    rc = set_err(e, SYSID_E_DEVICE, "dump copy failed");
  (void)hipFree(e->d_dump);
  e->d_dump = nullptr;
  return rc;
}

int32_t sysid_set_gram_chunk_bytes(sysid_engine* e, uint64_t bytes) {
  if (!e) return set_err(nullptr, SYSID_E_INVALID, "null engine");
  if (bytes != 0 && bytes < ((uint64_t)1 << 20))
    return set_err(e, SYSID_E_INVALID, "Gram chunk of %llu bytes: at least 1 MiB (or 0 = the default)",
                   (unsigned long long)bytes);
  e->gram_chunk = bytes ? (size_t)bytes : (size_t)4 << 30;
  return SYSID_OK;
}

int32_t sysid_gram_rows(const sysid_engine* e, uint32_t flags) {
  if (!e) return SYSID_E_INVALID;
  return gram_nullspace(e, flags);
}

int32_t sysid_debug_k1_config(const sysid_engine* e, int32_t* cfg4) {
  if (!e || !cfg4) return SYSID_E_INVALID;
  cfg4[0] = e->k1m[0].waves;
  cfg4[1] = e->k1m[0].bpc;
  cfg4[2] = (int32_t)e->k1m[0].lds;
  cfg4[3] = e->k1_maxch_tpl;
  return SYSID_OK;
}

// The packed exchange's device side (sysid_rccl.cpp: sysid_allreduce_normal_equations): the upper triangle of the
// n x n Gram row by row (row i starts at i n - i (i - 1) / 2), then the row count; unpacked into both triangles.
__global__ void __launch_bounds__(256) xchg_pack(const double* __restrict__ G, int n, double rows,
                                                 double* __restrict__ x) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)n * n) return;
  const int i = (int)(e / n), j = (int)(e - (int64_t)i * n);
  if (j >= i) x[(int64_t)i * n - (int64_t)i * (i - 1) / 2 + (j - i)] = G[e];
  if (e == 0) x[(int64_t)n * (n + 1) / 2] = rows;
}
__global__ void __launch_bounds__(256) xchg_unpack(const double* __restrict__ x, int n, double* __restrict__ G) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)n * n) return;
  const int r = (int)(e / n), c = (int)(e - (int64_t)r * n);
  const int i = r < c ? r : c, j = r < c ? c : r;
  G[e] = x[(int64_t)i * n - (int64_t)i * (i - 1) / 2 + (j - i)];
}

size_t sysid_exchange_bytes(const sysid_engine* e) {
  if (!e) return 0;
  const size_t n = (size_t)e->ncol;
  return (n * (n + 1) / 2 + 1) * sizeof(double);
}

// sysid_rccl.cpp's hooks (one library, so the RCCL translation unit stays free of device code)
int32_t sysid_internal_xchg_pack(const sysid_engine* e, const double* d_gram, double rows, double* d_x, void* stream) {
  const int n = e->ncol;
  // a NULL stream is the null stream of the CURRENT device: the engine's for this call (the caller's device is
  // restored on return, DevScope)
  DevScope dev_scope(e->device);
  if (dev_scope.st != hipSuccess) return SYSID_E_DEVICE;
  hipLaunchKernelGGL(xchg_pack, dim3((unsigned)(((int64_t)n * n + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), d_gram, n, rows, d_x);
  return hipGetLastError() == hipSuccess ? SYSID_OK : SYSID_E_DEVICE;
}
int32_t sysid_internal_xchg_unpack(const sysid_engine* e, const double* d_x, double* d_gram, void* stream) {
  const int n = e->ncol;
  DevScope dev_scope(e->device);
  if (dev_scope.st != hipSuccess) return SYSID_E_DEVICE;
  hipLaunchKernelGGL(xchg_unpack, dim3((unsigned)(((int64_t)n * n + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), d_x, n, d_gram);
  return hipGetLastError() == hipSuccess ? SYSID_OK : SYSID_E_DEVICE;
}

int32_t sysid_debug_set_stage_chunks(sysid_engine* e, int32_t chunks) {
  if (!e || chunks < 0 || chunks > 64) return set_err(e, SYSID_E_INVALID, "stage chunks %d outside 0..64", chunks);
  e->stage_chunks = chunks;
  return SYSID_OK;
}

int32_t sysid_debug_k2_config(const sysid_engine* e, int32_t* cfg4) {
  if (!e || !cfg4) return SYSID_E_INVALID;
  cfg4[0] = e->ntc;
  cfg4[1] = e->k2d[0].nslots;
  cfg4[2] = e->k2d[1].nslots;
  cfg4[3] = e->k2d[2].nslots;
  return SYSID_OK;
}

}  // extern "C"
