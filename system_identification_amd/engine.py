"""ctypes binding of libsysid.so (include/sysid.h).

The product path has no CPU fallback: if the HIP library is missing, or no GPU is visible when a
compute entry point is called, this module raises.  ``load_library()`` only loads the shared object
(it is safe without a GPU; the CPU test-suite uses it to check the exported symbols).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .model import Model

SYSID_OK = 0
SYSID_E_INVALID = -1
SYSID_E_MODEL = -2
SYSID_E_DEVICE = -3
SYSID_E_NOMEM = -4
SYSID_E_CONTACT = -5

EMIT_Y = 1
EMIT_TAU = 2
EMIT_FRICTION = 4
EMIT_GRAM = 8
EMIT_ALL = 15
GRAM_F32, GRAM_BF16 = 16, 32
GRAM_PROJECTOR = 64   # Gram-only from the reference's P·A rows (nv per sample)
GRAM_NULLSPACE = 128  # Gram-only from the nullspace rows Zᵀ·A (nv - rank(J_c) per sample)
GRAM_ROWS = {"auto": 0, "projector": GRAM_PROJECTOR, "nullspace": GRAM_NULLSPACE}
GRAM_PRECISION = {"f64": 0, "f32": GRAM_F32, "bf16": GRAM_BF16}

LIB_NAME = "libsysid.so"
LIB_PATH = os.environ.get("SYSID_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

# (name, restype, argtypes) — one entry per function declared in include/sysid.h
_c = ctypes
_dp = _c.POINTER(_c.c_double)
_vp = _c.c_void_p
_fp = _c.POINTER(_c.c_float)
SIGNATURES = [
    ("sysid_abi_version", _c.c_int32, []),
    ("sysid_model_create", _c.c_int32, [_vp, _c.c_size_t, _c.c_int32, _c.POINTER(_vp)]),
    ("sysid_destroy", None, [_vp]),
    ("sysid_last_error", _c.c_char_p, [_vp]),
    ("sysid_dims", _c.c_int32, [_vp] + [_c.POINTER(_c.c_int32)] * 7),
    ("sysid_build", _c.c_int32, [_vp, _dp, _dp, _dp, _dp, _dp, _c.c_int64, _c.c_int64, _c.c_uint32,
                                 _dp, _dp, _dp, _dp, _dp, _dp, _dp]),
    ("sysid_build_f32qc", _c.c_int32, [_vp, _fp, _dp, _dp, _dp, _fp, _c.c_int64, _c.c_int64, _c.c_uint32,
                                       _dp, _dp, _dp, _dp, _dp, _dp, _dp]),
    ("sysid_workspace_bytes", _c.c_size_t, [_vp, _c.c_int64, _c.c_uint32]),
    ("sysid_build_device", _c.c_int32, [_vp, _vp, _c.c_int64, _c.c_int64, _c.c_uint32, _vp, _c.c_int64,
                                        _vp, _vp, _c.c_size_t, _vp]),
    ("sysid_check_contacts", _c.c_int32, [_vp, _dp, _c.c_int64, _c.c_int64, _c.POINTER(_c.c_int64)]),
    ("sysid_debug_body_column", _c.c_int32, [_dp, _c.c_int32, _dp]),
    ("sysid_debug_body_column_device", _c.c_int32, [_dp, _dp]),
    ("sysid_debug_lds", _c.c_int32, [_vp, _dp, _dp, _dp, _dp, _dp, _dp, _c.c_int64]),
    ("sysid_debug_layout", _c.c_int32, [_vp, _c.POINTER(_c.c_int32)]),
    ("sysid_debug_k1_config", _c.c_int32, [_vp, _c.POINTER(_c.c_int32)]),
    ("sysid_gram_rows", _c.c_int32, [_vp, _c.c_uint32]),
    ("sysid_set_gram_chunk_bytes", _c.c_int32, [_vp, _c.c_uint64]),
    ("sysid_debug_k2_config", _c.c_int32, [_vp, _c.POINTER(_c.c_int32)]),
    ("sysid_debug_set_stage_chunks", _c.c_int32, [_vp, _c.c_int32]),
    ("sysid_time_stages", _c.c_int32, [_vp, _vp, _c.c_int64, _c.c_int64, _c.c_uint32, _vp, _c.c_int64, _vp,
                                       _vp, _c.c_size_t, _c.c_int32, _dp]),
    ("sysid_gram_workspace_bytes", _c.c_size_t, [_vp, _c.c_int64]),
    ("sysid_build_full", _c.c_int32, [_vp, _dp, _dp, _dp, _dp, _dp, _dp, _c.c_int64, _c.c_int64, _dp, _dp]),
    ("sysid_dat_shape", _c.c_int32, [_c.c_char_p, _c.POINTER(_c.c_int64), _c.POINTER(_c.c_int64)]),
    ("sysid_dat_read", _c.c_int32, [_c.c_char_p, _c.POINTER(_c.c_float), _c.c_int64, _c.c_int64, _c.c_int32]),
    ("sysid_io_last_error", _c.c_char_p, []),
    ("sysid_rccl_unique_id", _c.c_int32, [_vp]),
    ("sysid_rccl_comm_init", _c.c_int32, [_c.POINTER(_vp), _c.c_int32, _vp, _c.c_int32, _c.c_int32]),
    ("sysid_rccl_comm_destroy", _c.c_int32, [_vp]),
    ("sysid_allreduce_gram", _c.c_int32, [_vp, _vp, _vp, _vp]),
    ("sysid_rccl_last_error", _c.c_char_p, []),
    ("sysid_exchange_bytes", _c.c_size_t, [_vp]),
    ("sysid_allreduce_normal_equations", _c.c_int32, [_vp, _vp, _vp, _c.c_double, _vp, _vp]),
    ("sysid_tau_error", _c.c_int32, [_vp, _dp, _dp, _dp, _dp, _dp, _c.c_int64, _c.c_int64, _dp, _dp]),
    ("sysid_tau_error_workspace_bytes", _c.c_size_t, [_vp, _c.c_int64]),
    ("sysid_tau_error_device", _c.c_int32, [_vp, _vp, _c.c_int64, _c.c_int64, _vp, _vp, _vp, _c.c_size_t, _vp]),
    ("sysid_build_gram_device", _c.c_int32, [_vp, _vp, _c.c_int64, _c.c_int64, _c.c_uint32, _vp, _vp, _c.c_size_t,
                                             _vp]),
]

_LIB = None


class EngineError(RuntimeError):
    pass


def load_library(path: str = LIB_PATH):
    """Load libsysid.so and declare every C-ABI signature.  Raises if the library is not built."""
    global _LIB
    if _LIB is not None and path == LIB_PATH:
        return _LIB
    # torch bundles its own libamdhip64.so.7; load it first so libsysid binds to the same HIP runtime
    # (two runtimes in one process cannot share a device or a stream).
    import torch  # noqa: F401
    if not os.path.exists(path):
        raise EngineError(
            f"{path} is missing: the HIP engine is not built (run `python -c 'import __graft_entry__ as g; "
            "g.build()'`).  There is no CPU fallback.")
    lib = ctypes.CDLL(path)
    for name, res, args in SIGNATURES:
        if os.environ.get("SYSID_LIB") and not hasattr(lib, name):
            continue  # an older A/B build (SYSID_LIB): its missing entry points stay undeclared
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path == LIB_PATH:
        _LIB = lib
    return lib


def _raise(code: int, msg: str):
    if code in (SYSID_E_INVALID, SYSID_E_MODEL, SYSID_E_CONTACT):
        raise ValueError(msg)
    raise EngineError(msg)


def _ptr(a):
    return a.ctypes.data_as(_dp) if a is not None else None


PINNED_MIN_BYTES = 8 << 20
PINNED_MAX_BYTES = 1 << 30  # larger outputs: pageable (the C side page-locks them for the copy, host_copy)


def host_empty(shape, dtype=np.float64):
    """An output array for the host entry points.  Outputs of 8 MiB .. 1 GiB live in page-locked memory from
    PyTorch's caching host allocator: the DMA engine writes them at full PCIe rate, and a repeated call reuses
    blocks that are already pinned and paged in (a fresh np.empty pays one page fault per 4 KiB on first touch,
    which cost more than the copy itself: ~23 ms vs ~7 ms for Spot 20k's 374 MB Y_proj).

    That allocator rounds every block up to a power of two and keeps it cached, page-locked, after the array
    is dropped (release_pinned_cache() returns it to the OS).  Hence the 1 GiB cap: a larger output (e.g. a
    G1 full-output call's ~8 GB Y_proj) is plain np.empty, and sysid_build page-locks it only for the
    duration of its copy (hipHostRegister).  A failed pinned allocation also falls back to np.empty."""
    nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
    if nbytes < PINNED_MIN_BYTES or nbytes > PINNED_MAX_BYTES:
        return np.empty(shape, dtype=dtype)
    import torch
    tdt = {np.dtype(np.float64): torch.float64, np.dtype(np.float32): torch.float32}[np.dtype(dtype)]
    try:
        return torch.empty(tuple(shape), dtype=tdt, pin_memory=True).numpy()
    except RuntimeError:
        return np.empty(shape, dtype=dtype)


def release_pinned_cache():
    """Return the page-locked blocks cached by host_empty (PyTorch's caching host allocator) to the OS;
    arrays still alive keep theirs."""
    import torch
    torch._C._host_emptyCache()


def _require_gpu():
    import torch
    if not torch.cuda.is_available():
        raise EngineError("no HIP device visible: the MI355X engine has no CPU fallback")


class Engine:
    """One model on one device.  Wraps ``sysid_engine*``."""

    def __init__(self, model: Model, device: int = 0):
        _require_gpu()
        self.lib = load_library()
        self.model = model
        blob = model.pack()
        self._blob = ctypes.create_string_buffer(blob, len(blob))
        h = ctypes.c_void_p()
        rc = self.lib.sysid_model_create(self._blob, len(blob), int(device), ctypes.byref(h))
        if rc != SYSID_OK:
            _raise(rc, self.lib.sysid_last_error(None).decode())
        self._h = h
        self.device = device
        dims = [ctypes.c_int32() for _ in range(7)]
        self.lib.sysid_dims(self._h, *[ctypes.byref(d) for d in dims])
        self.nq, self.nv, self.nj, self.nb, self.n_contact, self.panel_cols, self.panel_ld = (d.value for d in dims)
        self.wy = 10 * self.nb
        self.w = self.wy + 2 * self.nj
        self.in_rows = self.nq + 2 * self.nv + self.nj + self.n_contact

    def close(self):
        if getattr(self, "_h", None):
            self.lib.sysid_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != SYSID_OK:
            _raise(rc, self.lib.sysid_last_error(self._h).decode())

    # ---- host-buffer path --------------------------------------------------------------------
    def build(self, q, dq, ddq, tau, cnt, flags: int = EMIT_ALL) -> dict:
        """Channel-major (channels x N) inputs -> stacked outputs (+ Gram), all float64 numpy.  q and contact as
        float32 arrays (what read_data returns, demo/spot_identification.py:10-14) go to sysid_build_f32qc and
        travel to the device as float32 / contact flags; otherwise everything is float64 (sysid_build)."""
        f32 = getattr(q, "dtype", None) == np.float32 and getattr(cnt, "dtype", None) == np.float32
        ins = []
        for a, rows, name in ((q, self.nq, "q"), (dq, self.nv, "dq"), (ddq, self.nv, "ddq"),
                              (tau, self.nj, "tau"), (cnt, self.n_contact, "contact")):
            wide = not (f32 and name in ("q", "contact"))
            a = np.ascontiguousarray(np.asarray(a, dtype=np.float64 if wide else np.float32))
            if a.ndim == 1:
                a = a.reshape(-1, 1)
            if a.shape[0] != rows:
                raise ValueError(f"{name}: expected {rows} channels, got shape {a.shape}")
            ins.append(a)
        N = ins[0].shape[1]
        for a in ins:
            if a.shape[1] != N:
                raise ValueError("all inputs must have the same number of samples")
        R = N * self.nv
        out = {}
        Y = host_empty((R, self.wy)) if flags & EMIT_Y else None
        t = host_empty((R,)) if flags & EMIT_TAU else None
        Bv = host_empty((R, self.nj)) if flags & EMIT_FRICTION else None
        Bc = host_empty((R, self.nj)) if flags & EMIT_FRICTION else None
        G = np.empty((self.w, self.w)) if flags & EMIT_GRAM else None
        g = np.empty(self.w) if flags & EMIT_GRAM else None
        btb = np.zeros(1) if flags & EMIT_GRAM else None
        if f32:
            fp = lambda a: a.ctypes.data_as(_fp)  # noqa: E731
            rc = self.lib.sysid_build_f32qc(self._h, fp(ins[0]), _ptr(ins[1]), _ptr(ins[2]), _ptr(ins[3]), fp(ins[4]),
                                            N, N, int(flags), _ptr(Y), _ptr(t), _ptr(Bv), _ptr(Bc), _ptr(G), _ptr(g),
                                            _ptr(btb))
        else:
            rc = self.lib.sysid_build(self._h, *[_ptr(a) for a in ins], N, N, int(flags),
                                      _ptr(Y), _ptr(t), _ptr(Bv), _ptr(Bc), _ptr(G), _ptr(g), _ptr(btb))
        self._check(rc)
        if Y is not None:
            out["Y_proj"] = Y
        if t is not None:
            out["tau_proj"] = t
        if Bv is not None:
            out["B_v"], out["B_c"] = Bv, Bc
        if G is not None:
            out["gram"], out["Atb"], out["btb"], out["num_rows"] = G, g, float(btb[0]), R
        return out

    def build_full(self, q, dq, ddq, tau, ee_force, cnt):
        """Unprojected regressor Y (N·nv x 10 nb) and F = Sᵀ tau + J_cᵀ lambda (N·nv,), K1 in full-force mode."""
        ins = []
        for a, rows, name in ((q, self.nq, "q"), (dq, self.nv, "dq"), (ddq, self.nv, "ddq"), (tau, self.nj, "tau"),
                              (ee_force, 3 * self.n_contact, "ee_force"), (cnt, self.n_contact, "contact")):
            a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
            if a.ndim == 1:
                a = a.reshape(-1, 1)
            if a.shape[0] != rows:
                raise ValueError(f"{name}: expected {rows} channels, got shape {a.shape}")
            ins.append(a)
        N = ins[0].shape[1]
        for a in ins:
            if a.shape[1] != N:
                raise ValueError("all inputs must have the same number of samples")
        Y = host_empty((N * self.nv, self.wy))
        F = host_empty((N * self.nv,))
        self._check(self.lib.sysid_build_full(self._h, *[_ptr(a) for a in ins], N, N, _ptr(Y), _ptr(F)))
        return Y, F

    def tau_error(self, q, dq, ddq, tau, cnt, phi) -> np.ndarray:
        """Sum over samples of the squared torque-prediction error of every row (nv,), K4 on the device."""
        ins = []
        for a, rows, name in ((q, self.nq, "q"), (dq, self.nv, "dq"), (ddq, self.nv, "ddq"),
                              (tau, self.nj, "tau"), (cnt, self.n_contact, "contact")):
            a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
            if a.ndim == 1:
                a = a.reshape(-1, 1)
            if a.shape[0] != rows:
                raise ValueError(f"{name}: expected {rows} channels, got shape {a.shape}")
            ins.append(a)
        N = ins[0].shape[1]
        phi = np.ascontiguousarray(np.asarray(phi, dtype=np.float64).reshape(-1))
        if phi.size != self.wy:
            raise ValueError(f"phi: expected {self.wy} parameters, got {phi.size}")
        err = np.zeros(self.nv)
        self._check(self.lib.sysid_tau_error(self._h, *[_ptr(a) for a in ins], N, N, _ptr(phi), _ptr(err)))
        return err

    def tau_error_device(self, bufs: dict, N: int, d_phi, d_err, stream=None):
        """K4 on a panel written by build_device; d_phi (10 nb,) and d_err (nv,) float64 CUDA tensors."""
        import torch
        ws = torch.empty(max(int(self.lib.sysid_tau_error_workspace_bytes(self._h, int(N))), 256),
                         dtype=torch.uint8, device=bufs["panel"].device)
        st = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        self._check(self.lib.sysid_tau_error_device(
            self._h, ctypes.c_void_p(bufs["panel"].data_ptr()), int(bufs["panel"].stride(0)), int(N),
            ctypes.c_void_p(d_phi.data_ptr()), ctypes.c_void_p(d_err.data_ptr()), ctypes.c_void_p(ws.data_ptr()),
            int(ws.numel()), ctypes.c_void_p(st)))
        return ws  # keep alive until the stream has consumed it

    # ---- device-buffer path (torch tensors on this engine's device) ----------------------------
    def workspace_bytes(self, N: int, flags: int = EMIT_ALL) -> int:
        return int(self.lib.sysid_workspace_bytes(self._h, int(N), int(flags)))

    def alloc_device(self, N: int, flags: int = EMIT_ALL) -> dict:
        import torch
        dev = torch.device("cuda", self.device)
        R = N * self.nv
        return {
            "panel": torch.empty((R, self.panel_ld), dtype=torch.float64, device=dev),
            "gram": torch.empty((self.panel_cols, self.panel_cols), dtype=torch.float64, device=dev),
            "ws": torch.empty(max(self.workspace_bytes(N, flags), 256), dtype=torch.uint8, device=dev),
        }

    def _check_inputs(self, d_in, N: int):
        """The C side cannot see tensor extents: a mismatched N would read other samples or fault, so the
        shapes are checked here, before anything is enqueued."""
        import torch
        if d_in.dtype != torch.float64 or not d_in.is_cuda or d_in.dim() != 2 or d_in.shape[0] != self.in_rows:
            raise ValueError(f"d_in must be a 2-D float64 CUDA tensor with {self.in_rows} channel rows")
        if d_in.device.index != self.device:
            raise ValueError(f"d_in is on {d_in.device}, the engine on cuda:{self.device}")
        if d_in.stride(1) != 1 or (d_in.shape[0] > 1 and d_in.stride(0) < d_in.shape[1]):
            raise ValueError("d_in must be channel-major with unit sample stride (a row-contiguous channel block)")
        if not 0 <= int(N) <= d_in.shape[1]:
            raise ValueError(f"N = {N} samples, but d_in holds {d_in.shape[1]}")

    def _check_buffer(self, t, name: str, dtype, min_numel: int):
        import torch
        if not isinstance(t, torch.Tensor) or t.dtype != dtype or not t.is_cuda or t.device.index != self.device:
            raise ValueError(f"{name} must be a {dtype} tensor on cuda:{self.device}")
        if not t.is_contiguous() and not (t.dim() == 2 and t.stride(1) == 1):
            raise ValueError(f"{name} must have unit stride along its last dimension")
        if t.numel() < min_numel:
            raise ValueError(f"{name} holds {t.numel()} elements, {min_numel} needed")

    def build_device(self, d_in, N: int, flags: int, bufs: dict, stream=None):
        """Stream-ordered launch on device tensors.  ``d_in`` is the (in_rows x ld) channel block."""
        import torch
        self._check_inputs(d_in, N)
        P = bufs["panel"]
        self._check_buffer(P, "panel", torch.float64, 0)
        if P.dim() != 2 or P.stride(1) != 1 or P.shape[1] < self.panel_cols or P.shape[0] < int(N) * self.nv:
            raise ValueError(f"panel must be a row-major (>= {int(N) * self.nv}) x (>= {self.panel_cols}) float64 "
                             f"tensor, got {tuple(P.shape)} with strides {P.stride()}")
        if flags & EMIT_GRAM:
            self._check_buffer(bufs["gram"], "gram", torch.float64, self.panel_cols * self.panel_cols)
            if not bufs["gram"].is_contiguous():
                raise ValueError("gram must be contiguous")
        self._check_buffer(bufs["ws"], "ws", torch.uint8, self.workspace_bytes(N, flags))
        ld = d_in.stride(0)
        st = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        rc = self.lib.sysid_build_device(
            self._h, ctypes.c_void_p(d_in.data_ptr()), int(N), int(ld), int(flags),
            ctypes.c_void_p(bufs["panel"].data_ptr()), int(bufs["panel"].stride(0)),
            ctypes.c_void_p(bufs["gram"].data_ptr()), ctypes.c_void_p(bufs["ws"].data_ptr()),
            int(bufs["ws"].numel()), ctypes.c_void_p(st))
        self._check(rc)

    # ---- Gram-only device path (panel produced chunk by chunk inside the workspace) -------------
    def gram_workspace_bytes(self, N: int) -> int:
        return int(self.lib.sysid_gram_workspace_bytes(self._h, int(N)))

    def alloc_gram_device(self, N: int) -> dict:
        import torch
        dev = torch.device("cuda", self.device)
        return {
            "gram": torch.empty((self.panel_cols, self.panel_cols), dtype=torch.float64, device=dev),
            "ws": torch.empty(max(self.gram_workspace_bytes(N), 256), dtype=torch.uint8, device=dev),
        }

    def build_gram_device(self, d_in, N: int, bufs: dict, stream=None, precision: str = "f64",
                          rows: str = "auto"):
        """Normal equations of N samples without materialising the N·nv-row panel (stream-ordered).
        precision: "f64" (parity), "f32" or "bf16" (MFMA in reduced precision, error reported).
        rows: "nullspace" (each sample's nv - rank(J_c) rows Zᵀ·A, ZᵀZ = P), "projector" (the reference's nv
        rows P·A) or "auto" (nullspace for f64 / f32 unless the model runs the Q-form K1; projector otherwise and for bf16); all give Σ AᵀPA."""
        import torch
        self._check_inputs(d_in, N)
        self._check_buffer(bufs["gram"], "gram", torch.float64, self.panel_cols * self.panel_cols)
        if not bufs["gram"].is_contiguous():
            raise ValueError("gram must be contiguous")
        self._check_buffer(bufs["ws"], "ws", torch.uint8, self.gram_workspace_bytes(N))
        st = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        rc = self.lib.sysid_build_gram_device(
            self._h, ctypes.c_void_p(d_in.data_ptr()), int(N), int(d_in.stride(0)),
            GRAM_PRECISION[precision] | GRAM_ROWS[rows],
            ctypes.c_void_p(bufs["gram"].data_ptr()), ctypes.c_void_p(bufs["ws"].data_ptr()),
            int(bufs["ws"].numel()), ctypes.c_void_p(st))
        self._check(rc)

    def set_stage_chunks(self, chunks: int) -> None:
        """Tests: stage the host entry points' inputs in `chunks` equal chunks (0 = the default bounds)."""
        self._check(self.lib.sysid_debug_set_stage_chunks(self._h, int(chunks)))

    def set_gram_chunk_bytes(self, nbytes: int) -> None:
        """Chunk panel size of the Gram-only path (>= 1 MiB; 0 = the 4 GiB default).  alloc_gram_device /
        gram_workspace_bytes follow it, so set it before allocating."""
        self._check(self.lib.sysid_set_gram_chunk_bytes(self._h, int(nbytes)))

    def gram_rows(self, precision: str = "f64", rows: str = "auto") -> str:
        """The rows build_gram_device uses: "nullspace" (Zᵀ·A) or "projector" (P·A)."""
        rc = self.lib.sysid_gram_rows(self._h, GRAM_PRECISION[precision] | GRAM_ROWS[rows])
        self._check(min(rc, 0))
        return "nullspace" if rc == 1 else "projector"

    def k1_config(self) -> list:
        """K1 launch shape of the f64 panel [waves per workgroup, workgroups per CU, LDS bytes, chain slots]."""
        cfg = (ctypes.c_int32 * 4)()
        self._check(self.lib.sysid_debug_k1_config(self._h, cfg))
        return list(cfg)

    def k2_config(self) -> list:
        """K2 Gram deal [tile columns, tile slots of the f64, f32 and bf16 deals]."""
        cfg = (ctypes.c_int32 * 4)()
        self._check(self.lib.sysid_debug_k2_config(self._h, cfg))
        return list(cfg)

    def time_stages(self, d_in, N: int, flags: int, bufs: dict, iters: int = 10) -> list:
        """Mean ms per step in each stage [regressor/projector, Gram SYRK, Gram reduce] (HIP events).  With
        Gram-only buffers (alloc_gram_device: no "panel") the chunked Gram-only path is timed, its chunks summed."""
        self._check_inputs(d_in, N)
        ms = np.zeros(3)
        panel = bufs.get("panel")
        rc = self.lib.sysid_time_stages(
            self._h, ctypes.c_void_p(d_in.data_ptr()), int(N), int(d_in.stride(0)), int(flags),
            ctypes.c_void_p(panel.data_ptr() if panel is not None else None),
            int(panel.stride(0)) if panel is not None else 0,
            ctypes.c_void_p(bufs["gram"].data_ptr()), ctypes.c_void_p(bufs["ws"].data_ptr()),
            int(bufs["ws"].numel()), int(iters), _ptr(ms))
        self._check(rc)
        return ms.tolist()

    def views(self, bufs: dict, N: int) -> dict:
        """Reference-shaped views of the device panel / Gram (no copies)."""
        P = bufs["panel"][: N * self.nv]
        G = bufs["gram"]
        W = self.w
        return {"Y_proj": P[:, : self.wy], "B_v": P[:, self.wy: self.wy + self.nj],
                "B_c": P[:, self.wy + self.nj: W], "tau_proj": P[:, W],
                "gram": G[:W, :W], "Atb": G[:W, W], "btb": G[W, W]}
