"""ctypes wrapper of oracle/_build/libsysid_oracle.so (CPU ORACLE — test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.  Built by
__graft_entry__.build() with gcc from oracle/sysid_oracle.c.
"""
import ctypes
import os

import numpy as np

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libsysid_oracle.so")
_dp = ctypes.POINTER(ctypes.c_double)


def _lib():
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} missing: run __graft_entry__.build()")
    lib = ctypes.CDLL(LIB_PATH)
    lib.oracle_create.restype = ctypes.c_void_p
    lib.oracle_create.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.oracle_destroy.argtypes = [ctypes.c_void_p]
    lib.oracle_build.restype = ctypes.c_int
    lib.oracle_build.argtypes = [ctypes.c_void_p] + [_dp] * 5 + [ctypes.c_int64, ctypes.c_int64] + [_dp] * 8 + [ctypes.c_int]
    return lib


class COracle:
    def __init__(self, model):
        self.lib = _lib()
        self.model = model
        blob = model.pack()
        self._blob = ctypes.create_string_buffer(blob, len(blob))
        self.h = self.lib.oracle_create(self._blob, len(blob))
        if not self.h:
            raise ValueError("oracle: bad model")

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.oracle_destroy(self.h)

    def build(self, q, dq, ddq, tau, cnt, nthreads=1, gram=True, stacked=True, ymax=False):
        """The stacked arrays and normal equations; ymax=True adds "Y_max", each sample's max |Y| of its
        unprojected regressor (the per-sample scale of the Y_proj parity metric, tests/parity.py)."""
        m = self.model
        ins = [np.ascontiguousarray(np.asarray(a, dtype=np.float64)) for a in (q, dq, ddq, tau, cnt)]
        N = ins[0].shape[1]
        R, W = N * m.nv, 10 * m.nb + 2 * m.nj
        Y = np.empty((R, 10 * m.nb)) if stacked else None
        t = np.empty(R) if stacked else None
        Bv = np.empty((R, m.nj)) if stacked else None
        Bc = np.empty((R, m.nj)) if stacked else None
        G = np.empty((W, W)) if gram else None
        g = np.empty(W) if gram else None
        bb = np.zeros(1)
        ym = np.empty(N) if ymax else None
        p = lambda a: a.ctypes.data_as(_dp) if a is not None else None  # noqa: E731
        self.lib.oracle_build(self.h, *[p(a) for a in ins], N, ins[0].strides[0] // 8,
                              p(Y), p(t), p(Bv), p(Bc), p(G), p(g), p(bb), p(ym), int(nthreads))
        return {"Y_proj": Y, "tau_proj": t, "B_v": Bv, "B_c": Bc, "gram": G, "Atb": g, "btb": float(bb[0]),
                "Y_max": ym}
