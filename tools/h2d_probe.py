"""H2D copy shapes of the host entry point's input staging (dev tool): one 1-D copy of a packed chunk against
the 2-D copy (one row per input channel) the staged path sends, from page-locked memory, timed with HIP events.
usage: python tools/h2d_probe.py [rows=71] [N=20000] [chunks=2]"""
import ctypes
import sys

import torch

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 71
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
chunks = int(sys.argv[3]) if len(sys.argv) > 3 else 2
hip = ctypes.CDLL("libamdhip64.so")
H2D = 1
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipMemcpy2DAsync.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                 ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]

src = torch.ones(rows * N, dtype=torch.float64).pin_memory()
dst = torch.empty(rows * N, dtype=torch.float64, device="cuda")
st = torch.cuda.current_stream()
sh = ctypes.c_void_p(st.cuda_stream)
CH = (N + chunks - 1) // chunks
total = rows * N * 8


def run(kind):
    for c in range(chunks):
        c0 = c * CH
        n = min(CH, N - c0)
        if kind == "2d":  # the staged path: rows of [c0, c0 + n) of every channel, pitch N
            r = hip.hipMemcpy2DAsync(ctypes.c_void_p(dst.data_ptr() + c0 * 8), N * 8, ctypes.c_void_p(src.data_ptr() + c0 * 8),
                                     N * 8, n * 8, rows, H2D, sh)
        elif kind == "1d":  # the chunk packed contiguously (rows x n), one copy
            off = rows * c0 * 8
            r = hip.hipMemcpyAsync(ctypes.c_void_p(dst.data_ptr() + off), ctypes.c_void_p(src.data_ptr() + off),
                                   rows * n * 8, H2D, sh)
        else:  # one copy per channel row
            r = 0
            for k in range(rows):
                off = (k * N + c0) * 8
                r |= hip.hipMemcpyAsync(ctypes.c_void_p(dst.data_ptr() + off), ctypes.c_void_p(src.data_ptr() + off),
                                        n * 8, H2D, sh)
        assert r == 0, r


for kind in ("1d", "2d", "rows", "1d", "2d"):
    best = 1e9
    for _ in range(10):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record(st)
        run(kind)
        b.record(st)
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b))
    print(f"{kind:5s} {chunks} chunk(s), {rows} rows x {N}: {best:.4f} ms = {total / best / 1e6:.1f} GB/s", flush=True)
