"""Experiment: can K1 (VALU) and K2 (MFMA) run concurrently on two streams?  (dev tool, lib_exp.so)"""
import sys, os, ctypes, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from system_identification_amd import engine as E
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import generate, channel_block
robot = sys.argv[1] if len(sys.argv) > 1 else "spot"
N = 20000
m = load_robot(robot); d = generate(m, N, 1); eng = E.Engine(m)
lib = eng.lib
V = ctypes.c_void_p
lib.sysid_exp_k2.argtypes = [V, V, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, V, V, ctypes.c_size_t, V]
lib.sysid_exp_k1.argtypes = [V, V, ctypes.c_int64, ctypes.c_int64, V, ctypes.c_int64, V]
din = torch.from_numpy(channel_block(d)).cuda()
b1 = eng.alloc_device(N, E.EMIT_ALL); b2 = eng.alloc_device(N, E.EMIT_ALL)
eng.build_device(din, N, E.EMIT_ALL, b1); eng.build_device(din, N, E.EMIT_ALL, b2); torch.cuda.synchronize()
sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
def k1(buf, s): lib.sysid_exp_k1(eng._h, V(din.data_ptr()), N, din.stride(0), V(buf["panel"].data_ptr()), buf["panel"].stride(0), V(s.cuda_stream))
def k2(buf, s): lib.sysid_exp_k2(eng._h, V(buf["panel"].data_ptr()), N, buf["panel"].stride(0), 0, 1, V(buf["gram"].data_ptr()), V(buf["ws"].data_ptr()), buf["ws"].numel(), V(s.cuda_stream))
def timeit(fn, it=20):
    fn(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it): fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e3
print(robot, "blocks/CU env:", os.environ.get("SYSID_K1_BLOCKS_PER_CU"))
print("K1 alone   %.3f ms" % timeit(lambda: k1(b1, sA)))
print("K2+K3 alone %.3f ms" % timeit(lambda: k2(b2, sB)))
print("K1 then K2 same stream %.3f ms" % timeit(lambda: (k1(b1, sA), k2(b2, sA))))
print("K1 || K2 two streams %.3f ms" % timeit(lambda: (k1(b1, sA), k2(b2, sB))))
print("K2 || K1 two streams %.3f ms" % timeit(lambda: (k2(b2, sB), k1(b1, sA))))
