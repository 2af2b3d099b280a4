"""Scratch timing of the three kernels (dev tool)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from system_identification_amd.engine import Engine, EMIT_ALL
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import generate, channel_block

robot = sys.argv[1] if len(sys.argv) > 1 else "spot"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
m = load_robot(robot)
d = generate(m, N, 1)
eng = Engine(m)
din = torch.from_numpy(channel_block(d)).cuda()
bufs = eng.alloc_device(N, EMIT_ALL)
eng.build_device(din, N, EMIT_ALL, bufs); torch.cuda.synchronize()
ms = eng.time_stages(din, N, EMIT_ALL, bufs, iters=20)
print(robot, N, "ms per kernel [K1, K2, K3]:", ["%.4f" % x for x in ms], "total %.4f" % sum(ms))
bytes_k1 = N * ((m.nq + 2 * m.nv + m.nj + m.n_ee) * 8 + m.nv * (eng.w + 1) * 8)
W = eng.w
flops_k2 = N * (m.nv * W * (W + 1) + 2 * m.nv * W)
if ms[1] > 0:
    print("K1 %.1f GB/s   K2 %.2f TF/s   samples/s %.3e" % (bytes_k1 / ms[0] / 1e6, flops_k2 / ms[1] / 1e9, N / sum(ms) * 1e3))
else:  # fused K1 + Gram (ms[0] = the fused kernel)
    print("fused K12 %.2f TF/s (Gram flops), %.1f GB/s (K1 bytes)   samples/s %.3e" % (
        flops_k2 / ms[0] / 1e9, bytes_k1 / ms[0] / 1e6, N / sum(ms) * 1e3))
import ctypes
from system_identification_amd import engine as _E
cfg = (ctypes.c_int32 * 4)()
eng.lib.sysid_debug_k1_config(eng._h, cfg)
print("k1 config [waves/block, blocks/CU, lds bytes, maxch]:", list(cfg))
# whole step as the product runs it (pipelined K1 -> K2 when the panel is large enough)
for _ in range(3): eng.build_device(din, N, EMIT_ALL, bufs)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(20): eng.build_device(din, N, EMIT_ALL, bufs)
torch.cuda.synchronize()
st_ms = (time.perf_counter() - t) / 20 * 1e3
print("step (build_device) %.4f ms  samples/s %.3e  env chunks=%s ks=%s" % (st_ms, N / st_ms * 1e3, os.environ.get("SYSID_PIPE_CHUNKS"), os.environ.get("SYSID_PIPE_KS")))
