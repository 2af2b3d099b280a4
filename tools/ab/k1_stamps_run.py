"""Run K1 with the stamp build and print per-phase time shares:
SYSID_LIB=<stamps lib> python tools/ab/k1_stamps_run.py <robot> <N> [f64 | bf16]
(f64: stacked outputs, a lib patched with STAMP_PREC=0; bf16: the Gram-only projector rows, STAMP_PREC=2)"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from system_identification_amd.engine import Engine, EMIT_ALL, EMIT_Y
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import generate, channel_block
robot = sys.argv[1]; N = int(sys.argv[2]); prec = sys.argv[3] if len(sys.argv) > 3 else "f64"
m = load_robot(robot); d = generate(m, N, 1); e = Engine(m)
din = torch.from_numpy(channel_block(d)).cuda()
if prec == "f64":
    bufs = e.alloc_device(N, EMIT_ALL)
    run = lambda: e.build_device(din, N, EMIT_Y, bufs)
else:
    bufs = e.alloc_gram_device(N)
    run = lambda: e.build_gram_device(din, N, bufs, precision=prec, rows="projector")
run(); torch.cuda.synchronize()
f = e.lib.sysid_debug_k1_stamps
f.restype = ctypes.c_int32
out = (ctypes.c_ulonglong * 10)()
f(out, 1)
for _ in range(5):
    run()
torch.cuda.synchronize()
f(out, 0)
v = np.array(list(out), dtype=np.float64)
names = ["top", "FK poses", "axes+cpts", "v/a_gf", "J_c", "GS/P", "tp/H1/claim", "Y_proj", "friction"]
tot = v[:9].sum()
print(f"{robot} N={N} {prec}: waves {int(v[9])}, per-wave cycles per launch {tot / v[9] * 1 / 5:.0f}")
for n, x in zip(names, v[:9]):
    print(f"  {n:12s} {100 * x / tot:5.1f}%")
