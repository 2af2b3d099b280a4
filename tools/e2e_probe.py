"""Host entry point (PCIe-inclusive) timing probe (dev tool): page-locking vs pageable copies, output first
touch, pinned destination upper bound.  python tools/e2e_probe.py [robot] [N]"""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from system_identification_amd.engine import EMIT_ALL, EMIT_GRAM, Engine
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import generate

robot = sys.argv[1] if len(sys.argv) > 1 else "spot"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
m = load_robot(robot)
d = generate(m, N, 1)
ins = [d[k] for k in ("q", "dq", "ddq", "tau", "contact")]
e = Engine(m)
for flags, name in ((EMIT_ALL, "full"), (EMIT_GRAM, "gram")):
    e.build(*ins, flags)
    ts = []
    for _ in range(4):
        t = time.perf_counter(); e.build(*ins, flags); ts.append(time.perf_counter() - t)
    print(f"{name}: build {min(ts)*1e3:.2f} ms (reps {[round(x*1e3,2) for x in ts]})  register={os.environ.get('SYSID_HOST_REGISTER')}")
R = N * m.nv
t = time.perf_counter(); a = np.empty((R, e.wy)); a[::512] = 0; a.fill(0.0); t1 = time.perf_counter() - t
print(f"np.empty + fill of Y ({a.nbytes/1e6:.0f} MB): {t1*1e3:.2f} ms")
src = torch.empty((R, e.wy), dtype=torch.float64, device="cuda")
pin = torch.empty((R, e.wy), dtype=torch.float64, pin_memory=True)
for _ in range(2):
    torch.cuda.synchronize(); t = time.perf_counter(); pin.copy_(src, non_blocking=True); torch.cuda.synchronize()
    dt = time.perf_counter() - t
print(f"D2H into pinned: {dt*1e3:.2f} ms = {a.nbytes/dt/1e9:.1f} GB/s")
cpu = torch.from_numpy(np.empty((R, e.wy)))
for _ in range(2):
    torch.cuda.synchronize(); t = time.perf_counter(); cpu.copy_(src); torch.cuda.synchronize()
    dt = time.perf_counter() - t
print(f"D2H into pageable (touched): {dt*1e3:.2f} ms = {a.nbytes/dt/1e9:.1f} GB/s")
