"""Where the host entry point's e2e time goes (dev tool; run with SYSID_TRACE_HOST=1 for the C-side phases).
Prints the Python-side wall time of Engine.build per call next to the C phases on stderr, and the raw H2D rate of
the same bytes from pinned and pageable memory for comparison.
usage: SYSID_TRACE_HOST=1 python tools/e2e_breakdown.py [robot] [N] [reps]"""
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
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
m = load_robot(robot)
e = Engine(m)
d = generate(m, N, config_index=1)
ins = [d[k] for k in ("q", "dq", "ddq", "tau", "contact")]
nbytes = sum(a.nbytes for a in ins)
for name, flags in (("gram_only", EMIT_GRAM), ("full", EMIT_ALL)):
    e.build(*ins, flags)
    for _ in range(reps):
        t0 = time.perf_counter()
        e.build(*ins, flags)
        print(f"{name}: python wall {1e3 * (time.perf_counter() - t0):.3f} ms", flush=True)
        sys.stderr.flush()
x = torch.empty(nbytes // 8, dtype=torch.float64).pin_memory()
y = torch.empty(nbytes // 8, dtype=torch.float64, device="cuda")
z = np.ones(nbytes // 8)
for src, tag in ((x, "pinned"), (torch.from_numpy(z), "pageable")):
    best = 1e9
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        y.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    print(f"H2D {nbytes / 1e6:.1f} MB from {tag}: {1e3 * best:.3f} ms = {nbytes / best / 1e9:.1f} GB/s", flush=True)
