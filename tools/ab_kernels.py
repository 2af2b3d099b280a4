"""Per-kernel HIP-event times of one library build over several workloads (dev tool; SYSID_LIB selects the build):
spot 20k full outputs, spot 20k Gram-only f64 (engine's rows), g1 20k full outputs, g1 125k Gram-only bf16.
usage: SYSID_LIB=<lib> python tools/ab_kernels.py [workload ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from system_identification_amd.engine import EMIT_ALL, Engine
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import channel_block, generate

WL = {"spot_full": ("spot", 20000, None), "spot_go": ("spot", 20000, "f64"),
      "g1_full": ("g1_29dof", 20000, None), "g1_bf16": ("g1_29dof", 125000, "bf16")}
names = sys.argv[1:] or list(WL)
lib = os.path.basename(os.environ.get("SYSID_LIB", "libsysid.so"))
for name in names:
    robot, N, prec = WL[name]
    m = load_robot(robot)
    e = Engine(m)
    d = generate(m, N, 1)
    din = torch.from_numpy(channel_block(d)).cuda()
    settle = float(os.environ.get("SYSID_AB_SETTLE_MS", "0"))  # untimed steps first: clocks at their operating point
    if prec is None:
        bufs = e.alloc_device(N, EMIT_ALL)
        e.build_device(din, N, EMIT_ALL, bufs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < settle:
            for _ in range(16):
                e.build_device(din, N, EMIT_ALL, bufs)
            torch.cuda.synchronize()
        ms = e.time_stages(din, N, EMIT_ALL, bufs, iters=30)
    else:
        from system_identification_amd.engine import GRAM_PRECISION
        bufs = e.alloc_gram_device(N)
        e.build_gram_device(din, N, bufs, precision=prec)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < settle:
            for _ in range(8):
                e.build_gram_device(din, N, bufs, precision=prec)
            torch.cuda.synchronize()
        ms = e.time_stages(din, N, EMIT_ALL | GRAM_PRECISION[prec], bufs, iters=20)
    print(f"AB {lib} {name} K1 {ms[0]:.4f} K2 {ms[1]:.4f} K3 {ms[2]:.4f}", flush=True)
    del bufs, din
    torch.cuda.empty_cache()
