"""Dev tool: steps of the device entry point with D batches in flight (D streams, D buffer sets) vs one stream.

    python tools/inflight_probe.py [robot] [N] [D...]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from system_identification_amd.engine import EMIT_ALL, Engine  # noqa: E402
from system_identification_amd.model import load_robot  # noqa: E402
from system_identification_amd.synthetic import channel_block, generate  # noqa: E402

robot = sys.argv[1] if len(sys.argv) > 1 else "spot"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
depths = [int(x) for x in sys.argv[3:]] or [1, 2, 3]
m = load_robot(robot)
eng = Engine(m)
d_in = torch.from_numpy(channel_block(generate(m, N, 1))).cuda()
steps = 40
for D in depths:
    streams = [torch.cuda.Stream() for _ in range(D)]
    bufs = [eng.alloc_device(N, EMIT_ALL) for _ in range(D)]
    for k in range(2 * D):
        eng.build_device(d_in, N, EMIT_ALL, bufs[k % D], stream=streams[k % D].cuda_stream)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for k in range(steps):
        eng.build_device(d_in, N, EMIT_ALL, bufs[k % D], stream=streams[k % D].cuda_stream)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / steps * 1e3
    print(f"{robot} {N} batches in flight {D}: {ms:.4f} ms per step, {N / ms * 1e3:.4e} samples/s", flush=True)
    ok = all(torch.equal(bufs[0]["gram"], b["gram"]) for b in bufs[1:])
    print("  Grams of all buffer sets bitwise equal:", ok, flush=True)
