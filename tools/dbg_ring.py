"""Repeatability of the fused Gram-only ring form (dev tool): runs it `reps` times on one engine and compares every
run with the first and with the unfused projector-row Gram (deterministic).  usage: python tools/dbg_ring.py [N] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from system_identification_amd.engine import Engine
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import channel_block, generate

N = int(sys.argv[1]) if len(sys.argv) > 1 else 100001
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
m = load_robot("spot")
e = Engine(m)
d = generate(m, N, config_index=7)
din = torch.from_numpy(channel_block(d)).cuda()


def gram(rows):
    b = e.alloc_gram_device(N)
    b["gram"].fill_(float("nan"))
    e.build_gram_device(din, N, b, precision="f64", rows=rows)
    torch.cuda.synchronize()
    return b["gram"].cpu().numpy()


e.set_fusion(False)
ref = gram("projector")
e.set_fusion(True)
lib = os.path.basename(os.environ.get("SYSID_LIB", "libsysid.so"))
first = None
for r in range(reps):
    G = gram("auto")
    rel = np.abs(G - ref).max() / np.abs(ref).max()
    bad = np.argwhere(np.abs(G - ref) > 1e-9 * np.abs(ref).max())
    same = first is None or np.array_equal(G, first)
    first = G if first is None else first
    print(f"{lib} N={N} rep {r}: vs unfused {rel:.2e}, entries off {len(bad)} (e.g. {bad[:4].tolist()}), "
          f"bitwise == rep 0: {same}", flush=True)
