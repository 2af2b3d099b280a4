"""Debug: nullspace Gram-only repeatability (eager x3, then a captured graph), workspace row counts / list."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from system_identification_amd.engine import Engine, EMIT_ALL
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import generate, channel_block
robot = sys.argv[1] if len(sys.argv) > 1 else "spot"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
m = load_robot(robot); d = generate(m, N, 6); e = Engine(m)
din = torch.from_numpy(channel_block(d)).cuda()
gb = e.alloc_gram_device(N)
ws = gb["ws"]
def snap(tag):
    torch.cuda.synchronize()
    head = ws[1024:1024 + 256].view(torch.int32)
    G = gb["gram"].cpu().numpy()
    print(f"{tag}: total rows {int(head[0])}  G[0,0] {G[0,0]:.6e}  |G| {np.linalg.norm(G):.6e}", flush=True)
    return G
for k in range(3):
    e.build_gram_device(din, N, gb)
    G0 = snap(f"eager {k}")
expect = int((m.nv - 3 * (d["contact"] != 0).sum(axis=0)).sum())
print("expected rows (full-rank contacts):", expect)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, capture_error_mode="thread_local"):
    e.build_gram_device(din, N, gb, stream=torch.cuda.current_stream().cuda_stream)
for k in range(3):
    gb["gram"].fill_(float("nan"))
    g.replay()
    G1 = snap(f"replay {k}")
e.build_gram_device(din, N, gb)
snap("eager after")
