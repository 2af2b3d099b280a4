"""Diagnose the nullspace Gram-only graph replay after a 0xFF workspace (dev tool).
Prints, per case, whether the Gram matches the clean eager run, and the workspace head: the eight K1 claim
counters (u64, 128 B apart), the live-row total and the first segment sums.
usage: python tools/dbg_ns_graph.py [N]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from system_identification_amd.engine import Engine
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import channel_block, generate

robot = sys.argv[1] if len(sys.argv) > 1 else "spot"
rows = sys.argv[2] if len(sys.argv) > 2 else "nullspace"
N = int(sys.argv[3]) if len(sys.argv) > 3 else 4099
m = load_robot(robot)
e = Engine(m)
d = generate(m, N, config_index=8)
din = torch.from_numpy(channel_block(d)).cuda()
b = e.alloc_gram_device(N)


def head(tag):
    torch.cuda.synchronize()
    ws = b["ws"]
    cnt = ws[:1024].view(torch.int64)[::16].tolist()
    nrows = ws[1024:1028].view(torch.int32).item()
    rseg = ws[1024 + 256:1024 + 256 + 20].view(torch.int32).tolist()
    G = b["gram"]
    print(f"{robot} {rows} {tag}: equal {bool(torch.equal(G, G0))} nan {int(torch.isnan(G).sum())} "
          f"zero {bool((G == 0).all())} counters {cnt} rows {nrows} rseg {rseg}", flush=True)


# the order of tests/test_gpu_fused.py::test_no_state_carried_in_the_workspace
e.build_gram_device(din, N, b, rows=rows)
torch.cuda.synchronize()
G0 = b["gram"].clone()
b["ws"].fill_(255)
b["gram"].fill_(float("nan"))
e.build_gram_device(din, N, b, rows=rows)
head("eager after 0xFF")
s = torch.cuda.Stream()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    e.build_gram_device(din, N, b, rows=rows, stream=torch.cuda.current_stream().cuda_stream)
for i in range(3):
    b["ws"].fill_(255)
    b["gram"].fill_(float("nan"))
    g.replay()
    head(f"replay {i} after 0xFF")
b["ws"].fill_(255)
torch.cuda.synchronize()
b["gram"].fill_(float("nan"))
g.replay()
head("replay after 0xFF + synchronize")
