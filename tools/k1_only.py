"""Run K1 (and optionally the Gram) a few times for PMC collection (dev tool)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from system_identification_amd.engine import Engine, EMIT_ALL, EMIT_Y
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import generate, channel_block
robot = sys.argv[1] if len(sys.argv) > 1 else "spot"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
flags = EMIT_ALL if (len(sys.argv) > 3 and sys.argv[3] == "gram") else EMIT_Y
m = load_robot(robot); d = generate(m, N, 1); eng = Engine(m)
din = torch.from_numpy(channel_block(d)).cuda(); bufs = eng.alloc_device(N, EMIT_ALL)
for _ in range(3):
    eng.build_device(din, N, flags, bufs)
torch.cuda.synchronize()
