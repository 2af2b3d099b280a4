"""Gram-only launches for PMC collection (dev tool): python tools/k1_gram_only.py <robot> <N> <f64|f32|bf16> [nullspace|projector]"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from system_identification_amd.engine import Engine
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import generate, channel_block
robot, N, prec = sys.argv[1], int(sys.argv[2]), sys.argv[3]
rows = sys.argv[4] if len(sys.argv) > 4 else "nullspace"
m = load_robot(robot); d = generate(m, N, 1); e = Engine(m)
din = torch.from_numpy(channel_block(d)).cuda(); b = e.alloc_gram_device(N)
for _ in range(3):
    e.build_gram_device(din, N, b, precision=prec, rows=rows)
torch.cuda.synchronize()
