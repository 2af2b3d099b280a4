"""Gram-only stage times, nullspace rows vs projector rows, interleaved rounds (dev tool).
usage: python tools/gram_only_time.py <robot> <N> <f64|f32|bf16> [rounds]"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from system_identification_amd.engine import Engine, EMIT_ALL, GRAM_PRECISION, GRAM_PROJECTOR, GRAM_NULLSPACE
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import generate, channel_block
robot, N, prec = sys.argv[1], int(sys.argv[2]), sys.argv[3]
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 5
m = load_robot(robot); d = generate(m, N, 1); e = Engine(m)
din = torch.from_numpy(channel_block(d)).cuda()
b = e.alloc_gram_device(N)
res = {"nullspace": [], "projector": []}
for r in range(rounds):
    for mode in res:
        fl = EMIT_ALL | GRAM_PRECISION[prec] | (GRAM_PROJECTOR if mode == "projector" else GRAM_NULLSPACE)
        res[mode].append(e.time_stages(din, N, fl, b, iters=20))
for mode, v in res.items():
    v = np.median(np.array(v), axis=0)
    print(f"{robot} {N} {prec} {mode:9s}: K1(+list) {v[0]:.4f}  K2 {v[1]:.4f}  K3 {v[2]:.4f}  sum {v.sum():.4f} ms", flush=True)
