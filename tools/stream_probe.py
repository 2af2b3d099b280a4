"""Streamed-input probe (dev tool): one Spot 20k Gram-only host call with SYSID_STREAM_PARTS set by the caller; prints
whether K1's waits were satisfied, the call's wall time and the host phase stamps (SYSID_TRACE_HOST).  Exits 0 either
way (the failure is the measurement).  usage: SYSID_STREAM_PARTS=2 python tools/stream_probe.py [reps] [robot] [N]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from system_identification_amd.engine import EMIT_GRAM, Engine, EngineError
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import generate

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
robot = sys.argv[2] if len(sys.argv) > 2 else "spot"
N = int(sys.argv[3]) if len(sys.argv) > 3 else 20000
m = load_robot(robot)
e = Engine(m)
d = generate(m, N, config_index=1)
ins = [d[k] for k in ("q", "dq", "ddq", "tau", "contact")]
for i in range(reps):
    t0 = time.perf_counter()
    try:
        e.build(*ins, EMIT_GRAM)
        print(f"call {i}: ok {1e3 * (time.perf_counter() - t0):.3f} ms", flush=True)
    except EngineError as x:
        print(f"call {i}: FAILED after {1e3 * (time.perf_counter() - t0):.1f} ms: {x}", flush=True)
