"""Host entry point e2e times (dev tool): best of `reps` calls of Engine.build, Gram-only and full outputs, with q and
contact in float32 (read_data's dtypes) or float64.  Env knobs of the staging (SYSID_STAGE_CHUNKS, _SPLIT, _BOUNDS)
are read once per process: run one process per setting.
usage: python tools/e2e_time.py [robot] [N] [reps] [f32|f64] [gram|all] [auto|nullspace|projector]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from system_identification_amd.engine import EMIT_ALL, EMIT_GRAM, GRAM_ROWS, Engine
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import generate

robot = sys.argv[1] if len(sys.argv) > 1 else "spot"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
dt = sys.argv[4] if len(sys.argv) > 4 else "f32"
which = sys.argv[5] if len(sys.argv) > 5 else "gram"
rows = sys.argv[6] if len(sys.argv) > 6 else "auto"
m = load_robot(robot)
e = Engine(m)
d = generate(m, N, config_index=1)
cast = (lambda a: a.astype(np.float32)) if dt == "f32" else (lambda a: a)
ins = [cast(d["q"]), d["dq"], d["ddq"], d["tau"], cast(d["contact"])]
env = {k: v for k, v in os.environ.items() if k.startswith("SYSID_STAGE")}
for name, flags in (("gram_only", EMIT_GRAM | GRAM_ROWS[rows]), ("full", EMIT_ALL)):
    if which == "gram" and name == "full":
        continue
    e.build(*ins, flags)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        e.build(*ins, flags)
        ts.append(time.perf_counter() - t0)
    ts = np.array(ts) * 1e3
    print(f"{robot} {N} {dt} {name} rows={rows} {env}: best {ts.min():.3f} ms  median {np.median(ts):.3f} ms", flush=True)
