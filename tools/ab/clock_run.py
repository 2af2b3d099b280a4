"""In-kernel clocks of K1 and K2 (a tools/ab/k1k2_clock.py build): >= 2 s of back-to-back Spot 20k full-output steps,
then the counters are reset and N more steps stamped.  SYSID_LIB=<lib> python tools/ab/clock_run.py [steps]"""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from system_identification_amd.engine import Engine, EMIT_ALL
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import generate, channel_block
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
m = load_robot("spot"); N = 20000; d = generate(m, N, 1); e = Engine(m)
din = torch.from_numpy(channel_block(d)).cuda()
bufs = e.alloc_device(N, EMIT_ALL)
run = lambda: e.build_device(din, N, EMIT_ALL, bufs)
readers = [getattr(e.lib, "sysid_debug_clock0"), getattr(e.lib, "sysid_debug_clock2")]
for f in readers:
    f.restype = ctypes.c_int32
out = (ctypes.c_ulonglong * 2)()
for label, settle in (("cold (first steps)", 0.0), ("after 2.5 s of steps", 2.5)):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < settle:
        for _ in range(16):
            run()
        torch.cuda.synchronize()
    for f in readers:
        f(out, 1)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(steps if settle > 0 else 10):
        run()
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / (steps if settle > 0 else 10)
    res = []
    for name, f in zip(("K1", "K2"), readers):
        f(out, 0)
        res.append(f"{name} {out[0] / max(out[1], 1) * 0.1:.3f} GHz")
    print(f"{label}: {ms:.4f} ms/step, in-kernel clocks: " + ", ".join(res), flush=True)
