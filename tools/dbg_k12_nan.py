"""Diagnose NaN in the fused full-output Gram after a NaN-filled workspace/panel (dev tool).
usage: python tools/dbg_k12_nan.py [N ...]"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from system_identification_amd.engine import Engine, EMIT_ALL
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import generate, channel_block
m = load_robot("spot"); e = Engine(m)
import ctypes
_lib = ctypes.CDLL(os.environ["SYSID_LIB"]) if os.environ.get("SYSID_LIB") else None
_diag = getattr(_lib, "sysid_debug_k12_diag", None) if _lib is not None else None


def diag(bad_wg):
    if _diag is None:
        return
    buf = (ctypes.c_longlong * (256 * 8 * 10))()
    _diag(buf, 256 * 8 * 10)
    d = np.frombuffer(buf, dtype=np.int64).reshape(256, 8, 10)
    t0 = d[:, :, 1][d[:, :, 0] > 0].min()
    k1_end = (d[:, :4, 2] - t0) / 100.0  # microseconds
    g_end = (d[:, 4:, 2] - t0) / 100.0
    print(f"   K1 end us: median {np.median(k1_end):.0f} max {k1_end.max():.0f}; Gram end us: median "
          f"{np.median(g_end):.0f} max {g_end.max():.0f}; gram bad waves {int(d[:, 4:, 3].sum())}", flush=True)
    for b in bad_wg[:4]:
        print(f"   WG {b}: start us {[(int(x) - t0) / 100.0 for x in d[b, :, 1]]}", flush=True)
        print(f"      K1 [end us, ready, f0, f1]: {[((int(r[2]) - t0) / 100.0, int(r[3]), int(r[4]), int(r[5])) for r in d[b, :4]]}", flush=True)
        print(f"      Gram [end us, bad, np, nfast, ready0..3]: {[((int(r[2]) - t0) / 100.0, *map(int, r[3:])) for r in d[b, 4:]]}", flush=True)
for N in [int(x) for x in sys.argv[1:]] or [4099, 4098, 20000]:
    d = generate(m, N, 8)
    din = torch.from_numpy(channel_block(d)).cuda()
    for fill_ws, fill_panel in ((False, True), (True, False), (True, True)):
        f = e.alloc_device(N, EMIT_ALL)
        f["ws"].zero_(); f["panel"].zero_()
        e.build_device(din, N, EMIT_ALL, f); torch.cuda.synchronize()
        G0 = f["gram"].clone(); P0 = f["panel"][: N * e.nv].clone()
        if fill_ws: f["ws"].fill_(255)
        if fill_panel: f["panel"].fill_(float("nan"))
        e.build_device(din, N, EMIT_ALL, f); torch.cuda.synchronize()
        G = f["gram"]; P = f["panel"][: N * e.nv]
        grid = min(256, (N + 1) // 2)
        slab = f["ws"][1024:1024 + grid * 55 * 2048].view(torch.float64).view(grid, 55, 256)
        bad_wg = torch.isnan(slab).any(dim=2).any(dim=1).nonzero().flatten().tolist()
        bad_tiles = torch.isnan(slab).any(dim=2).sum(dim=0).tolist()
        prow = torch.isnan(P).any(dim=1).nonzero().flatten().tolist()
        print(f"N={N} fill_ws={fill_ws} fill_panel={fill_panel}: gram nan {int(torch.isnan(G).sum())}, "
              f"equal {bool(torch.equal(G, G0))}, panel equal {bool(torch.equal(P, P0))}, panel nan rows {len(prow)} "
              f"{prow[:5]}, nan WGs {len(bad_wg)} {bad_wg[:8]}, tiles with nan per slot {[i for i, x in enumerate(bad_tiles) if x]}",
              flush=True)
        diag(bad_wg)
        del f
