"""Whole-N oracle parity at BASELINE.json's one-GPU configurations: every sample of the
stacked panel and the whole Gram / Aᵀb / bᵀb against the C oracle (oracle/sysid_oracle.c, OpenMP on the box's
16 threads) at north_star's 1e-6 — not sampled subsets.

* config 1 Solo-12 2k, config 2 Spot 20k (the headline workload) and config 3 G1 20k: the whole panel, per sample
  block, and the whole normal equations;
* config 4 Spot 200k and config 5 G1 1M (f64 Gram-only): the whole normal equations (tests/test_gpu_configs.py
  holds their shard-sum and sampled-panel checks).
Per-block metric: max |a - b| over the block / max(max |b| over the block, 1e-4 x the sample's unprojected scale):
its |tau| for tau_proj, its joint |dq| for B_v, 1 for B_c, and its unprojected regressor's max |Y| for Y_proj (the
C oracle reports it per sample, oracle_build's ymax), as the sampled tests do (tests/parity.py).  Run times are
printed (pytest -s) and listed by --durations (tests/conftest.py).
Reference: demo/spot_identification.py:84-87, src/solver.py:186-190."""
import time

import numpy as np
import pytest

from oracle.ref_c import COracle
from system_identification_amd.engine import EMIT_ALL, Engine
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import channel_block, generate

pytestmark = pytest.mark.gpu

TOL = 1e-6
CH = ("q", "dq", "ddq", "tau", "contact")
FLOOR = 1e-4


def rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def block_errors(a, b, N, nv, floor):
    """Per-sample relative errors of a stacked (N nv x c) array: max over the block / max(block max, floor_s)."""
    a3, b3 = a.reshape(N, nv, -1), b.reshape(N, nv, -1)
    num = np.abs(a3 - b3).max(axis=(1, 2))
    den = np.maximum(np.abs(b3).max(axis=(1, 2)), np.maximum(floor, 1e-300))
    return num / den


def check_normal_equations(G, o, W, what):
    eg, ea = rel(G[:W, :W], o["gram"]), rel(G[:W, W], o["Atb"])
    eb = abs(G[W, W] - o["btb"]) / abs(o["btb"])
    print(f"{what}: Gram {eg:.2e}  Atb {ea:.2e}  btb {eb:.2e}")
    assert eg < TOL and ea < TOL and eb < TOL, (what, eg, ea, eb)


@pytest.mark.parametrize("robot,N,cfg", [("solo12", 2000, 0), ("spot", 20000, 1), ("g1_29dof", 20000, 2)])
def test_whole_panel_and_gram_vs_oracle(robot, N, cfg):
    import torch
    model = load_robot(robot)
    e = Engine(model)
    d = generate(model, N, config_index=cfg)
    din = torch.from_numpy(channel_block(d)).cuda()
    bufs = e.alloc_device(N, EMIT_ALL)
    e.build_device(din, N, EMIT_ALL, bufs)
    torch.cuda.synchronize()
    P = bufs["panel"][: N * model.nv].cpu().numpy()
    G = bufs["gram"].cpu().numpy()
    t0 = time.perf_counter()
    o = COracle(model).build(*[d[k] for k in CH], nthreads=16, ymax=True)
    t_o = time.perf_counter() - t0
    nv, wy, nj, W = model.nv, e.wy, e.nj, e.w
    bd = model.base_dof
    tau_s = np.abs(d["tau"]).max(axis=0)
    dq_s = np.abs(d["dq"][bd:]).max(axis=0)
    errs = {
        "Y_proj": block_errors(P[:, :wy], o["Y_proj"], N, nv, FLOOR * o["Y_max"]),
        "tau_proj": block_errors(P[:, W], o["tau_proj"], N, nv, FLOOR * tau_s),
        "B_v": block_errors(P[:, wy:wy + nj], o["B_v"], N, nv, FLOOR * dq_s),
        "B_c": block_errors(P[:, wy + nj:W], o["B_c"], N, nv, FLOOR),
    }
    worst = {k: (float(v.max()), int(v.argmax())) for k, v in errs.items()}
    print(f"{robot} {N}: oracle {t_o:.2f} s on 16 threads; worst block "
          + ", ".join(f"{k} {v[0]:.1e} (sample {v[1]})" for k, v in worst.items()))
    for k, (v, s) in worst.items():
        assert v < TOL, (k, s, v)
    assert np.all(P[:, W + 1:e.panel_cols] == 0.0)  # the pad column is written as zeros
    check_normal_equations(G, o, W, f"{robot} {N}")


def test_config4_spot_200k_whole_gram_vs_oracle():
    import torch
    model = load_robot("spot")
    e = Engine(model)
    N = 200000
    d = generate(model, N, config_index=3)
    din = torch.from_numpy(channel_block(d)).cuda()
    bufs = e.alloc_device(N, EMIT_ALL)
    e.build_device(din, N, EMIT_ALL, bufs)
    torch.cuda.synchronize()
    G = bufs["gram"].cpu().numpy()
    del bufs
    t0 = time.perf_counter()
    o = COracle(model).build(*[d[k] for k in CH], nthreads=16, stacked=False)
    print(f"Spot 200k: oracle {time.perf_counter() - t0:.1f} s on 16 threads")
    check_normal_equations(G, o, e.w, "Spot 200k (config 4 whole)")


def test_config5_g1_1m_whole_gram_vs_oracle():
    """config 5 whole: the f64 Gram-only normal equations of all 1M G1 samples against the oracle's."""
    import torch
    model = load_robot("g1_29dof")
    e = Engine(model)
    N = 1000000
    d = generate(model, N, config_index=5)
    din = torch.from_numpy(channel_block(d)).cuda()
    b = e.alloc_gram_device(N)
    e.build_gram_device(din, N, b, precision="f64")
    torch.cuda.synchronize()
    G = b["gram"].cpu().numpy()
    del b, din
    t0 = time.perf_counter()
    o = COracle(model).build(*[d[k] for k in CH], nthreads=16, stacked=False)
    print(f"G1 1M: oracle {time.perf_counter() - t0:.1f} s on 16 threads")
    check_normal_equations(G, o, e.w, "G1 1M (config 5 whole, f64 Gram-only)")
