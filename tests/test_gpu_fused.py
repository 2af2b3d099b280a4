"""The fused K1 + Gram kernel (k12_fused_panel_gram) against the unfused K1 -> K2 -> K3 path and
the C oracle: Spot and Solo-12 (the quadruped K1, 10-tile Gram), ragged sample counts (an odd last pair, fewer
pairs than CUs, one sample), bitwise repeatability and graph replay.  Reference: demo/spot_identification.py:84-87
(the stacked panel) and src/solver.py:186-190 (the Gram the objective implies).  The fused kernel is off by default
(measured slower than K1 -> K2 -> K3): every test here turns it on explicitly."""
import numpy as np
import pytest

from oracle.ref_c import COracle
from system_identification_amd.engine import EMIT_ALL, Engine
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import channel_block, generate

pytestmark = pytest.mark.gpu

CH = ("q", "dq", "ddq", "tau", "contact")


def rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def run(e, d, N, fused):
    import torch
    e.set_fusion(fused)
    din = torch.from_numpy(channel_block(d)).cuda()
    bufs = e.alloc_device(N, EMIT_ALL)
    bufs["gram"].fill_(np.nan)
    e.build_device(din, N, EMIT_ALL, bufs)
    torch.cuda.synchronize()
    return bufs["panel"][: N * e.nv].cpu().numpy(), bufs["gram"].cpu().numpy()


def test_fused_where_supported():
    for robot, want in (("spot", True), ("solo12", True), ("g1_29dof", False), ("snake14", False)):
        e = Engine(load_robot(robot))
        assert not e.fused(EMIT_ALL), robot  # off by default
        e.set_fusion(True)
        assert e.fused(EMIT_ALL) == want, robot
        e.set_fusion(False)
        assert not e.fused(EMIT_ALL)


@pytest.mark.parametrize("robot,N", [("spot", 1), ("spot", 3), ("spot", 64), ("spot", 513), ("spot", 20000),
                                     ("solo12", 2000), ("solo12", 4001)])
def test_fused_matches_unfused_and_oracle(robot, N):
    model = load_robot(robot)
    e = Engine(model)
    d = generate(model, N, config_index=5)
    P1, G1 = run(e, d, N, True)
    P0, G0 = run(e, d, N, False)
    # the panel: the same K1 code on the same samples
    assert rel(P1, P0) <= 1e-15, robot
    # the Gram: another summation order only
    W = e.panel_cols
    assert np.all(np.isfinite(G1))
    assert rel(G1, G0) <= 1e-13, (robot, N, rel(G1, G0))
    assert np.array_equal(G1, G1.T)
    # whole-N C oracle (OpenMP): Gram, Atb, btb at north_star's 1e-6
    o = COracle(model).build(*[d[k] for k in CH], nthreads=16, stacked=False)
    Wg = W - 1
    assert rel(G1[:Wg, :Wg], o["gram"]) < 1e-6
    assert rel(G1[:Wg, Wg], o["Atb"]) < 1e-6
    assert abs(G1[Wg, Wg] - o["btb"]) <= 1e-6 * abs(o["btb"])


def test_fused_bitwise_repeatable_and_graph_replay():
    import torch
    model = load_robot("spot")
    e = Engine(model)
    e.set_fusion(True)
    N = 20000
    d = generate(model, N, config_index=6)
    din = torch.from_numpy(channel_block(d)).cuda()
    bufs = e.alloc_device(N, EMIT_ALL)
    e.build_device(din, N, EMIT_ALL, bufs)
    torch.cuda.synchronize()
    P, G = bufs["panel"].clone(), bufs["gram"].clone()
    for _ in range(3):
        bufs["gram"].zero_()
        e.build_device(din, N, EMIT_ALL, bufs)
        torch.cuda.synchronize()
        assert torch.equal(bufs["gram"], G) and torch.equal(bufs["panel"], P)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        e.build_device(din, N, EMIT_ALL, bufs, stream=s.cuda_stream)  # warm outside the capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        e.build_device(din, N, EMIT_ALL, bufs, stream=torch.cuda.current_stream().cuda_stream)
    for _ in range(3):
        bufs["gram"].zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(bufs["gram"], G) and torch.equal(bufs["panel"], P)


@pytest.mark.parametrize("robot,N", [("spot", 1), ("spot", 7), ("spot", 513), ("spot", 20000), ("spot", 100001),
                                     ("solo12", 3001)])
def test_fused_gram_only_ring(robot, N):
    """The fused Gram-only form (rows through per-wave rings of three sample pairs, never a panel): against the
    full-output fused Gram (the same rows, the same summation order: bitwise), the unfused nullspace-row path
    (1e-10) and the C oracle (1e-6, whole N); bitwise repeatable."""
    import torch
    from system_identification_amd.engine import EMIT_GRAM
    model = load_robot(robot)
    e = Engine(model)
    e.set_fusion(True)
    assert e.fused(EMIT_GRAM) and e.gram_rows("f64") == "projector"
    d = generate(model, N, config_index=7)
    din = torch.from_numpy(channel_block(d)).cuda()

    def gram_only(rows="auto"):
        b = e.alloc_gram_device(N)
        b["gram"].fill_(float("nan"))
        e.build_gram_device(din, N, b, precision="f64", rows=rows)
        torch.cuda.synchronize()
        return b["gram"].cpu().numpy()
    G = gram_only()
    assert np.all(np.isfinite(G)) and np.array_equal(G, G.T)
    assert np.array_equal(G, gram_only())
    _, Gfull = run(e, d, N, True)
    assert np.array_equal(G, Gfull)  # same rows, same deal, same order
    Gz = gram_only("nullspace")
    assert rel(G, Gz) <= 1e-10, rel(G, Gz)
    o = COracle(model).build(*[d[k] for k in CH], nthreads=16, stacked=False)
    W = e.w
    assert rel(G[:W, :W], o["gram"]) < 1e-6 and rel(G[:W, W], o["Atb"]) < 1e-6
    assert abs(G[W, W] - o["btb"]) <= 1e-6 * abs(o["btb"])


@pytest.mark.parametrize("robot,rows,fuse", [("spot", "auto", True), ("spot", "auto", False),
                                           ("spot", "nullspace", False), ("g1_29dof", "auto", False)])
def test_no_state_carried_in_the_workspace(robot, rows, fuse):
    """Every launch sequence derives its counters, row lists, rings and slabs from the current launch only
    (VERDICT r3 item 6): a workspace filled with 0xFF bytes (-1 ints, NaN doubles) beforehand gives the same Gram
    bitwise as a clean one, eagerly and under graph replay, for the fused ring, the nullspace row list and the
    chunked projector rows; the full-output path likewise (fused on the quadrupeds)."""
    import torch
    model = load_robot(robot)
    e = Engine(model)
    e.set_fusion(fuse)
    N = 4099
    d = generate(model, N, config_index=8)
    din = torch.from_numpy(channel_block(d)).cuda()
    b = e.alloc_gram_device(N)
    e.build_gram_device(din, N, b, rows=rows)
    torch.cuda.synchronize()
    G0 = b["gram"].clone()
    b["ws"].fill_(255)
    b["gram"].fill_(float("nan"))
    e.build_gram_device(din, N, b, rows=rows)
    torch.cuda.synchronize()
    assert torch.equal(b["gram"], G0)
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        e.build_gram_device(din, N, b, rows=rows, stream=torch.cuda.current_stream().cuda_stream)
    for _ in range(2):
        b["ws"].fill_(255)
        b["gram"].fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(b["gram"], G0)
    f = e.alloc_device(N, EMIT_ALL)
    e.build_device(din, N, EMIT_ALL, f)
    torch.cuda.synchronize()
    P0, F0 = f["panel"].clone(), f["gram"].clone()
    f["ws"].fill_(255)
    f["panel"].fill_(float("nan"))
    e.build_device(din, N, EMIT_ALL, f)
    torch.cuda.synchronize()
    assert torch.equal(f["gram"], F0) and torch.equal(f["panel"][: N * e.nv], P0[: N * e.nv])


@pytest.mark.parametrize("form", ["ring", "full"])
def test_fused_give_up_poisons_the_gram_and_returns(form, monkeypatch):
    """The fused kernel's waits are bounded.  With a short bound (SYSID_K12_SPIN_LOG2, a test knob read at model
    creation) they give up: in the Gram-only ring form the K1 waves' waits for their ring slots, with the Gram waves
    held back (SYSID_K12_STALL_POLLS); in the full-output form the Gram waves' waits for their K1 waves' steps.
    The workgroup's abort word then makes every Gram wave write NaN tiles, later waits return at once, and the
    launch completes promptly (a K1-side give-up used to overwrite unread ring slots silently and leave
    later waits spinning for ~1 s each)."""
    import time
    import torch
    monkeypatch.setenv("SYSID_K12_SPIN_LOG2", "8" if form == "ring" else "2")
    monkeypatch.setenv("SYSID_K12_STALL_POLLS", "100000" if form == "ring" else "0")
    model = load_robot("spot")
    e = Engine(model)
    e.set_fusion(True)
    N = 20000
    d = generate(model, N, config_index=7)
    din = torch.from_numpy(channel_block(d)).cuda()
    t0 = time.perf_counter()
    if form == "ring":
        b = e.alloc_gram_device(N)
        e.build_gram_device(din, N, b, precision="f64")
    else:
        b = e.alloc_device(N, EMIT_ALL)
        e.build_device(din, N, EMIT_ALL, b)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    G = b["gram"].cpu().numpy()
    assert np.isnan(G).any(), form
    assert dt < 5.0, dt
    # the same engine without the knobs' effect on a fresh model builds the right Gram again
    monkeypatch.delenv("SYSID_K12_SPIN_LOG2")
    monkeypatch.delenv("SYSID_K12_STALL_POLLS")
    e2 = Engine(model)
    e2.set_fusion(True)
    b2 = e2.alloc_gram_device(N)
    e2.build_gram_device(din, N, b2, precision="f64")
    torch.cuda.synchronize()
    assert np.all(np.isfinite(b2["gram"].cpu().numpy()))
