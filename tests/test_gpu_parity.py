"""GPU parity: the HIP path, called through the C ABI, against the CPU oracles.

Tolerance: north_star's 1e-6 relative.  Per-sample blocks are compared relative to the block's own largest
magnitude; the Gram normwise (max-abs relative).  At full sizes, size-independent properties are checked
(linearity over sample shards, determinism, symmetry/PSD, Gram == panelᵀ·panel, sampled rows vs the C
oracle)."""
import os

import numpy as np
import pytest

from oracle import ref_numpy as ref
from system_identification_amd import engine as E
from system_identification_amd.engine import EMIT_ALL, EMIT_GRAM, Engine
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import channel_block, generate
from tests.parity import rel as rel_floor
from tests.parity import unprojected_scales

pytestmark = pytest.mark.gpu

TOL = 1e-6
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_ENGINES = {}


def eng(robot):
    if robot not in _ENGINES:
        _ENGINES[robot] = Engine(load_robot(robot))
    return _ENGINES[robot]


def rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


def check_blocks(out, Y, t, Bv, Bc, model, q, dq, ddq, tau):
    """Per-sample blocks, relative to the block's magnitude floored by the unprojected scale (tests/parity.py)."""
    nv = model.nv
    for s, sc in enumerate(unprojected_scales(model, q, dq, ddq, tau)):
        sl = slice(s * nv, (s + 1) * nv)
        for a, b, c in ((out["Y_proj"][sl], Y[sl], sc[0]), (out["tau_proj"][sl], t[sl], sc[1]),
                        (out["B_v"][sl], Bv[sl], sc[2]), (out["B_c"][sl], Bc[sl], sc[3])):
            assert rel_floor(a, b, c) < TOL, s


@pytest.mark.parametrize("robot,N,cfg", [("solo12", 48, 0), ("spot", 64, 1), ("g1_29dof", 24, 2),
                                         ("solo12_fixed", 48, 3), ("snake14", 40, 5)])
def test_panel_and_gram_vs_oracle(robot, N, cfg):
    """snake14 (an authored robot with a 14-joint tail, tools/make_robots.py) is the one model whose chains
    need the 16-slot K1 instantiations: K1_C16P here, K1_C16Q in the reduced-precision tests below."""
    model = load_robot(robot)
    d = generate(model, N, config_index=cfg)
    out = eng(robot).build(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"], EMIT_ALL)
    Y, t = ref.get_projected_y_tau(model, d["q"], d["dq"], d["ddq"], d["tau"], d["contact"])
    Bv, Bc = ref.get_projected_friction_regressors(model, d["q"], d["dq"], d["ddq"], d["contact"])
    G, g, btb, rows = ref.normal_equations(Y, t, Bv, Bc)
    check_blocks(out, Y, t, Bv, Bc, model, d["q"], d["dq"], d["ddq"], d["tau"])
    assert rel(out["gram"], G) < TOL
    assert rel(out["Atb"], g) < TOL
    assert abs(out["btb"] - btb) <= TOL * abs(btb)
    assert out["num_rows"] == rows
    if robot == "snake14":
        assert eng(robot).k1_config()[3] == 16  # the 16-slot chain instantiation ran


@pytest.mark.parametrize("robot", ["solo12", "spot", "g1_29dof", "solo12_fixed"])
def test_golden_fixtures(robot):
    g = dict(np.load(os.path.join(GOLD, f"{robot}.npz")))
    model = load_robot(robot)
    out = eng(robot).build(g["q"], g["dq"], g["ddq"], g["tau"], g["contact"], EMIT_ALL)
    check_blocks(out, g["Y_proj"], g["tau_proj"], g["B_v"], g["B_c"], model, g["q"], g["dq"], g["ddq"], g["tau"])
    assert rel(out["gram"], g["gram"]) < TOL and rel(out["Atb"], g["Atb"]) < TOL


def test_degenerate_inputs():
    model = load_robot("spot")
    e = eng("spot")
    d = generate(model, 6, config_index=4)
    cases = [np.zeros(4), np.ones(4), 2 * np.ones(4), np.array([2, 0, 0, 0.0]), np.array([0, 0, 0, 1.0]),
             np.array([1, 2, 0, 1.0])]
    cnt = np.stack(cases, axis=1)
    out = e.build(d["q"], d["dq"], d["ddq"], d["tau"], cnt, EMIT_ALL)
    Y, t = ref.get_projected_y_tau(model, d["q"], d["dq"], d["ddq"], d["tau"], cnt)
    Bv, Bc = ref.get_projected_friction_regressors(model, d["q"], d["dq"], d["ddq"], cnt)
    check_blocks(out, Y, t, Bv, Bc, model, d["q"], d["dq"], d["ddq"], d["tau"])
    # no contact: P = I, so the friction columns are exactly S^T diag(dq)
    assert np.array_equal(out["B_v"][:18], np.vstack([np.zeros((6, 12)), np.diag(d["dq"][6:, 0])]))
    # N = 1 and N = 0
    one = e.build(d["q"][:, :1], d["dq"][:, :1], d["ddq"][:, :1], d["tau"][:, :1], cnt[:, :1], EMIT_ALL)
    assert np.array_equal(one["Y_proj"], out["Y_proj"][:18])
    empty = e.build(d["q"][:, :0], d["dq"][:, :0], d["ddq"][:, :0], d["tau"][:, :0], cnt[:, :0], EMIT_ALL)
    assert empty["Y_proj"].shape == (0, 130) and not empty["gram"].any() and empty["btb"] == 0.0


def test_ill_conditioned_contact_jacobians():
    """solo12_fixed standing on nearly straight legs: cond(J_c) ~5/eps up to 5e8, and exactly singular legs
    (eps = 0, pinv drops 4 directions).  The Gram-Schmidt projector stays pinv-grade (tests/test_projector.py)."""
    model = load_robot("solo12_fixed")
    knees = [i for i, n in enumerate(model.joint_names) if n.endswith("KFE")]
    eps = [1e-2, 1e-4, 1e-6, 1e-8, 0.0]
    pats = [[1, 1, 1, 0], [1, 0, 2, 0], [1, 1, 1, 1], [0, 1, 1, 1]]
    n = len(eps) * len(pats)
    d = generate(model, n, config_index=3)
    cnt = np.zeros((4, n))
    for s in range(n):
        for j in knees:
            d["q"][model.idx_q[j], s] = eps[s % len(eps)]
        cnt[:, s] = pats[s // len(eps)]
    out = eng("solo12_fixed").build(d["q"], d["dq"], d["ddq"], d["tau"], cnt, EMIT_ALL)
    Y, t = ref.get_projected_y_tau(model, d["q"], d["dq"], d["ddq"], d["tau"], cnt)
    Bv, Bc = ref.get_projected_friction_regressors(model, d["q"], d["dq"], d["ddq"], cnt)
    nv = model.nv
    scales = unprojected_scales(model, d["q"], d["dq"], d["ddq"], d["tau"])
    for s in range(n):
        sl = slice(s * nv, (s + 1) * nv)
        pinned = cnt[:, s].all() and eps[s % len(eps)] != 0.0  # J_c square, invertible: P = 0 exactly
        for a, b, c in ((out["Y_proj"][sl], Y[sl], scales[s][0]), (out["tau_proj"][sl], t[sl], scales[s][1]),
                        (out["B_v"][sl], Bv[sl], scales[s][2]), (out["B_c"][sl], Bc[sl], scales[s][3])):
            if pinned:
                # both paths return rounding noise ~eps·cond(J_c) (cond up to 5e8 here): zero to the bar
                assert np.abs(a).max() <= TOL * c and np.abs(b).max() <= TOL * c, s
            else:
                assert rel_floor(a, b, c) < TOL, s
    G, g, _, _ = ref.normal_equations(Y, t, Bv, Bc)
    assert rel(out["gram"], G) < TOL and rel(out["Atb"], g) < TOL


def test_exactly_dependent_contact_rows():
    """Two contact slots on one foot frame (Spot with end-effector 1 := end-effector 0): with both in contact
    J_c repeats three rows exactly; pinv drops them, and so must the quadruped kernel's Gram-Schmidt."""
    import copy
    model = copy.deepcopy(load_robot("spot"))
    model.end_effector_names[1] = model.end_effector_names[0]
    N = 16
    d = generate(model, N, config_index=2)
    cnt = np.ones((4, N))
    cnt[2:, ::2] = 0.0
    out = Engine(model).build(d["q"], d["dq"], d["ddq"], d["tau"], cnt, EMIT_ALL)
    Y, t = ref.get_projected_y_tau(model, d["q"], d["dq"], d["ddq"], d["tau"], cnt)
    Bv, Bc = ref.get_projected_friction_regressors(model, d["q"], d["dq"], d["ddq"], cnt)
    check_blocks(out, Y, t, Bv, Bc, model, d["q"], d["dq"], d["ddq"], d["tau"])


def test_contact_contract_and_shape_errors():
    model = load_robot("spot")
    d = generate(model, 3, config_index=1)
    cnt = d["contact"].copy()
    cnt[:, 1] = [0.5, 0.0, 0.0, 0.0]  # int(sum) = 0 < one foot in contact: the reference raises
    with pytest.raises(ValueError):
        eng("spot").build(d["q"], d["dq"], d["ddq"], d["tau"], cnt, EMIT_ALL)
    with pytest.raises(ValueError):
        eng("spot").build(d["q"][:5], d["dq"], d["ddq"], d["tau"], d["contact"], EMIT_ALL)


@pytest.mark.parametrize("flags", [EMIT_ALL, EMIT_GRAM])
@pytest.mark.parametrize("f32", [False, True])
def test_contact_contract_checked_while_staging(flags, f32):
    """The host entry points check the contact contract in their packing threads, chunk by chunk (Stager::check):
    a violation in the last staged chunk still fails the call before any output is written, and the message names
    the first offending sample; the same inputs without the violations build normally afterwards."""
    model = load_robot("spot")
    e = eng("spot")
    N = 20001
    d = generate(model, N, config_index=1)
    cnt = d["contact"].copy()
    cnt[:, 19000] = [0.5, 0.0, 0.0, 0.0]
    cnt[:, 15000] = [0.0, 0.5, 0.0, 0.0]
    q = d["q"].astype(np.float32) if f32 else d["q"]
    c = cnt.astype(np.float32) if f32 else cnt
    with pytest.raises(ValueError, match="sample 15000"):
        e.build(q, d["dq"], d["ddq"], d["tau"], c, flags)
    ok = e.build(q, d["dq"], d["ddq"], d["tau"], d["contact"].astype(c.dtype), flags)
    ref_out = e.build(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"], flags)
    for k in ok:
        assert np.array_equal(np.asarray(ok[k]), np.asarray(ref_out[k])), k


def test_device_api_views_and_determinism():
    import torch
    model = load_robot("spot")
    e = eng("spot")
    N = 3000
    d = generate(model, N, config_index=5)
    din = torch.from_numpy(channel_block(d)).cuda()
    bufs = e.alloc_device(N, EMIT_ALL)
    e.build_device(din, N, EMIT_ALL, bufs)
    torch.cuda.synchronize()
    v = e.views(bufs, N)
    host = e.build(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"], EMIT_ALL)
    assert np.array_equal(v["Y_proj"].cpu().numpy(), host["Y_proj"])
    assert np.array_equal(v["gram"].cpu().numpy(), host["gram"])
    g1 = bufs["gram"].clone()
    p1 = bufs["panel"].clone()
    for _ in range(2):
        e.build_device(din, N, EMIT_ALL, bufs)
    torch.cuda.synchronize()
    assert torch.equal(g1, bufs["gram"]) and torch.equal(p1, bufs["panel"])  # bitwise deterministic
    # a non-default stream
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        e.build_device(din, N, EMIT_ALL, bufs, stream=s.cuda_stream)
    s.synchronize()
    assert torch.equal(g1, bufs["gram"])


@pytest.mark.parametrize("robot", ["spot", "g1_29dof"])
def test_null_stream_is_ordered_with_the_default_stream(robot):
    """stream=None / NULL is the device's null stream: a launch is ordered after PyTorch's default-stream writes
    of its buffers and before the reads and frees that follow.  (Round 3's illegal access and round 4's NaN panel:
    NULL used to select the engine's own non-blocking stream, which raced a 400 MB default-stream fill_.)"""
    import torch
    model = load_robot(robot)
    e = eng(robot)
    N = 20000
    d = generate(model, N, config_index=8)
    din = torch.from_numpy(channel_block(d)).cuda()
    bufs = e.alloc_device(N, EMIT_ALL)
    e.build_device(din, N, EMIT_ALL, bufs)
    torch.cuda.synchronize()
    P0, G0 = bufs["panel"][: N * e.nv].clone(), bufs["gram"].clone()
    gb = e.alloc_gram_device(N)
    e.build_gram_device(din, N, gb)
    torch.cuda.synchronize()
    H0 = gb["gram"].clone()
    for _ in range(2):
        bufs["panel"].fill_(float("nan"))
        bufs["ws"].fill_(255)
        bufs["gram"].fill_(float("nan"))
        e.build_device(din, N, EMIT_ALL, bufs)  # no synchronize: stream order alone
        assert torch.equal(bufs["panel"][: N * e.nv], P0) and torch.equal(bufs["gram"], G0)
        gb["ws"].fill_(255)
        gb["gram"].fill_(float("nan"))
        e.build_gram_device(din, N, gb)
        assert torch.equal(gb["gram"], H0)
    # a buffer freed right after the launch (the caching allocator reuses it on the same stream)
    tmp = e.alloc_device(N, EMIT_ALL)
    e.build_device(din, N, EMIT_ALL, tmp)
    del tmp
    junk = torch.full((N * e.nv, e.panel_ld), float("nan"), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    del junk


@pytest.mark.parametrize("robot,N", [("spot", 100000), ("g1_29dof", 20000)])
def test_full_size_properties(robot, N):
    import torch
    from oracle.ref_c import COracle
    model = load_robot(robot)
    e = eng(robot)
    d = generate(model, N, config_index=1)
    din = torch.from_numpy(channel_block(d)).cuda()
    bufs = e.alloc_device(N, EMIT_ALL)
    e.build_device(din, N, EMIT_ALL, bufs)
    torch.cuda.synchronize()
    panel = bufs["panel"][:, :e.panel_cols].cpu().numpy()
    G = bufs["gram"].cpu().numpy()
    # Gram == panel^T panel (fp64 on the host)
    assert rel(G, panel.T @ panel) < 1e-12
    assert np.array_equal(G, G.T)
    w = np.linalg.eigvalsh(G)
    assert w.min() >= -1e-10 * w.max()
    # linearity over shards: G(all) = G(first half) + G(second half)
    h = N // 2
    parts = []
    for s0, s1 in ((0, h), (h, N)):
        sub = {k: np.ascontiguousarray(d[k][:, s0:s1]) for k in ("q", "dq", "ddq", "tau", "contact")}
        dd = torch.from_numpy(channel_block(sub)).cuda()
        b2 = e.alloc_device(s1 - s0, EMIT_ALL)
        e.build_device(dd, s1 - s0, EMIT_ALL, b2)
        torch.cuda.synchronize()
        parts.append(b2["gram"].cpu().numpy())
    assert rel(parts[0] + parts[1], G) < 1e-12
    # sampled rows against the C oracle
    idx = np.random.default_rng(0).choice(N, 200, replace=False)
    sub = {k: np.ascontiguousarray(d[k][:, idx]) for k in ("q", "dq", "ddq", "tau", "contact")}
    o = COracle(model).build(sub["q"], sub["dq"], sub["ddq"], sub["tau"], sub["contact"], nthreads=4, gram=False)
    nv, wy, nj = model.nv, e.wy, e.nj
    for k, s in enumerate(idx):
        rows = panel[s * nv:(s + 1) * nv]
        A = np.hstack([o["Y_proj"][k * nv:(k + 1) * nv], o["B_v"][k * nv:(k + 1) * nv],
                       o["B_c"][k * nv:(k + 1) * nv], o["tau_proj"][k * nv:(k + 1) * nv, None]])
        assert rel(rows, A) < TOL


@pytest.mark.parametrize("robot,N", [("spot", 3000), ("g1_29dof", 700)])
def test_hip_graph_replay_matches_eager(robot, N):
    """The device entry points are stream-ordered and allocation-free: one step captured into a HIP graph
    (what bench.py replays) gives bitwise the eager results, replay after replay, full and Gram-only."""
    import torch
    model = load_robot(robot)
    e = eng(robot)
    d = generate(model, N, config_index=6)
    din = torch.from_numpy(channel_block(d)).cuda()
    bufs = e.alloc_device(N, EMIT_ALL)
    gb = e.alloc_gram_device(N)
    e.build_device(din, N, EMIT_ALL, bufs)
    e.build_gram_device(din, N, gb)
    torch.cuda.synchronize()
    W = e.w
    P, G, GO = bufs["panel"][: N * e.nv, : W + 1], bufs["gram"][: W + 1, : W + 1], gb["gram"][: W + 1, : W + 1]
    p0, g0, go0 = P.clone(), G.clone(), GO.clone()
    for t in (P, G, GO):  # the graph must rewrite every element the reference reads
        t.fill_(float("nan"))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        st = torch.cuda.current_stream().cuda_stream
        e.build_device(din, N, EMIT_ALL, bufs, stream=st)
        e.build_gram_device(din, N, gb, stream=st)
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(p0, P) and torch.equal(g0, G) and torch.equal(go0, GO)


@pytest.mark.parametrize("robot,N", [("spot", 50000), ("g1_29dof", 12000)])
def test_gram_only_chunked(robot, N):
    """Gram-only path (the panel produced in chunks on the device: 256 MiB chunks here, 5 of them) against
    the full-panel path, on the host API and on the device API; bitwise repeatable; the default 4 GiB chunk
    (one chunk here) gives the same Gram to rounding."""
    import torch
    model = load_robot(robot)
    e = Engine(model)
    e.set_gram_chunk_bytes(256 << 20)
    d = generate(model, N, config_index=3)
    full = e.build(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"], EMIT_ALL)
    only = e.build(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"], EMIT_GRAM)
    assert set(only) == {"gram", "Atb", "btb", "num_rows"}
    assert rel(only["gram"], full["gram"]) < 1e-12
    assert rel(only["Atb"], full["Atb"]) < 1e-12
    assert abs(only["btb"] - full["btb"]) <= 1e-12 * abs(full["btb"])
    din = torch.from_numpy(channel_block(d)).cuda()
    bufs = e.alloc_gram_device(N)
    e.build_gram_device(din, N, bufs)
    torch.cuda.synchronize()
    G1 = bufs["gram"].clone()
    # the host path chunks along its staged input DMA (each chunk's K1 starts when its inputs land): the same
    # Gram to rounding, summed in a different chunk order
    assert rel(G1[:e.w, :e.w].cpu().numpy(), only["gram"]) < 1e-12
    e.build_gram_device(din, N, bufs)
    torch.cuda.synchronize()
    assert torch.equal(G1, bufs["gram"])
    # too small a workspace is rejected, not overrun
    small = {"gram": bufs["gram"], "ws": bufs["ws"][:1024]}
    with pytest.raises(ValueError):
        e.build_gram_device(din, N, small)
    one = eng(robot).build(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"], EMIT_GRAM)
    assert rel(one["gram"], only["gram"]) < 1e-12
    with pytest.raises(ValueError):
        e.set_gram_chunk_bytes(1000)


@pytest.mark.parametrize("robot,N,chunks,ws_chunk", [("spot", 20001, 3, 0), ("spot", 4999, 2, 0), ("g1_29dof", 3001, 4, 0),
                                                    ("spot", 20001, 2, 8 << 20), ("g1_29dof", 3001, 2, 16 << 20),
                                                    ("spot", 20001, 0, 0), ("spot", 10000, 0, 0),
                                                    ("spot", 40000, 0, 64 << 20),
                                                    ("g1_29dof", 9001, 0, 0)])
def test_host_gram_only_staged_chunks(robot, N, chunks, ws_chunk):
    """Host Gram-only entry point with its inputs staged in `chunks` wire blocks (each chunk packed as its own block,
    sent as one DMA and widened by K0W into the row-major block its K1 reads), ragged last chunk, and staged chunks
    larger than the workspace's panel chunk (ws_chunk bytes: several K1 launches per staged block): the same normal
    equations as the device entry point on the row-major block, to rounding.  chunks = 0: the default bounds (a
    first chunk of one K1 round, then two chunks of whole rounds)."""
    import torch
    model = load_robot(robot)
    e = Engine(model)
    e.set_stage_chunks(chunks)
    if ws_chunk:
        e.set_gram_chunk_bytes(ws_chunk)
    d = generate(model, N, config_index=4)
    only = e.build(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"], EMIT_GRAM)
    din = torch.from_numpy(channel_block(d)).cuda()
    bufs = e.alloc_gram_device(N)
    e.build_gram_device(din, N, bufs)
    torch.cuda.synchronize()
    W = e.w
    G = bufs["gram"].cpu().numpy()
    assert rel(only["gram"], G[:W, :W]) < 1e-12
    assert rel(only["Atb"], G[:W, W]) < 1e-12
    assert abs(only["btb"] - G[W, W]) <= 1e-12 * abs(G[W, W])
    assert only["num_rows"] == N * model.nv


@pytest.mark.parametrize("flags", [EMIT_GRAM, EMIT_ALL])
def test_host_calls_restage_fresh_inputs(flags):
    """The host entry point reuses its page-locked staging block from call to call, and K0W reads the first chunk
    from it directly over PCIe: alternating calls on two different input sets of the same size (same chunk bounds,
    same staging offsets) must each give their own outputs, bitwise equal to a fresh engine's — a stale first
    chunk (cached or not yet rewritten) would return the other set's rows."""
    model = load_robot("spot")
    N = 20000
    sets = [generate(model, N, config_index=1), generate(model, N, config_index=4)]
    ins = [[x["q"].astype(np.float32), x["dq"], x["ddq"], x["tau"], x["contact"].astype(np.float32)] for x in sets]
    fresh = [Engine(model).build(*a, flags) for a in ins]
    assert not np.array_equal(fresh[0]["gram"], fresh[1]["gram"])
    e = Engine(model)
    for k in (0, 1, 0, 1, 1, 0):
        out = e.build(*ins[k], flags)
        for key in fresh[k]:
            assert np.array_equal(np.asarray(out[key]), np.asarray(fresh[k][key])), (k, key)


@pytest.mark.parametrize("robot,N", [("spot", 20001), ("g1_29dof", 3001), ("solo12", 7), ("spot", 1)])
def test_float32_q_contact_entry_point_is_bitwise_the_float64_one(robot, N):
    """sysid_build_f32qc (q and contact in float32, as read_data returns them, demo/spot_identification.py:10-14)
    against sysid_build on the same values in float64: the float32 -> float64 widening is exact and the contact
    bytes carry the non-zero test K1 applies (values 2 = LOST included), so every output is bitwise equal, stacked
    and Gram-only, large (staged chunks) and small (one inline-packed chunk)."""
    model = load_robot(robot)
    e = Engine(model)
    d = generate(model, N, config_index=7)
    assert np.any(d["contact"] == 2.0) or N < 100
    q32, c32 = d["q"].astype(np.float32), d["contact"].astype(np.float32)
    assert np.array_equal(q32.astype(np.float64), d["q"]) and np.array_equal(c32.astype(np.float64), d["contact"])
    for flags in (EMIT_ALL, EMIT_GRAM):
        a = e.build(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"], flags)
        b = e.build(q32, d["dq"], d["ddq"], d["tau"], c32, flags)
        assert set(a) == set(b)
        for k in a:
            assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), (flags, k)


@pytest.mark.parametrize("robot,N", [("spot", 3000), ("g1_29dof", 700)])
def test_tau_prediction_rmse_reduction(robot, N):
    """K4 (device reduction of the torque-prediction error) against the reference's loop over the
    oracle's stacked arrays (src/sys_identification.py:421-437), host and device forms."""
    import torch
    from system_identification_amd.sys_identification import SystemIdentification
    model = load_robot(robot)
    d = generate(model, N, config_index=4)
    s = SystemIdentification(robot, None, floating_base=True)
    phi = np.asarray(s.get_phi_prior(), dtype=np.float64)
    Y, t = ref.get_projected_y_tau(model, d["q"], d["dq"], d["ddq"], d["tau"], d["contact"])
    nv, bd = model.nv, model.base_dof
    err = ((Y @ phi) - t).reshape(N, nv)[:, bd:]
    total_ref = np.mean(np.square(np.linalg.norm(err, axis=1)))
    joint_ref = np.sqrt(np.mean(np.square(err), axis=0))
    total, joint = s.tau_prediction_rmse(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"], phi)
    assert abs(total - total_ref) <= TOL * total_ref
    assert rel(joint, joint_ref) < TOL
    e = eng(robot)
    din = torch.from_numpy(channel_block(d)).cuda()
    bufs = e.alloc_device(N, EMIT_ALL)
    e.build_device(din, N, EMIT_ALL, bufs)
    d_phi = torch.from_numpy(phi).cuda()
    d_err = torch.empty(nv, dtype=torch.float64, device="cuda")
    keep = e.tau_error_device(bufs, N, d_phi, d_err)
    torch.cuda.synchronize()
    del keep
    host_err = e.tau_error(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"], phi)
    assert np.array_equal(d_err.cpu().numpy(), host_err)  # same kernels, same order
    with pytest.raises(ValueError):
        e.tau_error(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"], phi[:-1])


@pytest.mark.parametrize("robot,N", [("spot", 20000), ("g1_29dof", 5000)])
def test_reduced_precision_gram(robot, N):
    """f32 / bf16 MFMA Grams (error reported, not gated) against the f64 Gram of the
    same panel; normwise relative error printed, bounded loosely (f32 ~1e-7, bf16 ~1e-3 expected)."""
    import torch
    model = load_robot(robot)
    e = eng(robot)
    d = generate(model, N, config_index=7)
    din = torch.from_numpy(channel_block(d)).cuda()
    out = {}
    for prec in ("f64", "f32", "bf16"):
        bufs = e.alloc_gram_device(N)
        e.build_gram_device(din, N, bufs, precision=prec)
        torch.cuda.synchronize()
        out[prec] = bufs["gram"].cpu().numpy()
    G = out["f64"]
    nrm = np.linalg.norm(G)
    errs = {p: np.linalg.norm(out[p] - G) / nrm for p in ("f32", "bf16")}
    print(f"{robot} N={N} Gram normwise rel. error: f32 {errs['f32']:.2e}  bf16 {errs['bf16']:.2e}")
    assert errs["f32"] < 1e-5
    assert errs["bf16"] < 3e-2
    assert np.array_equal(out["f32"], out["f32"].T) and np.array_equal(out["bf16"], out["bf16"].T)


@pytest.mark.parametrize("robot,N", [("spot", 20000), ("g1_29dof", 5000), ("snake14", 4000)])
def test_reduced_precision_gram_matches_rounded_panel(robot, N):
    """The f32 / bf16 Gram kernels (each with its own super-tile deal and K3 reduction) against the exact
    Gram of the panel rounded the way K1 rounds it (f64 -> f32, then -> bf16, both RNE): what remains is only
    the kernels' f32 accumulation, so the bound is tight (1e-5 normwise), unlike the error against the f64
    Gram that test_reduced_precision_gram reports.  (The Q-form models' bf16 rows come from K1's f32 row loop,
    ~1e-7 relative before the bf16 rounding: an entry near a rounding boundary may land one bf16 ulp away,
    far inside the bound.)  Gram-only output from the reference's P·A rows (the
    GRAM_PROJECTOR rows, the same rows the full path's f64 panel holds) vs that panel."""
    import torch
    model = load_robot(robot)
    e = eng(robot)
    d = generate(model, N, config_index=7)
    din = torch.from_numpy(channel_block(d)).cuda()
    bufs = e.alloc_device(N, EMIT_ALL)
    e.build_device(din, N, EMIT_ALL, bufs)
    torch.cuda.synchronize()
    p64 = bufs["panel"][:, :e.panel_cols]
    rounded = {"f32": p64.to(torch.float32).to(torch.float64),
               "bf16": p64.to(torch.float32).to(torch.bfloat16).to(torch.float64)}
    for prec, pr in rounded.items():
        ref = (pr.T @ pr).cpu().numpy()
        g = e.alloc_gram_device(N)
        e.build_gram_device(din, N, g, precision=prec, rows="projector")  # the same rows as the f64 panel
        torch.cuda.synchronize()
        G = g["gram"].cpu().numpy()
        err = np.linalg.norm(G - ref) / np.linalg.norm(ref)
        print(f"{robot} N={N} {prec} Gram vs the Gram of the {prec}-rounded panel: {err:.2e}")
        assert err < 1e-5, (prec, err)


@pytest.mark.parametrize("robot,N,cfg", [("solo12", 48, 0), ("spot", 64, 1), ("g1_29dof", 24, 2),
                                         ("solo12_fixed", 48, 3)])
def test_full_regressor_force_vs_oracle(robot, N, cfg):
    """get_full_regressor_force (:391-399) batched on the GPU against the oracle, per sample; LOST=2 values
    (whose lambda/J_c shapes disagree in the reference) are rejected."""
    from system_identification_amd.sys_identification import SystemIdentification
    model = load_robot(robot)
    d = generate(model, N, config_index=cfg)
    cnt = np.minimum(d["contact"], 1.0)
    f = np.random.default_rng(cfg).standard_normal((3 * model.n_ee, N)) * 50.0
    s = SystemIdentification(robot, None, floating_base=model.floating_base)
    Y, F = s.get_full_regressor_force(d["q"], d["dq"], d["ddq"], d["tau"], f, cnt)
    nv = model.nv
    for k in range(N):
        Yr, Fr = ref.get_full_regressor_force(model, d["q"][:, k], d["dq"][:, k], d["ddq"][:, k], d["tau"][:, k],
                                              f[:, k], cnt[:, k])
        assert rel(Y[k * nv:(k + 1) * nv], Yr) < TOL
        assert rel(F[k * nv:(k + 1) * nv], Fr) < TOL
    Y1, F1 = s.get_full_regressor_force(d["q"][:, 0], d["dq"][:, 0], d["ddq"][:, 0], d["tau"][:, 0], f[:, 0], cnt[:, 0])
    assert np.array_equal(Y1, Y[:nv]) and np.array_equal(F1, F[:nv])
    bad = cnt.copy()
    bad[0, 0] = 2.0
    with pytest.raises(ValueError):
        s.get_full_regressor_force(d["q"], d["dq"], d["ddq"], d["tau"], f, bad)


def test_rccl_gram_allreduce_single_rank():
    """sysid_allreduce_gram over a one-rank RCCL communicator is the identity on the Gram (the N > 1 path
    needs more GPUs than a test box has; its host logic is covered by the gloo tests)."""
    import torch
    from system_identification_amd.distributed import RcclGramComm
    e = eng("spot")
    N = 2000
    d = generate(load_robot("spot"), N, config_index=6)
    din = torch.from_numpy(channel_block(d)).cuda()
    bufs = e.alloc_gram_device(N)
    e.build_gram_device(din, N, bufs)
    torch.cuda.synchronize()
    G0 = bufs["gram"].clone()
    comm = RcclGramComm(e, rank=0, world=1)
    comm.allreduce_gram(bufs["gram"])
    torch.cuda.synchronize()
    assert torch.equal(G0, bufs["gram"])
    comm.close()


def test_sysid_api_and_demo_functions():
    from system_identification_amd.demo import get_projected_friction_regressors, get_projected_y_tau
    from system_identification_amd.sys_identification import SystemIdentification
    s = SystemIdentification("spot", None, floating_base=True)
    model = s.model
    d = generate(model, 20, config_index=6)
    i = 7
    Yp, tp = s.get_proj_regressor_torque(d["q"][:, i], d["dq"][:, i], d["ddq"][:, i], d["tau"][:, i], d["contact"][:, i])
    Yr, tr = ref.get_proj_regressor_torque(model, d["q"][:, i], d["dq"][:, i], d["ddq"][:, i], d["tau"][:, i],
                                           d["contact"][:, i])
    assert rel(Yp, Yr) < TOL and rel(tp, tr) < TOL
    Bv, Bc = s.get_proj_friction_regressors(d["q"][:, i], d["dq"][:, i], d["ddq"][:, i], d["contact"][:, i])
    Bvr, Bcr = ref.get_proj_friction_regressors(model, d["q"][:, i], d["dq"][:, i], d["ddq"][:, i], d["contact"][:, i])
    assert rel(Bv, Bvr) < TOL and rel(Bc, Bcr) < TOL
    Y, t = get_projected_y_tau(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"], s)
    Bv, Bc = get_projected_friction_regressors(d["q"], d["dq"], d["ddq"], d["contact"], s)
    Yr, tr = ref.get_projected_y_tau(model, d["q"], d["dq"], d["ddq"], d["tau"], d["contact"])
    assert np.vstack(Y).shape == Yr.shape and np.hstack(t).shape == tr.shape  # demo :84-87 still work
    assert rel(Y, Yr) < TOL and rel(t, tr) < TOL
    ne = s.build_normal_equations(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"])
    A = np.hstack([Y, Bv, Bc])
    assert rel(ne["gram"], A.T @ A) < 1e-12 and ne["num_rows"] == 20 * 18


def test_distributed_helper_single_rank_uses_engine():
    from system_identification_amd.distributed import build_normal_equations_distributed
    from system_identification_amd.sys_identification import SystemIdentification
    s = SystemIdentification("spot")
    d = generate(s.model, 500, config_index=7)
    ne = build_normal_equations_distributed(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"],
                                            s.build_normal_equations, rank=0, world=1)
    full = s.build_normal_equations(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"])
    assert np.array_equal(ne["gram"], full["gram"])


def test_kernel_helper_on_device():
    import ctypes
    from system_identification_amd.model import rpy_to_matrix
    lib = E.load_library()
    rng = np.random.default_rng(3)
    R = rpy_to_matrix(*rng.normal(size=3))
    t, v, a = rng.normal(size=3), rng.normal(size=6), rng.normal(size=6)
    b = np.concatenate([R.ravel(), t, v, a])
    out = np.zeros(64 * 6)
    P = ctypes.POINTER(ctypes.c_double)
    assert lib.sysid_debug_body_column_device(b.ctypes.data_as(P), out.ctypes.data_as(P)) == 0
    Fw = ref.force_act(R, t, ref.body_regressor(v, a))
    out = out.reshape(64, 6)
    for lane in range(64):
        assert np.abs(out[lane] - Fw[:, lane % 10]).max() < 1e-13


def _gram_only(e, din, N, prec="f64", rows="nullspace"):  # rows forced: "auto" picks projector for bf16
    import torch
    b = e.alloc_gram_device(N)
    e.build_gram_device(din, N, b, precision=prec, rows=rows)
    torch.cuda.synchronize()
    return b["gram"].cpu().numpy()


@pytest.mark.parametrize("robot,N,cfg", [("solo12", 2000, 0), ("spot", 20000, 1), ("g1_29dof", 5000, 2),
                                         ("solo12_fixed", 2000, 3), ("snake14", 3000, 6)])
def test_gram_only_nullspace_rows(robot, N, cfg):
    """Gram-only default: each sample contributes Zᵀ·A, its nv - rank(J_c) rows in an orthonormal basis Z of
    null(J_c) (ZᵀZ = P, Householder-completed from K1's Gram-Schmidt basis), gathered by the Gram kernels
    through k1s_row_list.  Against the reference's P·A rows (GRAM_PROJECTOR) and a sampled subset's oracle
    Gram; bitwise repeatable; f32 / bf16 errors against f64 bounded as for the projector rows."""
    import torch
    from oracle.ref_c import COracle
    model = load_robot(robot)
    e = eng(robot)
    d = generate(model, N, config_index=cfg)
    din = torch.from_numpy(channel_block(d)).cuda()
    Gz, Gp = _gram_only(e, din, N), _gram_only(e, din, N, rows="projector")
    err = rel(Gz, Gp)
    assert err < 1e-10, err
    assert np.array_equal(Gz, _gram_only(e, din, N))  # deterministic row list and summation order
    assert np.array_equal(Gz, Gz.T)
    idx = np.sort(np.random.default_rng(cfg).choice(N, 150, replace=False))
    sub = {k: np.ascontiguousarray(d[k][:, idx]) for k in ("q", "dq", "ddq", "tau", "contact")}
    o = COracle(model).build(sub["q"], sub["dq"], sub["ddq"], sub["tau"], sub["contact"], stacked=False)
    Gs = _gram_only(e, torch.from_numpy(channel_block(sub)).cuda(), len(idx))
    W = e.w
    assert rel(Gs[:W, :W], o["gram"]) < TOL and rel(Gs[:W, W], o["Atb"]) < TOL
    assert abs(Gs[W, W] - o["btb"]) <= TOL * o["btb"]
    nrm = np.linalg.norm(Gz)
    errs = {p: np.linalg.norm(_gram_only(e, din, N, prec=p) - Gz) / nrm for p in ("f32", "bf16")}
    print(f"{robot} N={N} nullspace rows: vs projector rows {err:.2e}; f32 {errs['f32']:.2e} bf16 {errs['bf16']:.2e}")
    assert errs["f32"] < 1e-5 and errs["bf16"] < 3e-2


@pytest.mark.parametrize("N", [32768, 32769, 31745])
def test_nullspace_row_list_one_and_two_launch_forms(N):
    """k1s_row_list sums the earlier segments' row counts itself for chunks of up to K1S_ONEPASS_SEGS = 32 segments
    of 1024 samples, and after k1s_seg_sums beyond: 32,768 samples (32 full segments, one launch), 32,769 (33
    segments, the last holding one sample: two launches), 31,745 (ragged 32nd segment).  Each Gram from the
    gathered nullspace rows equals the projector rows' Gram to 1e-10, bitwise repeatably."""
    import torch
    model = load_robot("spot")
    e = eng("spot")
    d = generate(model, N, config_index=4)
    din = torch.from_numpy(channel_block(d)).cuda()
    Gz, Gp = _gram_only(e, din, N), _gram_only(e, din, N, rows="projector")
    assert rel(Gz, Gp) < 1e-10
    assert np.array_equal(Gz, _gram_only(e, din, N))


def test_gram_only_nullspace_degenerate_and_ill_conditioned():
    """The nullspace rows on the hard contact cases, host entry point with EMIT_GRAM only (the Gram-only path)
    against the numpy oracle's Gram of the reference's stacked P·A (1e-6): Spot with no / all / LOST=2 /
    single feet, two contact slots on one foot (exactly dependent rows: rank 3 per duplicated pair), and
    solo12_fixed on nearly straight knees (cond(J_c) up to 5e8, exactly singular legs, and four feet down:
    J_c square and invertible, so a sample contributes no row at all)."""
    import copy
    model = load_robot("spot")
    d = generate(model, 6, config_index=4)
    cnt = np.stack([np.zeros(4), np.ones(4), 2 * np.ones(4), np.array([2, 0, 0, 0.0]), np.array([0, 0, 0, 1.0]),
                    np.array([1, 2, 0, 1.0])], axis=1)
    cases = [(model, eng("spot"), d, cnt)]
    dup = copy.deepcopy(load_robot("spot"))
    dup.end_effector_names[1] = dup.end_effector_names[0]
    d2 = generate(dup, 16, config_index=2)
    c2 = np.ones((4, 16))
    c2[2:, ::2] = 0.0
    cases.append((dup, Engine(dup), d2, c2))
    fx = load_robot("solo12_fixed")
    knees = [i for i, n in enumerate(fx.joint_names) if n.endswith("KFE")]
    eps = [1e-2, 1e-4, 1e-6, 1e-8, 0.0]
    pats = [[1, 1, 1, 0], [1, 0, 2, 0], [1, 1, 1, 1], [0, 1, 1, 1]]
    n = len(eps) * len(pats)
    d3 = generate(fx, n, config_index=3)
    c3 = np.zeros((4, n))
    for s in range(n):
        for j in knees:
            d3["q"][fx.idx_q[j], s] = eps[s % len(eps)]
        c3[:, s] = pats[s // len(eps)]
    cases.append((fx, eng("solo12_fixed"), d3, c3))
    for m, e, dd, c in cases:
        only = e.build(dd["q"], dd["dq"], dd["ddq"], dd["tau"], c, EMIT_GRAM)
        Y, t = ref.get_projected_y_tau(m, dd["q"], dd["dq"], dd["ddq"], dd["tau"], c)
        Bv, Bc = ref.get_projected_friction_regressors(m, dd["q"], dd["dq"], dd["ddq"], c)
        G, g, btb, rows = ref.normal_equations(Y, t, Bv, Bc)
        assert rel(only["gram"], G) < TOL and rel(only["Atb"], g) < TOL, m.robot_name
        assert abs(only["btb"] - btb) <= TOL * abs(btb) and only["num_rows"] == rows


@pytest.mark.parametrize("robot,N,cfg", [("spot", 20000, 1), ("solo12", 5000, 0)])
def test_narrow_gram_degenerate_start(robot, N, cfg):
    """The narrow f64 Gram (k2_gram_syrk, 10 tile columns, one workgroup per CU) of a panel whose first samples
    carry the degenerate contact patterns: against panelᵀ·panel of the returned panel, a second engine's build
    (bitwise: the deal and the split are fixed at model creation) and a second call (bitwise)."""
    model = load_robot(robot)
    es = eng(robot)
    assert es.k2_config()[0] == 10
    ed = Engine(model)
    d = generate(model, N, config_index=cfg)
    cnt = d["contact"].copy()
    cnt[:, :6] = np.stack([np.zeros(4), np.ones(4), 2 * np.ones(4), [2, 0, 0, 0.0], [0, 0, 0, 1.0],
                           [1, 2, 0, 1.0]], axis=1)  # degenerate patterns at the start
    a = es.build(d["q"], d["dq"], d["ddq"], d["tau"], cnt, EMIT_ALL)
    b = ed.build(d["q"], d["dq"], d["ddq"], d["tau"], cnt, EMIT_ALL)
    assert np.array_equal(a["Y_proj"], b["Y_proj"]) and np.array_equal(a["B_c"], b["B_c"])
    A = np.hstack([a["Y_proj"], a["B_v"], a["B_c"], a["tau_proj"][:, None]])
    G = np.block([[a["gram"], a["Atb"][:, None]], [a["Atb"][None, :], np.array([[a["btb"]]])]])
    ref_g = A.T @ A
    err = rel(G, ref_g)
    print(f"{robot} {N}: Gram vs panel^T panel {err:.2e}")
    assert err < 1e-12
    assert np.array_equal(a["gram"], b["gram"]) and np.array_equal(a["Atb"], b["Atb"]) and a["btb"] == b["btb"]
    assert np.array_equal(a["gram"], a["gram"].T)
    # bitwise reproducible
    a2 = es.build(d["q"], d["dq"], d["ddq"], d["tau"], cnt, EMIT_ALL)
    assert np.array_equal(a["gram"], a2["gram"]) and np.array_equal(a["Atb"], a2["Atb"])


def test_solo12_gram_ill_conditioned_contacts():
    """solo12 (floating base) on nearly straight legs, cond(J_c) up to ~5e8, with partial, value-2 and full
    contact patterns: the Gram stays within the parity bar of the oracle's."""
    model = load_robot("solo12")
    knees = [i for i, n in enumerate(model.joint_names) if n.endswith("KFE")]
    eps = [1e-2, 1e-4, 1e-6, 1e-8, 0.0]
    pats = [[1, 1, 1, 0], [1, 0, 2, 0], [1, 1, 1, 1], [0, 1, 1, 1]]
    n = len(eps) * len(pats)
    d = generate(model, n, config_index=3)
    cnt = np.zeros((4, n))
    for s in range(n):
        for j in knees:
            d["q"][model.idx_q[j], s] = eps[s % len(eps)]
        cnt[:, s] = pats[s // len(eps)]
    out = eng("solo12").build(d["q"], d["dq"], d["ddq"], d["tau"], cnt, EMIT_ALL)
    Y, t = ref.get_projected_y_tau(model, d["q"], d["dq"], d["ddq"], d["tau"], cnt)
    Bv, Bc = ref.get_projected_friction_regressors(model, d["q"], d["dq"], d["ddq"], cnt)
    G, g, btb, _ = ref.normal_equations(Y, t, Bv, Bc)
    assert rel(out["gram"], G) < TOL and rel(out["Atb"], g) < TOL
    assert abs(out["btb"] - btb) <= TOL * abs(btb)
