"""GPU tests at BASELINE.json's one-GPU configurations and of the launch contract.

* config 1: Solo-12, 2k samples, through the reference's own flow (demo/solo_identification.py:57-91): .dat
  logs written in the reference format, read_data with the Butterworth filter, the batched
  get_projected_y_tau / get_projected_friction_regressors, the Gram, the llsq solve and the RMSE report;
  every stacked array is compared with the C oracle on the same filtered arrays (and a slice with the numpy
  oracle), at north_star's 1e-6.
* config 4's per-GPU shard: Spot 25k (200k / 8) full outputs, through the device and the host entry points.
* config 4 whole on one GPU: Spot 200k full outputs (4.5 GB panel): sampled C-oracle rows, Gram ==
  panelᵀ·panel, and Gram == the sum of the 8 contiguous shard Grams the 8-GPU all-reduce adds.
* config 5's per-GPU share: G1 125k Gram-only in f64 / f32 / bf16 (1M samples / 8 GPUs).
* config 5 whole on one GPU: G1 1M Gram-only in f64 (== the sum of its 8 shard Grams, a sampled subset
  against the oracle's Gram) and in f32 / bf16 (errors against f64 reported).
* launch state: concurrent launches on two streams, a rejected launch, a corrupted counter."""
import numpy as np
import pytest

from oracle import ref_numpy as ref
from oracle.ref_c import COracle
from system_identification_amd.engine import EMIT_ALL, EMIT_GRAM, Engine
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import channel_block, generate
from tests.parity import rel as rel_floor
from tests.parity import unprojected_scales

pytestmark = pytest.mark.gpu

TOL = 1e-6
CH = ("q", "dq", "ddq", "tau", "contact")


def rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


def check_stacked_vs_oracle(model, out, o, ins, idx=None):
    """Per-sample blocks against the oracle's stacked arrays (relative to the block scale, tests/parity.py)."""
    nv = model.nv
    scales = unprojected_scales(model, *ins[:4])
    for s in (range(len(scales)) if idx is None else idx):
        sl = slice(s * nv, (s + 1) * nv)
        sc = scales[s]
        for name, k in (("Y_proj", 0), ("tau_proj", 1), ("B_v", 2), ("B_c", 3)):
            assert rel_floor(out[name][sl], o[name][sl], sc[k]) < TOL, (name, s)


def test_solo12_2k_reference_flow(tmp_path, capsys):
    """BASELINE config 1 end to end on the HIP path (demo/solo_identification.py:57-91)."""
    from system_identification_amd import demo
    from system_identification_amd.datio import read_data, write_dat
    from system_identification_amd.solver import Solver
    from system_identification_amd.sys_identification import SystemIdentification
    model = load_robot("solo12")
    N = 2000
    d = generate(model, N, config_index=0)
    write_dat(str(tmp_path), "solo", d)  # the reference's file names: solo_robot_{q,dq,ddq,tau,contact}.dat
    q, dq, ddq, tau, cnt = read_data(str(tmp_path), "solo", "butterworth")
    assert q.dtype == np.float32 and dq.dtype == np.float64 and q.shape == (model.nq, N)
    s = SystemIdentification("solo12", None, floating_base=True)
    Y, t = demo.get_projected_y_tau(q, dq, ddq, tau, cnt, s)
    Bv, Bc = demo.get_projected_friction_regressors(q, dq, ddq, cnt, s)
    Y, t, Bv, Bc = np.vstack(Y), np.hstack(t), np.vstack(Bv), np.vstack(Bc)  # demo :84-87
    ins = [np.asarray(a, dtype=np.float64) for a in (q, dq, ddq, tau, cnt)]
    o = COracle(model).build(*ins, nthreads=8)
    out = {"Y_proj": Y, "tau_proj": t, "B_v": Bv, "B_c": Bc}
    check_stacked_vs_oracle(model, out, o, ins)
    # the numpy oracle (the reference's own per-sample structure) on a slice pins the C oracle here too
    sl = slice(0, 64)
    Yr, tr = ref.get_projected_y_tau(model, *[a[:, sl] for a in ins])
    assert rel(Y[: 64 * model.nv], Yr) < TOL and rel(t[: 64 * model.nv], tr) < TOL
    ne = s.build_normal_equations(q, dq, ddq, tau, cnt)
    assert rel(ne["gram"], o["gram"]) < TOL and rel(ne["Atb"], o["Atb"]) < TOL
    assert abs(ne["btb"] - o["btb"]) <= TOL * o["btb"] and ne["num_rows"] == N * model.nv
    # the demo's solve, from the Gram, against the reference solver on the oracle's stacked arrays
    phi = demo.main(["--robot", "solo12", "--data", str(tmp_path), "--name", "solo", "--solver", "llsq"])
    printed = capsys.readouterr().out
    assert "Identified" in printed and "Prior" in printed
    phi_ref = Solver(o["Y_proj"], o["tau_proj"], s.get_num_links(), s.get_phi_prior(), s.get_robot_mass(),
                     None).solve_llsq_svd()
    pred, pred_ref = o["Y_proj"] @ phi, o["Y_proj"] @ phi_ref
    assert np.linalg.norm(pred - pred_ref) <= 1e-6 * np.linalg.norm(pred_ref)


@pytest.mark.parametrize("robot,N", [("spot", 25000)])
def test_config4_shard_full_outputs(robot, N):
    """Config 4's per-GPU shard (Spot 200k over 8 GPUs): device panel, host entry point (device de-interleave
    + contiguous copies) and sampled C-oracle rows."""
    import torch
    model = load_robot(robot)
    e = Engine(model)
    d = generate(model, N, config_index=11)
    din = torch.from_numpy(channel_block(d)).cuda()
    bufs = e.alloc_device(N, EMIT_ALL)
    e.build_device(din, N, EMIT_ALL, bufs)
    torch.cuda.synchronize()
    v = {k: x.cpu().numpy() for k, x in e.views(bufs, N).items() if k != "btb"}
    host = e.build(*[d[k] for k in CH], EMIT_ALL)
    for k in ("Y_proj", "tau_proj", "B_v", "B_c", "gram", "Atb"):
        assert np.array_equal(host[k], v[k]), k  # the host path returns exactly the device results
    idx = np.sort(np.random.default_rng(1).choice(N, 256, replace=False))
    sub = [np.ascontiguousarray(d[k][:, idx]) for k in CH]
    o = COracle(model).build(*sub, nthreads=8, gram=False)
    nv = model.nv
    rows = np.concatenate([np.arange(s * nv, (s + 1) * nv) for s in idx])
    out = {k: host[k][rows] for k in ("Y_proj", "tau_proj", "B_v", "B_c")}
    check_stacked_vs_oracle(model, out, o, sub)


def _shard_gram_sum(e, din, N, world, gram_only, prec="f64"):
    """The Grams of the `world` contiguous shards (distributed.shard_range), summed in rank order: what the
    all-reduce of BASELINE configs 4 / 5 adds up on 8 GPUs."""
    import torch
    from system_identification_amd.distributed import shard_range
    total = None
    for r in range(world):
        s0, s1 = shard_range(N, r, world)
        n = s1 - s0
        if gram_only:
            b = e.alloc_gram_device(n)
            e.build_gram_device(din[:, s0:s1], n, b, precision=prec)
        else:
            b = e.alloc_device(n, EMIT_ALL)
            e.build_device(din[:, s0:s1], n, EMIT_ALL, b)
        torch.cuda.synchronize()
        g = b["gram"].cpu().numpy()
        total = g if total is None else total + g
        del b
    return total


def test_config4_spot_200k_whole():
    """BASELINE config 4 (Spot 200k) whole on one GPU, full outputs: sampled rows against the C oracle at
    1e-6, Gram == panelᵀ·panel (device fp64 GEMM), and Gram == the sum of the 8 contiguous shard Grams to
    1e-12 -- the exact algebra the 8-GPU all-reduce relies on."""
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
    assert np.array_equal(G, G.T)
    P = bufs["panel"][:, : e.panel_cols]
    Gref = (P.T @ P).cpu().numpy()
    err_pp = rel(G, Gref)
    parts = _shard_gram_sum(e, din, N, 8, gram_only=False)
    err_sh = rel(parts, G)
    print(f"Spot 200k: Gram vs panel^T panel {err_pp:.2e}, vs the sum of 8 shard Grams {err_sh:.2e}")
    assert err_pp < 1e-12 and err_sh < 1e-12
    idx = np.sort(np.random.default_rng(4).choice(N, 256, replace=False))
    nv = model.nv
    rows = torch.from_numpy(np.concatenate([np.arange(s * nv, (s + 1) * nv) for s in idx])).cuda()
    panel_rows = bufs["panel"].index_select(0, rows).cpu().numpy()
    del bufs, P
    sub = [np.ascontiguousarray(d[k][:, idx]) for k in CH]
    o = COracle(model).build(*sub, nthreads=8, gram=False)
    wy, nj, W = e.wy, e.nj, e.w
    out = {"Y_proj": panel_rows[:, :wy], "B_v": panel_rows[:, wy:wy + nj], "B_c": panel_rows[:, wy + nj:W],
           "tau_proj": panel_rows[:, W]}
    check_stacked_vs_oracle(model, out, o, sub)


def test_config5_g1_1m_whole_gram_only():
    """BASELINE config 5 (G1 1M) whole on one GPU, Gram-only: f64 == the sum of the 8 shard Grams (1e-12), a
    sampled subset's Gram against the oracle (1e-6); f32 / bf16 at 1M with their normwise errors against f64
    printed (reported, not gated: north_star), and each reduced precision also summed over the 8 shards."""
    import torch
    model = load_robot("g1_29dof")
    e = Engine(model)
    N = 1000000
    d = generate(model, N, config_index=5)
    din = torch.from_numpy(channel_block(d)).cuda()
    G = {}
    for prec in ("f64", "f32", "bf16"):
        b = e.alloc_gram_device(N)
        e.build_gram_device(din, N, b, precision=prec)
        torch.cuda.synchronize()
        G[prec] = b["gram"].cpu().numpy()
        del b
    G64 = G["f64"]
    assert np.array_equal(G64, G64.T)
    err_sh = rel(_shard_gram_sum(e, din, N, 8, gram_only=True), G64)
    w = np.linalg.eigvalsh(G64)
    assert w.min() >= -1e-10 * w.max()
    idx = np.sort(np.random.default_rng(5).choice(N, 96, replace=False))
    sub = [np.ascontiguousarray(d[k][:, idx]) for k in CH]
    o = COracle(model).build(*sub, nthreads=8, stacked=False)
    dsub = torch.from_numpy(channel_block(dict(zip(CH, sub)))).cuda()
    b = e.alloc_gram_device(len(idx))
    e.build_gram_device(dsub, len(idx), b)
    torch.cuda.synchronize()
    Gs = b["gram"].cpu().numpy()
    W = e.w
    err_o = max(rel(Gs[:W, :W], o["gram"]), rel(Gs[:W, W], o["Atb"]))
    nrm = np.linalg.norm(G64)
    errs = {p: float(np.linalg.norm(G[p] - G64) / nrm) for p in ("f32", "bf16")}
    sh = {p: rel(_shard_gram_sum(e, din, N, 8, gram_only=True, prec=p), G[p]) for p in ("f32", "bf16")}
    print(f"G1 1M Gram-only: f64 vs the sum of 8 shard Grams {err_sh:.2e}, sampled subset vs oracle {err_o:.2e}; "
          f"normwise error vs f64: f32 {errs['f32']:.2e} bf16 {errs['bf16']:.2e}; "
          f"shard sums f32 {sh['f32']:.2e} bf16 {sh['bf16']:.2e}")
    assert err_sh < 1e-12 and err_o < TOL
    assert errs["f32"] < 1e-5 and errs["bf16"] < 3e-2
    assert sh["f32"] < 1e-5 and sh["bf16"] < 1e-3


def test_host_entry_point_odd_friction_width():
    """G1 (nj = 29, odd): the 8-byte friction columns of the de-interleave; host == device bitwise."""
    import torch
    model = load_robot("g1_29dof")
    e = Engine(model)
    N = 333
    d = generate(model, N, config_index=12)
    din = torch.from_numpy(channel_block(d)).cuda()
    bufs = e.alloc_device(N, EMIT_ALL)
    e.build_device(din, N, EMIT_ALL, bufs)
    torch.cuda.synchronize()
    v = {k: x.cpu().numpy() for k, x in e.views(bufs, N).items() if k != "btb"}
    host = e.build(*[d[k] for k in CH], EMIT_ALL)
    for k in ("Y_proj", "tau_proj", "B_v", "B_c"):
        assert np.array_equal(host[k], v[k]), k
    only_t = e.build(*[d[k] for k in CH], 2)  # EMIT_TAU alone
    assert set(only_t) == {"tau_proj"} and np.array_equal(only_t["tau_proj"], v["tau_proj"])


def test_config5_share_gram_only_precisions():
    """Config 5's per-GPU share (G1 1M over 8 GPUs = 125k): Gram-only in f64, f32 and bf16.  f64: linearity
    over two uneven shards (chunk boundaries fall elsewhere), a sampled subset against the oracle's Gram,
    symmetry; f32 / bf16: normwise error against f64, reported (north_star: reported, not gated)."""
    import torch
    model = load_robot("g1_29dof")
    e = Engine(model)
    N = 125000
    d = generate(model, N, config_index=4)
    din = torch.from_numpy(channel_block(d)).cuda()
    G = {}
    for prec in ("f64", "f32", "bf16"):
        b = e.alloc_gram_device(N)
        e.build_gram_device(din, N, b, precision=prec)
        torch.cuda.synchronize()
        G[prec] = b["gram"].cpu().numpy()
        del b
    G64 = G["f64"]
    assert np.array_equal(G64, G64.T)
    h = 47011
    parts = []
    for s0, s1 in ((0, h), (h, N)):
        b = e.alloc_gram_device(s1 - s0)
        e.build_gram_device(din[:, s0:], s1 - s0, b)
        torch.cuda.synchronize()
        parts.append(b["gram"].cpu().numpy())
        del b
    assert rel(parts[0] + parts[1], G64) < 1e-12
    idx = np.sort(np.random.default_rng(2).choice(N, 96, replace=False))
    sub = [np.ascontiguousarray(d[k][:, idx]) for k in CH]
    o = COracle(model).build(*sub, nthreads=8, stacked=False)
    dsub = torch.from_numpy(channel_block(dict(zip(CH, sub)))).cuda()
    b = e.alloc_gram_device(len(idx))
    e.build_gram_device(dsub, len(idx), b)
    torch.cuda.synchronize()
    Gs = b["gram"].cpu().numpy()
    W = e.w
    assert rel(Gs[:W, :W], o["gram"]) < TOL and rel(Gs[:W, W], o["Atb"]) < TOL
    nrm = np.linalg.norm(G64)
    errs = {p: float(np.linalg.norm(G[p] - G64) / nrm) for p in ("f32", "bf16")}
    print(f"G1 125k Gram-only normwise error vs f64: f32 {errs['f32']:.2e}  bf16 {errs['bf16']:.2e}")
    assert errs["f32"] < 1e-5 and errs["bf16"] < 3e-2


def test_two_streams_concurrent_launches_bitwise():
    """Per-launch state lives in the caller's workspace: one handle, two streams, two workspaces, launches
    interleaved without host synchronisation — each result equals the sequential one bit for bit."""
    import torch
    model = load_robot("spot")
    e = Engine(model)
    N = 6000
    d1, d2 = generate(model, N, config_index=13), generate(model, N, config_index=14)
    x1, x2 = (torch.from_numpy(channel_block(x)).cuda() for x in (d1, d2))
    b1, b2 = e.alloc_device(N, EMIT_ALL), e.alloc_device(N, EMIT_ALL)
    e.build_device(x1, N, EMIT_ALL, b1)
    e.build_device(x2, N, EMIT_ALL, b2)
    torch.cuda.synchronize()
    ref1, ref2 = b1["panel"].clone(), b2["panel"].clone()
    g1, g2 = b1["gram"].clone(), b2["gram"].clone()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(4):
        b1["panel"].fill_(float("nan"))
        b2["panel"].fill_(float("nan"))
        torch.cuda.synchronize()
        for _ in range(3):
            e.build_device(x1, N, EMIT_ALL, b1, stream=s1.cuda_stream)
            e.build_device(x2, N, EMIT_ALL, b2, stream=s2.cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(b1["panel"], ref1) and torch.equal(b2["panel"], ref2)
        assert torch.equal(b1["gram"], g1) and torch.equal(b2["gram"], g2)


def test_rejected_launch_enqueues_nothing_and_counter_is_reset():
    """An argument error returns before any enqueue (the panel is untouched), and a workspace whose counter
    holds garbage (an aborted launch) still gives the correct result: the counter is zeroed per launch."""
    import torch
    from system_identification_amd import engine as E
    model = load_robot("spot")
    e = Engine(model)
    N = 3000
    d = generate(model, N, config_index=15)
    din = torch.from_numpy(channel_block(d)).cuda()
    bufs = e.alloc_device(N, EMIT_ALL)
    e.build_device(din, N, EMIT_ALL, bufs)
    torch.cuda.synchronize()
    P0, G0 = bufs["panel"].clone(), bufs["gram"].clone()
    bufs["panel"].fill_(-7.0)
    torch.cuda.synchronize()
    import ctypes
    short = int(e.workspace_bytes(N, EMIT_ALL)) - 1024
    rc = e.lib.sysid_build_device(e._h, ctypes.c_void_p(din.data_ptr()), N, din.stride(0), EMIT_ALL,
                                  ctypes.c_void_p(bufs["panel"].data_ptr()), bufs["panel"].stride(0),
                                  ctypes.c_void_p(bufs["gram"].data_ptr()), ctypes.c_void_p(bufs["ws"].data_ptr()),
                                  short, None)
    assert rc == E.SYSID_E_INVALID
    torch.cuda.synchronize()
    assert bool((bufs["panel"] == -7.0).all())  # nothing ran
    bufs["ws"][:1024].fill_(0xA5)  # counters left mid-count by an aborted launch
    e.build_device(din, N, EMIT_ALL, bufs)
    torch.cuda.synchronize()
    assert torch.equal(bufs["panel"], P0) and torch.equal(bufs["gram"], G0)
    with pytest.raises(ValueError):  # more samples than the input block holds: caught before the C call
        e.build_device(din[:, : N // 2], N, EMIT_ALL, bufs)
