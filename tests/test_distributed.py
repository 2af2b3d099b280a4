"""Multi-rank normal equations on CPU (gloo, world_size 2): sharding + one all-reduce reproduces the
single-process Gram.  The per-rank compute is the C oracle here; on the GPU box it
is the HIP engine (same host code, system_identification_amd/distributed.py)."""
import os
import socket

import numpy as np
import pytest

from system_identification_amd.distributed import (pack_normal_equations, shard_range, unpack_normal_equations)


def test_shard_range_covers_all_samples():
    for N in (0, 1, 7, 20000, 200001):
        for W in (1, 2, 3, 8):
            r = [shard_range(N, k, W) for k in range(W)]
            assert r[0][0] == 0 and r[-1][1] == N
            assert all(r[k][1] == r[k + 1][0] for k in range(W - 1))
            assert max(b - a for a, b in r) - min(b - a for a, b in r) <= 1


def test_pack_round_trip():
    rng = np.random.default_rng(0)
    A = rng.normal(size=(50, 7))
    b = rng.normal(size=50)
    ne = {"gram": A.T @ A, "Atb": A.T @ b, "btb": float(b @ b), "num_rows": 50}
    buf, rows = pack_normal_equations(ne)
    back = unpack_normal_equations(buf, rows)
    assert np.array_equal(back["gram"], ne["gram"]) and back["btb"] == ne["btb"] and back["num_rows"] == 50


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, robot, N, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    from oracle.ref_c import COracle
    from system_identification_amd.distributed import build_normal_equations_distributed
    from system_identification_amd.model import load_robot
    from system_identification_amd.synthetic import generate
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = load_robot(robot)
    d = generate(m, N, config_index=3)
    orc = COracle(m)

    def partial(q, dq, ddq, tau, cnt):
        o = orc.build(q, dq, ddq, tau, cnt, nthreads=1, stacked=False)
        return {"gram": o["gram"], "Atb": o["Atb"], "btb": o["btb"], "num_rows": q.shape[1] * m.nv}

    ne = build_normal_equations_distributed(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"], partial, rank, world)
    if rank == 0:
        np.savez(out_path, **ne)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_ranks_match_single_process(tmp_path):
    import torch.multiprocessing as mp
    from oracle.ref_c import COracle
    from system_identification_amd.model import load_robot
    from system_identification_amd.synthetic import generate
    robot, N = "spot", 301
    out = str(tmp_path / "ne.npz")
    mp.start_processes(_worker, args=(2, _free_port(), robot, N, out), nprocs=2, start_method="spawn")
    got = dict(np.load(out))
    m = load_robot(robot)
    d = generate(m, N, config_index=3)
    ref = COracle(m).build(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"], nthreads=1, stacked=False)
    assert int(got["num_rows"]) == N * m.nv
    assert np.abs(got["gram"] - ref["gram"]).max() <= 1e-12 * np.abs(ref["gram"]).max()
    assert np.abs(got["Atb"] - ref["Atb"]).max() <= 1e-12 * np.abs(ref["Atb"]).max()
    assert abs(float(got["btb"]) - ref["btb"]) <= 1e-12 * ref["btb"]


def _worker_uneven(rank, world, port, robot, splits, out_path):
    """Each rank holds a shard of a DIFFERENT size (e.g. the tail rank of an uneven split) and exchanges the
    packed (W+1)^2 buffer + row count through allreduce_normal_equations."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    from oracle.ref_c import COracle
    from system_identification_amd.distributed import allreduce_normal_equations
    from system_identification_amd.model import load_robot
    from system_identification_amd.synthetic import generate
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = load_robot(robot)
    d = generate(m, splits[-1], config_index=5)
    s0, s1 = splits[rank], splits[rank + 1]
    o = COracle(m).build(*[d[k][:, s0:s1] for k in ("q", "dq", "ddq", "tau", "contact")], nthreads=1, stacked=False)
    ne = {"gram": o["gram"], "Atb": o["Atb"], "btb": o["btb"], "num_rows": (s1 - s0) * m.nv}
    out = allreduce_normal_equations(ne)
    np.savez(out_path + f".{rank}.npz", **out)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_uneven_shards_allreduce(tmp_path):
    import torch.multiprocessing as mp
    from oracle.ref_c import COracle
    from system_identification_amd.model import load_robot
    from system_identification_amd.synthetic import generate
    robot, splits = "spot", [0, 37, 260]  # 37 and 223 samples
    out = str(tmp_path / "ne")
    mp.start_processes(_worker_uneven, args=(2, _free_port(), robot, splits, out), nprocs=2, start_method="spawn")
    m = load_robot(robot)
    d = generate(m, splits[-1], config_index=5)
    ref = COracle(m).build(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"], nthreads=1, stacked=False)
    got = [dict(np.load(out + f".{r}.npz")) for r in range(2)]
    for g in got:  # every rank holds the full normal equations, with the exact total row count
        assert int(g["num_rows"]) == splits[-1] * m.nv
        assert np.abs(g["gram"] - ref["gram"]).max() <= 1e-12 * np.abs(ref["gram"]).max()
        assert np.abs(g["Atb"] - ref["Atb"]).max() <= 1e-12 * np.abs(ref["Atb"]).max()
        assert abs(float(g["btb"]) - ref["btb"]) <= 1e-12 * ref["btb"]
    assert np.array_equal(got[0]["gram"], got[1]["gram"])


def test_row_count_survives_the_float_buffer():
    """The row count rides in the all-reduced float64 buffer: exact for any count below 2^53, through
    allreduce_normal_equations itself (a one-rank gloo group)."""
    import tempfile
    import torch.distributed as dist
    from system_identification_amd.distributed import allreduce_normal_equations
    ne = {"gram": np.eye(3), "Atb": np.arange(3.0), "btb": 2.5, "num_rows": 2 ** 40 + 12345}
    with tempfile.TemporaryDirectory() as tmp:
        dist.init_process_group("gloo", init_method=f"file://{tmp}/rdv", rank=0, world_size=1)
        try:
            out = allreduce_normal_equations(ne)
        finally:
            dist.destroy_process_group()
    assert out["num_rows"] == 2 ** 40 + 12345 and isinstance(out["num_rows"], int)
    assert np.array_equal(out["gram"], ne["gram"]) and np.array_equal(out["Atb"], ne["Atb"]) and out["btb"] == 2.5


def test_packed_upper_triangle_layout():
    """pack_upper is the device exchange format (xchg_pack: row i of the upper triangle at i n - i (i - 1) / 2,
    the row count last): §8e's 12,091 doubles for Spot and 64,621 for G1, n = W + 1 of the real models (the Gram
    the engine exchanges, sysid_exchange_bytes; not the padded panel stride), and a bitwise-symmetric unpack."""
    from system_identification_amd.distributed import pack_upper, unpack_upper
    from system_identification_amd.model import load_robot
    for robot, want in (("spot", 12091), ("g1_29dof", 64621)):
        m = load_robot(robot)
        n = 10 * m.nb + 2 * m.nj + 1  # W + 1 (SURVEY §8 notation: W = 10 nb + 2 nj)
        assert n == {"spot": 155, "g1_29dof": 359}[robot]
        rng = np.random.default_rng(n)
        A = rng.normal(size=(n + 5, n))
        G = A.T @ A
        x = pack_upper(G, 17)
        assert x.size == want
        for i in (0, 1, n // 2, n - 1):
            off = i * n - i * (i - 1) // 2
            assert np.array_equal(x[off:off + n - i], G[i, i:])
        back, rows = unpack_upper(x, n)
        assert rows == 17 and np.array_equal(back, back.T) and np.array_equal(np.triu(back), np.triu(G))


class _StubLib:
    """The five RCCL entry points of libsysid.so as RcclGramComm calls them (ctypes-style arguments), with
    scripted failures; records what it was given."""

    def __init__(self, fail_id=False, fail_init=False):
        self.fail_id, self.fail_init = fail_id, fail_init
        self.init_ids, self.destroyed = [], 0

    def sysid_rccl_unique_id(self, buf):
        if self.fail_id:
            return -3
        buf.raw = bytes((7 * k + 3) % 256 for k in range(128))
        return 0

    def sysid_rccl_last_error(self):
        return b"stub: scripted failure"

    def sysid_rccl_comm_init(self, comm_ref, world, uid, rank, device):
        self.init_ids.append(bytes(uid.raw))
        if self.fail_init:
            return -3
        comm_ref._obj.value = 4096 + rank
        return 0

    def sysid_rccl_comm_destroy(self, comm):
        self.destroyed += 1
        return 0


def _worker_exchange(rank, world, port, scenario, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import json
    import torch
    import torch.distributed as dist
    from system_identification_amd.distributed import make_gram_exchange
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = _StubLib(fail_id=(scenario == "id_fails" and rank == 0), fail_init=(scenario == "init_fails" and rank == 1))

    class Eng:
        pass
    eng = Eng()
    eng.lib, eng.device, eng._h = lib, 0, None

    def share_id(raw):
        box = [raw if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        return box[0]

    def all_ok(flag):
        t = torch.tensor([int(flag)], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return int(t.item()) == 1
    comm, name = make_gram_exchange(eng, rank, world, share_id, all_ok)
    with open(out_path + f".{rank}.json", "w") as f:
        json.dump({"comm": comm is not None, "name": name, "ids": [i.hex() for i in lib.init_ids],
                   "destroyed": lib.destroyed}, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("scenario", ["ok", "init_fails", "id_fails"])
def test_rccl_exchange_setup_world2(tmp_path, scenario):
    """RcclGramComm's id sharing and bench.py's fallback (distributed.make_gram_exchange) on two gloo ranks with a
    stub library: every rank initialises with rank 0's 128-byte id; if the C-ABI set-up fails on any rank, EVERY
    rank falls back to torch.distributed (and a communicator that did come up is destroyed)."""
    import json
    import torch.multiprocessing as mp
    out = str(tmp_path / "x")
    mp.start_processes(_worker_exchange, args=(2, _free_port(), scenario, out), nprocs=2, start_method="spawn")
    r = [json.load(open(out + f".{k}.json")) for k in range(2)]
    want_id = bytes((7 * k + 3) % 256 for k in range(128)).hex()
    if scenario == "ok":
        assert all(x["comm"] for x in r) and all(x["ids"] == [want_id] for x in r)
        assert all("sysid_allreduce_normal_equations" in x["name"] for x in r)
    elif scenario == "init_fails":
        assert not any(x["comm"] for x in r)
        assert r[0]["ids"] == [want_id] and r[1]["ids"] == [want_id]
        assert r[0]["destroyed"] == 1 and "another rank" in r[0]["name"]
        assert "init failed" in r[1]["name"]
    else:  # rank 0 has no id: nobody calls comm_init, both fall back
        assert not any(x["comm"] for x in r) and all(x["ids"] == [] for x in r)
        assert all("init failed" in x["name"] for x in r)


def test_rccl_exchange_checks_buffers_before_the_c_call():
    """RcclGramComm hands raw pointers to the C ABI, which trusts the sizes: the wrapper refuses a Gram that is not
    (W+1)^2 float64 elements on the engine's device, and an exchange buffer that is not sysid_exchange_bytes long,
    before any C call (an out-of-bounds read / write otherwise)."""
    import torch
    from system_identification_amd.distributed import RcclGramComm

    class _Lib:
        calls = 0

        def sysid_exchange_bytes(self, h):
            return (155 * 156 // 2 + 1) * 8

        def sysid_allreduce_normal_equations(self, *a):
            _Lib.calls += 1
            return 0

        def sysid_allreduce_gram(self, *a):
            _Lib.calls += 1
            return 0

    class _Eng:
        w, device, _h = 154, 0, None

    comm = RcclGramComm.__new__(RcclGramComm)
    comm.lib, comm.engine, comm._comm = _Lib(), _Eng(), None
    good_cpu = torch.zeros(155 * 155, dtype=torch.float64)  # right size, wrong device (no GPU here)
    with pytest.raises(ValueError, match="gram"):
        comm.allreduce_gram(torch.zeros(155 * 154, dtype=torch.float64))
    with pytest.raises(ValueError, match="gram"):
        comm.allreduce_gram(good_cpu.float())
    with pytest.raises(ValueError, match="gram"):
        comm.allreduce_normal_equations(good_cpu, 10.0, torch.zeros(12091, dtype=torch.float64))
    assert _Lib.calls == 0
