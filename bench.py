"""Benchmark: regressor + projector + Gram build on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--robot spot] [--samples 20000 | --total-samples T]
                    [--gram-only [--precision f64|f32|bf16]] [--no-cpu-baseline] [--no-e2e] [--graph]

One "step" = one pass of the hot path over one batch of synthetic samples already resident in HBM:
K1 (per-sample regressor Y, contact projector P, stacked [Y_proj | B_v | B_c | tau_proj] panel written
to HBM in the reference's row layout) + K2/K3 (Gram AᵀA, Aᵀb, bᵀb on fp64 MFMA) + for N > 1 one RCCL
all-reduce of the Gram through the engine's own C-ABI exchange (sysid_allreduce_gram).  Samples are
sharded: with --samples every rank processes its own batch (weak scaling); with --total-samples the job's
samples are split over the ranks (strong scaling, BASELINE config 4: --total-samples 200000).
Rank 0 prints one JSON line.  For N > 1 launch with
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "regressor samples/sec + Gram-build GF/s, 12-DoF, 20k samples, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_MFMA_PEAK_TFS = 78.6  # AMD public spec for MI355X fp64 matrix (not in the container guide)
MFMA_PEAK_TFS = {"f64": FP64_MFMA_PEAK_TFS, "f32": 157.3, "bf16": 2500.0}  # MI355X_MICROARCH.md (dense)
BOX_CPU_SHARE = 16        # host threads a one-GPU box grants a job (OMP_NUM_THREADS there)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 steps after 100 warmup steps (~0.12 s of Spot work): 20 steps after 5 read 10% low (0.422 vs 0.383 ms
    # per step, profiles/r02_v3/steps_warmup.txt) -- the GPU had not reached its steady state yet
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--robot", default="spot")
    ap.add_argument("--samples", type=int, default=20000, help="samples per GPU (weak scaling)")
    ap.add_argument("--total-samples", type=int, default=0,
                    help="samples of the whole job, split over the ranks (strong scaling; config 4 = 200000)")
    ap.add_argument("--gram-only", action="store_true",
                    help="normal equations only (SURVEY.md §8d config 5): the panel is produced chunk by chunk on "
                         "the device and never returned")
    ap.add_argument("--precision", default="f64", choices=["f64", "f32", "bf16"],
                    help="Gram arithmetic for --gram-only (f32/bf16: config 5 throughput, error reported)")
    ap.add_argument("--rows", default="auto", choices=["auto", "nullspace", "projector"],
                    help="--gram-only rows per sample: nullspace (nv - rank(J_c) rows Z^T A), projector (the "
                         "reference's nv rows P A) or auto (the engine's choice, Engine.gram_rows: nullspace unless the "
                         "model runs the Q-form K1 (G1, snake14) or the Gram is bf16; the JSON names it as rows_used)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer (PCIe-inclusive) legs")
    ap.add_argument("--graph", action="store_true",
                    help="replay one captured HIP graph per step instead of eager launches (measured no gain)")
    ap.add_argument("--cpu-threads", type=int, default=BOX_CPU_SHARE,
                    help="threads of the extra multi-core C oracle timing (0 = off; 16 = the GPU box's CPU share)")
    ap.add_argument("--ref-samples", type=int, default=2000,
                    help="samples of the numpy reference-structure CPU leg (0 = off)")
    ap.add_argument("--exchange-overlap", default="off", choices=["on", "off"],
                    help="N > 1: on = step i's Gram all-reduce on its own stream while step i + 1 computes (the Gram "
                         "output double-buffered); off (default) = the all-reduce in line after K3.  On one GPU with "
                         "a one-rank communicator the overlap's two cross-stream waits per step cost 4.7%% (0.330 vs "
                         "0.316 ms, profiles/r03_o) while the in-line one-rank all-reduce costs nothing measurable")
    ap.add_argument("--exchange-world1", action="store_true",
                    help="test mode: run the C-ABI RCCL exchange on a one-rank communicator at N = 1, so the "
                         "(overlapped) exchange path runs on a single GPU; not a driver configuration")
    ap.add_argument("--settle-ms", type=float, default=0.0,
                    help="untimed steps run back to back for at least this long before the warmup steps (0 = off, "
                         "the default: the timed region follows exactly --warmup steps).  The steady-state figure "
                         "after a 250 ms settle is reported separately as `steady_state` (N = 1), never as `value`")
    ap.add_argument("--no-steady-state", action="store_true",
                    help="skip the labelled steady-state re-timing after the timed region")
    return ap.parse_args()


def pmc_traffic(kernel, robot, samples):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary for this workload
    (profiles/<round>/pmc_summary.json: FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, separate passes)."""
    import glob
    import re

    def version(path):  # r01_v10 after r01_v9 (numbers as numbers), r03_p after r03_m (round, then the tag)
        # type-stable key: numbers sort before words at the same position (r03_2 vs r03_j compares (0, 2) < (1, 'j'))
        return [(0, int(t), "") if t.isdigit() else (1, 0, t)
                for t in re.findall(r"\d+|[a-z]+", os.path.basename(os.path.dirname(path)))]

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_summary.json")), key=version, reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        cfg = d.get("_config", {})
        if cfg.get("robot") != robot or cfg.get("samples") != samples or kernel not in d:
            continue
        k = d[kernel]
        if "FETCH_bytes_corrected_x2" in k and "WRITE_bytes" in k:
            return round(k["FETCH_bytes_corrected_x2"] + k["WRITE_bytes"]), os.path.relpath(path, ROOT)
    return None, None


def cpu_baseline(model, data, n_sample, nthreads=1):
    """The C restatement of the reference path (oracle/sysid_oracle.c) on n_sample samples (OpenMP over the
    samples when nthreads > 1)."""
    from oracle.ref_c import COracle
    o = COracle(model)
    sl = {k: data[k][:, :n_sample].copy() for k in ("q", "dq", "ddq", "tau", "contact")}
    t0 = time.perf_counter()
    o.build(sl["q"], sl["dq"], sl["ddq"], sl["tau"], sl["contact"], nthreads=nthreads)
    dt = time.perf_counter() - t0
    return n_sample / dt, dt


def cpu_reference_structure(model, data, n_sample):
    """BASELINE.md CPU leg (i): the reference's own loop structure — per-sample get_proj_regressor_torque and
    get_proj_friction_regressors (two FK passes, two SVD pinvs per sample), np.vstack / np.hstack
    (demo/spot_identification.py:37-56, 84-87) and AᵀA — with pinocchio's algorithms restated in numpy
    (oracle/ref_numpy.py), on one core (BLAS limited to one thread)."""
    from threadpoolctl import threadpool_limits
    from oracle import ref_numpy as ref
    sl = {k: data[k][:, :n_sample].copy() for k in ("q", "dq", "ddq", "tau", "contact")}
    with threadpool_limits(limits=1):
        t0 = time.perf_counter()
        Y, t = ref.get_projected_y_tau(model, sl["q"], sl["dq"], sl["ddq"], sl["tau"], sl["contact"])
        Bv, Bc = ref.get_projected_friction_regressors(model, sl["q"], sl["dq"], sl["ddq"], sl["contact"])
        ref.normal_equations(Y, t, Bv, Bc)
        dt = time.perf_counter() - t0
    return n_sample / dt, dt


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def e2e_legs(eng, data, N, reps=10):
    """§8(d) end-to-end samples/s of the host entry point (numpy in -> numpy out, PCIe both ways):
    full outputs (stacked Y_proj, tau_proj, B_v, B_c + Gram) and Gram only (inputs in, 190 KB out).  The inputs in
    read_data's dtypes (demo/spot_identification.py:10-25): q and contact float32 as loaded, dq / ddq / tau float64
    (filtered); the engine sends them in its wire format (sysid_build_f32qc).  `ms` is the best of `reps` calls
    (samples_per_s from it), `median_ms` their median."""
    import numpy as np
    from system_identification_amd.engine import EMIT_ALL, EMIT_GRAM
    ins = [data["q"].astype(np.float32), data["dq"], data["ddq"], data["tau"], data["contact"].astype(np.float32)]
    in_bytes = sum(a.nbytes for a in ins)
    res = {}
    for name, flags in (("full", EMIT_ALL), ("gram_only", EMIT_GRAM)):
        eng.build(*ins, flags)  # warm: device buffers grown once
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            out = eng.build(*ins, flags)
            ts.append(time.perf_counter() - t0)
        best = min(ts)
        out_bytes = sum(v.nbytes for v in out.values() if hasattr(v, "nbytes"))
        res[name] = {"samples_per_s": round(N / best, 1), "ms": round(best * 1e3, 3),
                     "median_ms": round(float(np.median(ts)) * 1e3, 3), "calls": reps,
                     "pcie_bytes": int(in_bytes + out_bytes),
                     "pcie_GBps": round((in_bytes + out_bytes) / best / 1e9, 2)}
    return res


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one process per GPU)")
    # Dev rehearsal of the multi-rank path on a one-GPU box (SYSID_BENCH_REHEARSE=1; never the driver's runs): every
    # rank on cuda:0 and the process group over gloo.  RCCL refuses two ranks on one GPU, so the engine's C-ABI
    # exchange fails to come up and every rank takes the torch.distributed fallback: the rehearsal runs the
    # orchestration (shards, barriers, max-over-ranks timing, the exchange check, rank 0's line), not RCCL.
    rehearse = world > 1 and os.environ.get("SYSID_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from system_identification_amd.distributed import RcclGramComm, make_gram_exchange, shard_range
    from system_identification_amd.engine import EMIT_ALL, GRAM_PRECISION, GRAM_ROWS, Engine
    from system_identification_amd.model import load_robot
    from system_identification_amd.synthetic import channel_block, generate

    model = load_robot(args.robot)
    strong = args.total_samples > 0
    if strong:
        s0, s1 = shard_range(args.total_samples, rank, world)
        N = s1 - s0
        total_per_step = args.total_samples
    else:
        N = args.samples
        total_per_step = N * world
    data = generate(model, N, config_index=1 + rank)  # each rank its own shard of the log
    eng = Engine(model, device=local)
    d_in = torch.from_numpy(channel_block(data)).cuda(local)
    flags = EMIT_ALL
    tflags = EMIT_ALL | GRAM_PRECISION[args.precision] | GRAM_ROWS[args.rows]
    rows_used = args.rows if args.rows != "auto" else eng.gram_rows(args.precision)
    # one explicit (non-null) stream for every launch, the exchange and the step events
    stream = torch.cuda.Stream(device=local)
    torch.cuda.set_stream(stream)

    comm, exchange_name = None, None
    if world == 1 and args.exchange_world1:
        comm = RcclGramComm(eng, 0, 1)
        exchange_name = "sysid_allreduce_normal_equations (RCCL, C ABI, one-rank communicator: test mode)"
    if world > 1:
        # the engine's own exchange step (C ABI: sysid_rccl_unique_id / _comm_init /
        # sysid_allreduce_normal_equations); the 128-byte RCCL id travels from rank 0 over the torch process group.
        # Should the C-ABI communicator fail to come up on some rank, every rank runs the same all-reduce through
        # torch.distributed (RCCL) and the JSON says so (distributed.make_gram_exchange).
        def share_id(raw):
            box = [raw if rank == 0 else None]
            dist.broadcast_object_list(box, src=0)
            return box[0]

        def all_ok(flag):
            t = torch.tensor([int(flag)], dtype=torch.int32, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            return int(t.item()) == 1
        comm, exchange_name = make_gram_exchange(eng, rank, world, share_id, all_ok)
        if rehearse:
            exchange_name = "rehearsal on one GPU over gloo: " + exchange_name

    if args.gram_only:
        # config 5: 16 GiB chunk panels (the library default is 4 GiB; 16 GiB measured 2-3% faster on G1 1M)
        eng.set_gram_chunk_bytes(16 << 30)
        bufs = eng.alloc_gram_device(N)

        def launch(s, b=bufs):
            eng.build_gram_device(d_in, N, b, stream=s, precision=args.precision, rows=args.rows)
    else:
        bufs = eng.alloc_device(N, flags)

        def launch(s, b=bufs):
            eng.build_device(d_in, N, flags, b, stream=s)

    xbuf = comm.exchange_buffer() if comm is not None else None
    rows_local = float(N * model.nv)

    def exchange():
        if comm is not None:
            comm.allreduce_normal_equations(bufs["gram"], rows_local, xbuf, stream=stream.cuda_stream)
        elif world > 1:
            dist.all_reduce(bufs["gram"])

    # Overlapped exchange (the C-ABI communicator, eager launches): step i's all-reduce runs on its own stream
    # after step i's K3 while step i + 1's K1 / K2 / K3 run on the launch stream into the other Gram buffer; a
    # buffer is reused (step i + 2) only after its all-reduce has finished.  Every all-reduce of the timed steps
    # completes inside the timed region (the device-wide synchronize that closes it).
    overlap = comm is not None and args.exchange_overlap == "on" and not args.graph
    bufsets = [bufs]
    if overlap:
        bufsets.append(dict(bufs, gram=torch.zeros_like(bufs["gram"])))
        xbufs = [xbuf, comm.exchange_buffer()]
        comm_stream = torch.cuda.Stream(device=local)
        k_done = [torch.cuda.Event(), torch.cuda.Event()]
        x_done = [torch.cuda.Event(), torch.cuda.Event()]
        x_used = [False, False]
        step_no = [0]
        exchange_name += ", overlapped with the next step (own stream, Gram double-buffered)"

    # One step's launches (memsets + K1 + K2 + K3) captured once into a HIP graph and replayed: the same
    # kernels over the same buffers, without the per-launch host gaps.  The RCCL all-reduce stays eager.
    graph_used = False
    if args.graph:
        launch(stream.cuda_stream)  # warm the engine (first-launch setup outside the capture)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            launch(torch.cuda.current_stream(local).cuda_stream)
        graph_used = True

        def compute():
            g.replay()
    else:
        def compute():
            launch(stream.cuda_stream)

    def step():
        if overlap:
            b = step_no[0] % 2
            step_no[0] += 1
            if x_used[b]:
                stream.wait_event(x_done[b])  # buffer b's previous all-reduce has read it
            launch(stream.cuda_stream, bufsets[b])
            k_done[b].record(stream)
            comm_stream.wait_event(k_done[b])
            comm.allreduce_normal_equations(bufsets[b]["gram"], rows_local, xbufs[b], stream=comm_stream.cuda_stream)
            x_done[b].record(comm_stream)
            x_used[b] = True
        else:
            compute()
            exchange()

    # Optional clock settle (untimed, every rank; off by default): steps back to back until --settle-ms of wall
    # time has passed.  By default the timed region follows exactly the --warmup steps the caller asked for, so a
    # short run measures what a one-shot identification sees, clock ramp included (step_times shows it); the
    # settled figure is re-measured after the timed region and reported apart (`steady_state`).
    def settle_for(ms_budget):
        n, t_s = 0, time.perf_counter()
        while ms_budget > 0 and (time.perf_counter() - t_s) * 1e3 < ms_budget:
            for _ in range(8):
                compute()
            n += 8
            torch.cuda.synchronize()
        return {"steps": n, "ms": round((time.perf_counter() - t_s) * 1e3, 1)}

    settle = settle_for(args.settle_ms)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # per-step device times from HIP events recorded on the launch stream between the steps (no host
    # synchronisation inside the timed region): the warm-up evidence VERDICT r2 asked for, not the value
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    marks[0].record(stream)
    for i in range(args.steps):
        step()
        marks[i + 1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # Exchange check, right after the timed region and before anything else writes the Gram buffers (the steady-state
    # re-timing, time_stages and the e2e legs build this rank's local, un-reduced Gram into them): every rank must
    # hold the same reduced Gram in each buffer; with
    # the one-rank test communicator the all-reduce is the identity, so each buffer must equal a fresh local
    # build bitwise (K1-K3 are deterministic).
    exchange_check = None
    if comm is not None:
        sums = torch.stack([b_["gram"].sum() for b_ in bufsets] + [b_["gram"].abs().sum() for b_ in bufsets])
        if world > 1:
            hi, lo = sums.clone(), sums.clone()
            dist.all_reduce(hi, op=dist.ReduceOp.MAX)
            dist.all_reduce(lo, op=dist.ReduceOp.MIN)
            exchange_check = {"ranks_agree": bool(torch.equal(hi, lo)), "buffers": len(bufsets)}
        else:
            ref_g = dict(bufs, gram=torch.zeros_like(bufs["gram"]))
            launch(stream.cuda_stream, ref_g)
            torch.cuda.synchronize()
            exchange_check = {"bitwise_equal_local_build": all(bool(torch.equal(b_["gram"], ref_g["gram"]))
                                                               for b_ in bufsets), "buffers": len(bufsets)}
        # the packed exchange carries the row count: the job's N·nv (the Solver's 1/num_rows, solver.py:190)
        exchange_check["num_rows"] = float(xbuf[-1].item())
        exchange_check["num_rows_ok"] = exchange_check["num_rows"] == float(total_per_step * model.nv)
    elif world > 1:  # the torch.distributed fallback: every rank must hold the same summed Gram too
        sums = torch.stack([bufs["gram"].sum(), bufs["gram"].abs().sum()])
        hi, lo = sums.clone(), sums.clone()
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        exchange_check = {"ranks_agree": bool(torch.equal(hi, lo)), "buffers": 1}

    # Labelled side figures, all after the timed region: the steady state (250 ms of untimed steps, then the same
    # K steps re-timed; rank 0 at N = 1) and the host-entry-point legs (SURVEY §8d's end-to-end rate,
    # PCIe-inclusive).  Neither is `value`.
    steady = None
    if world == 1 and not args.no_steady_state:
        pre = settle_for(250.0)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            compute()
        torch.cuda.synchronize()
        el2 = time.perf_counter() - t1
        steady = {"ms_per_step": round(el2 / args.steps * 1e3, 5),
                  "samples_per_s": round(total_per_step * args.steps / el2, 1),
                  "settle": pre, "note": "the same K steps re-timed after 250 ms of untimed back-to-back steps "
                                         "(clocks at their operating point); not the headline value"}
    # per-kernel device time (HIP events on the engine's stream), for the roofline.  Gram-only: the chunked
    # path itself, each stage summed over its chunks.  Measured right after the timed region and the steady-state
    # re-timing, before the host-entry-point legs (whose host-bound gaps let the clocks drop again), so it sees the
    # kernels at the clocks rocprofv3's average over the same run sees them.
    n_time = N
    ms = eng.time_stages(d_in, N, tflags if args.gram_only else flags, bufs, iters=max(5, args.steps))
    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e:
        e2e = e2e_legs(eng, data, N)
        torch.cuda.synchronize()

    nv, W = model.nv, eng.w
    in_b = (model.nq + 2 * nv + model.nj + model.n_ee) * 8
    esize = {"f64": 8, "f32": 4, "bf16": 2}[args.precision] if args.gram_only else 8
    panel_b = nv * (W + 1) * esize  # Gram-only at reduced precision: K1 writes the chunk panel in f32 / bf16
    bytes_k1 = in_b + panel_b                                                       # SURVEY §8d per sample
    flops_k2 = nv * W * (W + 1) + 2 * nv * W                                       # SYRK + Aᵀb per sample
    k1_gbs = n_time * bytes_k1 / (ms[0] * 1e-3) / 1e9
    k2_tfs = n_time * flops_k2 / (ms[1] * 1e-3) / 1e12 if ms[1] > 0 else 0.0
    rows_per_sample = float(nv)
    if args.gram_only and rows_used == "nullspace" and 3 * model.n_ee <= 12:
        # the Gram kernel's own work: nv - rank(J_c) rows per sample (rank 3 per foot in contact: the synthetic
        # gaits' J_c have full row rank); roofline.achieved counts these executed flops, the algorithmic
        # nv-row count stays in K2_TFps / gram_gflops
        rows_per_sample = float(np.mean(nv - 3 * (data["contact"] != 0).sum(axis=0)))
    k2_exec_tfs = k2_tfs * rows_per_sample / nv
    if ms[0] >= ms[1]:
        traffic, src = pmc_traffic("k1_regressor_panel", args.robot, N) if not args.gram_only else (None, None)
        roof = {"kernel": "k1_regressor_panel", "bound": "hbm", "achieved": round(k1_gbs, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(k1_gbs / HBM_PEAK_GBS, 4),
                "traffic": traffic, "traffic_source": src, "algorithmic_bytes_per_launch": n_time * bytes_k1,
                "avg_launch_ms": round(ms[0], 5)}
    else:
        traffic, src = pmc_traffic("k2_gram_syrk", args.robot, N) if not args.gram_only else (None, None)
        peak = MFMA_PEAK_TFS[args.precision if args.gram_only else "f64"]
        roof = {"kernel": "k2_gram_syrk", "bound": "mfma", "achieved": round(k2_exec_tfs, 3),
                "peak": peak, "unit": "TFLOP/s", "frac": round(k2_exec_tfs / peak, 4),
                "traffic": traffic, "traffic_source": src,
                "algorithmic_flops_per_launch": round(n_time * flops_k2 * rows_per_sample / nv),
                "rows_per_sample": round(rows_per_sample, 3), "avg_launch_ms": round(ms[1], 5)}

    ms_step = elapsed / args.steps * 1e3
    per_step = np.array([marks[i].elapsed_time(marks[i + 1]) for i in range(args.steps)])
    q = max(1, args.steps // 4)
    step_stats = {"min_ms": round(float(per_step.min()), 5), "median_ms": round(float(np.median(per_step)), 5),
                  "max_ms": round(float(per_step.max()), 5),
                  "first_quartile_mean_ms": round(float(per_step[:q].mean()), 5),
                  "last_quartile_mean_ms": round(float(per_step[-q:].mean()), 5),
                  "source": "HIP events on the launch stream between consecutive timed steps (rank 0)"}
    # step-level floor: the bytes the step must move (inputs + panel written by K1 and read back by K2; Gram-only
    # chunks may stay on-die and are not counted) at HBM peak, and the Gram flops at the MFMA peak
    step_bytes = N * (in_b + (0 if args.gram_only else 2 * panel_b))
    hbm_floor = step_bytes / (HBM_PEAK_GBS * 1e9) * 1e3
    mfma_floor = N * flops_k2 / (MFMA_PEAK_TFS[args.precision if args.gram_only else "f64"] * 1e12) * 1e3
    value = total_per_step * args.steps / elapsed
    result = {
        "metric": METRIC, "value": round(value, 1), "unit": "samples/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 5),
        "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None,
        "hip_graph": graph_used,
        "dtype": "f64" if not args.gram_only or args.precision == "f64" else f"f64 panel, {args.precision} Gram",
        "data": "synthetic (SURVEY.md §8d recipe: sinusoidal joints in URDF limits, wobbling base, "
                "inverse-dynamics torques + noise, trot contacts with LOST=2); no .dat ships with the reference",
        "config": {"workload": f"{args.robot} " + (f"{args.total_samples} samples split over {world} GPU(s)" if strong
                                                    else f"{N} samples per GPU") + ", " + (
                       f"Gram only ({rows_used} rows chunked on the device, {args.precision} Gram)"
                       if args.gram_only else
                       "full outputs (stacked Y_proj/tau_proj/B_v/B_c panel + Gram)"),
                   "robot": args.robot, "samples_per_gpu": N, "total_samples_per_step": total_per_step,
                   "nv": nv, "W": W, "parallelism": f"dp{world}",
                   "exchange": exchange_name,
                   "exchange_check": exchange_check,
                   "timed_region": ("K1 + K2 per panel chunk + K3 (Gram-only)" if args.gram_only else "K1 + K2 + K3")
                   + ", HBM-resident inputs and outputs" + (", + the Gram all-reduce" if comm is not None or world > 1
                                                             else "")},
        "step_times": step_stats,
        "settle": settle,
        "steady_state": steady,
        "gram_gflops": round(total_per_step * flops_k2 / (ms_step * 1e-3) / 1e9, 2),
        "kernel_ms": {"K1_regressor_panel": round(ms[0], 5), "K2_gram_syrk": round(ms[1], 5),
                      "K3_gram_reduce": round(ms[2], 5), "samples_timed": n_time},
        "K1_GBps": round(k1_gbs, 1), "K2_TFps": round(k2_tfs, 3),
        "roofline": roof,
        "step_roofline": {"hbm_bytes": step_bytes, "hbm_floor_ms": round(hbm_floor, 5),
                          "mfma_floor_ms": round(mfma_floor, 5), "floor_ms": round(max(hbm_floor, mfma_floor), 5),
                          "frac": round(max(hbm_floor, mfma_floor) / ms_step, 4)},
    }
    if e2e is not None:
        result["e2e"] = e2e
        result["e2e_full_samples_per_s"] = result["e2e"]["full"]["samples_per_s"]
        result["e2e_gram_only_samples_per_s"] = result["e2e"]["gram_only"]["samples_per_s"]
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # the contract: rank 0 at N = 1 only
        n_cpu = min(N, 20000)
        v, dt = cpu_baseline(model, data, n_cpu)
        host = {"cpu_model": cpu_model(), "nproc": os.cpu_count(), "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}
        result["cpu_baseline"] = {
            "value": round(v, 1), "unit": "samples/s", "cores": 1, "kind": "port",
            "sample": f"{n_cpu} {args.robot} samples, oracle/sysid_oracle.c single thread: reference structure "
                      f"(2 FK passes + 2 SVD pinv per sample, stacking, AᵀA), {dt:.2f} s", "host": host}
        if args.cpu_threads > 1:
            v2, dt2 = cpu_baseline(model, data, n_cpu, nthreads=args.cpu_threads)
            result["cpu_baseline_multicore"] = {
                "value": round(v2, 1), "unit": "samples/s", "cores": args.cpu_threads, "kind": "port",
                "sample": f"the same {n_cpu} samples, oracle/sysid_oracle.c with OpenMP over the samples on "
                          f"{args.cpu_threads} threads = the GPU box's CPU share (os.cpu_count() = {os.cpu_count()} "
                          f"is the whole host), {dt2:.2f} s"}
        if args.ref_samples > 0:
            n_ref = min(N, args.ref_samples)
            v3, dt3 = cpu_reference_structure(model, data, n_ref)
            result["cpu_baseline_reference_structure"] = {
                "value": round(v3, 1), "unit": "samples/s", "cores": 1, "kind": "port",
                "sample": f"{n_ref} {args.robot} samples: the reference's per-sample Python loop "
                          "(demo/spot_identification.py:37-56, 84-87) over oracle/ref_numpy.py (pinocchio restated "
                          f"in numpy; BLAS 1 thread) + AᵀA, {dt3:.2f} s"}
    if comm is not None:
        comm.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
