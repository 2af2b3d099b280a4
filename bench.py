"""Benchmark: regressor + projector + Gram build on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--robot spot] [--samples 20000] [--gram-only]

One "step" = one pass of the hot path over one batch of synthetic samples already resident in HBM:
K1 (per-sample regressor Y, contact projector P, stacked [Y_proj | B_v | B_c | tau_proj] panel written
to HBM in the reference's row layout) + K2/K3 (Gram AᵀA, Aᵀb, bᵀb on fp64 MFMA) + for N > 1 one RCCL
all-reduce of the Gram.  Samples are sharded: every rank processes its own --samples (weak scaling).
Rank 0 prints one JSON line.  For N > 1 launch with
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--robot", default="spot")
    ap.add_argument("--samples", type=int, default=20000, help="samples per GPU")
    ap.add_argument("--gram-only", action="store_true",
                    help="normal equations only (SURVEY.md §8d config 5): the panel is produced chunk by chunk on "
                         "the device and never returned")
    ap.add_argument("--precision", default="f64", choices=["f64", "f32", "bf16"],
                    help="Gram arithmetic for --gram-only (f32/bf16: config 5 throughput, error reported)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", action="store_true",
                    help="replay one captured HIP graph per step instead of eager launches (measured no gain)")
    ap.add_argument("--cpu-threads", type=int, default=min(16, os.cpu_count() or 1),
                    help="threads of the extra all-core C oracle timing (0 = off; 16 = the GPU box's CPU share)")
    return ap.parse_args()


def pmc_traffic(kernel, robot, samples):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary for this workload
    (profiles/<round>/pmc_summary.json: FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, separate passes)."""
    import glob
    import re

    def version(path):  # r01_v10 sorts after r01_v9: compare the numbers, not the strings
        return [int(n) for n in re.findall(r"\d+", os.path.basename(os.path.dirname(path)))]

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


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


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
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from system_identification_amd.engine import EMIT_ALL, Engine
    from system_identification_amd.model import load_robot
    from system_identification_amd.synthetic import channel_block, generate

    model = load_robot(args.robot)
    N = args.samples
    data = generate(model, N, config_index=1 + rank)  # each rank its own shard of the log
    eng = Engine(model, device=local)
    d_in = torch.from_numpy(channel_block(data)).cuda(local)
    from system_identification_amd.engine import GRAM_PRECISION
    flags = EMIT_ALL
    tflags = EMIT_ALL | (GRAM_PRECISION[args.precision] if args.gram_only else 0)  # kernels timed below
    stream = torch.cuda.current_stream(local)
    if args.gram_only:
        bufs = eng.alloc_gram_device(N)

        def step():
            eng.build_gram_device(d_in, N, bufs, stream=stream.cuda_stream, precision=args.precision)
            if world > 1:
                dist.all_reduce(bufs["gram"])
    else:
        bufs = eng.alloc_device(N, flags)

        def step():
            eng.build_device(d_in, N, flags, bufs, stream=stream.cuda_stream)
            if world > 1:
                dist.all_reduce(bufs["gram"])

    # One step's launches (memset + K1 + K2 + K3) captured once into a HIP graph and replayed: the same
    # kernels over the same buffers, without the per-launch host gaps.  The RCCL all-reduce stays eager.
    graph_used = False
    if args.graph:
        if args.gram_only:
            def launch(s):
                eng.build_gram_device(d_in, N, bufs, stream=s, precision=args.precision)
        else:
            def launch(s):
                eng.build_device(d_in, N, flags, bufs, stream=s)
        launch(stream.cuda_stream)  # warm the engine (first-launch setup outside the capture)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            launch(torch.cuda.current_stream(local).cuda_stream)
        graph_used = True

        def step():
            g.replay()
            if world > 1:
                dist.all_reduce(bufs["gram"])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-kernel device time (HIP events on the engine's stream), for the roofline.  Gram-only runs the
    # same kernels chunk by chunk; they are timed on one chunk-sized batch.
    n_time = N
    if args.gram_only:
        n_time = min(N, max(4096, (512 << 20) // (model.nv * eng.panel_ld * 8)))
        tb = eng.alloc_device(n_time, flags)
        ms = eng.time_stages(d_in, n_time, tflags, tb, iters=max(5, args.steps))
        del tb
    else:
        ms = eng.time_stages(d_in, N, flags, bufs, iters=max(5, args.steps))
    nv, W = model.nv, eng.w
    bytes_k1 = (model.nq + 2 * nv + model.nj + model.n_ee) * 8 + nv * (W + 1) * 8   # SURVEY §8d per sample
    flops_k2 = nv * W * (W + 1) + 2 * nv * W                                       # SYRK + Aᵀb per sample
    k1_gbs = n_time * bytes_k1 / (ms[0] * 1e-3) / 1e9
    k2_tfs = n_time * flops_k2 / (ms[1] * 1e-3) / 1e12
    if ms[0] >= ms[1]:
        traffic, src = pmc_traffic("k1_regressor_panel", args.robot, N) if not args.gram_only else (None, None)
        roof = {"kernel": "k1_regressor_panel", "bound": "hbm", "achieved": round(k1_gbs, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(k1_gbs / HBM_PEAK_GBS, 4),
                "traffic": traffic, "traffic_source": src, "algorithmic_bytes_per_launch": n_time * bytes_k1,
                "avg_launch_ms": round(ms[0], 5)}
    else:
        traffic, src = pmc_traffic("k2_gram_syrk", args.robot, N) if not args.gram_only else (None, None)
        peak = MFMA_PEAK_TFS[args.precision if args.gram_only else "f64"]
        roof = {"kernel": "k2_gram_syrk", "bound": "mfma", "achieved": round(k2_tfs, 3),
                "peak": peak, "unit": "TFLOP/s", "frac": round(k2_tfs / peak, 4),
                "traffic": traffic, "traffic_source": src, "algorithmic_flops_per_launch": n_time * flops_k2,
                "avg_launch_ms": round(ms[1], 5)}

    total_samples = N * world * args.steps
    value = total_samples / elapsed
    result = {
        "metric": METRIC, "value": round(value, 1), "unit": "samples/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "hip_graph": graph_used,
        "dtype": "f64" if not args.gram_only or args.precision == "f64" else f"f64 panel, {args.precision} Gram",
        "data": "synthetic (SURVEY.md §8d recipe: sinusoidal joints in URDF limits, wobbling base, "
                "inverse-dynamics torques + noise, trot contacts with LOST=2); no .dat ships with the reference",
        "config": {"workload": f"{args.robot} {N} samples per GPU, " + (
                       f"Gram only (panel chunked on the device, {args.precision} Gram)" if args.gram_only else
                       "full outputs (stacked Y_proj/tau_proj/B_v/B_c panel + Gram)"),
                   "robot": args.robot, "samples_per_gpu": N,
                   "nv": nv, "W": W, "parallelism": f"dp{world}"},
        "gram_gflops": round(N * world * flops_k2 / (elapsed / args.steps) / 1e9, 2),
        "kernel_ms": {"K1_regressor_panel": round(ms[0], 5), "K2_gram_syrk": round(ms[1], 5),
                      "K3_gram_reduce": round(ms[2], 5), "samples_timed": n_time},
        "K1_GBps": round(k1_gbs, 1), "K2_TFps": round(k2_tfs, 3),
        "roofline": roof,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # the contract: rank 0 at N = 1 only
        n_cpu = min(N, 20000)
        v, dt = cpu_baseline(model, data, n_cpu)
        result["cpu_baseline"] = {
            "value": round(v, 1), "unit": "samples/s", "cores": 1, "kind": "port",
            "sample": f"{n_cpu} {args.robot} samples, oracle/sysid_oracle.c single thread: reference structure "
                      f"(2 FK passes + 2 SVD pinv per sample, stacking, AᵀA), {dt:.2f} s",
            "host": {"cpu_model": cpu_model(), "nproc": os.cpu_count(),
                     "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")},
        }
        if args.cpu_threads > 1:
            v2, dt2 = cpu_baseline(model, data, n_cpu, nthreads=args.cpu_threads)
            result["cpu_baseline_allcores"] = {
                "value": round(v2, 1), "unit": "samples/s", "cores": args.cpu_threads, "kind": "port",
                "sample": f"the same {n_cpu} samples, oracle/sysid_oracle.c with OpenMP over the samples, {dt2:.2f} s"}
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
