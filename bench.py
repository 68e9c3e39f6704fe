#!/usr/bin/env python3
"""MI355X inference-codelet benchmark (BASELINE.json metric: inferences/sec + p50 latency).

A *step* is one task per worker: each of the `--workers` workers of a GPU
(StarPU's STARPU_NWORKER_PER_CUDA=4 analogue, models/resnet18.yml:6) calls the
HIP codelet (libspi_hip.so, through the C-ABI) on its own HIP stream over one
synthetic batch already resident in HBM.  Default workload = BASELINE.json
configs[1]: ResNet-18, batch 8, fp16 MFMA, one MI355X.

Multi-GPU: one process per GPU (torch.distributed.run), one weight replica
per device, tasks sharded across devices with no data-path collective
("scaling": "weak"); a gloo barrier brackets the timed region and the time is
the max over ranks.  `value` = inferences of all ranks / that time.

Also reported: p50 per-task device latency (HIP events on the worker stream,
linear-interpolated percentile as src/core/latency_statistics.hpp:52-93), p50
end-to-end latency including pinned H2D + D2H (serial, one task in flight),
the dominant kernel's roofline (HIP events on its launch stream) and the CPU
codelet baseline (oracle: ATen CPU forward of the same TorchScript-able module,
rank 0 only, bounded sample).
"""
from __future__ import annotations

import argparse
import ctypes as C
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_METRIC = "inferences/sec + p50 latency, ResNet-18 bs=1 & BERT-base seq=128, 1/2/4/8 GPU"
WORKLOADS = {
    "resnet18": "ResNet-18 bs=8 fp16, single MI355X HIP codelet (conv-as-implicit-GEMM MFMA)",
    "bert_base": "bert-base-uncased seq=128 bs=8 fp16, 1xMI355X (QKV GEMM + softmax + LayerNorm fused)",
    "resnet152": "ResNet-152 bs=32 fp16, StarPU-style HIP workers per MI355X (request-parallel, no RCCL)",
    "vit_l_16": "ViT-L/16 224^2 bs=16 fp16 (patch-embed GEMM + MFMA attention, LDS-tiled)",
}
PEAK_TFLOPS = {"fp16": 2500.0, "fp16x3": 2500.0, "fp32": 157.3}  # MI355X dense (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def percentile(samples, p):
    """Linear-interpolated percentile (latency_statistics.hpp:52-93)."""
    xs = sorted(samples)
    if not xs:
        return float("nan")
    if len(xs) == 1:
        return xs[0]
    pos = (p / 100.0) * (len(xs) - 1)
    lo = int(np.floor(pos))
    hi = min(lo + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (pos - lo)


def reduce_max_elapsed(elapsed: float, world: int) -> float:
    """Max over ranks of the barrier-bracketed timed region (control plane only, gloo)."""
    if world <= 1:
        return elapsed
    import torch
    import torch.distributed as dist

    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shard_requests(n: int, rank: int, world: int) -> list:
    """Request-level sharding across independent per-GPU workers (no data-path collective):
    contiguous blocks, as an eager shared queue drained by per-device workers would end up."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return list(range(lo, lo + base + (1 if rank < extra else 0)))


def make_inputs(name, batch, rng, seq=128):
    if name.startswith("bert"):
        ids = rng.integers(0, 30522, size=(batch, seq), dtype=np.int64)
        mask = np.ones((batch, seq), dtype=np.int64)  # all-ones mask
        return [ids, mask], (batch, seq, 768)
    return [rng.random((batch, 3, 224, 224), dtype=np.float32)], (batch, 1000)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="resnet18", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--precision", default="fp16", choices=["fp16", "fp16x3", "fp32"])
    ap.add_argument("--workers", type=int, default=4, help="worker streams per GPU")
    ap.add_argument("--graphs", type=int, default=1, help="capture the forward body into hipGraphs")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--latency-iters", type=int, default=40)
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    spi = importlib.import_module("starpu-inference-server_amd")
    zoo = importlib.import_module("starpu-inference-server_amd.zoo")
    N = spi._native
    lib = spi.lib

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = local_rank
    torch.cuda.set_device(dev)

    model = zoo.build(args.model, seed=0)
    seq = 128
    replica = spi.ModelReplica(model, dev, args.precision, max_batch=args.batch,
                               seq_len=seq if args.model.startswith("bert") else 0)
    replica.set_graphs(bool(args.graphs))

    rng = np.random.default_rng(rank)
    W = args.workers
    streams = [torch.cuda.Stream(dev) for _ in range(W)]
    host_inputs, out_shape = make_inputs(args.model, args.batch, rng, seq)
    d_in = [[torch.from_numpy(x).to(dev) for x in host_inputs] for _ in range(W)]
    d_out = [torch.empty(out_shape, device=dev, dtype=torch.float32) for _ in range(W)]
    torch.cuda.synchronize(dev)

    # Prebuilt codelet arguments per worker (the task's cl_arg + buffers).
    calls = []
    for w in range(W):
        params = spi.make_params([list(x.shape) for x in d_in[w]], [x.dtype for x in d_in[w]],
                                 models_gpu=[replica], device_ids=[dev])
        a = params.to_args()
        bufs = spi.buffer_array([spi.tensor_interface(x) for x in d_in[w]] + [spi.tensor_interface(d_out[w])])
        calls.append((a, bufs, streams[w]))

    def run_task(w, ev=None):
        a, bufs, st = calls[w]
        lib.spi_set_worker_context(w, dev, C.c_void_p(st.cuda_stream))
        if ev is not None:
            ev[0].record(st)
        lib.spi_hip_inference_func(bufs, C.byref(a))
        if ev is not None:
            ev[1].record(st)
        if a.status != N.SPI_OK:
            raise RuntimeError(a.error.decode())

    for _ in range(args.warmup):
        for w in range(W):
            run_task(w)
    torch.cuda.synchronize(dev)

    events = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(W)]
              for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        for w in range(W):
            run_task(w, events[k][w])
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = reduce_max_elapsed(t1 - t0, world)
    task_lat_ms = [s.elapsed_time(e) for step in events for (s, e) in step]
    inferences = world * W * args.batch * args.steps
    value = inferences / elapsed
    ms_per_step = elapsed * 1e3 / args.steps

    # Serial end-to-end latency: pinned host -> H2D -> codelet -> D2H, one task in flight.
    st0 = streams[0]
    pinned_in = [torch.from_numpy(x).pin_memory() for x in host_inputs]
    pinned_out = torch.empty(out_shape, dtype=torch.float32).pin_memory()
    e2e = []
    for i in range(args.latency_iters + 3):
        ts = time.perf_counter()
        with torch.cuda.stream(st0):
            for hsrc, dst in zip(pinned_in, d_in[0]):
                dst.copy_(hsrc, non_blocking=True)
            run_task(0)
            pinned_out.copy_(d_out[0], non_blocking=True)
        st0.synchronize()
        if i >= 3:
            e2e.append((time.perf_counter() - ts) * 1e3)

    # Dominant kernel (per-op HIP events on the launch stream, same workload).
    ops = replica.profile(d_in[0], d_out[0], st0.cuda_stream)
    totals = {}
    for op in ops:
        t = totals.setdefault(op["name"], [0.0, 0, op["flops"], op["bytes"]])
        t[0] += op["ms"]
        t[1] += 1
    dom_name, (dom_ms_total, dom_count, dom_flops, dom_bytes) = max(totals.items(), key=lambda kv: kv[1][0])
    dom_ms = dom_ms_total / dom_count
    fwd_ms = sum(op["ms"] for op in ops)
    fwd_flops = sum(op["flops"] for op in ops)
    achieved_tf = dom_flops / (dom_ms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.precision]

    result = {
        "metric": BASELINE_METRIC,
        "value": round(value, 2),
        "unit": "inferences/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic (seeded U[0,1) images / uniform token ids, all-ones mask); random-init weights "
                "of the reference architecture (no checkpoints offline)",
        "config": {
            "workload": WORKLOADS[args.model],
            "batch_per_task": args.batch,
            "workers_per_gpu": W,
            "tasks_per_step_per_gpu": W,
            "graphs": bool(args.graphs),
            "parallelism": f"replicas x{world} (request sharding, no collective)",
        },
        "p50_task_latency_ms": round(percentile(task_lat_ms, 50), 4),
        "p95_task_latency_ms": round(percentile(task_lat_ms, 95), 4),
        "p50_e2e_latency_ms_incl_h2d_d2h": round(percentile(e2e, 50), 4),
        "e2e_inferences_per_s_serial": round(args.batch / (percentile(e2e, 50) * 1e-3), 2),
        "model_gflop_per_inference": round(replica.flops(1) / 1e9, 4),
        "forward_device_ms_profiled": round(fwd_ms, 4),
        "model_tflops_per_gpu": round(replica.flops(1) * value / world / 1e12, 3),
        "roofline": {
            "bound": "mfma",
            "kernel": dom_name,
            "launches_per_forward": dom_count,
            "achieved": round(achieved_tf, 3),
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": round(achieved_tf / peak, 5),
            "traffic": None,
            "algorithmic_flops_per_launch": dom_flops,
            "avg_launch_ms": round(dom_ms, 5),
            "forward_frac": round(fwd_flops / (fwd_ms * 1e-3) / 1e12 / peak, 5),
        },
    }

    if rank == 0 and args.cpu_seconds > 0:
        from oracle.cpu_codelet import cpu_inference

        cores = torch.get_num_threads()
        n, t_cpu = 0, 0.0
        x_cpu = host_inputs
        cpu_inference(model, x_cpu)  # warm-up
        while t_cpu < args.cpu_seconds and n < 200:
            ts = time.perf_counter()
            cpu_inference(model, x_cpu)
            t_cpu += time.perf_counter() - ts
            n += 1
        result["cpu_baseline"] = {
            "value": round(n * args.batch / t_cpu, 3),
            "unit": "inferences/s",
            "cores": cores,
            "kind": "port",
            "sample": f"{n} forwards of the same {args.model} batch {args.batch} fp32 on host ATen "
                      f"(torch {torch.__version__}, {cores} intra-op threads), {t_cpu:.1f}s",
            "p50_ms": round(t_cpu / n * 1e3, 3),
        }
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
