#!/usr/bin/env python3
"""MI355X inference-codelet benchmark (BASELINE.json metric: inferences/sec + p50 latency).

Headline workload = BASELINE.json configs[1]: ResNet-18, batch 8 per task, fp16
MFMA, one MI355X -- run in the parity-grade fp16x3 mode (split-fp16 MFMA,
fp32-grade results; plain fp16 operands miss the 1e-3 bar on this network,
DESIGN.md 3).  A *step* is one task per worker: each of the `--workers` workers
of a GPU (STARPU_NWORKER_PER_CUDA=4, models/resnet18.yml:6) calls the HIP
codelet (libspi_hip.so, through the C-ABI) on its own HIP stream over one
synthetic batch already resident in HBM.

Multi-GPU: one process per GPU (torch.distributed.run), one weight replica per
device, tasks sharded across devices with no data-path collective
("scaling": "weak"); a gloo barrier brackets the timed region and the time is
the max over ranks; `value` = inferences of all ranks / that time.

Also reported (rank 0): p50 per-task device latency (hipEvents on the worker
stream, linear-interpolated percentile as src/core/latency_statistics.hpp:52-93),
p50 end-to-end latency including pinned H2D + D2H, the dominant kernel's
roofline (hipEvents on its launch stream), the CPU codelet baseline (oracle =
ATen CPU forward of the same module, bounded sample) and, single-GPU only,
extras: plain-fp16 throughput, BERT-base seq128 bs8, ResNet-18 bs1 latency and
the PCIe-inclusive mini-runtime path.
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
    "resnet152": "ResNet-152 bs=32 fp16, HIP workers per MI355X (request-parallel, no RCCL)",
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


class Harness:
    """Prebuilt codelet calls (cl_arg + buffers + stream) for `workers` workers of one device."""

    def __init__(self, spi, replica, name, dev, batch, workers, rng, streams=None):
        import torch

        self.spi, self.lib, self.N = spi, spi.lib, spi._native
        self.torch = torch
        self.dev = dev
        self.replica = replica
        self.batch = batch
        # Reuse the worker streams of an earlier harness when given: each new HIP
        # stream takes a hardware queue, and queues beyond GPU_MAX_HW_QUEUES are shared.
        self.streams = list(streams) if streams is not None else [torch.cuda.Stream(dev) for _ in range(workers)]
        self.host_inputs, self.out_shape = make_inputs(name, batch, rng)
        self.d_in = [[torch.from_numpy(x).to(dev) for x in self.host_inputs] for _ in range(workers)]
        self.d_out = [torch.empty(self.out_shape, device=dev, dtype=torch.float32) for _ in range(workers)]
        torch.cuda.synchronize(dev)
        self.calls = []
        for w in range(workers):
            params = spi.make_params([list(x.shape) for x in self.d_in[w]], [x.dtype for x in self.d_in[w]],
                                     models_gpu=[replica], device_ids=[dev])
            bufs = spi.buffer_array([spi.tensor_interface(x) for x in self.d_in[w]] +
                                    [spi.tensor_interface(self.d_out[w])])
            self.calls.append((params.to_args(), bufs, self.streams[w]))

    def task(self, w, ev=None):
        a, bufs, st = self.calls[w]
        self.lib.spi_set_worker_context(w, self.dev, C.c_void_p(st.cuda_stream))
        if ev is not None:
            ev[0].record(st)
        self.lib.spi_hip_inference_func(bufs, C.byref(a))
        if ev is not None:
            ev[1].record(st)
        if a.status != self.N.SPI_OK:
            raise RuntimeError(a.error.decode())

    def throughput(self, steps, warmup, world=1, dist=None):
        """Timed region: `steps` rounds of one task per worker, no instrumentation
        inside (timing events on every task cost ~25 % of throughput on ROCm).
        Per-task latency comes from a separate pass of the same load with events."""
        torch = self.torch
        W = len(self.calls)
        for _ in range(warmup):
            for w in range(W):
                self.task(w)
        torch.cuda.synchronize(self.dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(self.dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            for w in range(W):
                self.task(w)
        torch.cuda.synchronize(self.dev)
        t1 = time.perf_counter()
        if world > 1:
            dist.barrier()
        elapsed = reduce_max_elapsed(t1 - t0, world)
        return elapsed, self.loaded_latency(min(steps, 50))

    def loaded_latency(self, steps):
        """Device latency of each task (events on its worker stream) with every worker busy."""
        torch = self.torch
        W = len(self.calls)
        events = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(W)]
                  for _ in range(steps)]
        for k in range(steps):
            for w in range(W):
                self.task(w, events[k][w])
        torch.cuda.synchronize(self.dev)
        return [s.elapsed_time(e) for step in events for (s, e) in step]

    def serial_e2e(self, iters):
        """pinned host -> H2D -> codelet -> D2H -> sync, one task in flight."""
        torch = self.torch
        st = self.streams[0]
        pinned_in = [torch.from_numpy(x).pin_memory() for x in self.host_inputs]
        pinned_out = torch.empty(self.out_shape, dtype=torch.float32).pin_memory()
        out = []
        for i in range(iters + 3):
            ts = time.perf_counter()
            with torch.cuda.stream(st):
                for h, d in zip(pinned_in, self.d_in[0]):
                    d.copy_(h, non_blocking=True)
                self.task(0)
                pinned_out.copy_(self.d_out[0], non_blocking=True)
            st.synchronize()
            if i >= 3:
                out.append((time.perf_counter() - ts) * 1e3)
        return out

    def dominant_kernel(self, precision, model=""):
        ops = self.replica.profile(self.d_in[0], self.d_out[0], self.streams[0].cuda_stream)
        totals = {}
        for op in ops:
            t = totals.setdefault(op["name"], [0.0, 0, op["flops"], op["bytes"]])
            t[0] += op["ms"]
            t[1] += 1
        name, (tot, cnt, flops, nbytes) = max(totals.items(), key=lambda kv: kv[1][0])
        ms = tot / cnt
        fwd_ms = sum(o["ms"] for o in ops)
        fwd_flops = sum(o["flops"] for o in ops)
        peak = PEAK_TFLOPS[precision]
        traffic, src = measured_traffic(model, self.batch, precision, name)
        common = {"kernel": name, "launches_per_forward": cnt, "traffic": traffic, "traffic_source": src,
                  "avg_launch_ms": round(ms, 5), "forward_share": round(tot / fwd_ms, 4),
                  "forward_frac": round(fwd_flops / (fwd_ms * 1e-3) / 1e12 / peak, 5)}
        if flops == 0:  # a byte-moving op dominates: HBM roofline on its algorithmic bytes
            ach = nbytes / (ms * 1e-3) / 1e9
            return {"bound": "hbm", "achieved": round(ach, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(ach / PEAK_HBM_GBS, 5), "algorithmic_bytes_per_launch": nbytes, **common}
        ach = flops / (ms * 1e-3) / 1e12
        return {"bound": "mfma", "achieved": round(ach, 3), "peak": peak, "unit": "TFLOP/s",
                "frac": round(ach / peak, 5), "algorithmic_flops_per_launch": flops,
                "mfma_issue_per_flop": 3 if precision == "fp16x3" else 1, **common}


def measured_traffic(model, batch, precision, op):
    """HBM bytes per launch of `op` from the committed PMC profile
    profiles/<round>/traffic_<model>_bs<batch>_<precision>.json (tools/pmc_traffic.sh:
    separate FETCH_SIZE / WRITE_SIZE passes, gfx950 FETCH x2 correction), or None."""
    import glob

    hits = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"traffic_{model}_bs{batch}_{precision}.json")))
    if not hits:
        return None, None
    with open(hits[-1]) as f:
        ops = json.load(f).get("ops", {})
    if op not in ops:
        return None, None
    return ops[op]["hbm_bytes_per_launch"], os.path.relpath(hits[-1], ROOT)


def runtime_e2e(spi, replica, name, batch, inflight=8, requests=160, workers=4, req_batch=None, coalesce=1,
                delay_us=0):
    """Closed loop through the mini-runtime (host buffers, pinned slots, H2D/D2H):
    inf/s = inferences / (last response - first request) (inference_client.cpp:259-270).
    req_batch < batch: requests of req_batch samples, merged by the runtime's dynamic
    batching into codelet calls of up to `batch` (coalesce jobs, delay_us wait)."""
    rtmod = importlib.import_module("starpu-inference-server_amd.runtime")
    rb = req_batch or batch
    host_inputs, out_shape = make_inputs(name, rb, np.random.default_rng(7))
    if name.startswith("bert"):
        in_specs = [((x.shape[1],), np.int64) for x in host_inputs]
    else:
        in_specs = [((3, 224, 224), np.float32)]
    out_elems = int(np.prod(out_shape[1:]))
    rt = rtmod.Runtime([replica], in_specs, [(out_elems, np.float32)], max_batch=batch, workers_per_device=workers,
                       coalesce_max_jobs=coalesce, coalesce_delay_us=delay_us)
    outs = [np.empty(out_shape, np.float32) for _ in range(inflight)]
    submitted = 0
    t0 = time.perf_counter()
    while submitted < requests:
        done = len(rt.completions)
        while submitted < requests and submitted - done < inflight:
            rt.submit(submitted, host_inputs, [outs[submitted % inflight]])
            submitted += 1
        time.sleep(0.0002)
    rt.drain()
    first = min(c.submit_ns for c in rt.completions)
    last = max(c.complete_ns for c in rt.completions)
    lat = [c.latency_ms for c in rt.completions]
    ok, failed = rt.stats()
    jobs_per_call = float(np.mean([c.task_jobs for c in rt.completions]))
    rt.close()
    return {"value": round(requests * rb / ((last - first) * 1e-9), 2), "unit": "inferences/s",
            "p50_latency_ms": round(percentile(lat, 50), 4), "p95_latency_ms": round(percentile(lat, 95), 4),
            "requests": requests, "request_batch": rb, "max_batch": batch, "inflight": inflight,
            "workers": workers, "coalesce_max_jobs": coalesce, "coalesce_delay_us": delay_us,
            "mean_jobs_per_codelet_call": round(jobs_per_call, 2), "failed": failed,
            "wall_s": round(time.perf_counter() - t0, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="resnet18", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--precision", default="fp16x3", choices=["fp16", "fp16x3", "fp32"])
    ap.add_argument("--workers", type=int, default=4, help="worker streams per GPU")
    ap.add_argument("--graphs", type=int, default=1, help="capture the forward body into hipGraphs")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--latency-iters", type=int, default=40)
    ap.add_argument("--extras", type=int, default=1, help="single-GPU extra measurements (0 = skip)")
    args = ap.parse_args()
    # One HIP hardware queue per worker stream: HIP maps streams onto
    # GPU_MAX_HW_QUEUES queues round-robin (default 4, shared with torch's own
    # streams), and worker streams that share a queue run serially -- measured
    # 28.4k -> 38.1k inf/s at 4 workers going from 4 to 8 queues (16 measured
    # the same as 8).  Room for two sets of worker streams: the harness's and the
    # mini-runtime extra's own.  Must be set before the first HIP call (DESIGN.md,
    # INTEGRATION.md).
    queues = min(32, max(int(os.environ.get("GPU_MAX_HW_QUEUES", "4")), 2 * args.workers + 4))
    os.environ["GPU_MAX_HW_QUEUES"] = str(queues)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    spi = importlib.import_module("starpu-inference-server_amd")
    zoo = importlib.import_module("starpu-inference-server_amd.zoo")

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    # SPI_BENCH_SHARE_DEVICE=1: every rank on device 0 (multi-rank rehearsal on a 1-GPU box only).
    dev = 0 if os.environ.get("SPI_BENCH_SHARE_DEVICE") == "1" else local_rank
    torch.cuda.set_device(dev)

    seq = 128
    model = zoo.build(args.model, seed=0)
    replica = spi.ModelReplica(model, dev, args.precision, max_batch=args.batch,
                               seq_len=seq if args.model.startswith("bert") else 0, graphs=bool(args.graphs))
    h = Harness(spi, replica, args.model, dev, args.batch, args.workers, np.random.default_rng(rank))
    elapsed, task_lat = h.throughput(args.steps, args.warmup, world, dist)
    value = world * args.workers * args.batch * args.steps / elapsed

    result = {
        "metric": BASELINE_METRIC,
        "value": round(value, 2),
        "unit": "inferences/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic (seeded U[0,1) images / uniform token ids, all-ones mask); random-init weights "
                "of the reference architecture (no checkpoints offline)",
        "config": {
            "workload": WORKLOADS[args.model],
            "batch_per_task": args.batch,
            "workers_per_gpu": args.workers,
            "tasks_per_step_per_gpu": args.workers,
            "precision_mode": {"fp16x3": "split-fp16 MFMA (hi/lo fp16 operands, fp32 accumulate): fp32-grade parity",
                               "fp16": "fp16 MFMA operands, fp32 accumulate", "fp32": "fp32 MFMA"}[args.precision],
            "graphs": bool(args.graphs),
            "hip_hw_queues": queues,
            "parallelism": f"replicas x{world} (request sharding, no collective)",
        },
        "p50_task_latency_ms": round(percentile(task_lat, 50), 4),
        "p95_task_latency_ms": round(percentile(task_lat, 95), 4),
    }
    if rank == 0:
        e2e = h.serial_e2e(args.latency_iters)
        result["p50_e2e_latency_ms_incl_h2d_d2h"] = round(percentile(e2e, 50), 4)
        result["e2e_inferences_per_s_serial"] = round(args.batch / (percentile(e2e, 50) * 1e-3), 2)
        result["model_gflop_per_inference"] = round(replica.flops(1) / 1e9, 4)
        result["model_tflops_per_gpu"] = round(replica.flops(1) * value / world / 1e12, 3)
        result["roofline"] = h.dominant_kernel(args.precision, args.model)

    if rank == 0 and args.cpu_seconds > 0:
        from oracle.cpu_codelet import cpu_inference

        cores = torch.get_num_threads()

        def cpu_sample(inputs, seconds, cap):
            cpu_inference(model, inputs)  # warm-up
            times = []
            while sum(times) < seconds and len(times) < cap:
                ts = time.perf_counter()
                cpu_inference(model, inputs)
                times.append(time.perf_counter() - ts)
            return times

        times = cpu_sample(h.host_inputs, args.cpu_seconds, 200)
        t_cpu = sum(times)
        result["cpu_baseline"] = {
            "value": round(len(times) * args.batch / t_cpu, 3), "unit": "inferences/s", "cores": cores,
            "kind": "port",
            "sample": f"{len(times)} forwards of the same {args.model} batch {args.batch} fp32 on host ATen "
                      f"(torch {torch.__version__}, {cores} intra-op threads), {t_cpu:.1f}s",
            "p50_ms": round(percentile([t * 1e3 for t in times], 50), 3)}
        if args.model == "resnet18":
            # BASELINE configs[0] (C1): the CPU codelet alone, ResNet-18 bs=1 fp32
            one = [x[:1] for x in h.host_inputs]
            t1 = cpu_sample(one, min(4.0, args.cpu_seconds), 400)
            result["cpu_baseline"]["c1_resnet18_bs1_fp32"] = {
                "value": round(len(t1) / sum(t1), 3), "unit": "inferences/s",
                "p50_ms": round(percentile([t * 1e3 for t in t1], 50), 3), "forwards": len(t1)}

    if rank == 0 and world == 1 and args.extras and args.model == "resnet18":
        extras = {}
        # plain fp16 operands on the same workload (faster, 1.8e-3 parity on this network)
        r16 = spi.ModelReplica(model, dev, "fp16", max_batch=args.batch, graphs=True)
        h16 = Harness(spi, r16, "resnet18", dev, args.batch, args.workers, np.random.default_rng(1), h.streams)
        el, lat = h16.throughput(args.steps, args.warmup)
        extras["resnet18_bs8_fp16_plain"] = {
            "value": round(args.workers * args.batch * args.steps / el, 2), "unit": "inferences/s",
            "p50_task_latency_ms": round(percentile(lat, 50), 4), "parity_normalised_max_err": 1.8e-3}
        # ResNet-18 bs=1 latency (the metric names it)
        r1 = spi.ModelReplica(model, dev, args.precision, max_batch=1, graphs=True)
        h1 = Harness(spi, r1, "resnet18", dev, 1, args.workers, np.random.default_rng(2), h.streams)
        el, lat = h1.throughput(args.steps, args.warmup)
        e2e1 = h1.serial_e2e(args.latency_iters)
        extras["resnet18_bs1"] = {"value": round(args.workers * args.steps / el, 2), "unit": "inferences/s",
                                  "p50_task_latency_ms": round(percentile(lat, 50), 4),
                                  "p50_e2e_latency_ms_incl_h2d_d2h": round(percentile(e2e1, 50), 4),
                                  "dtype": args.precision}
        # the PCIe-inclusive serving path through the mini-runtime (never `value`)
        extras["resnet18_bs8_runtime_pcie"] = runtime_e2e(spi, replica, "resnet18", args.batch)
        # bs=1 client requests, dynamically batched by the runtime into calls of <= 8
        extras["resnet18_bs1_requests_batched8_runtime_pcie"] = runtime_e2e(
            spi, replica, "resnet18", args.batch, inflight=64, requests=1280, req_batch=1, coalesce=args.batch,
            delay_us=500)
        del r16, h16, r1, h1
        # BERT-base seq128 bs8 fp16 (BASELINE configs[2])
        bmodel = zoo.build("bert_base", seed=0)
        rb = spi.ModelReplica(bmodel, dev, "fp16", max_batch=8, seq_len=seq, graphs=True)
        hb = Harness(spi, rb, "bert_base", dev, 8, args.workers, np.random.default_rng(3), h.streams)
        el, lat = hb.throughput(max(20, args.steps // 4), 5)
        e2eb = hb.serial_e2e(10)
        extras["bert_base_seq128_bs8_fp16"] = {
            "value": round(args.workers * 8 * max(20, args.steps // 4) / el, 2), "unit": "sequences/s",
            "p50_task_latency_ms": round(percentile(lat, 50), 4),
            "p50_e2e_latency_ms_incl_h2d_d2h": round(percentile(e2eb, 50), 4),
            "gflop_per_seq": round(rb.flops(1) / 1e9, 3), "roofline": hb.dominant_kernel("fp16", "bert_base")}
        result["extras"] = extras

    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
