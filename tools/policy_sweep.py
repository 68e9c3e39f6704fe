#!/usr/bin/env python3
"""Four-stream throughput of whole forwards under several GEMM plan policies, one
process, rounds interleaved (the bench's timed loop: `--workers` worker streams
replaying the captured forward back to back).

Each policy is a set of environment knobs read by the library (SPI_GEMM_256_MIN,
SPI_GEMM_HALO_CFG, SPI_GEMM_MAXSPLIT, ...); the knobs are re-read and a fresh
replica (fresh graphs) is built per policy.

usage: python tools/policy_sweep.py --model resnet18 --batch 8 --precision fp16x3 \
           --policy base= --policy 'l4=SPI_GEMM_HALO_CFG=7:128,s;0:0' ...
A policy is NAME=KEY=VALUE[&KEY=VALUE...] (NAME= alone: the defaults).
"""
import argparse
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KNOBS = ["SPI_STEM_FUSED", "SPI_GEMM_256_MIN", "SPI_GEMM_256_LONGK", "SPI_GEMM_HALO_CFG", "SPI_GEMM_WIN",
         "SPI_GEMM_MAXSPLIT", "SPI_GEMM_PLAN", "SPI_CONV_WRES", "SPI_LN_FOLD", "SPI_QKV_ATTN", "SPI_GEMM_256_ORDER", "SPI_GEMM_PLAN_LONGK"]


def parse(p):
    name, _, rest = p.partition("=")
    env = {}
    for kv in filter(None, rest.split("&")):
        k, _, v = kv.partition("=")
        env[k] = v
    return name, env


def make_streams(torch, workers, mode, ncu=256):
    if mode == "none":
        return [torch.cuda.Stream() for _ in range(workers)]
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    out = []
    for w in range(workers):
        bits = [(i // (ncu // workers) == w) if mode == "block" else (i % workers == w) for i in range(ncu)]
        words = (C.c_uint32 * (ncu // 32))(*[sum(1 << b for b in range(32) if bits[32 * j + b]) for j in range(ncu // 32)])
        st = C.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(C.byref(st), C.c_uint32(ncu // 32), words)
        if rc != 0:
            raise RuntimeError(f"hipExtStreamCreateWithCUMask failed: {rc}")
        out.append(torch.cuda.ExternalStream(st.value))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--precision", default="fp16x3")
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--tasks-per-step", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--policy", action="append", default=[])
    ap.add_argument("--cu-mask", default="none", choices=["none", "block", "stride"],
                    help="worker streams on disjoint CU subsets (hipExtStreamCreateWithCUMask): contiguous CU ids "
                         "(block) or every workers-th id (stride)")
    a = ap.parse_args()
    os.environ["GPU_MAX_HW_QUEUES"] = str(max(int(os.environ.get("GPU_MAX_HW_QUEUES", "4")), 2 * a.workers + 8))
    import torch

    bench = importlib.import_module("bench")
    spi = importlib.import_module("starpu-inference-server_amd")
    zoo = importlib.import_module("starpu-inference-server_amd.zoo")
    model = zoo.build(a.model, seed=0)
    pols = [parse(p) for p in (a.policy or ["base="])]
    streams = make_streams(torch, a.workers, a.cu_mask)
    seq = 128 if a.model.startswith("bert") else 0
    res = {n: [] for n, _ in pols}
    for _ in range(a.rounds):
        for name, env in pols:
            for k in KNOBS:
                os.environ.pop(k, None)
            os.environ.update(env)
            spi.lib.spi_debug_gemm_reload_env()
            rep = spi.ModelReplica(model, 0, a.precision, max_batch=a.batch, seq_len=seq, graphs=True)
            h = bench.Harness(spi, rep, a.model, 0, a.batch, a.workers, np.random.default_rng(0), streams)
            el = h.throughput(a.steps, 3, a.tasks_per_step)
            res[name].append(a.workers * a.tasks_per_step * a.steps * a.batch / el)
            del h, rep
            torch.cuda.synchronize()
    for name, env in pols:
        v = res[name]
        print(f"{name:24s} {np.median(v):10.1f} inf/s  (min {min(v):.1f} max {max(v):.1f})  {env}", flush=True)


if __name__ == "__main__":
    main()
