#!/usr/bin/env python3
"""Host enqueue cost of one codelet task vs its device time (is the bench host-bound?).

usage: python tools/host_overhead.py [--model resnet18] [--precision fp16x3] [--batch 8]
Prints, for graphs off/on and 1/4 workers: host microseconds inside
spi_hip_inference_func per task, device microseconds per task (events), and
tasks/s when the host issues back to back.
"""
import argparse
import importlib
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--precision", default="fp16x3")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    bench = importlib.import_module("bench")
    spi = importlib.import_module("starpu-inference-server_amd")
    zoo = importlib.import_module("starpu-inference-server_amd.zoo")
    m = zoo.build(a.model)
    bert = a.model.startswith("bert")
    rep = spi.ModelReplica(m, 0, a.precision, max_batch=a.batch, seq_len=128 if bert else 0)
    for graphs in (0, 1):
        rep.set_graphs(bool(graphs))
        for workers in (1, 4):
            h = bench.Harness(spi, rep, a.model, 0, a.batch, workers, np.random.default_rng(0))
            for w in range(workers):
                for _ in range(3):
                    h.task(w)
            torch.cuda.synchronize()
            host = []
            t0 = time.perf_counter()
            for i in range(a.iters):
                ts = time.perf_counter()
                h.task(i % workers)
                host.append(time.perf_counter() - ts)
            t_issue = time.perf_counter() - t0
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            # device time of one task alone (stream idle before and after)
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            dev = []
            for _ in range(20):
                torch.cuda.synchronize()
                h.task(0, ev)
                torch.cuda.synchronize()
                dev.append(ev[0].elapsed_time(ev[1]) * 1e3)
            print(f"graphs={graphs} workers={workers}: host/task {np.median(host) * 1e6:7.1f} us "
                  f"(issue loop {t_issue / a.iters * 1e6:7.1f} us/task), wall/task {wall / a.iters * 1e6:7.1f} us, "
                  f"device/task alone {np.median(dev):7.1f} us, {a.iters * a.batch / wall:8.0f} inf/s", flush=True)


if __name__ == "__main__":
    main()
