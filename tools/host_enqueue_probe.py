#!/usr/bin/env python3
"""Is the timed loop host-bound?  Times the enqueue loop (host) apart from the device drain, for
one enqueueing thread (bench.py's Harness.rounds) and for one thread per worker (StarPU's layout:
each worker thread calls the codelet on its own stream).

usage: python tools/host_enqueue_probe.py [--model resnet18 --batch 8 --precision fp16m]"""
import argparse
import importlib
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--precision", default="fp16m")
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--tasks", type=int, default=160, help="tasks per worker per timed pass")
    args = ap.parse_args()
    os.environ.setdefault("GPU_MAX_HW_QUEUES", str(2 * args.workers + 8))
    import torch
    bench = importlib.import_module("bench")
    spi = importlib.import_module("starpu-inference-server_amd")
    zoo = importlib.import_module("starpu-inference-server_amd.zoo")
    model = zoo.build(args.model, seed=0)
    rep = spi.ModelReplica(model, 0, args.precision, max_batch=args.batch,
                           seq_len=128 if args.model.startswith("bert") else 0, graphs=True)
    h = bench.Harness(spi, rep, args.model, 0, args.batch, args.workers, np.random.default_rng(3))
    W = args.workers
    h.rounds(10)
    torch.cuda.synchronize()

    # host cost of one codelet call with the device idle (queue empty)
    t = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h.task(0)
        t.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    print(f"one call, idle device: host {np.median(t) * 1e6:.1f} us (median of 20)")

    for rep_i in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h.rounds(args.tasks)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        n = args.tasks * W * args.batch
        print(f"single thread: enqueue {(t1 - t0) * 1e3:.1f} ms, drain {(t2 - t1) * 1e3:.1f} ms, "
              f"{n / (t2 - t0):.0f} inf/s, host us per call {(t1 - t0) / (args.tasks * W) * 1e6:.1f}")

        def worker(w, out):
            a0 = time.perf_counter()
            for _ in range(args.tasks):
                h.task(w)
            out[w] = time.perf_counter() - a0

        torch.cuda.synchronize()
        out = [0.0] * W
        ths = [threading.Thread(target=worker, args=(w, out)) for w in range(W)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"thread per worker: enqueue {(t1 - t0) * 1e3:.1f} ms (per thread max {max(out) * 1e3:.1f}), "
              f"drain {(t2 - t1) * 1e3:.1f} ms, {n / (t2 - t0):.0f} inf/s")


if __name__ == "__main__":
    main()
