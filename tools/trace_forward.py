#!/usr/bin/env python3
"""Run isolated single forwards (one task, stream drained before and after) so a
rocprofv3 --kernel-trace shows each forward's kernel durations and the idle gaps
between its dependent launches.

usage: rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -- \
           python tools/trace_forward.py [--model resnet18] [--precision fp16x3] [--graphs 1]
       python tools/trace_forward.py --analyze gpurun_out/trace   (gaps per forward)
"""
import argparse
import csv
import glob
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def analyze(path):
    files = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # forwards are separated by host syncs: split where the idle gap exceeds 200 us
    fwd, cur, last_end = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if last_end is not None and s - last_end > 200_000:
            fwd.append(cur)
            cur = []
        cur.append((s, e, r["Kernel_Name"]))
        last_end = e
    fwd.append(cur)
    n = max(len(f) for f in fwd)
    full = [f for f in fwd if len(f) == n][3:]
    busy = [sum(e - s for s, e, _ in f) / 1e3 for f in full]
    span = [(f[-1][1] - f[0][0]) / 1e3 for f in full]
    print(f"{len(full)} forwards of {n} kernels: span {np.median(span):.1f} us, kernels busy {np.median(busy):.1f} us, "
          f"gaps {np.median(span) - np.median(busy):.1f} us ({(np.median(span) - np.median(busy)) / max(n - 1, 1):.2f} us/launch)")
    f = full[len(full) // 2]
    for i, (s, e, name) in enumerate(f):
        gap = (s - f[i - 1][1]) / 1e3 if i else 0.0
        print(f"  gap {gap:6.2f}  dur {(e - s) / 1e3:7.2f}  {name[:100]}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--precision", default="fp16x3")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--graphs", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--analyze", default="")
    ap.add_argument("--ops-out", default="", help="write the forward's op names (launch order) to this JSON file")
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze)
        return
    import time

    import torch
    bench = importlib.import_module("bench")
    spi = importlib.import_module("starpu-inference-server_amd")
    zoo = importlib.import_module("starpu-inference-server_amd.zoo")
    m = zoo.build(a.model)
    rep = spi.ModelReplica(m, 0, a.precision, max_batch=a.batch, seq_len=128 if a.model.startswith("bert") else 0)
    h = bench.Harness(spi, rep, a.model, 0, a.batch, 1, np.random.default_rng(0))
    if a.ops_out:  # op names in launch order (one eager profiled forward; tools/pmc_traffic.py maps dispatches)
        import json
        rows = rep.launch_table(h.d_in[0], h.d_out[0], h.streams[0].cuda_stream)  # one entry per kernel launch
        with open(a.ops_out, "w") as f:
            json.dump([r["op"] for r in rows], f)
    rep.set_graphs(bool(a.graphs))
    for _ in range(a.iters):
        torch.cuda.synchronize()
        time.sleep(0.001)
        h.task(0)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
