#!/usr/bin/env python3
"""Per-op device times of one forward (HIP events around every launch).

usage: python tools/op_profile.py [--model resnet18] [--precision fp16] [--batch 8]
"""
import argparse
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--precision", default="fp16")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    spi = importlib.import_module("starpu-inference-server_amd")
    zoo = importlib.import_module("starpu-inference-server_amd.zoo")
    m = zoo.build(a.model)
    bert = a.model.startswith("bert")
    rep = spi.ModelReplica(m, 0, a.precision, max_batch=a.batch, seq_len=128 if bert else 0)
    rng = np.random.default_rng(0)
    if bert:
        ins = [torch.from_numpy(rng.integers(0, 30522, (a.batch, 128))).cuda(),
               torch.ones(a.batch, 128, dtype=torch.int64, device="cuda")]
        out = torch.empty(a.batch, 128, 768, device="cuda")
    else:
        ins = [torch.from_numpy(rng.random((a.batch, 3, 224, 224), dtype=np.float32)).cuda()]
        out = torch.empty(a.batch, 1000, device="cuda")
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    runs = [rep.profile(ins, out, s.cuda_stream) for _ in range(a.reps)]
    ops = runs[-1]
    med = [float(np.median([r[i]["ms"] for r in runs])) for i in range(len(ops))]
    tot = sum(med)
    print(f"{rep.description}: {len(ops)} ops, sum {tot*1e3:.1f} us")
    for op, t in zip(ops, med):
        tf = op["flops"] / (t * 1e-3) / 1e12 if t > 0 else 0
        gbs = op["bytes"] / (t * 1e-3) / 1e9 if t > 0 else 0
        print(f"  {op['name']:<40s} {t*1e3:8.2f} us  {tf:8.1f} TF/s  {gbs:8.1f} GB/s")


if __name__ == "__main__":
    main()
