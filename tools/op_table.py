#!/usr/bin/env python3
"""Per-op device time of one forward, isolated and under the bench's four-stream load
(bench.Harness.op_profile: hipEvents around every launch on worker 0's stream).

usage: python tools/op_table.py [--model resnet18] [--precision fp16x3] [--batch 8]"""
import argparse
import importlib
import os
import sys

os.environ["GPU_MAX_HW_QUEUES"] = "16"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--precision", default="fp16x3")
    ap.add_argument("--batch", type=int, default=8)
    a = ap.parse_args()
    import bench
    spi = importlib.import_module("starpu-inference-server_amd")
    zoo = importlib.import_module("starpu-inference-server_amd.zoo")
    m = zoo.build(a.model)
    rep = spi.ModelReplica(m, 0, a.precision, max_batch=a.batch, seq_len=128 if a.model.startswith("bert") else 0,
                           graphs=True)
    h = bench.Harness(spi, rep, a.model, 0, a.batch, 4, np.random.default_rng(0))
    el = h.throughput(20, 3, 8)
    print(f"{rep.description}: {4 * 8 * 20 * a.batch / el:.0f} inf/s (4 streams)")
    iso = h.op_profile(False, 7)
    load = h.op_profile(True, 7)
    ti = sum(v[0] for v in iso.values())
    tl = sum(v[0] for v in load.values())
    print(f"{'op':44s} {'n':>3s} {'iso_us':>8s} {'load_us':>8s} {'iso%':>6s} {'load%':>6s} {'TF/s iso':>9s}")
    for k in sorted(iso, key=lambda k: -load[k][0]):
        t, n, f, b = iso[k]
        tflops = f * n / (t * 1e-3) / 1e12 if t > 0 else 0
        print(f"{k[:44]:44s} {n:3d} {t * 1e3:8.1f} {load[k][0] * 1e3:8.1f} {100 * t / ti:6.1f} {100 * load[k][0] / tl:6.1f} "
              f"{tflops:9.1f}")
    print(f"{'total':44s}     {ti * 1e3:8.1f} {tl * 1e3:8.1f}")


if __name__ == "__main__":
    main()
