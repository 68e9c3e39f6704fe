#!/usr/bin/env python3
"""Per-op device time of one forward, isolated and under the four-stream load (bench.Harness
.op_profile), plus each op's back-to-back steady-state launch time (Model::profile_op).

usage: python tools/loaded_ops.py [--model resnet18] [--precision fp16m] [--batch 8]"""
import argparse
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--precision", default="fp16m")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--workers", type=int, default=4)
    a = ap.parse_args()
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
    import torch
    bench = importlib.import_module("bench")
    spi = importlib.import_module("starpu-inference-server_amd")
    zoo = importlib.import_module("starpu-inference-server_amd.zoo")
    m = zoo.build(a.model, seed=0)
    rep = spi.ModelReplica(m, 0, a.precision, max_batch=a.batch, seq_len=128 if a.model.startswith("bert") else 0,
                           graphs=True)
    h = bench.Harness(spi, rep, a.model, 0, a.batch, a.workers, np.random.default_rng(0))
    h.rounds(4)
    torch.cuda.synchronize()
    iso = h.op_profile(False)
    lo = h.op_profile(True)
    tot_i = sum(v[0] for v in iso.values())
    tot_l = sum(v[0] for v in lo.values())
    print(f"{'op':36s} {'n':>3s} {'iso us':>8s} {'load us':>8s} {'share':>6s} {'b2b us':>8s} {'TF/s b2b':>9s}")
    for name, (t_l, cnt, fl, by) in sorted(lo.items(), key=lambda kv: -kv[1][0]):
        b2b = rep.profile_op(h.d_in[0], h.d_out[0], h.streams[0].cuda_stream, name, 50)
        print(f"{name:36s} {cnt:3d} {iso[name][0] * 1e3 / cnt:8.2f} {t_l * 1e3 / cnt:8.2f} {t_l / tot_l:6.3f} "
              f"{b2b['ms'] * 1e3:8.2f} {fl / (b2b['ms'] * 1e-3) / 1e12 if fl else 0:9.1f}", flush=True)
    print(f"forward: isolated {tot_i * 1e3:.1f} us, loaded {tot_l * 1e3:.1f} us (sum of per-op event times)")


if __name__ == "__main__":
    main()
