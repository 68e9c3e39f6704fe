#!/usr/bin/env python3
"""How many kernels from different worker streams run at the same time?

Each stream gets its own chain of R long GEMM launches whose grid is G workgroups
(SPI_GEMM_PLAN forces 64x64 tiles, no split: G = (M/64) * (N/64)); with W streams
the wall time of all chains is compared with one chain alone.  W kernels that
truly overlap (G * W well under the CUs) keep the time flat; a runtime or
hardware limit on concurrent kernels shows as time growing with W.

usage: SPI_GEMM_PLAN=64,64,2,1 python tools/stream_concurrency.py [--wg 16] [--k 16384]
"""
import argparse
import importlib
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--wg", type=int, default=16, help="workgroups per launch (M = 64 * wg, N = 64)")
    ap.add_argument("--k", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    assert os.environ.get("SPI_GEMM_PLAN"), "set SPI_GEMM_PLAN=64,64,2,1 (one tile per workgroup, no split)"
    ops = importlib.import_module("starpu-inference-server_amd.ops")
    M, N, K = 64 * a.wg, 64, a.k
    w = (np.random.default_rng(0).standard_normal((N, K)) * 0.01).astype(np.float32)
    wp = ops.pack_weight("fp16", w)
    A = torch.randn(M, K, device="cuda").half()
    for W in (1, 2, 4, 6, 8):
        streams = [torch.cuda.Stream() for _ in range(W)]
        outs = [torch.empty(M, N, device="cuda") for _ in range(W)]
        wss = [ops.workspace() for _ in range(W)]
        for i in range(W):  # warm
            ops.gemm("fp16", A, wp, N, out=outs[i], ws=wss[i], stream=streams[i].cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            for i in range(W):
                ops.gemm("fp16", A, wp, N, out=outs[i], ws=wss[i], stream=streams[i].cuda_stream)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.reps * 1e6
        print(f"streams={W} wg/launch={a.wg}: {dt:8.1f} us per round of {W} launches "
              f"({dt / W:7.1f} us per launch)", flush=True)


if __name__ == "__main__":
    main()
