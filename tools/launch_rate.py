#!/usr/bin/env python3
"""Kernel-boundary rate: how many dependent kernels per second the GPU retires
when W streams each replay a hipGraph of K small dependent kernels (the shape of
a captured forward: ResNet-18 ~24 kernels, BERT-base ~86).

usage: python tools/launch_rate.py [--kernels 24] [--bytes 1048576] [--reps 200]
Prints, for 1/2/4 streams: kernels/s retired and microseconds per kernel per
stream.  If four streams of trivial kernels retire only ~2e5 kernels/s, a
forward of K kernels cannot exceed 2e5/K forwards/s whatever its kernels cost.
"""
import argparse
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", type=int, default=24)
    ap.add_argument("--bytes", type=int, default=1 << 20, help="bytes each kernel reads and writes")
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    n = a.bytes // 4
    for W in (1, 2, 4):
        streams = [torch.cuda.Stream() for _ in range(W)]
        bufs = [torch.zeros(n, device="cuda") for _ in range(W)]
        graphs = []
        for w in range(W):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(streams[w]):
                bufs[w].add_(1.0)  # warm
                torch.cuda.current_stream().synchronize()
                with torch.cuda.graph(g, stream=streams[w]):
                    for _ in range(a.kernels):
                        bufs[w].add_(1.0)
            graphs.append(g)
        torch.cuda.synchronize()
        for w in range(W):
            with torch.cuda.stream(streams[w]):
                graphs[w].replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            for w in range(W):
                with torch.cuda.stream(streams[w]):
                    graphs[w].replay()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        k = a.reps * W * a.kernels
        print(f"streams={W} kernels/graph={a.kernels} bytes/kernel={a.bytes}: {k / dt:10.0f} kernels/s, "
              f"{dt / (a.reps * a.kernels) * 1e6:6.2f} us per kernel per stream", flush=True)


if __name__ == "__main__":
    main()
