#!/usr/bin/env python3
"""Host-to-device bandwidth of pinned 4.8 MB transfers (one ResNet bs8 task's input) on 1, 2, 4
streams, and of pageable -> pinned host copies (the runtime's staging), for the e2e ceiling."""
import time

import numpy as np
import torch

N = 8 * 3 * 224 * 224 * 4
REPS = 200
for nst in [1, 2, 4]:
    streams = [torch.cuda.Stream() for _ in range(nst)]
    src = [torch.empty(N, dtype=torch.uint8).pin_memory() for _ in range(nst)]
    dst = [torch.empty(N, dtype=torch.uint8, device="cuda") for _ in range(nst)]
    for i in range(nst):
        with torch.cuda.stream(streams[i]):
            dst[i].copy_(src[i], non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for r in range(REPS):
        i = r % nst
        with torch.cuda.stream(streams[i]):
            dst[i].copy_(src[i], non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"H2D pinned, {nst} stream(s): {REPS * N / dt / 1e9:.1f} GB/s", flush=True)
    out = torch.empty(1000 * 8 * 4, dtype=torch.uint8).pin_memory()
d2h_src = torch.empty(N, dtype=torch.uint8, device="cuda")
d2h_dst = torch.empty(N, dtype=torch.uint8).pin_memory()
torch.cuda.synchronize()
t0 = time.perf_counter()
for r in range(REPS):
    d2h_dst.copy_(d2h_src, non_blocking=True)
torch.cuda.synchronize()
print(f"D2H pinned: {REPS * N / (time.perf_counter() - t0) / 1e9:.1f} GB/s", flush=True)
a = np.random.default_rng(0).random(N // 4, dtype=np.float32)
b = torch.empty(N // 4, dtype=torch.float32).pin_memory().numpy()
t0 = time.perf_counter()
for r in range(50):
    np.copyto(b, a)
print(f"host pageable -> pinned memcpy, 1 thread: {50 * N / (time.perf_counter() - t0) / 1e9:.1f} GB/s", flush=True)
