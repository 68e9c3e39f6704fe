#!/usr/bin/env python3
"""Library reference point (not a product path): torch.matmul (hipBLASLt / rocBLAS) fp16 on the
transformer GEMM shapes, back-to-back launches timed with events, beside tools/gemm_bench.py."""
import torch

SHAPES = [("bert_qkv", 1024, 2304, 768), ("bert_out", 1024, 768, 768), ("bert_ff1", 1024, 3072, 768),
          ("bert_ff2", 1024, 768, 3072), ("vit_qkv", 3152, 3072, 1024), ("vit_ff1", 3152, 4096, 1024),
          ("vit_ff2", 3152, 1024, 4096), ("sq4096", 4096, 4096, 4096)]
for name, M, N, K in SHAPES:
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    w = torch.randn(N, K, device="cuda", dtype=torch.float16)
    for _ in range(3):
        torch.matmul(a, w.t())
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    s.record()
    for _ in range(reps):
        torch.matmul(a, w.t())
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    print(f"torch {name:10s} M={M:5d} N={N:5d} K={K:5d} {ms * 1e3:8.2f} us {2 * M * N * K / (ms * 1e-3) / 1e12:8.1f} TF/s",
          flush=True)
