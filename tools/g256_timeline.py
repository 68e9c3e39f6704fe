#!/usr/bin/env python3
"""Where a gemm256 launch spends its time, per workgroup, from the -DSPI_G256_TIMELINE build
(s_memrealtime at entry, after the prologue's first wait, after the k-loop, at exit).

For each shape (ViT-L bs16 / BERT-base bs8 transformer GEMMs with their model epilogues) the
GEMM is launched `reps` times back to back and the last launch's stamps are read:

  span        first entry -> last exit
  skew        first entry -> last entry
  pro / loop / epi   per workgroup: entry -> first wait done -> k-loop done -> exit (mean / max)

usage: SPI_HIP_LIB=tools/libspi_g256tl.so python tools/g256_timeline.py
(build: tools/build_variant.sh tools/libspi_g256tl.so WORKTREE -DSPI_G256_TIMELINE)"""
import ctypes as C
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ops = importlib.import_module("starpu-inference-server_amd.ops")

SHAPES = [("vit_qkv", 3152, 3072, 1024, "f16", None), ("vit_ff1", 3152, 4096, 1024, "f16", "gelu"),
          ("vit_out", 3152, 1024, 1024, "f32res", None), ("vit_ff2", 3152, 1024, 4096, "f32res", None),
          ("sq4096", 4096, 4096, 4096, "f16", None)]


def main():
    lib = ops.lib
    fn = lib.spi_debug_g256_timeline
    fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_size_t]
    ws = ops.workspace()
    rng = np.random.default_rng(0)
    for name, M, N, K, epi, act in SHAPES:
        A = torch.randn(M, K, device="cuda").half()
        wp = ops.pack_weight("fp16", rng.standard_normal((N, K)).astype(np.float32) * 0.05)
        bias = torch.randn(N, device="cuda") * 0.1
        res = torch.randn(M, N, device="cuda") if epi == "f32res" else None
        out = torch.empty(M, N, device="cuda", dtype=torch.float32 if epi == "f32res" else torch.float16)
        for _ in range(20):
            ops.gemm("fp16", A, wp, N, bias=bias, residual=res, out=out, act=act, ws=ws)
        torch.cuda.synchronize()
        wgs = ((M + 255) // 256) * (N // 256)
        buf = (C.c_ulonglong * (wgs * 6))()
        fn(buf, wgs * 6)
        t = np.frombuffer(buf, dtype=np.uint64).reshape(wgs, 6).astype(np.int64)
        t0 = t[:, 0].min()
        e, p1, l1, x = (t[:, 0] - t0) * 10e-3, (t[:, 1] - t0) * 10e-3, (t[:, 2] - t0) * 10e-3, (t[:, 3] - t0) * 10e-3
        pro, loop, epi_t = p1 - e, l1 - p1, x - l1
        print(f"{name:8s} M={M} N={N} K={K} wgs={wgs}: span {x.max():6.2f} us  skew {e.max():5.2f}  "
              f"pro {pro.mean():5.2f}/{pro.max():5.2f}  loop {loop.mean():6.2f}/{loop.max():6.2f} "
              f"({loop.mean() / (K // 64) * 1e3:5.0f} ns per k-tile)  epi {epi_t.mean():5.2f}/{epi_t.max():5.2f}",
              flush=True)


if __name__ == "__main__":
    main()
