#!/usr/bin/env python3
"""Fused stem (stem_pool) launch time: 200 back-to-back launches between two events,
per precision and rows-per-workgroup, ResNet bs8 @ 224."""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ops = importlib.import_module("starpu-inference-server_amd.ops")
lib = ops.lib
import ctypes as C

B = int(os.environ.get("B", "8"))
x = torch.rand(B, 3, 224, 224, device="cuda")
w = torch.randn(64, 3, 7, 7) * 0.1
b = torch.randn(64, device="cuda") * 0.1
host = np.empty(lib.spi_op_stem_pool_bytes(), dtype=np.uint8)
lib.spi_op_stem_pool_pack(np.ascontiguousarray(w.numpy()).ctypes.data, host.ctypes.data)
wp = torch.from_numpy(host).cuda()
y = torch.empty(B, 56, 56, 64 * 2, device="cuda", dtype=torch.float16)
s = torch.cuda.current_stream().cuda_stream
flops = 2.0 * B * 112 * 112 * 64 * 147
only = os.environ.get("STEM_ONLY")  # e.g. "fp16m:1"
for prec, name in [(1, "fp16"), (2, "fp16m"), (3, "fp16x3s")]:
    for rows in (0, 1, 2):
        if only and only != f"{name}:{rows}":
            continue
        call = lambda: lib.spi_op_stem_pool(prec, ops._ptr(x), B, 224, 224, ops._ptr(wp), ops._ptr(b), ops._ptr(y),
                                            rows, C.c_void_p(s))
        for _ in range(10):
            call()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            call()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 200 * 1e3
        print(f"stem_pool {name:8s} rows/wg {rows}: {us:7.2f} us  {flops / us / 1e6:7.1f} TF/s (algorithmic)", flush=True)
