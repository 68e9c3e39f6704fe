#!/usr/bin/env python3
"""Isolate a failing 3x3 conv case: the same conv under SPI_GEMM_WIN x SPI_GEMM_MAXSPLIT x
residual, each printed with its plan, normalised error and non-finite count."""
import ctypes as C
import importlib
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.cpu_codelet import normalized_max_error  # noqa: E402

ops = importlib.import_module("starpu-inference-server_amd.ops")
B, H, cin, cout = [int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (8, 14, 256, 256))]
prec = sys.argv[5] if len(sys.argv) > 5 else "fp16"
split = prec == "fp16x3s"
g = torch.Generator().manual_seed(1)
x = torch.randn(B, H, H, cin, generator=g)
w = torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (cin * 9)) ** 0.5
b = torch.randn(cout, generator=g)
r = torch.randn(B, H, H, cout, generator=g)
xin = ops.to_split(x) if split else x.half()
x_val = ops.from_split(xin) if split else xin.float()
wp = ops.pack_weight(prec, ops.conv_weight_matrix(w, cin))
os.environ["SPI_GEMM_HALO_CFG"] = "0"
os.environ["SPI_CONV_WRES"] = "0"
for res in (False, True):
    rin = (ops.to_split(r) if split else r.half()) if res else None
    ref = F.conv2d(x_val.permute(0, 3, 1, 2), w if split else w.half().float(), b, 1, 1).permute(0, 2, 3, 1)
    if res:
        ref = ref + (ops.from_split(rin) if split else rin.float())
    ref = F.relu(ref)
    for win in ("0", "1"):
        for ms in ("1", "0"):
            os.environ["SPI_GEMM_WIN"] = win
            if ms == "0":
                os.environ.pop("SPI_GEMM_MAXSPLIT", None)
            else:
                os.environ["SPI_GEMM_MAXSPLIT"] = ms
            ops.lib.spi_debug_gemm_reload_env()
            pl = (C.c_int * 8)()
            ops.lib.spi_debug_conv_plan(3 if split else 1, B, H, H, cin, cout, 3, 3, 1, 1, pl)
            for rep in range(2):
                out = ops.conv2d(prec, xin.cuda(), wp, cout, 3, 3, 1, 1, bias=b.cuda(), act="relu",
                                 residual=rin.cuda() if res else None)
                torch.cuda.synchronize()
                o = ops.from_split(out.cpu()) if split else out.float().cpu()
                bad = (~torch.isfinite(o)).sum().item()
                err = normalized_max_error(torch.nan_to_num(o, 0.0, 0.0, 0.0).numpy(), ref.numpy())
                diff = (torch.nan_to_num(o, 0.0, 0.0, 0.0) - ref).abs()
                worst = diff.flatten().argmax().item()
                print(f"res={res} win={win} maxsplit={ms} plan={list(pl)} rep={rep} err={err:.3e} nonfinite={bad} "
                      f"worst_flat={worst} (row {worst // cout}, col {worst % cout})", flush=True)
