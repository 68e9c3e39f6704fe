#!/usr/bin/env python3
"""Micro-benchmark of the GEMM / implicit-GEMM conv kernel on model layer shapes.

Times `--reps` back-to-back launches with HIP events on one stream (steady
state, no host gaps) and prints TFLOP/s per shape.
"""
import argparse
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ops = importlib.import_module("starpu-inference-server_amd.ops")

# (name, B, H, Cin, Cout, k, stride)  ResNet-18 bs8 layer shapes (+ stem with Cin padded to 8)
CONVS = [("stem7x7", 8, 224, 8, 64, 7, 2), ("l1_3x3", 8, 56, 64, 64, 3, 1), ("l2_3x3s2", 8, 56, 64, 128, 3, 2),
         ("l2_ds1x1", 8, 56, 64, 128, 1, 2), ("l2_3x3", 8, 28, 128, 128, 3, 1), ("l3_3x3s2", 8, 28, 128, 256, 3, 2),
         ("l3_ds1x1", 8, 28, 128, 256, 1, 2), ("l3_3x3", 8, 14, 256, 256, 3, 1), ("l4_3x3s2", 8, 14, 256, 512, 3, 2),
         ("l4_ds1x1", 8, 14, 256, 512, 1, 2), ("l4_3x3", 8, 7, 512, 512, 3, 1)]
# (name, M, N, K)  BERT-base bs8 S128 / ViT-L bs16
GEMMS = [("bert_qkv", 1024, 2304, 768), ("bert_out", 1024, 768, 768), ("bert_ff1", 1024, 3072, 768),
         ("bert_ff2", 1024, 768, 3072), ("vit_qkv", 3152, 3072, 1024), ("vit_ff1", 3152, 4096, 1024),
         ("vit_ff2", 3152, 1024, 4096), ("sq4096", 4096, 4096, 4096)]


EAGER = False


def timeit(fn, reps):
    """Device time per launch: `reps` launches captured in one graph, replayed
    (--eager: plain launches, for PMC profiling)."""
    fn()
    if EAGER:
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (3 * reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prec", default="fp16")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--only", default="")
    ap.add_argument("--plans", default="", help="';'-separated SPI_GEMM_PLAN values to sweep ('' = the chooser)")
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--halo-cfgs", default="", help="';'-separated SPI_GEMM_HALO_CFG values to sweep ('' = the chooser)")
    ap.add_argument("--model-epi", action="store_true",
                    help="the transformer plans' epilogues: qkv bias->fp16, ff1 bias+GELU->fp16, out/ff2 "
                         "bias+fp32 residual->fp32 (default: no bias, fp32 out)")
    ap.add_argument("--kscan", default="", help="MxN: time an f16+bias GEMM of that shape for K = 64 .. 4096")
    ap.add_argument("--epi-variants", action="store_true", help="with --model-epi: GELU launches also without GELU")
    ap.add_argument("--batch", type=int, default=0, help="override the conv batch (ResNet-152 bs32: 32)")
    ap.add_argument("--envs", default="", help="';'-separated knob sets KEY=VAL[&KEY=VAL] to sweep "
                                               "(e.g. 'SPI_CONV_WRES=0;SPI_GEMM_MAXSPLIT=1')")
    a = ap.parse_args()
    global EAGER
    EAGER = a.eager
    plans = a.plans.split(";") if a.plans else [""]
    if a.halo_cfgs:
        plans = [("halo", c) for c in a.halo_cfgs.split(";")]
    if a.envs:
        plans = [("env", c) for c in a.envs.split(";")]

    def sweep(fn, label, fl):
        for plan in plans:
            if isinstance(plan, tuple) and plan[0] == "env":
                for other in plans:  # knobs of the other sets: back to their defaults
                    for kv in filter(None, other[1].split("&")):
                        os.environ.pop(kv.partition("=")[0], None)
                for kv in filter(None, plan[1].split("&")):
                    k, _, v = kv.partition("=")
                    os.environ[k] = v
                plan = plan[1] or "default"
            elif isinstance(plan, tuple):
                os.environ["SPI_GEMM_HALO_CFG"] = plan[1]
                plan = "halo " + plan[1]
            else:
                os.environ["SPI_GEMM_PLAN"] = plan
            ops.lib.spi_debug_gemm_reload_env()  # knobs are cached in the library
            try:
                ms = timeit(fn, a.reps)
            except ops.OpError as e:
                print(f"{label}  skipped: {e}  [{plan}]", flush=True)
                continue
            print(f"{label}  {ms*1e3:8.2f} us  {fl/ms/1e9:8.1f} TF/s  [{plan or 'auto'}]", flush=True)
        os.environ["SPI_GEMM_PLAN"] = ""
        os.environ["SPI_GEMM_HALO_CFG"] = ""
        for k in ("SPI_CONV_WRES", "SPI_GEMM_MAXSPLIT"):
            os.environ.pop(k, None)
        ops.lib.spi_debug_gemm_reload_env()
    dt = ops.act_dtype(a.prec)
    ws = ops.workspace()
    if a.kscan:  # ViT-L FFN1's M x N over K: the slope is the k-loop, the intercept the fixed cost
        M, N_ = (int(v) for v in a.kscan.split("x"))
        rng = np.random.default_rng(0)
        for K in (64, 128, 256, 512, 1024, 2048, 4096):
            A = torch.randn(M, K, device="cuda").to(dt)
            wp = ops.pack_weight(a.prec, rng.standard_normal((N_, K)).astype(np.float32) * 0.05)
            bias = torch.randn(N_, device="cuda") * 0.1
            out = torch.empty(M, N_, device="cuda", dtype=dt)
            sweep(lambda: ops.gemm(a.prec, A, wp, N_, bias=bias, out=out, ws=ws),
                  f"gemm kscan M={M:6d} N={N_:4d} K={K:5d} f16", 2.0 * M * N_ * K)
        return
    rng = np.random.default_rng(0)
    for name, B, H, cin, cout, k, st in CONVS:
        if a.only and a.only not in name:
            continue
        B = a.batch or B
        x = torch.randn(B, H, H, cin, device="cuda").to(dt)
        w = rng.standard_normal((cout, k * k * cin)).astype(np.float32) * 0.05
        wp = ops.pack_weight(a.prec, w)
        pad = k // 2
        oh = (H + 2 * pad - k) // st + 1
        out = torch.empty(B, oh, oh, cout, device="cuda", dtype=dt)
        fl = 2.0 * B * oh * oh * cout * k * k * cin
        sweep(lambda: ops.conv2d(a.prec, x, wp, cout, k, k, st, pad, ws=ws, out=out),
              f"conv {name:10s} M={B*oh*oh:6d} N={cout:4d} K={k*k*cin:5d}", fl)
    for name, M, N_, K in GEMMS:
        if a.only and a.only not in name:
            continue
        A = torch.randn(M, K, device="cuda").to(dt)
        w = rng.standard_normal((N_, K)).astype(np.float32) * 0.05
        wp = ops.pack_weight(a.prec, w)
        fl = 2.0 * M * N_ * K
        if a.model_epi:
            bias = torch.randn(N_, device="cuda") * 0.1
            f16 = "qkv" in name or "ff1" in name
            act = "gelu" if "ff1" in name else None
            res = None if f16 else torch.randn(M, N_, device="cuda")
            out = torch.empty(M, N_, device="cuda", dtype=dt if f16 else torch.float32)
            sweep(lambda: ops.gemm(a.prec, A, wp, N_, bias=bias, residual=res, out=out, act=act, ws=ws),
                  f"gemm {name:10s} M={M:6d} N={N_:4d} K={K:5d} {'gelu ' if act else ''}{'f16' if f16 else 'f32+res'}", fl)
            if act and a.epi_variants:  # the same launch without the activation: what the GELU costs
                sweep(lambda: ops.gemm(a.prec, A, wp, N_, bias=bias, out=out, ws=ws),
                      f"gemm {name:10s} M={M:6d} N={N_:4d} K={K:5d} f16 (no GELU)", fl)
            continue
        out = torch.empty(M, N_, device="cuda", dtype=torch.float32)
        sweep(lambda: ops.gemm(a.prec, A, wp, N_, out=out, ws=ws), f"gemm {name:10s} M={M:6d} N={N_:4d} K={K:5d}", fl)


if __name__ == "__main__":
    main()
