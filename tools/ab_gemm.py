#!/usr/bin/env python3
"""Interleaved A/B of the GEMM / implicit-GEMM conv kernels between two builds of
the library, one process (cdna_hip_programming.md rule 24).

usage: ab_gemm.py LIB_A LIB_B [--prec fp16,fp16x3] [--set resnet18|gemm|all]

Conv shapes are ResNet-18 at bs8 224x224 (NHWC, folded BN -> bias, ReLU, the
second conv of each basic block with its residual), i.e. the headline's kernels.
"""
import argparse
import ctypes as C
import os

import numpy as np
import torch

V = C.c_void_p
PREC = {"fp32": 0, "fp16": 1, "fp16x3": 2, "fp16x3s": 3}  # fp16x3s: split activation layout
# (B, H, Cin, Cout, k, stride, residual)
RESNET18 = [(8, 224, 8, 64, 7, 2, False), (8, 56, 64, 64, 3, 1, False), (8, 56, 64, 64, 3, 1, True),
            (8, 56, 64, 128, 3, 2, False), (8, 28, 128, 128, 3, 1, True), (8, 56, 64, 128, 1, 2, False),
            (8, 28, 128, 256, 3, 2, False), (8, 14, 256, 256, 3, 1, True), (8, 14, 256, 512, 3, 2, False),
            (8, 7, 512, 512, 3, 1, True)]
GEMMS = [(1024, 3072, 768), (1024, 768, 3072), (3152, 3072, 1024), (3152, 4096, 1024), (3152, 1024, 4096),
         (3152, 1024, 1024), (4096, 4096, 4096)]


def load(path):
    lib = C.CDLL(path, mode=C.RTLD_LOCAL)
    lib.spi_op_gemm.argtypes = [C.c_int32, V, C.c_int32, C.c_int32, C.c_int32, V, C.c_int32, V, V, C.c_int32,
                                C.c_int32, V, C.c_int32, C.c_int32, C.c_int32, V, V]
    lib.spi_op_conv2d.argtypes = [C.c_int32, V, C.c_int32, C.c_int32, C.c_int32, C.c_int32, V, C.c_int32,
                                  C.c_int32, C.c_int32, C.c_int32, C.c_int32, V, V, V, C.c_int32, V, V]
    lib.spi_op_packed_bytes.restype = C.c_size_t
    lib.spi_op_workspace_bytes.restype = C.c_size_t
    lib.spi_op_pack_weight.argtypes = [C.c_int32, V, C.c_int32, C.c_int32, V]
    return lib


def packed(lib, prec, n, k):
    w = (np.random.default_rng(0).standard_normal((n, k)) * 0.05).astype(np.float32)
    host = np.empty(lib.spi_op_packed_bytes(prec, n, k, None, None), np.uint8)
    lib.spi_op_pack_weight(prec, w.ctypes.data, n, k, host.ctypes.data)
    return torch.from_numpy(host).cuda()


def time_pair(fns, reps=20, rounds=7):
    res = [[] for _ in fns]
    for _ in range(rounds):
        for i, f in enumerate(fns):
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(reps):
                f()
            e1.record()
            torch.cuda.synchronize()
            res[i].append(e0.elapsed_time(e1) / reps * 1e3)
    return [float(np.median(r)) for r in res]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs=2)
    ap.add_argument("--prec", default="fp16,fp16x3")
    ap.add_argument("--set", default="all", choices=["resnet18", "gemm", "all"])
    ap.add_argument("--env-a", default="", help="knobs for lib A only, e.g. 'SPI_GEMM_NG=2' (comma-separated)")
    ap.add_argument("--env-b", default="", help="knobs for lib B only")
    ap.add_argument("--act", type=int, default=0, help="GEMM activation: 0 none, 1 relu, 2 gelu")
    ap.add_argument("--out16", action="store_true", help="GEMMs: fp16 output (the transformer epilogues)")
    a = ap.parse_args()
    if a.libs[0] == a.libs[1]:  # same file twice: load a private copy so each keeps its own knobs
        import shutil
        import tempfile
        cp = os.path.join(tempfile.mkdtemp(), "libspi_b.so")
        shutil.copy(a.libs[1], cp)
        a.libs[1] = cp
    libs = [load(p) for p in a.libs]
    for lib, spec in zip(libs, [a.env_a, a.env_b]):  # knobs are cached per library: set, reload, restore
        kv = [s.split("=", 1) for s in spec.split(",") if s]
        old = {k: os.environ.get(k) for k, _ in kv}
        os.environ.update(dict(kv))
        lib.spi_debug_gemm_reload_env()
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    ws = [torch.zeros(l.spi_op_workspace_bytes(), dtype=torch.uint8, device="cuda") for l in libs]
    s = torch.cuda.current_stream().cuda_stream
    for pname in a.prec.split(","):
        prec = PREC[pname]
        dt = torch.float16 if pname == "fp16" else torch.float32
        split = pname == "fp16x3s"  # split layout: [.., C] as 2C fp16 (hi | lo per 32-block)

        def act(*shape):
            if split:
                return torch.randn(*shape[:-1], 2 * shape[-1], device="cuda").half()
            return torch.randn(*shape, device="cuda").to(dt)
        tot = [0.0, 0.0]
        if a.set in ("resnet18", "all"):
            for (B, H, cin, cout, k, st, has_res) in RESNET18:
                if split and cin < 32:
                    continue
                x = act(B, H, H, cin)
                wp = packed(libs[0], prec, cout, k * k * cin)
                bias = torch.randn(cout, device="cuda")
                oh = (H + 2 * (k // 2) - k) // st + 1
                res = act(B, oh, oh, cout) if has_res else None
                ys = [torch.empty_like(act(B, oh, oh, cout)) for _ in libs]
                fns = [(lambda l=l, y=y, w=w: l.spi_op_conv2d(
                    prec, x.data_ptr(), B, H, H, cin, wp.data_ptr(), cout, k, k, st, k // 2, bias.data_ptr(),
                    res.data_ptr() if res is not None else None, y.data_ptr(), 1, w.data_ptr(), s))
                       for l, y, w in zip(libs, ys, ws)]
                t = time_pair(fns)
                tot = [tot[0] + t[0], tot[1] + t[1]]
                flop = 2 * B * oh * oh * cout * k * k * cin
                same = torch.equal(ys[0], ys[1])
                print(f"{pname:6s} conv {H:3d}x{H:<3d} {cin:3d}->{cout:3d} k{k} s{st}{' +res' if has_res else '     '}: "
                      f"A {t[0]:7.2f} us  B {t[1]:7.2f} us  B/A {t[1] / t[0]:5.3f}  "
                      f"({flop / t[1] / 1e6:5.0f} TF/s){'' if same else '  OUTPUT DIFFERS'}")
            print(f"{pname:6s} resnet18 conv sum: A {tot[0]:.1f} us  B {tot[1]:.1f} us  B/A {tot[1] / tot[0]:.3f}")
        if a.set in ("gemm", "all"):
            for M, N, K in GEMMS:
                A = act(M, K)
                wp = packed(libs[0], prec, N, K)
                o16 = split or a.out16
                outs = [torch.empty_like(act(M, N)) if o16 else torch.empty(M, N, device="cuda") for _ in libs]
                bias = torch.randn(N, device="cuda")
                fns = [(lambda l=l, o=o, w=w: l.spi_op_gemm(prec, A.data_ptr(), M, K, K, wp.data_ptr(), N, bias.data_ptr(),
                                                           None, 0, 0, o.data_ptr(), 0 if o16 else 1, N, a.act,
                                                           w.data_ptr(), s))
                       for l, o, w in zip(libs, outs, ws)]
                t = time_pair(fns)
                print(f"{pname:6s} gemm {M}x{N}x{K}: A {t[0]:.2f} us ({2 * M * N * K / t[0] / 1e6:.0f} TF/s)  "
                      f"B {t[1]:.2f} us ({2 * M * N * K / t[1] / 1e6:.0f} TF/s)  B/A {t[1] / t[0]:.3f}")


if __name__ == "__main__":
    main()
