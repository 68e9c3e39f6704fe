#!/usr/bin/env python3
"""Interleaved A/B of spi_op_gemm between two builds of the library, one process
(cdna_hip_programming.md rule 24).  usage: ab_gemm.py LIB_A LIB_B"""
import ctypes as C
import sys

import numpy as np
import torch

SHAPES = [(3152, 3072, 1024), (4096, 4096, 4096), (1024, 3072, 768), (1024, 768, 3072)]


def load(path):
    lib = C.CDLL(path, mode=C.RTLD_LOCAL)
    lib.spi_op_gemm.argtypes = [C.c_int32, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_int32,
                                C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32, C.c_int32,
                                C.c_int32, C.c_void_p, C.c_void_p]
    lib.spi_op_packed_bytes.restype = C.c_size_t
    lib.spi_op_workspace_bytes.restype = C.c_size_t
    lib.spi_op_pack_weight.argtypes = [C.c_int32, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]
    return lib


def main():
    libs = [load(p) for p in sys.argv[1:3]]
    ws = torch.zeros(libs[0].spi_op_workspace_bytes(), dtype=torch.uint8, device="cuda")
    for M, N, K in SHAPES:
        A = torch.randn(M, K, device="cuda").half()
        w = (np.random.default_rng(0).standard_normal((N, K)) * 0.05).astype(np.float32)
        nb = libs[0].spi_op_packed_bytes(1, N, K, None, None)
        host = np.empty(nb, np.uint8)
        libs[0].spi_op_pack_weight(1, w.ctypes.data, N, K, host.ctypes.data)
        W = torch.from_numpy(host).cuda()
        out = torch.empty(M, N, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        res = {0: [], 1: []}
        for rnd in range(6):
            for i, lib in enumerate(libs):
                def f():
                    lib.spi_op_gemm(1, A.data_ptr(), M, K, K, W.data_ptr(), N, None, None, 0, 0, out.data_ptr(),
                                    1, N, 0, ws.data_ptr(), s)
                f()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(20):
                    f()
                e1.record()
                torch.cuda.synchronize()
                res[i].append(e0.elapsed_time(e1) / 20 * 1e3)
        a, b = np.median(res[0]), np.median(res[1])
        print(f"M={M} N={N} K={K}: A {a:.2f} us ({2*M*N*K/a/1e6:.0f} TF/s)  B {b:.2f} us ({2*M*N*K/b/1e6:.0f} TF/s)")


if __name__ == "__main__":
    main()
