#!/usr/bin/env python3
"""Phase shares of the GEMM main loop from the s_memtime diagnostic build
(tools/libspi_stamps.so, built with -DSPI_GEMM_STAMPS).  Shares only: the
stamps' own waits forbid overlaps the real kernel has (guide 7, In-kernel stamps)."""
import ctypes as C
import sys

import numpy as np
import torch

lib = C.CDLL(sys.argv[1] if len(sys.argv) > 1 else "tools/libspi_stamps.so")
V = C.c_void_p
lib.spi_op_conv2d.argtypes = [C.c_int32, V, C.c_int32, C.c_int32, C.c_int32, C.c_int32, V, C.c_int32, C.c_int32,
                              C.c_int32, C.c_int32, C.c_int32, V, V, V, C.c_int32, V, V]
lib.spi_op_gemm.argtypes = [C.c_int32, V, C.c_int32, C.c_int32, C.c_int32, V, C.c_int32, V, V, C.c_int32, C.c_int32,
                            V, C.c_int32, C.c_int32, C.c_int32, V, V]
lib.spi_op_packed_bytes.restype = C.c_size_t
lib.spi_op_workspace_bytes.restype = C.c_size_t
lib.spi_op_pack_weight.argtypes = [C.c_int32, V, C.c_int32, C.c_int32, V]
lib.spi_debug_gemm_stamps.argtypes = [V, C.c_size_t]


def packed(prec, n, k):
    w = (np.random.default_rng(0).standard_normal((n, k)) * 0.05).astype(np.float32)
    host = np.empty(lib.spi_op_packed_bytes(prec, n, k, None, None), np.uint8)
    lib.spi_op_pack_weight(prec, w.ctypes.data, n, k, host.ctypes.data)
    return torch.from_numpy(host).cuda()


def report(name, nblocks):
    buf = np.zeros(65536 * 8, np.uint64)
    torch.cuda.synchronize()
    lib.spi_debug_gemm_stamps(buf.ctypes.data, buf.size)
    st = buf.reshape(-1, 8)[:nblocks].astype(np.float64)
    tot, wait, issue, comp, steps = st[:, 0], st[:, 1], st[:, 2], st[:, 3], st[:, 4]
    print(f"{name:32s} blocks={nblocks:5d} steps={steps.mean():5.1f} loop_cycles={tot.mean():9.0f} "
          f"per_step={tot.mean() / steps.mean():7.0f}  wait {wait.sum() / tot.sum() * 100:5.1f}%  "
          f"issue {issue.sum() / tot.sum() * 100:5.1f}%  compute {comp.sum() / tot.sum() * 100:5.1f}%")


def main():
    ws = torch.zeros(lib.spi_op_workspace_bytes(), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for prec, pname, dt in [(1, "fp16", torch.float16), (2, "fp16x3", torch.float32)]:
        for (B, H, cin, cout, k, st) in [(8, 56, 64, 64, 3, 1), (8, 28, 128, 128, 3, 1), (8, 112, 64, 64, 3, 1)]:
            x = torch.randn(B, H, H, cin, device="cuda").to(dt)
            wp = packed(prec, cout, k * k * cin)
            oh = (H + 2 * (k // 2) - k) // st + 1
            y = torch.empty(B, oh, oh, cout, device="cuda", dtype=dt)
            for _ in range(3):
                lib.spi_op_conv2d(prec, x.data_ptr(), B, H, H, cin, wp.data_ptr(), cout, k, k, st, k // 2, None, None,
                                  y.data_ptr(), 1, ws.data_ptr(), s)
            report(f"{pname} conv {H}x{H}x{cin}->{cout}", (B * oh * oh + 63) // 64 * ((cout + 63) // 64))
        for (M, N, K) in [(1024, 3072, 768), (4096, 4096, 4096)]:
            A = torch.randn(M, K, device="cuda").to(dt)
            wp = packed(prec, N, K)
            out = torch.empty(M, N, device="cuda")
            for _ in range(3):
                lib.spi_op_gemm(prec, A.data_ptr(), M, K, K, wp.data_ptr(), N, None, None, 0, 0, out.data_ptr(), 1, N,
                                0, ws.data_ptr(), s)
            report(f"{pname} gemm {M}x{N}x{K}", ((M + 127) // 128) * ((N + 127) // 128))


if __name__ == "__main__":
    main()
