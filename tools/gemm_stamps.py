#!/usr/bin/env python3
"""Phase shares of the GEMM main loop from the s_memtime diagnostic build
(tools/libspi_stamps.so, built with -DSPI_GEMM_STAMPS).  Shares only: the
stamps' own waits forbid overlaps the real kernel has (guide 7, In-kernel stamps).

Conv layers run in the headline's mode (precision 3: fp16x3 on split
activations) and plain fp16; `loop_cycles` is the K loop of one workgroup,
`kernel_us` the event-timed launch (so kernel - loop = prologue + epilogue)."""
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


def plan_blocks(M, N, K, estep, T=128):
    """Workgroups of the default plan rule (gemm.hip choose_plan, tput:T, default 128)."""
    tiles = lambda bm, bn: -(-M // bm) * -(-N // bn)
    ks = -(-K // 64) * 64 // estep
    if N > 64 and tiles(128, 128) >= T:
        return tiles(128, 128), "128x128"
    if tiles(128, 64) >= T:
        return tiles(128, 64), "128x64"
    t64 = tiles(64, 64)
    sp = 1 if t64 >= T else max(1, min(-(-T // t64), ks // 6))
    kt = -(-ks // sp)
    sp = -(-ks // kt)
    return t64 * sp, f"64x64/{sp}"


def report(name, nblocks, plan, us):
    buf = np.zeros(65536 * 8, np.uint64)
    torch.cuda.synchronize()
    lib.spi_debug_gemm_stamps(buf.ctypes.data, buf.size)
    st = buf.reshape(-1, 8)[:nblocks].astype(np.float64)
    tot, wait, issue, comp, steps = st[:, 0], st[:, 1], st[:, 2], st[:, 3], st[:, 4]
    print(f"{name:34s} {plan:9s} wg={nblocks:5d} steps={steps.mean():5.1f} loop_cyc={tot.mean():7.0f} "
          f"({tot.mean() / 2.1e3:5.1f} us@2.1GHz) kernel={us:6.1f} us per_step={tot.mean() / steps.mean():6.0f}  "
          f"wait {wait.sum() / tot.sum() * 100:5.1f}%  issue {issue.sum() / tot.sum() * 100:5.1f}%  "
          f"mfma {comp.sum() / tot.sum() * 100:5.1f}%", flush=True)


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ws = torch.zeros(lib.spi_op_workspace_bytes(), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    convs = [(8, 56, 64, 64, 3, 1, True), (8, 56, 64, 128, 3, 2, False), (8, 28, 128, 128, 3, 1, True),
             (8, 14, 256, 256, 3, 1, True), (8, 7, 512, 512, 3, 1, True)]
    for prec, pname, estep in [(3, "fp16x3s", 32), (1, "fp16", 64)]:
        for (B, H, cin, cout, k, st, has_res) in convs:
            oh = (H + 2 * (k // 2) - k) // st + 1
            if prec == 3:
                x = torch.randn(B, H, H, 2 * cin, device="cuda").half()
                y = torch.empty(B, oh, oh, 2 * cout, device="cuda", dtype=torch.half)
                r = torch.randn(B, oh, oh, 2 * cout, device="cuda").half() if has_res else None
            else:
                x = torch.randn(B, H, H, cin, device="cuda").half()
                y = torch.empty(B, oh, oh, cout, device="cuda", dtype=torch.half)
                r = torch.randn(B, oh, oh, cout, device="cuda").half() if has_res else None
            wp = packed(prec, cout, k * k * cin)
            bias = torch.randn(cout, device="cuda")
            fn = lambda: lib.spi_op_conv2d(prec, x.data_ptr(), B, H, H, cin, wp.data_ptr(), cout, k, k, st, k // 2,
                                           bias.data_ptr(), r.data_ptr() if r is not None else None, y.data_ptr(), 1,
                                           ws.data_ptr(), s)
            us = timed(fn)
            fn()
            nb, plan = plan_blocks(B * oh * oh, cout, k * k * cin, estep)
            report(f"{pname} conv {H}x{H}x{cin}->{cout} s{st}{' +res' if has_res else ''}", nb, plan, us)


if __name__ == "__main__":
    main()
