#!/usr/bin/env python3
"""Phase cycles of the weight-resident layer-1 conv (conv_wres.hip) from the s_memtime
diagnostic build: tools/build_variant.sh tools/libspi_wres_stamps.so WORKTREE -DSPI_WRES_STAMPS
then  python tools/wres_stamps.py tools/libspi_wres_stamps.so.
Per workgroup (one band each since round 4): W + halo landed, compute, epilogue; total;
the shader clock from s_memtime / s_memrealtime (100 MHz).  Medians over workgroups."""
import ctypes as C
import os
import sys

import numpy as np
import torch

lib = C.CDLL(sys.argv[1])
bpws = [1]  # one band per workgroup (the multi-band variants were removed in round 4)
V = C.c_void_p
lib.spi_op_conv2d.argtypes = [C.c_int32, V, C.c_int32, C.c_int32, C.c_int32, C.c_int32, V, C.c_int32, C.c_int32,
                              C.c_int32, C.c_int32, C.c_int32, V, V, V, C.c_int32, V, V]
lib.spi_op_packed_bytes.restype = C.c_size_t
lib.spi_op_workspace_bytes.restype = C.c_size_t
lib.spi_op_pack_weight.argtypes = [C.c_int32, V, C.c_int32, C.c_int32, V]
lib.spi_debug_wres_stamps.argtypes = [V, C.c_size_t]
lib.spi_debug_gemm_reload_env.argtypes = []

B, H = 8, 56
w = (np.random.default_rng(0).standard_normal((64, 576)) * 0.05).astype(np.float32)
host = np.empty(lib.spi_op_packed_bytes(1, 64, 576, None, None), np.uint8)
lib.spi_op_pack_weight(1, w.ctypes.data, 64, 576, host.ctypes.data)
wp = torch.from_numpy(host).cuda()
x = torch.rand(B, H, H, 64, device="cuda").half()
y = torch.empty_like(x)
bias = torch.zeros(64, device="cuda")
ws = torch.zeros(lib.spi_op_workspace_bytes(), dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for bpw in bpws:
    for _ in range(20):
        lib.spi_op_conv2d(1, x.data_ptr(), B, H, H, 64, wp.data_ptr(), 64, 3, 3, 1, 1, bias.data_ptr(), None,
                          y.data_ptr(), 1, ws.data_ptr(), V(s))
    torch.cuda.synchronize()
    st = np.zeros(4096 * 10, np.uint64)
    lib.spi_debug_wres_stamps(st.ctypes.data, st.size)
    nwg = -(-B * 28 // bpw)
    t = st[: nwg * 10].reshape(nwg, 10).astype(np.int64)
    d = lambda a, b: np.median(t[:, b] - t[:, a])
    clk = np.median((t[:, 7] - t[:, 0]) / np.maximum(1, (t[:, 8] - t[:, 9])) * 100e6) / 1e9
    if bpw == 1 and os.environ.get("EPI"):
        print(f"  epilogue detail: barrier {d(2, 4):.0f} park {d(4, 5):.0f} barrier {d(5, 6):.0f} "
              f"stores+barrier {d(6, 3):.0f}", flush=True)
    print(f"bpw={bpw} wgs={nwg} clock~{clk:.2f} GHz | band0: wait {d(0, 1):.0f} compute {d(1, 2):.0f} "
          f"epilogue {d(2, 3):.0f}" + (f" | band1: wait {d(3, 4):.0f} compute {d(4, 5):.0f} epilogue {d(5, 6):.0f}"
                                       if bpw > 1 else "") + f" | total {d(0, 7):.0f} cycles", flush=True)
