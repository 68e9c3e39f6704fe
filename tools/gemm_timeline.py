#!/usr/bin/env python3
"""Where a GEMM / conv launch spends its time, per workgroup, from the -DSPI_GEMM_TIMELINE
build (s_memrealtime at entry, k-loop start, k-loop end and exit; HW_ID / XCC_ID).

For every gemm_kernel op of one ResNet-18 forward (the headline's replica, eager), the op is
launched `reps` times back to back on worker 0's stream (Model::profile_op) -- isolated, and
with the other workers replaying forwards (--loaded; only the profiling thread's launches stamp)
-- and the last launch's stamps are read:

  span      first entry -> last exit (the launch as the GPU runs it)
  skew      first entry -> last entry (dispatch of the grid)
  pro/loop/epi  per-workgroup entry -> loop start -> loop end -> exit (mean / max)
  per_cu    workgroups sharing a CU (max) -- the dispatcher may stack workgroups
  crit      the last workgroup to exit: its entry offset and its three phases

usage: SPI_HIP_LIB=tools/libspi_timeline.so python tools/gemm_timeline.py [--loaded]
(build: tools/build_variant.sh tools/libspi_timeline.so WORKTREE -DSPI_GEMM_TIMELINE)"""
import argparse
import collections
import ctypes as C
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def analyse(buf):
    st = buf.reshape(-1, 8)
    live = st[:, 0] != 0
    idx = np.nonzero(live)[0]
    if len(idx) == 0:
        return None
    s = st[idx].astype(np.float64)
    e, l0, l1, x, p1, p2 = s[:, 0], s[:, 1], s[:, 2], s[:, 3], s[:, 6], s[:, 7]
    us = 0.01  # s_memrealtime: 100 MHz
    hw = st[idx, 4].astype(np.uint64)
    hwid = hw & np.uint64(0xFFFFFFFF)
    xcc = (hw >> np.uint64(32)) & np.uint64(0xF)
    cu = (hwid >> np.uint64(8)) & np.uint64(0xFF)  # CU_ID[11:8], SH_ID[12], SE_ID[15:13]
    keys = collections.Counter(zip(xcc.tolist(), cu.tolist()))
    t0 = e.min()
    crit = int(np.argmax(x))
    kind = st[idx, 5]
    return {
        "wgs": len(idx),
        "span": (x.max() - t0) * us,
        "skew": (e.max() - t0) * us,
        "pro": ((l0 - e).mean() * us, (l0 - e).max() * us),
        "pro_split": ((p1 - e).mean() * us, (p2 - p1).mean() * us, (l0 - p2).mean() * us),
        "loop": ((l1 - l0).mean() * us, (l1 - l0).max() * us),
        "epi": ((x - l1).mean() * us, (x - l1).max() * us),
        "per_cu_max": max(keys.values()),
        "cus": len(keys),
        "xccs": len(set(xcc.tolist())),
        "crit": ((e[crit] - t0) * us, (l0[crit] - e[crit]) * us, (l1[crit] - l0[crit]) * us, (x[crit] - l1[crit]) * us,
                 int(kind[crit])),
        "reducers": int((kind == 2).sum()),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--precision", default="fp16m")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--loaded", action="store_true")
    a = ap.parse_args()
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
    import torch
    bench = importlib.import_module("bench")
    spi = importlib.import_module("starpu-inference-server_amd")
    zoo = importlib.import_module("starpu-inference-server_amd.zoo")
    lib = spi.lib
    lib.spi_debug_gemm_timeline.argtypes = [C.c_void_p, C.c_size_t]
    m = zoo.build(a.model, seed=0)
    rep = spi.ModelReplica(m, 0, a.precision, max_batch=a.batch, seq_len=128 if a.model.startswith("bert") else 0,
                           graphs=True)
    h = bench.Harness(spi, rep, a.model, 0, a.batch, 4, np.random.default_rng(0))
    h.rounds(4)
    torch.cuda.synchronize()
    ops = rep.profile(h.d_in[0], h.d_out[0], h.streams[0].cuda_stream)
    seen = []
    for op in ops:
        if op["name"] not in seen:
            seen.append(op["name"])
    buf = np.zeros(65536 * 8, np.uint64)
    print(f"{'op':34s} {'wgs':>4s} {'cus':>4s} {'x/cu':>4s} {'b2b':>6s} {'span':>6s} {'skew':>5s} "
          f"{'pro':>11s} {'loop':>11s} {'epi':>11s}  crit(start pro loop epi kind)", flush=True)
    for name in seen:
        torch.cuda.synchronize()
        lib.spi_debug_gemm_timeline_clear()
        if a.loaded:
            for _ in range(12):
                for w in range(1, 4):
                    h.task(w)
        r = rep.profile_op(h.d_in[0], h.d_out[0], h.streams[0].cuda_stream, name, a.reps)
        torch.cuda.synchronize()
        lib.spi_debug_gemm_timeline(buf.ctypes.data, buf.size)
        t = analyse(buf)
        if t is None:
            continue
        c = t["crit"]
        print(f"{name:34s} {t['wgs']:4d} {t['cus']:4d} {t['per_cu_max']:4d} {r['ms'] * 1e3:6.2f} {t['span']:6.2f} "
              f"{t['skew']:5.2f} {t['pro'][0]:5.2f}/{t['pro'][1]:5.2f} {t['loop'][0]:5.2f}/{t['loop'][1]:5.2f} "
              f"{t['epi'][0]:5.2f}/{t['epi'][1]:5.2f}  {c[0]:5.2f} {c[1]:5.2f} {c[2]:5.2f} {c[3]:5.2f} {c[4]}"
              f"  pro=decode {t['pro_split'][0]:.2f} + setup {t['pro_split'][1]:.2f} + issue {t['pro_split'][2]:.2f}"
              f"{'  reducers=%d' % t['reducers'] if t['reducers'] else ''}", flush=True)


if __name__ == "__main__":
    main()
