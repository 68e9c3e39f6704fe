#!/usr/bin/env python3
"""Where SDMA H2D stops paying: ResNet-18 / 34 / 50 / 101 / 152 at bs8 through the runtime's e2e
closed loop (4 workers, 32 in flight) with the H2D on the SDMA engines vs on the worker streams,
rounds interleaved in one process.  The models span 166 .. 26 KiB of fp32 input per GFLOP of the
forward -- the quantity SPI_H2D_AUTO's rule thresholds (runtime.cpp).  Basic-block nets run the
C2 mode (fp16m), bottleneck nets the C4 mode (fp16x3), as served."""
import importlib
import json
import os
import sys

os.environ["GPU_MAX_HW_QUEUES"] = "16"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

spi = importlib.import_module("starpu-inference-server_amd")
zoo = importlib.import_module("starpu-inference-server_amd.zoo")
rtmod = importlib.import_module("starpu-inference-server_amd.runtime")
NETS = [("resnet18", [2, 2, 2, 2], False), ("resnet34", [3, 4, 6, 3], False), ("resnet50", [3, 4, 6, 3], True),
        ("resnet101", [3, 4, 23, 3], True), ("resnet152", [3, 8, 36, 3], True)]
B = int(os.environ.get("BATCH", "8"))
x = np.random.default_rng(7).random((B, 3, 224, 224), dtype=np.float32)
for name, layers, bott in NETS:
    m = zoo.resnet(layers, bott, seed=0)
    prec = "fp16x3" if bott else "fp16m"
    rep = spi.ModelReplica(m, 0, prec, max_batch=B, graphs=True)
    kib_per_gflop = B * 602112 / 1024 / (rep.flops(B) / 1e9)
    res = {}
    for rnd in range(int(os.environ.get("ROUNDS", "2"))):
        for mode in ("worker_sdma", "worker_stream"):
            rt = rtmod.Runtime([rep], [((3, 224, 224), np.float32)], [(1000, np.float32)], max_batch=B,
                               workers_per_device=4, h2d_mode=mode, warmup_batches=-1)
            n = max(200, int(40000 / (rep.flops(B) / 1e9)))
            r = rt.loadgen([x], requests=n, inflight=32, warmup=64)
            rt.close()
            res.setdefault(mode, []).append(r["inferences_per_s"])
    sd, st = max(res["worker_sdma"]), max(res["worker_stream"])
    print(json.dumps({"model": name, "precision": prec, "batch": B, "kib_per_gflop": round(kib_per_gflop, 1),
                      "sdma": round(sd, 1), "stream": round(st, 1), "sdma_over_stream": round(sd / st, 3)}), flush=True)
    del rep, m
