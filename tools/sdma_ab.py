#!/usr/bin/env python3
"""SDMA vs stream H2D on a compute-bound config (ResNet-152 bs32 fp16x3, C4): interleaved
rounds in one process, each reporting the e2e rate, p50, and where the worker threads spent
their time (spi_runtime_worker_times: slot wait, host staging, H2D + codelet + D2H enqueue,
completion-event wait)."""
import importlib
import json
import os
import sys

os.environ["GPU_MAX_HW_QUEUES"] = "16"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402

spi = importlib.import_module("starpu-inference-server_amd")
zoo = importlib.import_module("starpu-inference-server_amd.zoo")
rtmod = importlib.import_module("starpu-inference-server_amd.runtime")
name, batch, prec = (sys.argv[1] if len(sys.argv) > 1 else "resnet152"), 32, "fp16x3"
if name == "vit_l_16":
    batch, prec = 16, "fp16"
m = zoo.build(name, seed=0)
rep = spi.ModelReplica(m, 0, prec, max_batch=batch, graphs=True)
x, out_shape = bench.make_inputs(name, batch, np.random.default_rng(7))
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for mode in ("worker_sdma", "worker_stream"):
        for wait in ("", "high", "0", "1", "2", "3"):
            if mode != "worker_sdma" and wait:
                continue
            os.environ.pop("SPI_H2D_SDMA_ENGINE", None)
            if wait:
                os.environ["SPI_H2D_SDMA_ENGINE"] = wait
            rt = rtmod.Runtime([rep], [((3, 224, 224), np.float32)], [(1000, np.float32)], max_batch=batch,
                               workers_per_device=4, h2d_mode=mode, warmup_batches=-1)
            r = rt.loadgen(x, requests=300, inflight=16, warmup=32)
            wt = rt.worker_times()
            rt.close()
            tot = {k: round(sum(w[k] for w in wt), 3) for k in ("slot_s", "stage_s", "enqueue_s", "event_s")}
            print(json.dumps({"round": rnd, "mode": mode + (f"/{wait}" if wait else ""),
                              "value": round(r["inferences_per_s"], 1), "p50": round(r["p50_ms"], 2),
                              "seconds": round(r["seconds"], 3), "tasks": sum(w["tasks"] for w in wt),
                              "worker_s": tot}), flush=True)
