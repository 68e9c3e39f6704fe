#!/usr/bin/env python3
"""H2D A/B through the mini-runtime, interleaved rounds in one process: SDMA copies (waited by the
worker thread) against the worker-stream hipMemcpyAsync copies.  Each line: e2e
rate, p50, and where the worker threads spent their time (spi_runtime_worker_times: slot wait,
host staging, H2D + codelet + D2H enqueue, completion-event wait).

usage: python tools/sdma_ab.py [resnet18|resnet152|vit_l_16|bert_base]   (ROUNDS=3, REQUESTS=400)
"""
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
name = sys.argv[1] if len(sys.argv) > 1 else "resnet152"
batch, prec = {"resnet18": (8, "fp16m"), "resnet152": (32, "fp16x3"), "vit_l_16": (16, "fp16"),
               "bert_base": (8, "fp16")}[name]
m = zoo.build(name, seed=0)
kw = {"seq_len": 128} if name.startswith("bert") else {}
rep = spi.ModelReplica(m, 0, prec, max_batch=batch, graphs=True, **kw)
x, out_shape = bench.make_inputs(name, batch, np.random.default_rng(7))
if name.startswith("bert"):
    in_specs = [((v.shape[1],), np.int64) for v in x]
else:
    in_specs = [((3, 224, 224), np.float32)]
out_elems = int(np.prod(out_shape[1:]))
requests = int(os.environ.get("REQUESTS", "400"))
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for label, mode in (("worker_sdma", "worker_sdma"), ("worker_stream", "worker_stream")):
        rt = rtmod.Runtime([rep], in_specs, [(out_elems, np.float32)], max_batch=batch, workers_per_device=4,
                           h2d_mode=mode, warmup_batches=-1)
        r = rt.loadgen(x, requests=requests, inflight=16, warmup=32)
        wt = rt.worker_times()
        rt.close()
        tot = {k: round(sum(w[k] for w in wt), 3) for k in ("slot_s", "stage_s", "enqueue_s", "event_s")}
        print(json.dumps({"model": name, "round": rnd, "mode": label,
                          "value": round(r["inferences_per_s"], 1), "p50": round(r["p50_ms"], 2),
                          "p99": round(r["p99_ms"], 2), "seconds": round(r["seconds"], 3),
                          "tasks": sum(w["tasks"] for w in wt), "worker_s": tot}), flush=True)
