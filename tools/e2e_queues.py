#!/usr/bin/env python3
"""Serving-path (mini-runtime + load generator) throughput and per-worker task counts under a given
GPU_MAX_HW_QUEUES (set before the first HIP call):
usage python tools/e2e_queues.py QUEUES [WORKERS] [device_stream|worker_stream|worker_copy]"""
import importlib, json, os, sys, time
os.environ["GPU_MAX_HW_QUEUES"] = sys.argv[1] if len(sys.argv) > 1 else "16"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
spi = importlib.import_module("starpu-inference-server_amd")
zoo = importlib.import_module("starpu-inference-server_amd.zoo")
rtmod = importlib.import_module("starpu-inference-server_amd.runtime")
rep = spi.ModelReplica(zoo.build("resnet18", seed=0), 0, "fp16m", max_batch=8, graphs=True)
x = np.random.default_rng(0).random((8, 3, 224, 224), dtype=np.float32)
WORKERS = int(sys.argv[2]) if len(sys.argv) > 2 else 4
MODE = sys.argv[3] if len(sys.argv) > 3 else "device_stream"
for rnd in range(2):
    rt = rtmod.Runtime([rep], [((3, 224, 224), np.float32)], [(1000, np.float32)], max_batch=8,
                       workers_per_device=WORKERS, h2d_mode=MODE)
    r = rt.loadgen([x], requests=4000, inflight=32, warmup=64)
    print(json.dumps({"queues": os.environ["GPU_MAX_HW_QUEUES"], "workers": WORKERS, "mode": MODE, "round": rnd, "inf_per_s": round(r["inferences_per_s"], 1),
                      "p50_ms": round(r["p50_ms"], 3), "tasks": [w["tasks"] for w in rt.worker_times()],
                      "event_s": [round(w["event_s"], 3) for w in rt.worker_times()]}), flush=True)
    rt.close()
