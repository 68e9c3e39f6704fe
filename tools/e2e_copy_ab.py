#!/usr/bin/env python3
"""Host staging threads A/B for the serving legs (ResNet-18 fp16m, 4 workers, the runtime's
default H2D mode), rounds interleaved in one process: bs8 requests, 32 in flight, and bs1 requests
through the adaptive batcher, 64 in flight, at copy_threads 4 / 8 / 12.

usage: python tools/e2e_copy_ab.py [ROUNDS]"""
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
rep = spi.ModelReplica(zoo.build("resnet18", seed=0), 0, "fp16m", max_batch=8, graphs=True)
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
for rnd in range(rounds):
    for ct in (4, 8, 12):
        r8 = bench.runtime_e2e(rtmod, rep, "resnet18", 8, 4000, inflight=32, workers=4, copy_threads=ct)
        r1 = bench.runtime_e2e(rtmod, rep, "resnet18", 8, 16000, inflight=64, req_batch=1, warmup=2000,
                               copy_threads=ct,
                               batching=rtmod.batching_config("adaptive", 1, 8, coalesce_timeout_us=200,
                                                              congestion=True, tick_us=500, entry_horizon_us=3000,
                                                              exit_horizon_us=7000))
        print(json.dumps({"round": rnd, "copy_threads": ct,
                          "bs8": [r8["value"], r8["p50_latency_ms"], r8["p99_latency_ms"]],
                          "bs1_adaptive": [r1["value"], r1["p50_latency_ms"], r1["p99_latency_ms"]]}), flush=True)
