"""Sweep the PCIe-inclusive serving path (mini-runtime + C++ load generator) over the
runtime's staging knobs, beside the device-resident rate of the same replica.

  python tools/e2e_sweep.py [--model resnet18] [--batch 8] [--requests 4000]
Writes one JSON line per configuration to stdout."""
import argparse
import importlib
import json
import os
import sys
import time

os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("SPI_QUEUES", "16")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--precision", default="fp16m")
    ap.add_argument("--requests", type=int, default=4000)
    ap.add_argument("--quick", type=int, default=0)
    args = ap.parse_args()
    spi = importlib.import_module("starpu-inference-server_amd")
    zoo = importlib.import_module("starpu-inference-server_amd.zoo")
    rtmod = importlib.import_module("starpu-inference-server_amd.runtime")
    m = zoo.build(args.model, seed=0)
    rep = spi.ModelReplica(m, 0, args.precision, max_batch=args.batch, graphs=True)
    x = np.random.default_rng(0).random((args.batch, 3, 224, 224), dtype=np.float32)
    import bench
    h = bench.Harness(spi, rep, args.model, 0, args.batch, 4, np.random.default_rng(1))
    el = h.throughput(200, 10)
    print(json.dumps({"device_resident_inf_per_s": round(4 * args.batch * 200 / el, 1),
                      "queues": os.environ["GPU_MAX_HW_QUEUES"]}), flush=True)
    del h
    grid = []
    for h2d in ["device_stream", "worker_stream", "worker_copy"]:
        for depth in [1, 2, 3]:
            for copy_threads in [1, 4]:
                for inflight in [8, 16]:
                    grid.append(dict(h2d_mode=h2d, pipeline_depth=depth, copy_threads=copy_threads,
                                     inflight=inflight))
    if args.quick:
        grid = [dict(h2d_mode=m, pipeline_depth=d, copy_threads=c, inflight=i) for m in ["device_stream", "worker_copy"]
                for d in [2, 3] for c in [4, 8] for i in [16, 32]]
    for g in grid:
        inflight = g.pop("inflight")
        rt = rtmod.Runtime([rep], [((3, 224, 224), np.float32)], [(1000, np.float32)], max_batch=args.batch,
                           workers_per_device=4, **g)
        t0 = time.perf_counter()
        r = rt.loadgen([x], requests=args.requests, inflight=inflight, warmup=64)
        rt.close()
        g["inflight"] = inflight
        print(json.dumps({**g, "inf_per_s": round(r["inferences_per_s"], 1), "p50_ms": round(r["p50_ms"], 4),
                          "p95_ms": round(r["p95_ms"], 4), "p99_ms": round(r["p99_ms"], 4),
                          "failed": r["failed"], "wall_s": round(time.perf_counter() - t0, 2)}), flush=True)


if __name__ == "__main__":
    main()
