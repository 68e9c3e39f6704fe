#!/usr/bin/env python3
"""Same-process A/B of the PCIe-inclusive serving rate (ResNet-18 bs8 fp16m, 4 workers, the bench's
e2e leg) over the runtime's H2D modes, rounds interleaved: `auto` (hipMemcpyAsync on the worker
stream) vs `worker_sdma` (hsa_amd_memory_async_copy on an SDMA engine, waited by the worker thread).

  python tools/e2e_h2d_ab.py [--rounds 3] [--requests 4000] [--modes auto,worker_sdma]"""
import argparse
import importlib
import json
import os
import sys

os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("SPI_QUEUES", "16")  # as bench.py (the box exports 4)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--requests", type=int, default=4000)
    ap.add_argument("--modes", default="auto,worker_sdma")
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--precision", default="fp16m")
    args = ap.parse_args()
    spi = importlib.import_module("starpu-inference-server_amd")
    zoo = importlib.import_module("starpu-inference-server_amd.zoo")
    rtmod = importlib.import_module("starpu-inference-server_amd.runtime")
    import bench
    rep = spi.ModelReplica(zoo.build(args.model, seed=0), 0, args.precision, max_batch=args.batch, graphs=True)
    for r in range(args.rounds):
        for spec in args.modes.split(","):
            mode = spec
            for inflight in (32, 16):
                out = bench.runtime_e2e(rtmod, rep, args.model, args.batch, args.requests, inflight, h2d_mode=mode)
                print(json.dumps({"round": r, "h2d_mode": spec, "inflight": inflight, **out}), flush=True)


if __name__ == "__main__":
    main()
