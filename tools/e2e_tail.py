"""Where the e2e tail comes from: the bench's e2e leg (ResNet-18 fp16m bs8, 4 workers, 32 in
flight) repeated under the runtime knob read at create (SPI_RT_COMPLETION),
interleaved rounds in one process; prints one JSON line per run with the latency breakdown."""
import importlib
import json
import os
import sys

os.environ["GPU_MAX_HW_QUEUES"] = "16"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

spi = importlib.import_module("starpu-inference-server_amd")
zoo = importlib.import_module("starpu-inference-server_amd.zoo")
rtmod = importlib.import_module("starpu-inference-server_amd.runtime")
m = zoo.resnet18()
rep = spi.ModelReplica(m, 0, "fp16m", max_batch=8, graphs=True)
variants = [{}, {"SPI_RT_COMPLETION": "spin"}]
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
for rnd in range(rounds):
    for v in variants:
        for k in ("SPI_RT_COMPLETION",):
            os.environ.pop(k, None)
        os.environ.update(v)
        for inflight in (32, 16):
            r = bench.runtime_e2e(rtmod, rep, "resnet18", 8, 4000, inflight=inflight, workers=4)
            print(json.dumps({"round": rnd, "knobs": v, "inflight": inflight, "value": r["value"],
                              "p50": r["p50_latency_ms"], "p95": r["p95_latency_ms"], "p99": r["p99_latency_ms"],
                              "breakdown": r["breakdown_ms"], "worst_at": r["worst_request_at"]}), flush=True)
