import importlib, json, os, sys, time
os.environ["GPU_MAX_HW_QUEUES"] = "16"
sys.path.insert(0, "/root/repo") if os.path.isdir("/root/repo") else None
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np
spi = importlib.import_module("starpu-inference-server_amd")
zoo = importlib.import_module("starpu-inference-server_amd.zoo")
rtmod = importlib.import_module("starpu-inference-server_amd.runtime")
m = zoo.build("resnet18", seed=0)
rep = spi.ModelReplica(m, 0, "fp16m", max_batch=8, graphs=True)
x = np.random.default_rng(0).random((8, 3, 224, 224), dtype=np.float32)
for cfg in [dict(h2d_mode="device_stream", pipeline_depth=2, inflight=32),
            dict(h2d_mode="device_stream", pipeline_depth=2, inflight=64),
            dict(h2d_mode="device_stream", pipeline_depth=4, inflight=64),
            dict(h2d_mode="worker_stream", pipeline_depth=2, inflight=32),
            dict(h2d_mode="device_stream", pipeline_depth=2, inflight=32, workers=3),
            dict(h2d_mode="device_stream", pipeline_depth=2, inflight=32, workers=2)]:
    inflight = cfg.pop("inflight"); workers = cfg.pop("workers", 4)
    rt = rtmod.Runtime([rep], [((3, 224, 224), np.float32)], [(1000, np.float32)], max_batch=8,
                       workers_per_device=workers, **cfg)
    r = rt.loadgen([x], requests=4000, inflight=inflight, warmup=64)
    rt.close()
    print(json.dumps({**cfg, "inflight": inflight, "workers": workers, "inf_per_s": round(r["inferences_per_s"], 1),
                      "p50_ms": round(r["p50_ms"], 3), "p95_ms": round(r["p95_ms"], 3),
                      "p50_queue_ms": round(r["p50_queue_ms"], 3)}), flush=True)

# where the worker threads' time goes at the default serving configuration
rt = rtmod.Runtime([rep], [((3, 224, 224), np.float32)], [(1000, np.float32)], max_batch=8, workers_per_device=4)
t0 = time.perf_counter()
r = rt.loadgen([x], requests=4000, inflight=32, warmup=64)
wall = time.perf_counter() - t0
for i, wt in enumerate(rt.worker_times()):
    print(json.dumps({"worker": i, "wall_s": round(wall, 3), **{k: round(v, 4) for k, v in wt.items()}}), flush=True)
rt.close()
