import os, sys, importlib, numpy as np
os.environ["GPU_MAX_HW_QUEUES"]="16"
sys.path.insert(0, os.getcwd())
import bench
spi = importlib.import_module("starpu-inference-server_amd"); zoo = importlib.import_module("starpu-inference-server_amd.zoo")
rtmod = importlib.import_module("starpu-inference-server_amd.runtime")
m = zoo.build("resnet152"); rep = spi.ModelReplica(m, 0, "fp16x3", max_batch=32, graphs=True)
for mode in ["device_stream", "worker_stream"]:
    print(mode, bench.runtime_e2e(rtmod, rep, "resnet152", 32, 60, inflight=16, workers=4, h2d_mode=mode), flush=True)
rep.set_graphs(False)
print("nographs", bench.runtime_e2e(rtmod, rep, "resnet152", 32, 60, inflight=16, workers=4), flush=True)
