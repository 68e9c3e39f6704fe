"""Host-side logic: latency statistics, bench contract helpers, multi-rank control (gloo)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_percentile_matches_reference_definition():
    """latency_statistics.hpp:52-93: sort, p<=0 -> min, p>=100 -> max, else lerp at p/100*(n-1)."""
    xs = [5.0, 1.0, 3.0, 2.0, 4.0]
    assert bench.percentile(xs, 0) == 1.0 and bench.percentile(xs, 100) == 5.0
    assert bench.percentile(xs, 50) == 3.0
    assert bench.percentile([1.0, 2.0], 50) == 1.5
    assert abs(bench.percentile(list(range(101)), 95) - 95.0) < 1e-12
    assert bench.percentile([7.0], 85) == 7.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    elapsed = bench.reduce_max_elapsed(0.5 + rank, world)
    shard = bench.shard_requests(100, rank, world)
    q.put((rank, elapsed, shard))
    dist.destroy_process_group()


def test_two_rank_gloo_max_time_and_request_sharding():
    """The N>1 bench path: barrier-bracketed timing reduced by MAX; requests sharded with no collective."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(abs(e - 1.5) < 1e-12 for _, e, _ in res)
    shards = [s for _, _, s in res]
    assert shards[0] + shards[1] == list(range(100))


def test_shard_requests_is_a_partition():
    for world in (1, 2, 3, 8):
        got = sorted(i for r in range(world) for i in bench.shard_requests(37, r, world))
        assert got == list(range(37))


def test_bench_gpus_2_spawns_two_ranks_control_path():
    """`python bench.py --gpus 2` (no launcher): two rank processes through the real control path
    (spawn_ranks, gloo rendezvous, barrier + max-over-ranks timing, e2e aggregation); the JSON
    line must say n_gpus 2 and carry the slowest rank's window."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20",
                          "--control-plane-only"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2
    assert line["ms_per_step"] >= 2.0  # rank 1 sleeps 2 ms per step: the max over ranks
    e = line["e2e"]
    assert e["requests"] == 200 and abs(e["seconds"] - 0.2) < 1e-9 and e["p50_latency_ms"] == 2.0
    assert abs(e["value"] - 200 * 8 / 0.2) < 1e-6 and len(e["per_rank"]) == 2


def test_fast_erf_in_gemm_epilogues_meets_fp32_bar():
    """The GELU epilogues' erf (csrc/device_math.hpp, coefficients parsed from the header)
    in fp32 against scipy's erf: max |error| < 5e-7, GELU error / max|x| < 1e-6, so GELU
    outputs stay inside the fp32 parity bar (1e-5 normalised)."""
    import importlib.util
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "fast_erf_check.py")
    spec = importlib.util.spec_from_file_location("fast_erf_check", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    e_erf, e_gelu = mod.max_error(n=400_001)
    assert e_erf < 5e-7 and e_gelu < 1e-6
    e16, g16 = mod.max_error(n=400_001, suffix="16")  # gemm256's lower-order form (fp16 operands)
    assert e16 < 3e-6 and g16 < 2e-6


def test_bench_compact_line_fits_the_driver_tail(tmp_path):
    """The printed line (bench.compact_line) carries the contract keys plus the metric's own
    shapes -- ResNet-18 bs1 rate / p50, C3-C5, the CI workload, the CPU layouts -- and stays
    under the 2000 bytes the driver's tail keeps; the full record goes to the detail file."""
    import contextlib
    import io
    import json
    long = "x" * 400  # long free-text fields must not reach the line
    lay = {"value": 700.0, "p50_ms": 20.0, "workers": 16, "threads_per_worker": 1, "tasks": 100}
    cfg_line = {"value": 24288.12, "unit": "sequences/s", "dtype": "fp16x3", "p50_task_latency_ms": 1.3532,
                "roofline": {"frac": 0.13612, "selection": long}, "e2e": {"value": 22175.24, "p50_latency_ms": 5.7508}}
    full = {
        "metric": bench.BASELINE_METRIC, "value": 116656.42, "unit": "inferences/s", "n_gpus": 8, "steps": 20,
        "warmup": 5, "ms_per_step": 2.1945, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "fp16m", "data": long,
        "config": {"workload": bench.WORKLOADS["resnet18"], "batch_per_task": 8, "workers_per_gpu": 4,
                   "tasks_per_step": 8, "parallelism": "replicas x8 (request sharding, no collective)",
                   "precision_mode": long},
        "roofline": {"bound": "mfma", "achieved": 149.146, "peak": 2500.0, "unit": "TFLOP/s", "frac": 0.05966,
                     "traffic": 14356821, "kernel": "conv3x3_c512_k512_s1_M392", "avg_launch_ms": 0.0124,
                     "frac_rocprof": 0.05709, "mfma_busy_pct": 3.86, "selection": long, "measured": long},
        "cpu_baseline": {"value": 784.734, "unit": "inferences/s", "cores": 16, "kind": "port", "sample": long,
                         "sample_short": "y" * 180, "host": {"nproc": 256, "numa_nodes": 2},
                         "layouts_summary": {f"bs{b}_{t}": [12345.678, 123.456, 16, 16] for b in (8, 1)
                                             for t in ("i", "ii", "iii")}},
        "e2e": {"value": 80824.12, "p50_latency_ms": 3.0912, "p99_latency_ms": 3.2145, "breakdown_ms": long},
        "p50_task_latency_ms": 0.273,
        "extras": {"resnet18_bs1_tasks": {"value": 20876.02, "p50_task_latency_ms": 0.1946,
                                          "p50_serial_e2e_latency_ms": 0.2147},
                   "c3_bert_base_seq128_bs8_fp16": cfg_line, "c4_resnet152_bs32_fp16x3": cfg_line,
                   "c5_vit_l_16_bs16_fp16": cfg_line,
                   "ci_perf_resnet152_schedule": {"value": 443.98, "p50_latency_ms": 9.5478, "config": long,
                                                  "mi355x_tuned": {"value": 443.98, "p50_latency_ms": 1.7066}}},
    }
    buf = io.StringIO()
    detail = tmp_path / "detail.json"
    with contextlib.redirect_stdout(buf):
        bench.emit(full, str(detail))
    text = buf.getvalue().strip()
    assert "\n" not in text and len(text) < 2000, len(text)
    line = json.loads(text)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line
    assert line["config"]["workload"] == bench.WORKLOADS["resnet18"]
    assert line["resnet18_bs1"]["p50_task_ms"] == 0.1946 and line["c3_bert"]["value"] == 24288.12
    assert line["ci_perf"]["tuned_p50_ms"] == 1.7066 and line["cpu_baseline"]["nproc"] == 256
    assert json.loads(detail.read_text())["data"] == long
