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
