"""End-to-end through the mini-runtime (StarPU stand-in): host buffers -> pinned
slots -> H2D -> HIP codelet -> D2H -> caller buffers, checked against the oracle."""
import importlib

import time

import numpy as np
import pytest

from oracle.cpu_codelet import cpu_inference, normalized_max_error

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rtmod(spi, gpu):
    return importlib.import_module("starpu-inference-server_amd.runtime")


@pytest.mark.parametrize("h2d", ["worker_stream", "device_stream", "worker_sdma"])
def test_runtime_resnet_jobs_match_oracle(spi, zoo, rtmod, h2d):
    m = zoo.resnet18(image=64)
    rep = spi.ModelReplica(m, 0, "fp32", max_batch=4, image_size=64)
    rt = rtmod.Runtime([rep], [((3, 64, 64), np.float32)], [(1000, np.float32)], max_batch=4, workers_per_device=3,
                       h2d_mode=h2d)
    rng = np.random.default_rng(0)
    jobs = []
    for rid in range(12):
        b = 1 + rid % 4  # varying effective batch: nx resized per task
        x = rng.random((b, 3, 64, 64), dtype=np.float32)
        y = np.full((b, 1000), np.nan, dtype=np.float32)
        rt.submit(rid, [x], [y])
        jobs.append((x, y))
    rt.drain()
    assert rt.stats() == (12, 0)
    for x, y in jobs:
        assert normalized_max_error(y, cpu_inference(m, [x])[0]) < 1e-5
    workers = {c.worker_id for c in rt.completions}
    assert len(workers) >= 2  # the eager queue spreads tasks over workers
    for c in rt.completions:
        assert c.status == 0 and c.device_id == 0
        assert c.submit_ns <= c.dequeue_ns <= c.codelet_start_ns <= c.codelet_end_ns <= c.complete_ns
    rt.close()


@pytest.mark.parametrize("h2d", ["worker_stream", "device_stream", "worker_sdma"])
def test_runtime_bert_two_inputs(spi, zoo, rtmod, h2d):
    m = zoo.bert(layers=2)
    rep = spi.ModelReplica(m, 0, "fp16", max_batch=2, seq_len=32)
    rt = rtmod.Runtime([rep], [((32,), np.int64), ((32,), np.int64)], [(32 * 768, np.float32)], max_batch=2,
                       workers_per_device=2, h2d_mode=h2d)
    rng = np.random.default_rng(1)
    ids = rng.integers(0, 30522, (2, 32), dtype=np.int64)
    mask = np.ones((2, 32), dtype=np.int64)
    mask[1, 20:] = 0
    out = np.zeros((2, 32, 768), dtype=np.float32)
    rt.submit(7, [ids, mask], [out])
    rt.drain()
    assert rt.completions[0].status == 0
    err = normalized_max_error(out, cpu_inference(m, [ids, mask])[0])
    print(f"runtime bert L2 S32 fp16 {h2d} err={err:.3e}")
    assert err < 1e-3
    rt.close()


def test_runtime_reports_codelet_failures_and_queue_full(spi, zoo, rtmod):
    m = zoo.resnet18(image=64)
    rep = spi.ModelReplica(m, 0, "fp16", max_batch=2, image_size=64)
    # wrong per-sample shape -> the codelet's layout check fails, the job completes with an error
    rt = rtmod.Runtime([rep], [((3, 32, 32), np.float32)], [(1000, np.float32)], max_batch=2, workers_per_device=1)
    x = np.zeros((1, 3, 32, 32), np.float32)
    y = np.zeros((1, 1000), np.float32)
    rt.submit(1, [x], [y])
    rt.drain()
    c = rt.completions[0]
    assert c.status != 0 and "Tensor layout mismatch" in c.error
    assert rt.stats() == (0, 1)
    rt.close()
    rt = rtmod.Runtime([rep], [((3, 64, 64), np.float32)], [(1000, np.float32)], max_batch=2, workers_per_device=1,
                       max_queue=1)
    xs = [np.zeros((2, 3, 64, 64), np.float32) for _ in range(64)]
    ys = [np.zeros((2, 1000), np.float32) for _ in range(64)]
    rejected = 0
    for i in range(64):
        try:
            rt.submit(i, [xs[i]], [ys[i]])
        except rtmod.QueueFullError:
            rejected += 1
    rt.drain()
    assert rejected > 0 and rt.stats()[0] == 64 - rejected
    rt.close()


def test_runtime_dynamic_batching_merges_and_slices(spi, zoo, rtmod):
    """Queued jobs of ragged sizes merged into one codelet call (merge_input_tensors,
    batch_composition_policy.cpp:153-193) and the outputs sliced back per job
    (slice_outputs_for_sub_job, batching_helpers.hpp:75-125): every job's rows equal
    its own forward."""
    m = zoo.resnet18(image=64)
    rep = spi.ModelReplica(m, 0, "fp32", max_batch=8, image_size=64)
    rt = rtmod.Runtime([rep], [((3, 64, 64), np.float32)], [(1000, np.float32)], max_batch=8,
                       workers_per_device=1, coalesce_max_jobs=8, coalesce_delay_us=200_000)
    rng = np.random.default_rng(3)
    sizes = [1, 3, 2, 1, 1, 4, 2, 1, 3, 1]
    jobs = []
    for rid, b in enumerate(sizes):
        x = rng.random((b, 3, 64, 64), dtype=np.float32)
        y = np.full((b, 1000), np.nan, dtype=np.float32)
        rt.submit(rid, [x], [y])
        jobs.append((x, y))
    rt.drain()
    assert rt.stats() == (len(sizes), 0)
    for x, y in jobs:
        assert normalized_max_error(y, cpu_inference(m, [x])[0]) < 1e-5
    by_id = {c.request_id: c for c in rt.completions}
    assert max(c.task_jobs for c in rt.completions) > 1  # something was merged
    for c in rt.completions:
        assert 1 <= c.task_jobs <= 8 and c.task_batch <= 8
        assert c.submit_ns <= c.dequeue_ns <= c.codelet_start_ns <= c.codelet_end_ns <= c.complete_ns
    # jobs merged into one call share its codelet stamps and batch
    groups = {}
    for rid, c in by_id.items():
        groups.setdefault((c.codelet_start_ns, c.worker_id), []).append(sizes[rid])
    for (start, _), members in groups.items():
        assert sum(members) == next(c.task_batch for c in rt.completions if c.codelet_start_ns == start)
    rt.close()


def test_runtime_bs1_requests_batched_to_8(spi, zoo, rtmod):
    """The serving shape of the reference's client: bs=1 requests, batched server-side."""
    m = zoo.resnet18(image=64)
    rep = spi.ModelReplica(m, 0, "fp16x3", max_batch=8, image_size=64)
    rt = rtmod.Runtime([rep], [((3, 64, 64), np.float32)], [(1000, np.float32)], max_batch=8,
                       workers_per_device=2, coalesce_max_jobs=8, coalesce_delay_us=50_000)
    rng = np.random.default_rng(4)
    xs = [rng.random((1, 3, 64, 64), dtype=np.float32) for _ in range(32)]
    ys = [np.zeros((1, 1000), np.float32) for _ in range(32)]
    for i in range(32):
        rt.submit(i, [xs[i]], [ys[i]])
    rt.drain()
    assert rt.stats() == (32, 0)
    ref = cpu_inference(m, [np.concatenate(xs)])[0]
    assert normalized_max_error(np.concatenate(ys), ref) < 1e-5
    assert sum(c.task_jobs for c in rt.completions) / len(rt.completions) > 1.5
    rt.close()


def test_runtime_two_replicas_on_one_device(spi, zoo, rtmod):
    """num_devices = 2 with device_ids [0, 0]: two weight replicas (clone_model_to_gpus,
    per_device) served by their own workers from one eager queue -- the multi-device path
    rehearsed on a one-GPU box.  Every task must match the oracle, whichever replica ran it."""
    m = zoo.resnet18(image=64)
    reps = spi.clone_model_to_gpus(m, [0, 0], precision="fp16x3", max_batch=4, image_size=64)
    rt = rtmod.Runtime(reps, [((3, 64, 64), np.float32)], [(1000, np.float32)], max_batch=4, workers_per_device=2)
    rng = np.random.default_rng(5)
    jobs = []
    for rid in range(24):
        x = rng.random((4, 3, 64, 64), dtype=np.float32)
        y = np.full((4, 1000), np.nan, dtype=np.float32)
        rt.submit(rid, [x], [y])
        jobs.append((x, y))
    rt.drain()
    assert rt.stats() == (24, 0)
    for x, y in jobs:
        assert normalized_max_error(y, cpu_inference(m, [x])[0]) < 1e-5
    by_worker = {c.worker_id for c in rt.completions}
    # workers 0-1 serve replica 0, workers 2-3 replica 1
    assert by_worker & {0, 1} and by_worker & {2, 3}
    rt.close()


def test_runtime_single_process_multi_device_adaptive(spi, zoo, rtmod):
    """bench.py's single-process serving leg (`e2e_single_process`: one runtime over every
    device's replica, one eager queue, one batcher -- StarPU's shape, starpu_setup.cpp:388-432,
    inference_runner.cpp:251-275) rehearsed with device_ids [0, 0] under the adaptive batcher:
    bs1 requests merged into tasks of up to 8, every request's row checked against the oracle,
    both replicas' workers serving."""
    m = zoo.resnet18(image=64)
    reps = spi.clone_model_to_gpus(m, [0, 0], precision="fp16m", max_batch=8, image_size=64, graphs=True)
    b = rtmod.batching_config("adaptive", 1, 8, coalesce_timeout_us=300, congestion=True, tick_us=500,
                              entry_horizon_us=2000, exit_horizon_us=5000)
    rt = rtmod.Runtime(reps, [((3, 64, 64), np.float32)], [(1000, np.float32)], max_batch=8, workers_per_device=2,
                       batching=b)
    rng = np.random.default_rng(21)
    xs = rng.random((96, 3, 64, 64), dtype=np.float32)
    ys = [np.full((1, 1000), np.nan, dtype=np.float32) for _ in range(96)]
    for rid in range(96):
        rt.submit(rid, [xs[rid:rid + 1]], [ys[rid]])
    rt.drain()
    assert rt.stats() == (96, 0)
    ref = cpu_inference(m, [xs])[0]
    # fp16m is held to 1e-3 at 224x224 only; the reduced 64x64 net sits at ~1.1e-3 and keeps the
    # plain-fp16 bound (test_parity_gpu.resnet_tol)
    assert normalized_max_error(np.concatenate(ys), ref) < 3e-3
    assert {c.worker_id for c in rt.completions} & {0, 1} and {c.worker_id for c in rt.completions} & {2, 3}
    assert max(c.task_jobs for c in rt.completions) > 1  # the batcher merged requests
    rt.close()


@pytest.mark.parametrize("h2d_mode", ["device_stream", "worker_stream", "worker_copy", "worker_sdma"])
def test_runtime_pipeline_with_small_slot_pool(spi, zoo, rtmod, h2d_mode):
    """Pipeline depth 3 per worker over a 2-slot pool (fewer slots than workers x depth): the
    worker must finalize its own finished tasks to free slots (SlotPoolBase::try_acquire /
    acquire / release) -- every ragged job still matches its own forward."""
    m = zoo.resnet18(image=64)
    rep = spi.ModelReplica(m, 0, "fp16x3", max_batch=4, image_size=64)
    rt = rtmod.Runtime([rep], [((3, 64, 64), np.float32)], [(1000, np.float32)], max_batch=4, workers_per_device=2,
                       pipeline_depth=3, slots_per_device=2, h2d_mode=h2d_mode, copy_threads=3)
    rng = np.random.default_rng(8)
    jobs = []
    for rid in range(40):
        b = 1 + rid % 4
        x = rng.random((b, 3, 64, 64), dtype=np.float32)
        y = np.full((b, 1000), np.nan, dtype=np.float32)
        rt.submit(rid, [x], [y])
        jobs.append((x, y))
    rt.drain()
    assert rt.stats() == (40, 0)
    for x, y in jobs:
        assert normalized_max_error(y, cpu_inference(m, [x])[0]) < 1e-5
    rt.close()


def test_runtime_fixed_worker_and_priority(spi, zoo, rtmod):
    """assign_fixed_worker_if_needed (inference_task.cpp:824-842): pinned jobs run on their worker.
    Priority (create_task, :690-753): queued jobs leave the queue highest priority first, and the
    default priority is max(min_prio, max_prio - request_id)."""
    m = zoo.resnet18(image=64)
    rep = spi.ModelReplica(m, 0, "fp32", max_batch=8, image_size=64)
    rt = rtmod.Runtime([rep], [((3, 64, 64), np.float32)], [(1000, np.float32)], max_batch=8, workers_per_device=3)
    x = np.random.default_rng(9).random((1, 3, 64, 64), dtype=np.float32)
    ys = [np.zeros((1, 1000), np.float32) for _ in range(12)]
    for i in range(12):
        rt.submit(i, [x], [ys[i]], fixed_worker=i % 3)
    rt.drain()
    assert all(c.worker_id == c.request_id % 3 and c.status == 0 for c in rt.completions)
    rt.close()

    big = spi.ModelReplica(zoo.resnet152(), 0, "fp32", max_batch=8)  # ~ms per task: the queue fills behind it
    rt = rtmod.Runtime([big], [((3, 224, 224), np.float32)], [(1000, np.float32)], max_batch=8, workers_per_device=1,
                       pipeline_depth=1, min_priority=-100, max_priority=100)
    xb = np.random.default_rng(10).random((8, 3, 224, 224), dtype=np.float32)
    yb = [np.zeros((8, 1000), np.float32) for _ in range(2)]
    xs = np.random.default_rng(11).random((1, 3, 224, 224), dtype=np.float32)
    small = [np.zeros((1, 1000), np.float32) for _ in range(6)]
    rt.submit(100, [xb], [yb[0]])          # occupies the only worker (fp32 ResNet-152 bs8: several ms)
    time.sleep(0.001)                      # let the worker dequeue it before the rest arrive
    rt.submit(101, [xb], [yb[1]])          # queued behind it, so the next three queue too
    for k, rid in enumerate([5, 3, 4]):     # default priorities 95, 97, 96
        rt.submit(rid, [xs], [small[k]])
    rt.submit(50, [xs], [small[3]], priority=-50)
    rt.submit(51, [xs], [small[4]], priority=99)
    rt.drain()
    order = [c.request_id for c in sorted(rt.completions, key=lambda c: c.dequeue_ns)]
    assert order[0] == 100
    assert order[1:] == [51, 3, 4, 5, 101, 50]  # 51 (99) > 3 (97) > 4 > 5 > 101 (max(-100, 100-101)=-1) > 50 (-50)
    rt.close()


@pytest.mark.parametrize("idle_dispatch", [False, True])
def test_runtime_adaptive_batching_under_load(spi, zoo, rtmod, idle_dispatch):
    """AdaptiveBatchingStrategy in the runtime: bs1 requests under a backlog grow the target
    (queue fill / in-flight pressure) and every merged job still gets its own rows back --
    also with idle_dispatch (no coalescing wait on an idle worker: batches form from the
    backlog alone)."""
    m = zoo.resnet18(image=64)
    rep = spi.ModelReplica(m, 0, "fp16x3", max_batch=8, image_size=64)
    b = rtmod.batching_config("adaptive", min_batch=1, batch_limit=8, coalesce_timeout_us=200, congestion=True,
                              tick_us=100, entry_horizon_us=400, exit_horizon_us=2000, idle_dispatch=idle_dispatch)
    rt = rtmod.Runtime([rep], [((3, 64, 64), np.float32)], [(1000, np.float32)], max_batch=8, workers_per_device=2,
                       max_queue=64, batching=b)
    rng = np.random.default_rng(12)
    xs = [rng.random((1, 3, 64, 64), dtype=np.float32) for _ in range(48)]
    ys = [np.zeros((1, 1000), np.float32) for _ in range(48)]
    for i in range(48):
        rt.submit(i, [xs[i]], [ys[i]])
    rt.drain()
    assert rt.stats() == (48, 0)
    ref = cpu_inference(m, [np.concatenate(xs)])[0]
    assert normalized_max_error(np.concatenate(ys), ref) < 1e-5
    assert max(c.task_batch for c in rt.completions) > 1
    assert 1 <= rt.batch_target <= 8
    rt.close()


def test_runtime_idle_dispatch_skips_the_coalescer(spi, zoo, rtmod):
    """idle_dispatch on a sparse open-loop schedule (one request every 2 ms, a 20 ms coalesce
    timeout): the reference's collector holds each request for the timeout while the GPU idles;
    with idle_dispatch the idle worker runs it at once, so p50 falls far below the timeout."""
    m = zoo.resnet18(image=64)
    rep = spi.ModelReplica(m, 0, "fp16", max_batch=8, image_size=64, graphs=True)
    x = np.random.default_rng(14).random((1, 3, 64, 64), dtype=np.float32)
    p50 = {}
    for idle in (False, True):
        b = rtmod.batching_config("adaptive", 1, 8, coalesce_timeout_us=20_000, idle_dispatch=idle)
        rt = rtmod.Runtime([rep], [((3, 64, 64), np.float32)], [(1000, np.float32)], max_batch=8,
                           workers_per_device=2, max_queue=64, batching=b)
        r = rt.loadgen([x], schedule=[(2000, 40)])
        assert r["completed"] == 40 and r["failed"] == 0
        p50[idle] = r["p50_ms"]
        rt.close()
    print(f"p50 coalescer {p50[False]:.2f} ms, idle dispatch {p50[True]:.2f} ms")
    assert p50[True] < 5.0 < p50[False]


def test_runtime_idle_dispatch_leaves_fixed_batching_alone(spi, zoo, rtmod):
    """idle_dispatch is the adaptive strategy's option (include/spi_runtime.h): under the FIXED
    kind the worker still merges up to coalesce_max_jobs jobs, waiting up to coalesce_delay_us
    for them.  A burst of 8 requests every 20 ms against a 10 ms delay: the tasks carry the
    burst whole (mean task batch well above 1) with or without the flag."""
    m = zoo.resnet18(image=64)
    rep = spi.ModelReplica(m, 0, "fp16", max_batch=8, image_size=64, graphs=True)
    x = np.random.default_rng(15).random((1, 3, 64, 64), dtype=np.float32)
    batch = {}
    for idle in (False, True):
        b = rtmod.batching_config("fixed", idle_dispatch=idle)
        rt = rtmod.Runtime([rep], [((3, 64, 64), np.float32)], [(1000, np.float32)], max_batch=8,
                           workers_per_device=1, max_queue=64, coalesce_max_jobs=8, coalesce_delay_us=10_000,
                           batching=b)
        r = rt.loadgen([x], schedule=[(0, 8), (20_000, 1), (0, 7), (20_000, 1), (0, 7)])
        assert r["completed"] == 24 and r["failed"] == 0
        batch[idle] = r["mean_task_batch"]
        rt.close()
    print(f"fixed kind: mean task batch {batch[False]:.2f} without idle_dispatch, {batch[True]:.2f} with")
    assert batch[False] > 3 and batch[True] > 3


def test_runtime_loadgen_closed_and_open_loop(spi, zoo, rtmod):
    """The C++ client loop: closed loop with k requests outstanding, and the open-loop
    (delta_us, repeat) schedule of ci/perf/ci_perf_resnet.csv with a bounded queue."""
    m = zoo.resnet18(image=64)
    rep = spi.ModelReplica(m, 0, "fp16x3", max_batch=8, image_size=64, graphs=True)
    rt = rtmod.Runtime([rep], [((3, 64, 64), np.float32)], [(1000, np.float32)], max_batch=8, workers_per_device=4,
                       max_queue=32, coalesce_max_jobs=8, coalesce_delay_us=100)
    x = np.random.default_rng(13).random((1, 3, 64, 64), dtype=np.float32)
    r = rt.loadgen([x], requests=400, inflight=16, warmup=16)
    assert r["completed"] == 400 and r["failed"] == 0 and r["inferences_per_s"] > 0
    assert 0 < r["p50_ms"] <= r["p95_ms"] <= r["p99_ms"] <= r["max_ms"]
    assert r["mean_task_batch"] >= 1
    r = rt.loadgen([x], schedule=[(300, 50), (50, 100), (500, 20)])
    assert r["completed"] + r["rejected"] == 170 and r["failed"] == 0
    rt.close()


def test_runtime_concurrent_graph_captures(spi, zoo, rtmod):
    """Graphs on, ragged batches across 4 workers: every new batch size is captured lazily on
    its worker thread while the other workers serve -- captures must not break each other
    (workspace allocation and capture are serialised; counters zeroed stream-ordered)."""
    m = zoo.resnet18(image=64)
    rep = spi.ModelReplica(m, 0, "fp16x3", max_batch=8, image_size=64, graphs=True)
    rt = rtmod.Runtime([rep], [((3, 64, 64), np.float32)], [(1000, np.float32)], max_batch=8, workers_per_device=4)
    rng = np.random.default_rng(14)
    jobs = []
    for rid in range(96):
        b = 1 + (rid * 5) % 8
        x = rng.random((b, 3, 64, 64), dtype=np.float32)
        y = np.full((b, 1000), np.nan, dtype=np.float32)
        rt.submit(rid, [x], [y])
        jobs.append((x, y))
    rt.drain()
    bad = [c.error for c in rt.completions if c.status != 0]
    assert not bad, bad[:3]
    for x, y in jobs:
        assert normalized_max_error(y, cpu_inference(m, [x])[0]) < 1e-5
    rt.close()


def test_replica_warmup_precaptures(spi, zoo, gpu):
    """spi_model_warmup: workspace + graph for (batch, seq) ready before the first task; the
    first task then gives the same bytes as an eager forward."""
    import torch
    m = zoo.bert(layers=2, init_std=0.05)
    rep = spi.ModelReplica(m, 0, "fp16", max_batch=2, seq_len=64, graphs=True)
    s = torch.cuda.Stream()
    rep.warmup(s.cuda_stream, 2, 48, True)
    with pytest.raises(spi.InferenceExecutionException, match="exceeds replica max_batch"):
        rep.warmup(s.cuda_stream, 3, 48, True)
    rng = np.random.default_rng(15)
    ids = torch.from_numpy(rng.integers(0, 30522, (2, 48), dtype=np.int64)).cuda()
    mask = torch.ones((2, 48), dtype=torch.int64, device="cuda")
    out_g = torch.empty((2, 48, 768), device="cuda")
    spi.run_hip(rep, [ids, mask], out_g, stream=s.cuda_stream)
    rep.set_graphs(False)
    out_e = torch.empty_like(out_g)
    spi.run_hip(rep, [ids, mask], out_e, stream=s.cuda_stream)
    assert torch.equal(out_g, out_e)
