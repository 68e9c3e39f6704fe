"""Python host over include/spi_runtime.h: the mini-runtime that stands in for
StarPU around the HIP codelet (eager priority queue, per-device HIP workers with
a pipeline of tasks in flight, pinned slot pools, parallel host staging, H2D on
a copy stream, completion callbacks, batching strategies) and the C++ load
generator that measures it like the reference client."""
from __future__ import annotations

import ctypes as C
import threading
from dataclasses import dataclass

import numpy as np

from . import _native as N
from ._native import lib
from .codelet import ModelReplica, spi_dtype

SPI_ERR_QUEUE_FULL = 8
BATCHING = {"fixed": 0, "disabled": 1, "adaptive": 2}
H2D_MODES = {"device_stream": 0, "worker_stream": 1, "worker_copy": 2, "auto": 3, "worker_sdma": 4}


class JobTiming(C.Structure):
    _fields_ = [("submit_ns", C.c_int64), ("dequeue_ns", C.c_int64), ("codelet_start_ns", C.c_int64),
                ("codelet_end_ns", C.c_int64), ("complete_ns", C.c_int64), ("device_id", C.c_int32),
                ("worker_id", C.c_int32), ("task_batch", C.c_int32), ("task_jobs", C.c_int32)]


DONE_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int32, C.c_int32, C.c_char_p, C.POINTER(JobTiming))


class BatchingConfig(C.Structure):
    """spi_batching_config (BatchingStrategyConfig, batching_strategy.hpp:12-24; times in us)."""
    _fields_ = [("kind", C.c_int32), ("min_batch_limit", C.c_int32), ("batch_limit", C.c_int32),
                ("coalesce_timeout_us", C.c_int32), ("congestion_enabled", C.c_int32),
                ("tick_interval_us", C.c_int32), ("entry_horizon_us", C.c_int32), ("exit_horizon_us", C.c_int32),
                ("fill_high", C.c_double), ("fill_low", C.c_double), ("rho_high", C.c_double),
                ("rho_low", C.c_double), ("idle_dispatch", C.c_int32), ("_pad1", C.c_int32)]


class BatchingPressure(C.Structure):
    _fields_ = [("queue_size", C.c_int64), ("queue_capacity", C.c_int64), ("prepared_depth", C.c_int64),
                ("inflight_tasks", C.c_int64), ("max_inflight_tasks", C.c_int64), ("congested", C.c_int32),
                ("_pad", C.c_int32)]


class BatchingState(C.Structure):
    _fields_ = [("target", C.c_int32), ("initialized", C.c_int32), ("low_streak", C.c_int32),
                ("has_marker", C.c_int32), ("last_update_ns", C.c_int64)]


class RuntimeConfig(C.Structure):
    _fields_ = [
        ("num_devices", C.c_int32),
        ("device_ids", C.c_int32 * N.SPI_MAX_REPLICAS),
        ("models", C.c_void_p * N.SPI_MAX_REPLICAS),
        ("workers_per_device", C.c_int32),
        ("max_batch", C.c_int32),
        ("max_queue", C.c_int32),
        ("num_inputs", C.c_int32),
        ("input_types", C.c_int32 * N.SPI_MAX_INPUTS),
        ("input_ndims", C.c_int32 * N.SPI_MAX_INPUTS),
        ("input_dims", (C.c_int64 * N.SPI_MAX_DIMS) * N.SPI_MAX_INPUTS),
        ("num_outputs", C.c_int32),
        ("output_types", C.c_int32 * N.SPI_MAX_OUTPUTS),
        ("output_elems", C.c_int64 * N.SPI_MAX_OUTPUTS),
        ("coalesce_max_jobs", C.c_int32),
        ("coalesce_delay_us", C.c_int32),
        ("pipeline_depth", C.c_int32),
        ("slots_per_device", C.c_int32),
        ("copy_threads", C.c_int32),
        ("h2d_mode", C.c_int32),
        ("min_priority", C.c_int32),
        ("max_priority", C.c_int32),
        ("batching", BatchingConfig),
        ("warmup_batches", C.c_int32),
        ("_pad0", C.c_int32),
    ]


class JobDesc(C.Structure):
    _fields_ = [("request_id", C.c_int32), ("fixed_worker", C.c_int32), ("has_priority", C.c_int32),
                ("priority", C.c_int32), ("batch", C.c_int64), ("inputs", C.POINTER(C.c_void_p)),
                ("outputs", C.POINTER(C.c_void_p)), ("done", DONE_FN), ("user", C.c_void_p)]


class ScheduleSegment(C.Structure):
    _fields_ = [("delta_us", C.c_int64), ("repeat", C.c_int64)]


class LoadgenConfig(C.Structure):
    _fields_ = [("requests", C.c_int64), ("inflight", C.c_int32), ("num_segments", C.c_int32),
                ("segments", C.POINTER(ScheduleSegment)), ("request_batch", C.c_int64),
                ("warmup_requests", C.c_int32), ("_pad", C.c_int32)]


class LoadgenResult(C.Structure):
    _fields_ = [("completed", C.c_int64), ("failed", C.c_int64), ("rejected", C.c_int64),
                ("inferences", C.c_int64), ("seconds", C.c_double), ("inferences_per_s", C.c_double),
                ("p50_ms", C.c_double), ("p95_ms", C.c_double), ("p99_ms", C.c_double), ("mean_ms", C.c_double),
                ("max_ms", C.c_double), ("mean_jobs_per_task", C.c_double), ("mean_task_batch", C.c_double),
                ("p50_queue_ms", C.c_double), ("p99_queue_ms", C.c_double), ("p50_stage_ms", C.c_double),
                ("p99_stage_ms", C.c_double), ("p50_device_ms", C.c_double), ("p99_device_ms", C.c_double),
                ("worst_at_frac", C.c_double), ("error", C.c_char * N.SPI_ERROR_LEN)]


for _name, _res, _args in [
    ("spi_runtime_config_init", None, [C.POINTER(RuntimeConfig)]),
    ("spi_runtime_create", C.c_void_p, [C.POINTER(RuntimeConfig), C.c_char_p, C.c_size_t]),
    ("spi_runtime_submit", C.c_int, [C.c_void_p, C.c_int32, C.c_int64, C.POINTER(C.c_void_p),
                                     C.POINTER(C.c_void_p), DONE_FN, C.c_void_p]),
    ("spi_runtime_submit_job", C.c_int, [C.c_void_p, C.POINTER(JobDesc)]),
    ("spi_runtime_drain", C.c_int, [C.c_void_p]),
    ("spi_runtime_stats", None, [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    ("spi_runtime_num_workers", C.c_int32, [C.c_void_p]),
    ("spi_runtime_worker_times", C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_int64)]),
    ("spi_runtime_batch_target", C.c_int32, [C.c_void_p]),
    ("spi_runtime_warmup_seconds", C.c_double, [C.c_void_p]),
    ("spi_runtime_h2d_mode", C.c_int32, [C.c_void_p]),
    ("spi_runtime_destroy", None, [C.c_void_p]),
    ("spi_runtime_loadgen", C.c_int, [C.c_void_p, C.POINTER(LoadgenConfig), C.POINTER(C.c_void_p),
                                      C.POINTER(LoadgenResult)]),
    ("spi_batching_decide", C.c_int, [C.POINTER(BatchingState), C.POINTER(BatchingConfig),
                                      C.POINTER(BatchingPressure), C.c_int64, C.POINTER(C.c_int32),
                                      C.POINTER(C.c_int32)]),
]:
    getattr(lib, _name).restype = _res
    getattr(lib, _name).argtypes = _args


class QueueFullError(RuntimeError):
    """RESOURCE_EXHAUSTED (docs/server_guide.md:120)."""


@dataclass
class Completion:
    request_id: int
    status: int
    error: str
    submit_ns: int
    dequeue_ns: int
    codelet_start_ns: int
    codelet_end_ns: int
    complete_ns: int
    device_id: int
    worker_id: int
    task_batch: int = 0
    task_jobs: int = 0

    @property
    def latency_ms(self) -> float:
        return (self.complete_ns - self.submit_ns) / 1e6


def batching_config(kind: str = "fixed", min_batch: int = 1, batch_limit: int = 0, coalesce_timeout_us: int = 0,
                    congestion: bool = False, tick_us: int = 500, entry_horizon_us: int = 3000,
                    exit_horizon_us: int = 7000, fill_high: float = 0.85, fill_low: float = 0.65,
                    rho_high: float = 1.10, rho_low: float = 0.90, idle_dispatch: bool = False) -> BatchingConfig:
    """Defaults follow the reference's perf config (ci/perf/resnet152_ci_perf.yml: fill 0.85/0.65,
    rho 1.10/0.90, entry/exit horizons 3000/7000 with a 500 tick), in microseconds.
    idle_dispatch: this build's MI355X tuning -- an idle worker dispatches the queue at once
    instead of waiting out the coalesce timeout (include/spi_runtime.h)."""
    b = BatchingConfig()
    b.kind = BATCHING[kind]
    b.min_batch_limit = min_batch
    b.batch_limit = batch_limit
    b.coalesce_timeout_us = coalesce_timeout_us
    b.congestion_enabled = int(congestion)
    b.tick_interval_us, b.entry_horizon_us, b.exit_horizon_us = tick_us, entry_horizon_us, exit_horizon_us
    b.fill_high, b.fill_low, b.rho_high, b.rho_low = fill_high, fill_low, rho_high, rho_low
    b.idle_dispatch = int(idle_dispatch)
    return b


class Runtime:
    """Eager priority queue over `workers_per_device` HIP workers per replica."""

    def __init__(self, replicas: list[ModelReplica], input_specs, output_specs, max_batch: int,
                 workers_per_device: int = 4, max_queue: int = 0, coalesce_max_jobs: int = 1,
                 coalesce_delay_us: int = 0, pipeline_depth: int = 2, slots_per_device: int = 0,
                 copy_threads: int = 4, h2d_mode: str = "auto", min_priority: int = 0,
                 max_priority: int = 0, batching: BatchingConfig | None = None, warmup_batches: int = 0):
        """input_specs: [(per-sample shape, dtype)]; output_specs: [(per-sample elems, dtype)].
        Fixed batching (default): coalesce_max_jobs > 1 merges up to that many queued jobs (while
        their samples fit max_batch), waiting up to coalesce_delay_us for more.  warmup_batches: 0 =
        every batch size 1..max_batch captured per worker before serving, k = 1..k and max_batch,
        -1 = max_batch only."""
        cfg = RuntimeConfig()
        lib.spi_runtime_config_init(C.byref(cfg))
        cfg.num_devices = len(replicas)
        for i, r in enumerate(replicas):
            cfg.device_ids[i] = r.device_id
            cfg.models[i] = r.handle.value
        cfg.workers_per_device = workers_per_device
        cfg.max_batch = max_batch
        cfg.max_queue = max_queue
        cfg.coalesce_max_jobs = coalesce_max_jobs
        cfg.coalesce_delay_us = coalesce_delay_us
        cfg.pipeline_depth = pipeline_depth
        cfg.slots_per_device = slots_per_device
        cfg.copy_threads = copy_threads
        cfg.h2d_mode = H2D_MODES[h2d_mode]
        cfg.min_priority, cfg.max_priority = min_priority, max_priority
        if batching is not None:
            cfg.batching = batching
        cfg.warmup_batches = warmup_batches
        cfg.num_inputs = len(input_specs)
        self.input_specs = input_specs
        for i, (shape, dt) in enumerate(input_specs):
            cfg.input_types[i] = spi_dtype(dt)
            cfg.input_ndims[i] = len(shape)
            for d, v in enumerate(shape):
                cfg.input_dims[i][d] = v
        cfg.num_outputs = len(output_specs)
        self.output_specs = output_specs
        for i, (elems, dt) in enumerate(output_specs):
            cfg.output_types[i] = spi_dtype(dt)
            cfg.output_elems[i] = elems
        err = C.create_string_buffer(256)
        h = lib.spi_runtime_create(C.byref(cfg), err, len(err))
        if not h:
            raise RuntimeError(f"runtime creation failed: {err.value.decode()}")
        self.handle = C.c_void_p(h)
        self.max_batch = max_batch
        self._replicas = replicas
        self._lock = threading.Lock()
        self._pending: dict[int, tuple] = {}
        self.completions: list[Completion] = []
        self._cb = DONE_FN(self._done)

    @property
    def num_workers(self) -> int:
        return lib.spi_runtime_num_workers(self.handle)

    def worker_times(self) -> list[dict]:
        """Per worker: tasks launched and the seconds its thread spent waiting for slots, staging
        inputs, enqueueing H2D + codelet + D2H and waiting on completion events."""
        out = []
        for w in range(self.num_workers):
            v = (C.c_int64 * 5)()
            if lib.spi_runtime_worker_times(self.handle, w, v) != N.SPI_OK:
                raise RuntimeError("spi_runtime_worker_times failed")
            out.append(dict(tasks=v[0], slot_s=v[1] / 1e9, stage_s=v[2] / 1e9, enqueue_s=v[3] / 1e9,
                            event_s=v[4] / 1e9))
        return out

    @property
    def h2d_mode(self) -> str:
        """The H2D mode in effect (SPI_H2D_AUTO resolved at create)."""
        v = lib.spi_runtime_h2d_mode(self.handle)
        return next(k for k, m in H2D_MODES.items() if m == v)

    @property
    def batch_target(self) -> int:
        return lib.spi_runtime_batch_target(self.handle)

    @property
    def warmup_seconds(self) -> float:
        """Wall time of the per-worker warm-up at create (graph captures, workspaces)."""
        return lib.spi_runtime_warmup_seconds(self.handle)

    def _done(self, _user, request_id, status, error, t):
        tt = t.contents
        c = Completion(request_id, status, (error or b"").decode(), tt.submit_ns, tt.dequeue_ns,
                       tt.codelet_start_ns, tt.codelet_end_ns, tt.complete_ns, tt.device_id, tt.worker_id,
                       tt.task_batch, tt.task_jobs)
        with self._lock:
            self._pending.pop(request_id, None)
            self.completions.append(c)

    def submit(self, request_id: int, inputs: list[np.ndarray], outputs: list[np.ndarray],
               fixed_worker: int | None = None, priority: int | None = None) -> None:
        d = JobDesc()
        d.request_id = request_id
        d.fixed_worker = -1 if fixed_worker is None else fixed_worker
        d.has_priority = int(priority is not None)
        d.priority = 0 if priority is None else priority
        d.batch = int(inputs[0].shape[0])
        ins = (C.c_void_p * len(inputs))(*[x.ctypes.data for x in inputs])
        outs = (C.c_void_p * len(outputs))(*[y.ctypes.data for y in outputs])
        d.inputs = C.cast(ins, C.POINTER(C.c_void_p))
        d.outputs = C.cast(outs, C.POINTER(C.c_void_p))
        d.done = self._cb
        with self._lock:
            self._pending[request_id] = (inputs, outputs, ins, outs)  # alive until the callback
        rc = lib.spi_runtime_submit_job(self.handle, C.byref(d))
        if rc != N.SPI_OK:
            with self._lock:
                self._pending.pop(request_id, None)
            if rc == SPI_ERR_QUEUE_FULL:
                raise QueueFullError("RESOURCE_EXHAUSTED: inference queue is full")
            raise RuntimeError(f"submit failed ({rc})")

    def loadgen(self, inputs: list[np.ndarray], requests: int = 0, inflight: int = 8,
                schedule: list[tuple[int, int]] | None = None, warmup: int = 0) -> dict:
        """The reference client's loop in C++ (closed loop, or the (delta_us, repeat) open-loop
        schedule of ci/perf/ci_perf_resnet.csv): inf/s = inferences / (last response - first
        request), linear-interpolated latency percentiles."""
        ins = [np.ascontiguousarray(x) for x in inputs]
        ptrs = (C.c_void_p * len(ins))(*[x.ctypes.data for x in ins])
        cfg = LoadgenConfig()
        cfg.requests = requests
        cfg.inflight = inflight
        segs = None
        if schedule:
            segs = (ScheduleSegment * len(schedule))(*[ScheduleSegment(d, r) for d, r in schedule])
            cfg.num_segments = len(schedule)
            cfg.segments = segs
        cfg.request_batch = int(ins[0].shape[0])
        cfg.warmup_requests = warmup
        r = LoadgenResult()
        rc = lib.spi_runtime_loadgen(self.handle, C.byref(cfg), ptrs, C.byref(r))
        out = {k: getattr(r, k) for k, _ in LoadgenResult._fields_ if k != "error"}
        out["error"] = r.error.decode()
        if rc not in (N.SPI_OK,) and not out["error"]:
            out["error"] = f"loadgen rc={rc}"
        return out

    def drain(self) -> None:
        lib.spi_runtime_drain(self.handle)

    def stats(self) -> tuple[int, int]:
        c, f = C.c_int64(), C.c_int64()
        lib.spi_runtime_stats(self.handle, C.byref(c), C.byref(f))
        return c.value, f.value

    def close(self) -> None:
        if getattr(self, "handle", None):
            lib.spi_runtime_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def batching_decide(state: BatchingState, config: BatchingConfig, pressure: BatchingPressure,
                    now_ns: int) -> tuple[int, int]:
    t, to = C.c_int32(), C.c_int32()
    rc = lib.spi_batching_decide(C.byref(state), C.byref(config), C.byref(pressure), now_ns, C.byref(t), C.byref(to))
    if rc != N.SPI_OK:
        raise RuntimeError(f"spi_batching_decide failed ({rc})")
    return t.value, to.value
