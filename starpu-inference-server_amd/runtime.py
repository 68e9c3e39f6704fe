"""Python host over include/spi_runtime.h: the mini-runtime that stands in for
StarPU around the HIP codelet (eager queue, per-device HIP workers, pinned slot
staging, H2D/D2H on the worker stream, completion callbacks, and optional
dynamic batching: queued jobs merged into one codelet call, outputs sliced back
per job)."""
from __future__ import annotations

import ctypes as C
import threading
from dataclasses import dataclass

import numpy as np

from . import _native as N
from ._native import lib
from .codelet import ModelReplica, spi_dtype

SPI_ERR_QUEUE_FULL = 8


class JobTiming(C.Structure):
    _fields_ = [("submit_ns", C.c_int64), ("dequeue_ns", C.c_int64), ("codelet_start_ns", C.c_int64),
                ("codelet_end_ns", C.c_int64), ("complete_ns", C.c_int64), ("device_id", C.c_int32),
                ("worker_id", C.c_int32), ("task_batch", C.c_int32), ("task_jobs", C.c_int32)]


DONE_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int32, C.c_int32, C.c_char_p, C.POINTER(JobTiming))


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
    ]


lib.spi_runtime_create.restype = C.c_void_p
lib.spi_runtime_create.argtypes = [C.POINTER(RuntimeConfig), C.c_char_p, C.c_size_t]
lib.spi_runtime_submit.restype = C.c_int
lib.spi_runtime_submit.argtypes = [C.c_void_p, C.c_int32, C.c_int64, C.POINTER(C.c_void_p),
                                   C.POINTER(C.c_void_p), DONE_FN, C.c_void_p]
lib.spi_runtime_drain.restype = C.c_int
lib.spi_runtime_drain.argtypes = [C.c_void_p]
lib.spi_runtime_stats.restype = None
lib.spi_runtime_stats.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
lib.spi_runtime_destroy.restype = None
lib.spi_runtime_destroy.argtypes = [C.c_void_p]


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


class Runtime:
    """Eager shared queue over `workers_per_device` HIP workers per replica."""

    def __init__(self, replicas: list[ModelReplica], input_specs, output_specs, max_batch: int,
                 workers_per_device: int = 4, max_queue: int = 0, coalesce_max_jobs: int = 1,
                 coalesce_delay_us: int = 0):
        """input_specs: [(per-sample shape, dtype)]; output_specs: [(per-sample elems, dtype)].
        coalesce_max_jobs > 1 merges up to that many queued jobs (while their samples fit
        max_batch) into one codelet call, waiting up to coalesce_delay_us for more."""
        cfg = RuntimeConfig()
        cfg.num_devices = len(replicas)
        for i, r in enumerate(replicas):
            cfg.device_ids[i] = r.device_id
            cfg.models[i] = r.handle.value
        cfg.workers_per_device = workers_per_device
        cfg.max_batch = max_batch
        cfg.max_queue = max_queue
        cfg.coalesce_max_jobs = coalesce_max_jobs
        cfg.coalesce_delay_us = coalesce_delay_us
        cfg.num_inputs = len(input_specs)
        self._in_dtypes = []
        for i, (shape, dt) in enumerate(input_specs):
            cfg.input_types[i] = spi_dtype(dt)
            cfg.input_ndims[i] = len(shape)
            for d, v in enumerate(shape):
                cfg.input_dims[i][d] = v
        cfg.num_outputs = len(output_specs)
        for i, (elems, dt) in enumerate(output_specs):
            cfg.output_types[i] = spi_dtype(dt)
            cfg.output_elems[i] = elems
        err = C.create_string_buffer(256)
        h = lib.spi_runtime_create(C.byref(cfg), err, len(err))
        if not h:
            raise RuntimeError(f"runtime creation failed: {err.value.decode()}")
        self.handle = C.c_void_p(h)
        self._replicas = replicas
        self._lock = threading.Lock()
        self._pending: dict[int, tuple] = {}
        self.completions: list[Completion] = []
        self._cb = DONE_FN(self._done)

    def _done(self, _user, request_id, status, error, t):
        tt = t.contents
        c = Completion(request_id, status, (error or b"").decode(), tt.submit_ns, tt.dequeue_ns,
                       tt.codelet_start_ns, tt.codelet_end_ns, tt.complete_ns, tt.device_id, tt.worker_id,
                       tt.task_batch, tt.task_jobs)
        with self._lock:
            self._pending.pop(request_id, None)
            self.completions.append(c)

    def submit(self, request_id: int, inputs: list[np.ndarray], outputs: list[np.ndarray]) -> None:
        batch = int(inputs[0].shape[0])
        ins = (C.c_void_p * len(inputs))(*[x.ctypes.data for x in inputs])
        outs = (C.c_void_p * len(outputs))(*[y.ctypes.data for y in outputs])
        with self._lock:
            self._pending[request_id] = (inputs, outputs, ins, outs)  # alive until the callback
        rc = lib.spi_runtime_submit(self.handle, request_id, batch, ins, outs, self._cb, None)
        if rc != N.SPI_OK:
            with self._lock:
                self._pending.pop(request_id, None)
            if rc == SPI_ERR_QUEUE_FULL:
                raise QueueFullError("RESOURCE_EXHAUSTED: inference queue is full")
            raise RuntimeError(f"submit failed ({rc})")

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
