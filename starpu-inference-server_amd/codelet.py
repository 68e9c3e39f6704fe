"""Host-side mirror of the reference's codelet interface over the C-ABI.

Names, argument meaning and error behaviour follow the reference so parity
tests read like its own tests:

* ``InferenceCodelet``  -- src/core/starpu_setup.cpp:559-568 (cpu/cuda funcs);
  ``hip_inference_func`` replaces ``cuda_inference_func`` (:807-846).
* ``InferenceParams``   -- src/core/inference_params.hpp:77-92, lowered to the
  POD ``spi_codelet_args``.
* ``StarPUCodeletException`` -- raised when the codelet reports a failure
  (the reference throws it from run_codelet_inference, :710-716).
* ``make_variable_interface`` / ``make_vector_interface`` -- the hand-built
  buffers of tests/common/test_helpers.hpp:247-267.
* ``ModelReplica`` / ``clone_model_to_gpus`` -- src/core/inference_runner.cpp:243-275.
"""
from __future__ import annotations

import contextlib
import ctypes as C
from dataclasses import dataclass, field
from typing import Iterable, Sequence

import numpy as np
import torch

from . import _native as N
from ._native import lib


class StarPUCodeletException(RuntimeError):
    """Codelet failure (the reference's StarPUCodeletException)."""

    def __init__(self, message: str, status: int = N.SPI_ERR_DEVICE):
        super().__init__(message)
        self.status = status


class InferenceExecutionException(RuntimeError):
    pass


_TORCH_TO_SPI = {
    torch.uint8: N.DTYPE_U8, torch.int8: N.DTYPE_I8, torch.int16: N.DTYPE_I16, torch.int32: N.DTYPE_I32,
    torch.int64: N.DTYPE_I64, torch.float16: N.DTYPE_F16, torch.float32: N.DTYPE_F32,
    torch.float64: N.DTYPE_F64, torch.bool: N.DTYPE_BOOL, torch.bfloat16: N.DTYPE_BF16,
}
_SPI_TO_TORCH = {v: k for k, v in _TORCH_TO_SPI.items()}
_SPI_TO_NUMPY = {
    N.DTYPE_U8: np.uint8, N.DTYPE_I8: np.int8, N.DTYPE_I16: np.int16, N.DTYPE_I32: np.int32,
    N.DTYPE_I64: np.int64, N.DTYPE_F16: np.float16, N.DTYPE_F32: np.float32, N.DTYPE_F64: np.float64,
    N.DTYPE_BOOL: np.bool_,
}


def spi_dtype(dtype) -> int:
    if isinstance(dtype, int):
        return dtype
    if isinstance(dtype, torch.dtype):
        return _TORCH_TO_SPI[dtype]
    return _TORCH_TO_SPI[getattr(torch, str(np.dtype(dtype)))]


# ---------------------------------------------------------------------------
# Buffers (StarPU data interfaces)
# ---------------------------------------------------------------------------
def make_variable_interface(ptr: int, nbytes: int) -> N.VariableInterface:
    """tests/common/test_helpers.hpp:247-267: id=VARIABLE, ptr, elemsize=bytes."""
    return N.VariableInterface(N.STARPU_VARIABLE_INTERFACE_ID, int(ptr), 0, 0, int(nbytes))


def make_vector_interface(ptr: int, nx: int, elemsize: int, allocsize: int | None = None) -> N.VectorInterface:
    alloc = nx * elemsize if allocsize is None else allocsize
    return N.VectorInterface(N.STARPU_VECTOR_INTERFACE_ID, int(ptr), 0, 0, int(nx), int(elemsize), 0, int(alloc))


def tensor_interface(t: torch.Tensor, vector: bool = True):
    """A vector interface over a contiguous tensor (host or device)."""
    if not t.is_contiguous():
        raise InferenceExecutionException("[ERROR] tensor must be contiguous")
    if vector:
        return make_vector_interface(t.data_ptr(), t.numel(), t.element_size())
    return make_variable_interface(t.data_ptr(), t.numel() * t.element_size())


def buffer_array(ifaces: Sequence) -> C.Array:
    """void** buffers: inputs (R) first, then outputs (W)."""
    arr = (C.c_void_p * max(1, len(ifaces)))()
    for i, f in enumerate(ifaces):
        arr[i] = C.addressof(f)
    arr._keep = list(ifaces)  # keep the interfaces alive with the array
    return arr


def buffer_byte_size(iface) -> int:
    n = C.c_size_t(0)
    st = lib.spi_buffer_byte_size(C.addressof(iface) if iface is not None else None, C.byref(n))
    if st == N.SPI_ERR_UNSUPPORTED:
        raise InferenceExecutionException(f"[ERROR] Unsupported StarPU buffer interface id {iface.id}")
    if st != N.SPI_OK:
        raise InferenceExecutionException("[ERROR] StarPU buffer is null" if iface is None else
                                          "[ERROR] StarPU buffer size exceeds size_t capacity")
    return n.value


# ---------------------------------------------------------------------------
# Model replicas
# ---------------------------------------------------------------------------
def named_tensors(module: torch.nn.Module) -> list[tuple[str, np.ndarray]]:
    """named_parameters() + floating named_buffers(), as contiguous fp32 arrays."""
    out = []
    seen = set()
    for name, t in list(module.named_parameters()) + list(module.named_buffers()):
        if name in seen or not torch.is_floating_point(t):
            continue
        seen.add(name)
        out.append((name, np.ascontiguousarray(t.detach().to(torch.float32).cpu().numpy())))
    return out


def load_model(path: str) -> torch.jit.ScriptModule:
    """torch::jit::load + eval (inference_runner.cpp:243-249)."""
    m = torch.jit.load(path, map_location="cpu")
    m.eval()
    return m


PRECISIONS = {"fp16": N.PREC_F16, "f16": N.PREC_F16, "fp32": N.PREC_F32, "f32": N.PREC_F32,
              "fp16x3": N.PREC_F16X3, "f16x3": N.PREC_F16X3, "fp16m": N.PREC_F16M, "f16m": N.PREC_F16M}
_FAMILIES = {None: N.FAMILY_AUTO, "auto": N.FAMILY_AUTO, "resnet": N.FAMILY_RESNET, "bert": N.FAMILY_BERT,
             "vit": N.FAMILY_VIT, "affine": N.FAMILY_AFFINE}


class ModelReplica:
    """One device-resident weight replica (BN-folded, MFMA-packed) -- a `spi_model*`."""

    def __init__(self, module: torch.nn.Module | str | None, device_id: int = 0, precision: str = "fp16",
                 max_batch: int = 8, family: str | None = None, num_heads: int = 0, seq_len: int = 0,
                 image_size: int = 0, eps: float = 0.0, affine: tuple[float, float] = (1.0, 0.0),
                 graphs: bool = False):
        if isinstance(module, str):
            # The reference's on-disk format: torch::jit::load + the C++ weight
            # extractor in libspi_torch.so (inference_runner.cpp:243-275).
            from .libtorch import TorchScriptModule
            ts = TorchScriptModule(module)
            rep = ts.replica(device_id, precision, max_batch, family=family, num_heads=num_heads, seq_len=seq_len,
                             image_size=image_size, eps=eps, graphs=graphs)
            self.__dict__.update(rep.__dict__)
            rep.handle = None  # ownership moved to self
            return
        tensors = named_tensors(module) if module is not None else []
        arr = (N.NamedTensor * max(1, len(tensors)))()
        keep = []
        for i, (name, a) in enumerate(tensors):
            bname = name.encode()
            keep.append(bname)
            keep.append(a)
            arr[i].name = bname
            arr[i].data = a.ctypes.data
            arr[i].dtype = N.DTYPE_F32
            arr[i].ndim = a.ndim
            for d, s in enumerate(a.shape):
                arr[i].shape[d] = s
        cfg = N.ModelConfig()
        cfg.family = _FAMILIES[family]
        cfg.precision = PRECISIONS[precision]
        cfg.max_batch = max_batch
        cfg.num_heads = num_heads
        cfg.seq_len = seq_len
        cfg.image_size = image_size
        cfg.eps = eps
        cfg.affine_scale, cfg.affine_shift = affine
        err = C.create_string_buffer(512)
        h = lib.spi_model_create(device_id, C.byref(cfg), arr, len(tensors), err, len(err))
        if not h:
            raise InferenceExecutionException(f"model replica creation failed: {err.value.decode()}")
        self.handle = C.c_void_p(h)
        self.device_id = device_id
        self.precision = precision
        self.max_batch = max_batch
        if graphs:
            self.set_graphs(True)

    @classmethod
    def from_handle(cls, handle: int, device_id: int, precision: str, max_batch: int,
                    graphs: bool = False) -> "ModelReplica":
        self = cls.__new__(cls)
        self.handle = C.c_void_p(handle)
        self.device_id = device_id
        self.precision = precision
        self.max_batch = max_batch
        if graphs:
            self.set_graphs(True)
        return self

    def set_graphs(self, on: bool) -> None:
        lib.spi_model_set_graphs(self.handle, 1 if on else 0)

    def warmup(self, stream: int, batch: int, seq: int = 0, with_mask: bool = True) -> None:
        """Allocate `stream`'s workspace and pre-capture its (batch, seq) graph (per-worker warm-up)."""
        if lib.spi_model_warmup(self.handle, C.c_void_p(stream), batch, seq, int(with_mask)) != N.SPI_OK:
            raise InferenceExecutionException(f"warmup failed: {N.last_error()}")

    @property
    def description(self) -> str:
        return lib.spi_model_describe(self.handle).decode()

    @property
    def weight_bytes(self) -> int:
        return lib.spi_model_weight_bytes(self.handle)

    @property
    def weight_digest(self) -> int:
        return lib.spi_model_weight_digest(self.handle)

    def flops(self, batch: int) -> float:
        return lib.spi_model_flops(self.handle, batch)

    def profile(self, inputs: Sequence[torch.Tensor], out: torch.Tensor, stream: int,
                max_ops: int = 4096) -> list[dict]:
        """One forward with every launch bracketed by hipEvents on `stream` (measurement only)."""
        ins = (C.c_void_p * max(1, len(inputs)))(*[x.data_ptr() for x in inputs])
        outs = (C.c_void_p * 1)(out.data_ptr())
        ms = (C.c_float * max_ops)()
        fl = (C.c_double * max_ops)()
        by = (C.c_double * max_ops)()
        name_len = 96
        names = C.create_string_buffer(name_len * max_ops)
        seq = int(inputs[0].shape[1]) if inputs[0].dim() >= 2 else 0
        n = lib.spi_model_profile(self.handle, C.c_void_p(stream), int(inputs[0].shape[0]), seq, ins, outs, ms, fl,
                                  by, names, name_len, max_ops)
        if n < 0:
            raise InferenceExecutionException(f"profile failed: {N.last_error()}")
        raw = names.raw
        return [dict(name=raw[i * name_len:(i + 1) * name_len].split(b"\0")[0].decode(), ms=ms[i], flops=fl[i],
                     bytes=by[i]) for i in range(n)]

    def launch_table(self, inputs: Sequence[torch.Tensor], out: torch.Tensor, stream: int) -> list[dict]:
        """One eager forward with every kernel launch recorded (measurement only): per launch its
        op (index, name), kernel (template id) and grid in workgroups."""
        ins = (C.c_void_p * max(1, len(inputs)))(*[x.data_ptr() for x in inputs])
        outs = (C.c_void_p * 1)(out.data_ptr())
        seq = int(inputs[0].shape[1]) if inputs[0].dim() >= 2 else 0
        size = 1 << 20
        while True:
            buf = C.create_string_buffer(size)
            n = lib.spi_model_launch_table(self.handle, C.c_void_p(stream), int(inputs[0].shape[0]), seq, ins, outs,
                                           buf, size)
            if n < 0:
                raise InferenceExecutionException(f"launch_table failed: {N.last_error()}")
            if n < size:
                break
            size = int(n) + 1
        rows = []
        for line in buf.value.decode().splitlines():
            i, name, kernel, gx, gy, gz, block = line.split("\t")
            rows.append(dict(op_index=int(i), op=name, kernel=kernel, grid=(int(gx), int(gy), int(gz)),
                             block=int(block)))
        return rows

    def profile_op(self, inputs: Sequence[torch.Tensor], out: torch.Tensor, stream: int, name: str,
                   reps: int = 200) -> dict:
        """One eager forward with op `name` launched `reps` times back to back between one pair
        of hipEvents on `stream`: its device time per launch (measurement only)."""
        ins = (C.c_void_p * max(1, len(inputs)))(*[x.data_ptr() for x in inputs])
        outs = (C.c_void_p * 1)(out.data_ptr())
        ms, fl, by = C.c_float(), C.c_double(), C.c_double()
        seq = int(inputs[0].shape[1]) if inputs[0].dim() >= 2 else 0
        rc = lib.spi_model_profile_op(self.handle, C.c_void_p(stream), int(inputs[0].shape[0]), seq, ins, outs,
                                      name.encode(), int(reps), C.byref(ms), C.byref(fl), C.byref(by))
        if rc != 0:
            raise InferenceExecutionException(f"profile_op failed: {N.last_error()}")
        return dict(name=name, ms=ms.value, flops=fl.value, bytes=by.value, reps=reps)

    def close(self) -> None:
        if getattr(self, "handle", None):
            lib.spi_model_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def clone_model_to_gpus(module: torch.nn.Module, device_ids: Iterable[int], **kw) -> list[ModelReplica]:
    """One replica per device (gpu_model_replication: per_device)."""
    return [ModelReplica(module, device_id=d, **kw) for d in device_ids]


# ---------------------------------------------------------------------------
# CPU forward binding (LibTorch model_cpu->forward of the reference)
# ---------------------------------------------------------------------------
def _append_ivalue(value, outputs: list) -> None:
    """append_ivalue (starpu_setup.cpp:496-513): Tensor / list / tuple / dict, depth-first."""
    if isinstance(value, torch.Tensor):
        outputs.append(value)
    elif isinstance(value, (list, tuple)):
        for v in value:
            _append_ivalue(v, outputs)
    elif isinstance(value, dict):
        for v in value.values():
            _append_ivalue(v, outputs)
    else:
        raise InferenceExecutionException("Unsupported model output type")


def _view(tv: N.TensorView) -> torch.Tensor:
    shape = tuple(tv.shape[d] for d in range(tv.ndim))
    n = int(np.prod(shape)) if shape else 1
    dt = _SPI_TO_NUMPY[tv.dtype]
    if n == 0:
        return torch.from_numpy(np.empty(shape, dtype=dt))
    buf = (C.c_char * (n * np.dtype(dt).itemsize)).from_address(tv.data)
    return torch.from_numpy(np.frombuffer(buf, dtype=dt).reshape(shape))


class TorchCpuForward:
    """Binds a torch / TorchScript module as the codelet's CPU forward callback.

    Mirrors cpu_inference_func's body: views over the buffers, forward under
    InferenceMode, IValue flattening, then copy_output_to_buffer's checks
    (numel, dtype, contiguity, byte size) and memcpy (tensor_builder.cpp:162-190).
    """

    def __init__(self, module: torch.nn.Module):
        self.module = module
        self._cb = N.CPU_FORWARD_FN(self._call)
        self.handle = C.c_void_p(id(self))

    def _call(self, _model, inputs, n_in, outputs, n_out, err, errlen):
        try:
            xs = [_view(inputs[i]) for i in range(n_in)]
            with torch.inference_mode():
                result = self.module(*xs)
            outs: list = []
            _append_ivalue(result, outs)
            if len(outs) != n_out:
                raise InferenceExecutionException("Mismatch between model outputs and StarPU buffers")
            for i in range(n_out):
                t = outs[i]
                tv = outputs[i]
                if not tv.data:
                    raise InferenceExecutionException("[ERROR] Output buffer pointer is null")
                if t.dtype != _SPI_TO_TORCH.get(tv.dtype):
                    raise InferenceExecutionException("[ERROR] Output type mismatch")
                if not t.is_contiguous():
                    raise InferenceExecutionException("[ERROR] Output tensor must be contiguous")
                if t.numel() != tv.shape[0]:
                    raise InferenceExecutionException("[ERROR] Output buffer size mismatch in bytes")
                C.memmove(tv.data, t.data_ptr(), t.numel() * t.element_size())
            return 0
        except Exception as e:  # noqa: BLE001 -- reported through the C status
            msg = str(e).encode()[: errlen - 1]
            C.memmove(err, msg + b"\0", len(msg) + 1)
            return 1


# ---------------------------------------------------------------------------
# InferenceParams -> spi_codelet_args
# ---------------------------------------------------------------------------
@dataclass
class InferenceParams:
    num_inputs: int = 0
    num_outputs: int = 0
    dims: list = field(default_factory=list)          # per input, dims[0] = batch
    input_types: list = field(default_factory=list)   # torch dtypes or spi codes
    output_types: list = field(default_factory=list)  # expected output dtypes (default fp32)
    models_gpu: list = field(default_factory=list)    # ModelReplica per device/worker
    device_ids: list = field(default_factory=list)
    worker_ids: list = field(default_factory=list)
    model_cpu: TorchCpuForward | None = None
    batch_size: int = 1
    request_id: int = 0
    max_inputs: int = N.SPI_MAX_INPUTS
    max_dims: int = N.SPI_MAX_DIMS

    def to_args(self) -> N.CodeletArgs:
        a = N.CodeletArgs()
        lib.spi_args_init(C.byref(a))
        a.num_inputs = self.num_inputs
        a.num_outputs = self.num_outputs
        a.request_id = self.request_id
        a.batch_size = self.batch_size
        a.max_inputs = self.max_inputs
        a.max_dims = self.max_dims
        for i, d in enumerate(self.dims[: N.SPI_MAX_INPUTS]):
            a.num_dims[i] = len(d)
            for j, v in enumerate(d[: N.SPI_MAX_DIMS]):
                a.dims[i][j] = int(v)
        for i, t in enumerate(self.input_types[: N.SPI_MAX_INPUTS]):
            a.input_types[i] = spi_dtype(t)
        for i, t in enumerate(self.output_types[: N.SPI_MAX_OUTPUTS]):
            a.output_types[i] = spi_dtype(t)
        a.num_replicas = len(self.models_gpu)
        for i, m in enumerate(self.models_gpu[: N.SPI_MAX_REPLICAS]):
            a.models_gpu[i] = m.handle.value if m is not None and m.handle else None
        a.num_device_ids = len(self.device_ids)
        for i, d in enumerate(self.device_ids[: N.SPI_MAX_REPLICAS]):
            a.device_ids[i] = d
        a.num_worker_ids = len(self.worker_ids)
        for i, w in enumerate(self.worker_ids[: N.SPI_MAX_REPLICAS]):
            a.worker_ids[i] = w
        if self.model_cpu is not None:
            a.model_cpu = self.model_cpu.handle
            a.cpu_forward = self.model_cpu._cb
        a._keep = (self.models_gpu, self.model_cpu)
        return a


def make_params(shapes: Sequence[Sequence[int]], dtypes: Sequence, num_outputs: int = 1,
                **kw) -> InferenceParams:
    """make_params_for_inputs (tests/common/test_helpers.hpp:270-300)."""
    return InferenceParams(num_inputs=len(shapes), num_outputs=num_outputs, dims=[list(s) for s in shapes],
                           input_types=list(dtypes), batch_size=int(shapes[0][0]) if shapes and shapes[0] else 1,
                           **kw)


def select_gpu_module(params: InferenceParams | N.CodeletArgs, worker_id: int, device_id: int) -> int:
    a = params.to_args() if isinstance(params, InferenceParams) else params
    idx = C.c_int32(-1)
    st = lib.spi_select_replica(C.byref(a), worker_id, device_id, C.byref(idx))
    if st != N.SPI_OK:
        if a.num_worker_ids > 0:
            raise StarPUCodeletException(
                f"[ERROR] No GPU model replica available for worker {worker_id} on device {device_id}",
                N.SPI_ERR_NO_REPLICA)
        raise StarPUCodeletException(f"[ERROR] No GPU model replica available for device {device_id}",
                                     N.SPI_ERR_NO_REPLICA)
    return idx.value


@contextlib.contextmanager
def worker_context(worker_id: int, device_id: int, stream: int | None):
    """What starpu_worker_get_id / _get_devid / starpu_hip_get_local_stream return."""
    lib.spi_set_worker_context(worker_id, device_id, C.c_void_p(stream or 0))
    try:
        yield
    finally:
        lib.spi_clear_worker_context()


class InferenceCodelet:
    """The codelet descriptor: cpu func + HIP func, variable buffers, async HIP."""

    nbuffers = -1  # STARPU_VARIABLE_NBUFFERS
    type = "STARPU_FORKJOIN"
    hip_flags = 1  # STARPU_HIP_ASYNC

    def __init__(self):
        self.cpu_funcs = [self.cpu_inference_func]
        self.hip_funcs = [self.hip_inference_func]

    @staticmethod
    def _run(fn, buffers, params):
        args = params.to_args() if isinstance(params, InferenceParams) else params
        arr = buffer_array(buffers) if buffers is not None else None
        fn(arr, C.byref(args))
        if args.status != N.SPI_OK:
            raise StarPUCodeletException(args.error.decode(), args.status)
        return args

    @classmethod
    def cpu_inference_func(cls, buffers, params) -> N.CodeletArgs:
        return cls._run(lib.spi_cpu_inference_func, buffers, params)

    @classmethod
    def hip_inference_func(cls, buffers, params) -> N.CodeletArgs:
        return cls._run(lib.spi_hip_inference_func, buffers, params)


def run_hip(replica: ModelReplica, inputs: Sequence[torch.Tensor], out: torch.Tensor,
            stream: int | None = None, device_id: int | None = None, worker_id: int = 0,
            sync: bool = True) -> N.CodeletArgs:
    """Convenience: one codelet call over device tensors on `stream`."""
    dev = replica.device_id if device_id is None else device_id
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    params = make_params([list(x.shape) for x in inputs], [x.dtype for x in inputs], models_gpu=[replica],
                         device_ids=[replica.device_id], output_types=[out.dtype])
    bufs = [tensor_interface(x) for x in inputs] + [tensor_interface(out)]
    with worker_context(worker_id, dev, stream):
        args = InferenceCodelet.hip_inference_func(bufs, params)
    if sync:
        lib.spi_stream_synchronize(C.c_void_p(stream))
    return args
