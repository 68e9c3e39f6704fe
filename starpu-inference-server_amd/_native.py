"""ctypes binding of the C-ABI in include/spi_codelet.h (libspi_hip.so).

The library is the product: every compute call goes through it.  There is no
CPU or PyTorch fallback -- if the shared object is missing or fails to load,
import fails loudly.

``torch`` is imported before the library is opened on purpose: torch's wheel
ships its own libamdhip64.so (SONAME libamdhip64.so.7).  Loading it first lets
the dynamic loader resolve our NEEDED entry to the same runtime, so device
pointers and streams from torch and from this library share one HIP runtime.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (pins the process-wide HIP runtime, see docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
# SPI_HIP_LIB: another build of the same library (A/B runs, tools/build_variant.sh).
LIB_PATH = os.environ.get("SPI_HIP_LIB") or os.path.join(_HERE, "libspi_hip.so")

SPI_ABI_VERSION = 1
SPI_MAX_INPUTS = 16
SPI_MAX_OUTPUTS = 16
SPI_MAX_DIMS = 8
SPI_MAX_REPLICAS = 32
SPI_ERROR_LEN = 256

# enum spi_interface_id
STARPU_VECTOR_INTERFACE_ID = 2
STARPU_VARIABLE_INTERFACE_ID = 5

# enum spi_dtype (at::ScalarType codes)
DTYPE_U8, DTYPE_I8, DTYPE_I16, DTYPE_I32, DTYPE_I64 = 0, 1, 2, 3, 4
DTYPE_F16, DTYPE_F32, DTYPE_F64, DTYPE_BOOL, DTYPE_BF16 = 5, 6, 7, 11, 15

# enum spi_device_type
DEVICE_UNKNOWN, DEVICE_CPU, DEVICE_GPU = 0, 1, 2

# enum spi_status
SPI_OK = 0
SPI_ERR_INVALID_ARGUMENT = 1
SPI_ERR_NO_REPLICA = 2
SPI_ERR_OUTPUT_MISMATCH = 3
SPI_ERR_UNSUPPORTED = 4
SPI_ERR_DEVICE = 5
SPI_ERR_MODEL = 6
SPI_ERR_CPU_FORWARD = 7

# enum spi_family / spi_precision
FAMILY_AUTO, FAMILY_RESNET, FAMILY_BERT, FAMILY_VIT, FAMILY_AFFINE = 0, 1, 2, 3, 4
PREC_F32, PREC_F16, PREC_F16X3, PREC_F16M = 0, 1, 2, 3


class VectorInterface(C.Structure):
    """struct starpu_vector_interface (StarPU 1.4)."""

    _fields_ = [
        ("id", C.c_int32),
        ("ptr", C.c_size_t),
        ("dev_handle", C.c_size_t),
        ("offset", C.c_size_t),
        ("nx", C.c_size_t),
        ("elemsize", C.c_size_t),
        ("slice_base", C.c_size_t),
        ("allocsize", C.c_size_t),
    ]


class VariableInterface(C.Structure):
    """struct starpu_variable_interface (StarPU 1.4)."""

    _fields_ = [
        ("id", C.c_int32),
        ("ptr", C.c_size_t),
        ("dev_handle", C.c_size_t),
        ("offset", C.c_size_t),
        ("elemsize", C.c_size_t),
    ]


class TensorView(C.Structure):
    _fields_ = [
        ("data", C.c_void_p),
        ("dtype", C.c_int32),
        ("ndim", C.c_int32),
        ("shape", C.c_int64 * SPI_MAX_DIMS),
    ]


# err is a raw char* the callback writes into (c_void_p: ctypes would hand a
# c_char_p argument to Python as an immutable bytes copy).
CPU_FORWARD_FN = C.CFUNCTYPE(
    C.c_int, C.c_void_p, C.POINTER(TensorView), C.c_int, C.POINTER(TensorView), C.c_int,
    C.c_void_p, C.c_size_t)


class CodeletArgs(C.Structure):
    """spi_codelet_args: the POD cl_arg (InferenceParams, inference_params.hpp:77-92)."""

    _fields_ = [
        ("abi_version", C.c_uint32),
        ("num_inputs", C.c_uint32),
        ("num_outputs", C.c_uint32),
        ("request_id", C.c_int32),
        ("batch_size", C.c_int64),
        ("verbosity", C.c_int32),
        ("_pad0", C.c_int32),
        ("dims", (C.c_int64 * SPI_MAX_DIMS) * SPI_MAX_INPUTS),
        ("num_dims", C.c_int64 * SPI_MAX_INPUTS),
        ("input_types", C.c_int32 * SPI_MAX_INPUTS),
        ("output_types", C.c_int32 * SPI_MAX_OUTPUTS),
        ("max_inputs", C.c_uint64),
        ("max_dims", C.c_uint64),
        ("model_cpu", C.c_void_p),
        ("cpu_forward", CPU_FORWARD_FN),
        ("num_replicas", C.c_int32),
        ("num_device_ids", C.c_int32),
        ("num_worker_ids", C.c_int32),
        ("_pad1", C.c_int32),
        ("device_ids", C.c_int32 * SPI_MAX_REPLICAS),
        ("worker_ids", C.c_int32 * SPI_MAX_REPLICAS),
        ("models_gpu", C.c_void_p * SPI_MAX_REPLICAS),
        ("codelet_start_ns", C.c_int64),
        ("codelet_end_ns", C.c_int64),
        ("inference_start_ns", C.c_int64),
        ("executed_on", C.c_int32),
        ("worker_id", C.c_int32),
        ("device_id", C.c_int32),
        ("status", C.c_int32),
        ("error", C.c_char * SPI_ERROR_LEN),
    ]


class NamedTensor(C.Structure):
    _fields_ = [
        ("name", C.c_char_p),
        ("data", C.c_void_p),
        ("dtype", C.c_int32),
        ("ndim", C.c_int32),
        ("shape", C.c_int64 * SPI_MAX_DIMS),
    ]


class ModelConfig(C.Structure):
    _fields_ = [
        ("family", C.c_int32),
        ("precision", C.c_int32),
        ("max_batch", C.c_int32),
        ("num_heads", C.c_int32),
        ("seq_len", C.c_int32),
        ("image_size", C.c_int32),
        ("eps", C.c_float),
        ("affine_scale", C.c_float),
        ("affine_shift", C.c_float),
        ("_pad", C.c_int32),
    ]


# name -> (restype, argtypes): every function declared in include/spi_codelet.h
_PROTOS = {
    "spi_hip_inference_func": (None, [C.c_void_p, C.c_void_p]),
    "spi_cpu_inference_func": (None, [C.c_void_p, C.c_void_p]),
    "spi_codelet_init": (C.c_int, [C.c_void_p]),
    "spi_set_worker_context": (None, [C.c_int32, C.c_int32, C.c_void_p]),
    "spi_clear_worker_context": (None, []),
    "spi_buffer_byte_size": (C.c_int, [C.c_void_p, C.POINTER(C.c_size_t)]),
    "spi_select_replica": (C.c_int, [C.POINTER(CodeletArgs), C.c_int32, C.c_int32, C.POINTER(C.c_int32)]),
    "spi_dtype_size": (C.c_size_t, [C.c_int32]),
    "spi_args_init": (None, [C.POINTER(CodeletArgs)]),
    "spi_model_create": (C.c_void_p, [C.c_int32, C.POINTER(ModelConfig), C.POINTER(NamedTensor), C.c_int32,
                                      C.c_char_p, C.c_size_t]),
    "spi_model_destroy": (None, [C.c_void_p]),
    "spi_model_weight_bytes": (C.c_size_t, [C.c_void_p]),
    "spi_model_weight_digest": (C.c_uint64, [C.c_void_p]),
    "spi_model_flops": (C.c_double, [C.c_void_p, C.c_int64]),
    "spi_model_describe": (C.c_char_p, [C.c_void_p]),
    "spi_model_set_graphs": (None, [C.c_void_p, C.c_int32]),
    "spi_model_warmup": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int32]),
    "spi_model_profile": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.POINTER(C.c_void_p),
                                    C.POINTER(C.c_void_p), C.POINTER(C.c_float), C.POINTER(C.c_double),
                                    C.POINTER(C.c_double), C.c_char_p, C.c_int32, C.c_int32]),
    "spi_model_profile_op": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.POINTER(C.c_void_p),
                                       C.POINTER(C.c_void_p), C.c_char_p, C.c_int32, C.POINTER(C.c_float),
                                       C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "spi_model_launch_table": (C.c_int64, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.POINTER(C.c_void_p),
                                          C.POINTER(C.c_void_p), C.c_char_p, C.c_size_t]),
    "spi_device_count": (C.c_int, []),
    "spi_set_device": (C.c_int, [C.c_int32]),
    "spi_device_malloc": (C.c_void_p, [C.c_size_t]),
    "spi_device_free": (None, [C.c_void_p]),
    "spi_host_malloc": (C.c_void_p, [C.c_size_t]),
    "spi_host_free": (None, [C.c_void_p]),
    "spi_memcpy_h2d": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "spi_memcpy_d2h": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "spi_memset_d": (C.c_int, [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p]),
    "spi_stream_create": (C.c_void_p, []),
    "spi_stream_destroy": (None, [C.c_void_p]),
    "spi_stream_synchronize": (C.c_int, [C.c_void_p]),
    "spi_last_error": (C.c_char_p, []),
    # include/spi_ops.h
    "spi_op_packed_bytes": (C.c_size_t, [C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_int32),
                                         C.POINTER(C.c_int32)]),
    "spi_op_pack_weight": (C.c_int, [C.c_int32, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]),
    "spi_op_workspace_bytes": (C.c_size_t, []),
    "spi_op_gemm": (C.c_int, [C.c_int32, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_int32,
                              C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32, C.c_int32,
                              C.c_int32, C.c_void_p, C.c_void_p]),
    "spi_op_conv2d": (C.c_int, [C.c_int32, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p,
                                C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]),
    "spi_op_avgpool_fc": (C.c_int, [C.c_int32, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_int32,
                                    C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]),
    "spi_op_stem_pool_bytes": (C.c_size_t, []),
    "spi_op_stem_pool_pack": (C.c_int, [C.c_void_p, C.c_void_p]),
    "spi_op_stem_pool": (C.c_int, [C.c_int32, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p,
                                   C.c_void_p, C.c_int32, C.c_void_p]),
    "spi_op_attention": (C.c_int, [C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32,
                                   C.c_float, C.c_void_p]),
    "spi_op_layernorm": (C.c_int, [C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.c_int32, C.c_int32, C.c_float, C.c_void_p]),
}


def _load() -> C.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C starpu-inference-server_amd/csrc` "
            "(or __graft_entry__.build()); there is no fallback path")
    lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    for name, (res, args) in _PROTOS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def last_error() -> str:
    msg = lib.spi_last_error()
    return msg.decode() if msg else ""
