"""MI355X-native StarPU inference codelet (gfx950 HIP kernels behind a C-ABI).

Import with ``importlib.import_module("starpu-inference-server_amd")`` (the
directory name is not a Python identifier).  Importing fails loudly when the
native library ``libspi_hip.so`` has not been built: there is no fallback.
"""
from . import _native
from ._native import lib
from .codelet import (InferenceCodelet, InferenceExecutionException, InferenceParams, ModelReplica,
                      StarPUCodeletException, TorchCpuForward, buffer_array, buffer_byte_size,
                      clone_model_to_gpus, load_model, make_params, make_variable_interface,
                      make_vector_interface, named_tensors, run_hip, select_gpu_module, tensor_interface,
                      worker_context)

__all__ = [
    "_native", "lib", "InferenceCodelet", "InferenceExecutionException", "InferenceParams", "ModelReplica",
    "StarPUCodeletException", "TorchCpuForward", "buffer_array", "buffer_byte_size", "clone_model_to_gpus",
    "load_model", "make_params", "make_variable_interface", "make_vector_interface", "named_tensors",
    "run_hip", "select_gpu_module", "tensor_interface", "worker_context",
]
