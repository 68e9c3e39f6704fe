"""CPU restatement of the reference's CPU codelet -- TEST INFRASTRUCTURE ONLY.

Follows InferenceCodelet::cpu_inference_func (src/core/starpu_setup.cpp:784-801)
and run_inference (:594-624):
  1. wrap each input buffer as a row-major view with dims taken from the layout
     (TensorBuilder::assign_tensor_view, src/core/tensor_builder.cpp:68-92);
  2. run model->forward under InferenceMode (starpu_setup.cpp:610, :795);
  3. flatten the IValue result depth-first: Tensor, TensorList, Tuple, List,
     GenericDict in insertion order (append_ivalue, :496-513);
  4. check output count == num_outputs (:612-614) and, per output, numel,
     dtype, contiguity and byte size before a plain memcpy
     (TensorBuilder::copy_output_to_buffer, tensor_builder.cpp:162-190).

The arithmetic of the forward lives in LibTorch (third-party; the reference pins
libtorch 2.2.2 cu118, Dockerfile:50-51).  Here it is PyTorch 2.10.0's ATen CPU
kernels -- the same operator library, a later version -- running the same
TorchScript graphs.  Parity anchoring: the reference's own golden vectors for
this boundary are its toy models (x+1 -> {2,3,4},
tests/integration/starpu/integration_starpu_setup.cpp:42-60; x+1.5,
tests/unit/core/unit_starpu_setup.cpp:2332-2433; x*2 / identity / tuple /
list outputs, tests/common/test_inference_runner.hpp:22-70); they are checked
in tests/test_oracle.py.  ResNet/BERT/ViT numerics are not pinned by any
reference fixture: for those the oracle is ATen itself.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np
import torch


class OracleError(RuntimeError):
    pass


def flatten_ivalue(value, out: list) -> list:
    """append_ivalue (starpu_setup.cpp:496-513)."""
    if isinstance(value, torch.Tensor):
        out.append(value)
    elif isinstance(value, (list, tuple)):
        for v in value:
            flatten_ivalue(v, out)
    elif isinstance(value, dict):
        for v in value.values():
            flatten_ivalue(v, out)
    else:
        raise OracleError("Unsupported model output type")
    return out


def cpu_inference(module: torch.nn.Module, inputs: Sequence[np.ndarray], dims: Sequence[Sequence[int]] | None = None,
                  num_outputs: int = 1, output_nbytes: Sequence[int] | None = None) -> list[np.ndarray]:
    """Run the CPU codelet semantics and return the bytes the W buffers would hold."""
    views = []
    for i, x in enumerate(inputs):
        shape = tuple(dims[i]) if dims is not None else x.shape
        if int(np.prod(shape)) > x.size:
            raise OracleError("[ERROR] Tensor layout mismatch")
        views.append(torch.from_numpy(np.ascontiguousarray(x).reshape(-1)[: int(np.prod(shape))].reshape(shape)))
    with torch.inference_mode():
        result = module(*views)
    outs = flatten_ivalue(result, [])
    if len(outs) != num_outputs:
        raise OracleError("Mismatch between model outputs and StarPU buffers")
    res = []
    for i, t in enumerate(outs):
        if not t.is_contiguous():
            raise OracleError("[ERROR] Output tensor must be contiguous")
        arr = t.detach().cpu().numpy().copy()
        if output_nbytes is not None and arr.nbytes != output_nbytes[i]:
            raise OracleError("[ERROR] Output buffer size mismatch in bytes")
        res.append(arr)
    return res


def normalized_max_error(got: np.ndarray, ref: np.ndarray) -> float:
    """max|got - ref| / max|ref| -- the parity metric (hard part 3)."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    denom = max(np.abs(ref).max(), 1e-30)
    return float(np.abs(got - ref).max() / denom)


def top1_agreement(got: np.ndarray, ref: np.ndarray) -> float:
    return float((np.asarray(got).argmax(-1) == np.asarray(ref).argmax(-1)).mean())
