"""CPU tests of the C-ABI boundary (no GPU needed).

Mirrors the reference's codelet tests that run without a device:
buffer_byte_size (src/core/starpu_setup.cpp:515-542), select_gpu_module
(tests/unit/core/unit_starpu_setup.cpp:4106-4183), the missing-replica error
(:2435-2472), the CPU codelet over hand-built buffers
(tests/integration/starpu/integration_starpu_setup.cpp:42-60) and
copy_output_to_buffer's checks (tests/unit/core/unit_tensor_builder.cpp:159-410).
"""
import ctypes as C
import glob
import os
import re
import subprocess

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions(pattern="*.h"):
    names = set()
    for path in glob.glob(os.path.join(ROOT, "include", pattern)):
        for line in open(path):
            if line.lstrip().startswith(("typedef", "*", "/*", "#")):
                continue
            m = re.match(r"^[A-Za-z_][\w \t\*]*?\b(spi_\w+)\s*\(", line)
            if m:
                names.add(m.group(1))
    return names


def exported(lib_path):
    out = subprocess.run(["nm", "-D", "--defined-only", lib_path], capture_output=True, text=True,
                         check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_library_exports_every_header_symbol(spi):
    import importlib
    torch_names = header_functions("spi_torch.h")
    names = header_functions() - torch_names
    assert len(names) >= 36 and len(torch_names) >= 8
    missing = sorted(names - exported(spi._native.LIB_PATH))
    assert not missing, f"declared but not exported by libspi_hip.so: {missing}"
    lt = importlib.import_module("starpu-inference-server_amd.libtorch")
    missing = sorted(torch_names - exported(lt.LIB_PATH))
    assert not missing, f"declared but not exported by libspi_torch.so: {missing}"
    importlib.import_module("starpu-inference-server_amd.runtime")  # binds include/spi_runtime.h
    for n in names:  # and every one is bound in ctypes
        assert n in spi._native._PROTOS or getattr(spi.lib, n).argtypes is not None, n
    for n in torch_names:
        assert n in lt._PROTOS, n


PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "spi_codelet.h"
#include "spi_runtime.h"
#define F(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
#define S(T) printf(#T " %zu\n", sizeof(T));
int main(void) {
  S(spi_vector_interface) F(spi_vector_interface, ptr) F(spi_vector_interface, nx) F(spi_vector_interface, elemsize) F(spi_vector_interface, slice_base) F(spi_vector_interface, allocsize)
  S(spi_variable_interface) F(spi_variable_interface, ptr) F(spi_variable_interface, elemsize)
  S(spi_tensor_view) S(spi_named_tensor) S(spi_model_config)
  S(spi_codelet_args) F(spi_codelet_args, dims) F(spi_codelet_args, input_types)
  F(spi_codelet_args, output_types) F(spi_codelet_args, model_cpu) F(spi_codelet_args, cpu_forward)
  F(spi_codelet_args, device_ids) F(spi_codelet_args, models_gpu) F(spi_codelet_args, codelet_start_ns)
  F(spi_codelet_args, executed_on) F(spi_codelet_args, status) F(spi_codelet_args, error)
  S(spi_runtime_config) F(spi_runtime_config, models) F(spi_runtime_config, workers_per_device)
  F(spi_runtime_config, input_dims) F(spi_runtime_config, num_outputs) F(spi_runtime_config, output_elems)
  F(spi_runtime_config, coalesce_max_jobs) F(spi_runtime_config, coalesce_delay_us)
  F(spi_runtime_config, pipeline_depth) F(spi_runtime_config, h2d_mode) F(spi_runtime_config, max_priority)
  F(spi_runtime_config, batching)
  S(spi_batching_config) F(spi_batching_config, exit_horizon_us) F(spi_batching_config, fill_high)
  F(spi_batching_config, rho_low) S(spi_batching_pressure) F(spi_batching_pressure, congested)
  S(spi_batching_state) F(spi_batching_state, last_update_ns)
  S(spi_job_desc) F(spi_job_desc, batch) F(spi_job_desc, done) F(spi_job_desc, user)
  S(spi_loadgen_config) F(spi_loadgen_config, segments) F(spi_loadgen_config, warmup_requests)
  S(spi_loadgen_result) F(spi_loadgen_result, p50_queue_ms) F(spi_loadgen_result, error)
  S(spi_schedule_segment)
  S(spi_job_timing) F(spi_job_timing, complete_ns) F(spi_job_timing, worker_id) F(spi_job_timing, task_jobs)
  return 0;
}
"""


def test_ctypes_layouts_match_the_c_header(spi, tmp_path):
    src = tmp_path / "probe.c"
    src.write_text(PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                             check=True).stdout.splitlines())
    import importlib
    rt = importlib.import_module("starpu-inference-server_amd.runtime")
    N = spi._native
    types = {"spi_runtime_config": rt.RuntimeConfig, "spi_job_timing": rt.JobTiming,
             "spi_batching_config": rt.BatchingConfig, "spi_batching_pressure": rt.BatchingPressure,
             "spi_batching_state": rt.BatchingState, "spi_job_desc": rt.JobDesc,
             "spi_loadgen_config": rt.LoadgenConfig, "spi_loadgen_result": rt.LoadgenResult,
             "spi_schedule_segment": rt.ScheduleSegment,
             "spi_vector_interface": N.VectorInterface, "spi_variable_interface": N.VariableInterface,
             "spi_tensor_view": N.TensorView, "spi_named_tensor": N.NamedTensor, "spi_model_config": N.ModelConfig,
             "spi_codelet_args": N.CodeletArgs}
    for key, val in got.items():
        if "." in key:
            t, f = key.split(".")
            assert getattr(types[t], f).offset == int(val), key
        else:
            assert C.sizeof(types[key]) == int(val), key


def test_buffer_byte_size(spi):
    N = spi._native
    var = spi.make_variable_interface(0x1000, 12)
    assert spi.buffer_byte_size(var) == 12
    vec = spi.make_vector_interface(0x1000, 5, 8)
    assert spi.buffer_byte_size(vec) == 40
    vec.nx = 0
    assert spi.buffer_byte_size(vec) == 0
    vec.nx = 1 << 40  # nx is size_t (StarPU 1.4): no 32-bit truncation
    assert spi.buffer_byte_size(vec) == (1 << 40) * 8
    # BufferByteSize.ThrowsWhenVectorSizeOverflows (unit_starpu_setup.cpp:2105-2124)
    over = spi.make_vector_interface(0x1000, 2, 2**64 - 1)
    with pytest.raises(spi.InferenceExecutionException, match="exceeds size_t capacity"):
        spi.buffer_byte_size(over)
    bad = N.VariableInterface(3, 0, 0, 0, 4)  # CSR id: unsupported
    with pytest.raises(spi.InferenceExecutionException, match="Unsupported StarPU buffer interface id 3"):
        spi.buffer_byte_size(bad)
    with pytest.raises(spi.InferenceExecutionException, match="buffer is null"):
        spi.buffer_byte_size(None)


@pytest.fixture(scope="module")
def fake_replicas(spi):
    # host-only replicas (device -1): valid spi_model handles without a GPU
    return [spi.ModelReplica(None, -1, "fp32", family="affine") for _ in range(2)]


def test_select_replica_mappings(spi, fake_replicas):
    r0, r1 = fake_replicas
    p = spi.InferenceParams(models_gpu=[r0])
    assert spi.select_gpu_module(p, worker_id=3, device_id=0) == 0          # index = device id
    p = spi.InferenceParams(models_gpu=[r0, r1], device_ids=[0, 2])
    assert spi.select_gpu_module(p, worker_id=5, device_id=2) == 1          # device id mapping
    p = spi.InferenceParams(models_gpu=[r0, r1], device_ids=[0, 0], worker_ids=[7, 9])
    assert spi.select_gpu_module(p, worker_id=9, device_id=0) == 1          # worker id mapping
    p = spi.InferenceParams(models_gpu=[r0], device_ids=[0], worker_ids=[7])
    with pytest.raises(spi.StarPUCodeletException, match="No GPU model replica available for worker 8 on device 0"):
        spi.select_gpu_module(p, worker_id=8, device_id=0)
    p = spi.InferenceParams(models_gpu=[None])
    with pytest.raises(spi.StarPUCodeletException, match="No GPU model replica available for device 0"):
        spi.select_gpu_module(p, worker_id=0, device_id=0)


def test_hip_codelet_without_replica_raises(spi):
    """unit_starpu_setup.cpp:2435-2472: no replica -> StarPUCodeletException (no device touched)."""
    params = spi.InferenceParams(num_inputs=0, num_outputs=0)
    with spi.worker_context(91, 0, None):
        with pytest.raises(spi.StarPUCodeletException, match=r"Codelet failure: \[ERROR\] No GPU model replica"):
            spi.InferenceCodelet.hip_inference_func(None, params)


def test_abi_version_mismatch_is_rejected(spi, fake_replicas):
    a = spi.InferenceParams(models_gpu=[fake_replicas[0]]).to_args()
    a.abi_version = 99
    with pytest.raises(spi.StarPUCodeletException, match="ABI version"):
        spi.InferenceCodelet.hip_inference_func(None, a)


def _cpu_call(spi, module, x, out, n_out=1):
    params = spi.make_params([list(x.shape)], [x.dtype], num_outputs=n_out,
                             model_cpu=spi.TorchCpuForward(module), output_types=[out.dtype] * n_out)
    bufs = [spi.make_variable_interface(x.data_ptr(), x.numel() * x.element_size()),
            spi.make_variable_interface(out.data_ptr(), out.numel() * out.element_size())]
    with spi.worker_context(4, -1, None):
        return spi.InferenceCodelet.cpu_inference_func(bufs, params)


def test_cpu_codelet_x_plus_one(spi, zoo):
    """integration_starpu_setup.cpp:42-60: x+1 on {1,2,3} -> {2,3,4}, executed_on CPU, stamps ordered."""
    x = torch.tensor([1.0, 2.0, 3.0])
    out = torch.zeros(3)
    import time
    before = time.monotonic_ns()
    args = _cpu_call(spi, zoo.AddConstant(1.0), x, out)
    after = time.monotonic_ns()
    assert out.tolist() == [2.0, 3.0, 4.0]
    assert args.executed_on == spi._native.DEVICE_CPU and args.worker_id == 4
    assert before <= args.codelet_start_ns <= args.inference_start_ns <= args.codelet_end_ns <= after


def test_cpu_codelet_output_checks(spi, zoo):
    x = torch.tensor([1.0, 2.0, 3.0])
    with pytest.raises(spi.StarPUCodeletException, match="Output buffer size mismatch"):
        _cpu_call(spi, zoo.AddConstant(1.0), x, torch.zeros(4))

    class Pair(torch.nn.Module):
        def forward(self, t):
            return t, t + 1

    with pytest.raises(spi.StarPUCodeletException, match="Mismatch between model outputs and StarPU buffers"):
        _cpu_call(spi, Pair(), x, torch.zeros(3))

    class Const(torch.nn.Module):
        def forward(self, t):
            return 5

    with pytest.raises(spi.StarPUCodeletException, match="Unsupported model output type"):
        _cpu_call(spi, Const(), x, torch.zeros(3))
    with pytest.raises(spi.StarPUCodeletException, match="Output type mismatch"):
        _cpu_call(spi, zoo.AddConstant(1.0), x, torch.zeros(3, dtype=torch.float64))


def test_cpu_codelet_without_model(spi):
    x = torch.ones(2)
    params = spi.make_params([[2]], [torch.float32])
    bufs = [spi.make_variable_interface(x.data_ptr(), 8), spi.make_variable_interface(x.data_ptr(), 8)]
    with pytest.raises(spi.StarPUCodeletException, match="No CPU model"):
        spi.InferenceCodelet.cpu_inference_func(bufs, params)


def test_layout_limits(spi, zoo):
    x = torch.ones(2)
    params = spi.make_params([[2]], [torch.float32], model_cpu=spi.TorchCpuForward(zoo.AddConstant(1.0)))
    params.max_inputs = 0
    bufs = [spi.make_variable_interface(x.data_ptr(), 8), spi.make_variable_interface(x.data_ptr(), 8)]
    with pytest.raises(spi.StarPUCodeletException, match="Too many input tensors"):
        spi.InferenceCodelet.cpu_inference_func(bufs, params)


def test_codelet_descriptor(spi):
    """InferenceCodelet ctor (starpu_setup.cpp:559-568): variable buffers, FORKJOIN, async GPU func."""
    cl = spi.InferenceCodelet()
    assert cl.nbuffers == -1 and cl.type == "STARPU_FORKJOIN" and cl.hip_flags == 1
    assert cl.cpu_funcs[0] == cl.cpu_inference_func and cl.hip_funcs[0] == cl.hip_inference_func
    # without <starpu.h> the C adapter reports itself unavailable rather than guessing the struct
    assert spi.lib.spi_codelet_init(None) == spi._native.SPI_ERR_UNSUPPORTED


@pytest.mark.parametrize("name,kw,gflop", [
    ("resnet18", {}, 3.628), ("resnet152", {}, 23.027), ("bert_base", {"seq_len": 128}, 22.35),
    ("vit_l_16", {}, 123.1)])
def test_host_replica_recognition_and_flops(spi, zoo, name, kw, gflop):
    """Recogniser + packer on the full architectures (host-only replica); FLOPs match SURVEY.md 8(d)."""
    m = zoo.build(name)
    r = spi.ModelReplica(m, -1, "fp16", max_batch=2, **kw)
    assert abs(r.flops(1) / 1e9 - gflop) / gflop < 2e-3
    assert r.weight_bytes > 0
    r16x3 = spi.ModelReplica(m, -1, "fp16x3", max_batch=2, **kw)
    assert "f16x3" in r16x3.description
    r16m = spi.ModelReplica(m, -1, "fp16m", max_batch=2, **kw)
    assert "f16m" in r16m.description
    if name.startswith("resnet"):  # + the downsample lo halves, stem / FC in split fp16
        assert r.weight_bytes < r16m.weight_bytes < r16x3.weight_bytes
    else:  # transformers: hi + lo halves of every GEMM weight (the fp32 embeddings / LN as fp16)
        assert r16m.weight_bytes > r.weight_bytes


def test_flops_match_torch_flop_counter(spi, zoo):
    from torch.utils.flop_counter import FlopCounterMode
    m = zoo.resnet18(image=64)
    with FlopCounterMode(display=False) as fc:
        m(torch.rand(2, 3, 64, 64))
    r = spi.ModelReplica(m, -1, "fp32", max_batch=2, image_size=64)
    assert abs(r.flops(2) - fc.get_total_flops()) / fc.get_total_flops() < 1e-6


def test_recognition_errors(spi, zoo):
    m = zoo.resnet18(image=64)
    sd = {k: v for k, v in m.state_dict().items() if "layer3.0.conv2" not in k}
    holder = torch.nn.Module()
    for k, v in sd.items():
        holder.register_buffer(k.replace(".", "__"), v)

    class Named(torch.nn.Module):
        def __init__(self, d):
            super().__init__()
            self.d = d

        def named_parameters(self, *a, **k):
            return iter([])

        def named_buffers(self, *a, **k):
            return iter(self.d.items())

    with pytest.raises(spi.InferenceExecutionException, match="missing parameter 'layer3.0.conv2.weight'"):
        spi.ModelReplica(Named(sd), -1, "fp16", image_size=64)
    with pytest.raises(spi.InferenceExecutionException, match="unrecognised model"):
        spi.ModelReplica(Named({"foo.weight": torch.zeros(2)}), -1, "fp16")


def _named(d):
    class Named(torch.nn.Module):
        def named_parameters(self, *a, **k):
            return iter([])

        def named_buffers(self, *a, **k):
            return iter(d.items())
    return Named()


def test_grouped_conv_resnext_is_rejected(spi, zoo):
    """ResNeXt (grouped 3x3, models/import_resnet.py variants) stores weight.shape[1] = C/groups;
    packing it as a dense conv would silently give garbage, so the channel chain is checked."""
    m = zoo.resnet([1, 1, 1, 1], True, image=64)
    sd = dict(m.state_dict())
    w = sd["layer1.0.conv2.weight"]  # [64, 64, 3, 3] -> groups=8: [64, 8, 3, 3]
    sd["layer1.0.conv2.weight"] = w[:, :8].clone()
    with pytest.raises(spi.InferenceExecutionException, match="grouped/unsupported conv"):
        spi.ModelReplica(_named(sd), -1, "fp16", image_size=64)
    # an identity residual whose channels do not line up is rejected too
    sd = dict(m.state_dict())
    sd = {k: v for k, v in sd.items() if not k.startswith("layer1.0.downsample")}
    with pytest.raises(spi.InferenceExecutionException, match="grouped/unsupported conv"):
        spi.ModelReplica(_named(sd), -1, "fp16", image_size=64)


def test_replicas_build_concurrently(spi, zoo):
    """spi_model_create is re-entrant: replicas packed from several threads at once
    (one per device, clone_model_to_gpus) equal the serially built one byte for byte."""
    import threading
    m = zoo.resnet([1, 1, 1, 1], False, image=64)
    ref = spi.ModelReplica(m, -1, "fp16x3", image_size=64)
    out = [None] * 4

    def build(i):
        out[i] = spi.ModelReplica(m, -1, "fp16x3", image_size=64)

    ts = [threading.Thread(target=build, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert all(r is not None and r.weight_digest == ref.weight_digest for r in out)
    other = spi.ModelReplica(m, -1, "fp16", image_size=64)
    assert other.weight_digest != ref.weight_digest


def test_torchscript_file_is_accepted(spi, zoo, tmp_path):
    """The reference's on-disk format: a traced TorchScript .pt (models/import_resnet.py)."""
    m = zoo.resnet18(image=64)
    path = str(tmp_path / "resnet18.pt")
    torch.jit.trace(m, torch.rand(1, 3, 64, 64)).save(path)
    r_file = spi.ModelReplica(path, -1, "fp16", image_size=64)
    r_mod = spi.ModelReplica(m, -1, "fp16", image_size=64)
    assert r_file.description == r_mod.description and r_file.weight_bytes == r_mod.weight_bytes


def test_no_fallback_when_library_missing(tmp_path):
    """Importing the package without the native library fails loudly."""
    import shutil
    import sys
    pkg = os.path.join(ROOT, "starpu-inference-server_amd")
    dst = tmp_path / "starpu-inference-server_amd"
    shutil.copytree(pkg, dst, ignore=shutil.ignore_patterns("*.so", "csrc", "__pycache__"))
    code = "import importlib, sys; sys.path.insert(0, %r); importlib.import_module('starpu-inference-server_amd')"
    r = subprocess.run([sys.executable, "-c", code % str(tmp_path)], capture_output=True, text=True)
    assert r.returncode != 0 and "libspi_hip.so is missing" in r.stderr


def test_runtime_rejects_invalid_config_without_touching_a_device(spi):
    import importlib
    rt = importlib.import_module("starpu-inference-server_amd.runtime")
    cfg = rt.RuntimeConfig()  # zero devices
    err = C.create_string_buffer(128)
    assert not spi.lib.spi_runtime_create(C.byref(cfg), err, 128)
    assert b"invalid runtime configuration" in err.value
    cfg.num_devices, cfg.max_batch, cfg.num_inputs, cfg.num_outputs = 1, 8, 1, 1
    cfg.input_types[0], cfg.input_ndims[0] = 6, 1
    cfg.input_dims[0][0] = 4
    cfg.output_types[0], cfg.output_elems[0] = 6, 4
    assert not spi.lib.spi_runtime_create(C.byref(cfg), err, 128)  # no replica for the device
    assert b"missing replica" in err.value
    assert spi.lib.spi_runtime_submit(None, 0, 1, None, None, rt.DONE_FN(), None) == spi._native.SPI_ERR_INVALID_ARGUMENT


def test_starpu_adapter_compiles_without_starpu(tmp_path):
    """csrc/spi_starpu_adapter.cpp builds in the default (no StarPU) configuration, and asking
    for the StarPU build without <starpu.h> fails at compile time with a clear message instead of
    guessing the interface layout."""
    import subprocess
    src = os.path.join(ROOT, "starpu-inference-server_amd", "csrc", "spi_starpu_adapter.cpp")
    ok = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", src], capture_output=True, text=True)
    assert ok.returncode == 0, ok.stderr
    bad = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-DSPI_WITH_STARPU", src], capture_output=True,
                         text=True)
    assert bad.returncode != 0 and "SPI_WITH_STARPU needs <starpu.h>" in bad.stderr
