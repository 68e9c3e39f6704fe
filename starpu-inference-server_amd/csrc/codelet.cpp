// C-ABI codelet entry points (include/spi_codelet.h).
//
// spi_hip_inference_func is the MI355X replacement for
// InferenceCodelet::cuda_inference_func (src/core/starpu_setup.cpp:807-846):
// worker/device/stream from the worker context, replica selection
// (select_gpu_module, :725-778), stamps and device bookkeeping
// (run_codelet_inference, :638-723), input views from params->layout
// (tensor_builder.cpp:68-124), the forward enqueued on the worker stream and
// the output written straight into the W buffer by the last kernel (no D2D
// copy_, which the reference needs at :834-844).  Nothing synchronises: the
// caller (StarPU with STARPU_HIP_ASYNC, or the mini-runtime) syncs the stream.
#include <hip/hip_runtime.h>
#include <time.h>

#include <cstdio>
#include <cstring>
#include <exception>
#include <stdexcept>
#include <string>

#include "../../include/spi_codelet.h"
#include "model.hpp"

#ifdef SPI_WITH_STARPU
#include <starpu.h>
#endif

namespace {

struct WorkerContext {
  bool set = false;
  int32_t worker = -1;
  int32_t device = -1;
  hipStream_t stream = nullptr;
};
thread_local WorkerContext tl_ctx;
thread_local std::string tl_last_error;

int64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

void set_error(spi_codelet_args* a, int status, const std::string& msg) {
  a->status = status;
  std::snprintf(a->error, SPI_ERROR_LEN, "%s", msg.c_str());
  tl_last_error = msg;
}

struct CodeletError : std::runtime_error {
  int status;
  CodeletError(int s, const std::string& m) : std::runtime_error(m), status(s) {}
};

void current_worker(int32_t* worker, int32_t* device, hipStream_t* stream) {
  if (tl_ctx.set) {
    *worker = tl_ctx.worker;
    *device = tl_ctx.device;
    *stream = tl_ctx.stream;
    return;
  }
#ifdef SPI_WITH_STARPU
  *worker = starpu_worker_get_id();
  *device = starpu_worker_get_devid(*worker);
  *stream = starpu_hip_get_local_stream();
#else
  *worker = -1;
  *device = -1;
  *stream = nullptr;
#endif
}

// validate_input_layout (tensor_builder.cpp:51-66) + refresh_input_cache checks.
void validate_layout(const spi_codelet_args* a, void** buffers) {
  if (a->num_inputs > a->max_inputs || a->num_inputs > SPI_MAX_INPUTS)
    throw CodeletError(SPI_ERR_INVALID_ARGUMENT, "[ERROR] Too many input tensors");
  if (a->num_outputs > SPI_MAX_OUTPUTS)
    throw CodeletError(SPI_ERR_INVALID_ARGUMENT, "[ERROR] Too many output tensors");
  if ((a->num_inputs + a->num_outputs) > 0 && buffers == nullptr)
    throw CodeletError(SPI_ERR_INVALID_ARGUMENT, "[ERROR] Too few input buffers");
  for (uint32_t i = 0; i < a->num_inputs; ++i) {
    if (buffers[i] == nullptr) throw CodeletError(SPI_ERR_INVALID_ARGUMENT, "[ERROR] StarPU buffer is null");
    if (a->num_dims[i] < 0)
      throw CodeletError(SPI_ERR_INVALID_ARGUMENT, "Invalid number of dimensions (must be non-negative)");
    if ((uint64_t)a->num_dims[i] > a->max_dims || a->num_dims[i] > SPI_MAX_DIMS)
      throw CodeletError(SPI_ERR_INVALID_ARGUMENT, "[ERROR] Tensor layout mismatch");
  }
  for (uint32_t i = 0; i < a->num_outputs; ++i)
    if (buffers[a->num_inputs + i] == nullptr)
      throw CodeletError(SPI_ERR_INVALID_ARGUMENT, "[ERROR] StarPU buffer is null");
}

size_t byte_size_or_throw(const void* iface) {
  size_t n = 0;
  const int st = spi_buffer_byte_size(iface, &n);
  if (st == SPI_ERR_INVALID_ARGUMENT) throw CodeletError(st, "[ERROR] StarPU buffer is null");
  if (st == SPI_ERR_UNSUPPORTED) {
    const int id = iface ? *static_cast<const int32_t*>(iface) : -1;
    throw CodeletError(st, "[ERROR] Unsupported StarPU buffer interface id " + std::to_string(id));
  }
  if (st != SPI_OK) throw CodeletError(st, "[ERROR] StarPU buffer size exceeds size_t capacity");
  return n;
}

uintptr_t buffer_ptr(const void* iface) { return static_cast<const spi_variable_interface*>(iface)->ptr; }

}  // namespace

extern "C" {

size_t spi_dtype_size(int32_t dtype) {
  switch (dtype) {
    case SPI_DTYPE_U8:
    case SPI_DTYPE_I8:
    case SPI_DTYPE_BOOL:
      return 1;
    case SPI_DTYPE_I16:
    case SPI_DTYPE_F16:
    case SPI_DTYPE_BF16:
      return 2;
    case SPI_DTYPE_I32:
    case SPI_DTYPE_F32:
      return 4;
    case SPI_DTYPE_I64:
    case SPI_DTYPE_F64:
      return 8;
    default:
      return 0;
  }
}

void spi_args_init(spi_codelet_args* a) {
  if (!a) return;
  std::memset(a, 0, sizeof(*a));
  a->abi_version = SPI_ABI_VERSION;
  a->batch_size = 1;
  a->max_inputs = SPI_MAX_INPUTS;
  a->max_dims = SPI_MAX_DIMS;
  a->worker_id = -1;
  a->device_id = -1;
  for (int i = 0; i < SPI_MAX_OUTPUTS; ++i) a->output_types[i] = SPI_DTYPE_F32;
}

// buffer_byte_size (starpu_setup.cpp:515-542)
int spi_buffer_byte_size(const void* iface, size_t* out) {
  if (!iface || !out) return SPI_ERR_INVALID_ARGUMENT;
  const int32_t id = *static_cast<const int32_t*>(iface);
  if (id == SPI_STARPU_VARIABLE_INTERFACE_ID) {
    *out = static_cast<const spi_variable_interface*>(iface)->elemsize;
    return SPI_OK;
  }
  if (id == SPI_STARPU_VECTOR_INTERFACE_ID) {
    const auto* v = static_cast<const spi_vector_interface*>(iface);
    if (v->elemsize != 0 && (size_t)v->nx > SIZE_MAX / v->elemsize) return SPI_ERR_OUTPUT_MISMATCH;
    *out = (size_t)v->nx * v->elemsize;
    return SPI_OK;
  }
  return SPI_ERR_UNSUPPORTED;
}

// select_gpu_module (starpu_setup.cpp:725-778)
int spi_select_replica(const spi_codelet_args* a, int32_t worker_id, int32_t device_id, int32_t* out) {
  if (!a || !out) return SPI_ERR_INVALID_ARGUMENT;
  auto fetch = [&](int idx) -> bool {
    return idx >= 0 && idx < a->num_replicas && idx < SPI_MAX_REPLICAS && a->models_gpu[idx] != nullptr;
  };
  if (a->num_worker_ids > 0) {
    if (worker_id >= 0)
      for (int i = 0; i < a->num_worker_ids && i < SPI_MAX_REPLICAS; ++i)
        if (a->worker_ids[i] == worker_id) {
          if (fetch(i)) {
            *out = i;
            return SPI_OK;
          }
          break;
        }
    return SPI_ERR_NO_REPLICA;
  }
  int idx = -1;
  if (device_id >= 0) {
    if (a->num_device_ids > 0) {
      for (int i = 0; i < a->num_device_ids && i < SPI_MAX_REPLICAS; ++i)
        if (a->device_ids[i] == device_id) {
          idx = i;
          break;
        }
    } else {
      idx = device_id;
    }
  }
  if (fetch(idx)) {
    *out = idx;
    return SPI_OK;
  }
  return SPI_ERR_NO_REPLICA;
}

void spi_set_worker_context(int32_t worker_id, int32_t device_id, void* hip_stream) {
  tl_ctx.set = true;
  tl_ctx.worker = worker_id;
  tl_ctx.device = device_id;
  tl_ctx.stream = static_cast<hipStream_t>(hip_stream);
}

void spi_clear_worker_context(void) { tl_ctx = WorkerContext{}; }

const char* spi_last_error(void) { return tl_last_error.c_str(); }
void spi_set_last_error(const char* msg) { tl_last_error = msg ? msg : ""; }

void spi_hip_inference_func(void** buffers, void* cl_arg) {
  auto* a = static_cast<spi_codelet_args*>(cl_arg);
  if (a == nullptr) return;
  a->codelet_start_ns = now_ns();
  a->status = SPI_OK;
  a->error[0] = '\0';
  try {
    if (a->abi_version != SPI_ABI_VERSION)
      throw CodeletError(SPI_ERR_INVALID_ARGUMENT, "[ERROR] spi_codelet_args ABI version mismatch");
    int32_t worker = -1, device = -1;
    hipStream_t stream = nullptr;
    current_worker(&worker, &device, &stream);
    int32_t idx = -1;
    if (spi_select_replica(a, worker, device, &idx) != SPI_OK) {
      if (a->num_worker_ids > 0)
        throw CodeletError(SPI_ERR_NO_REPLICA, "[ERROR] No GPU model replica available for worker " +
                                                   std::to_string(worker) + " on device " + std::to_string(device));
      throw CodeletError(SPI_ERR_NO_REPLICA,
                         "[ERROR] No GPU model replica available for device " + std::to_string(device));
    }
    spi::Model* m = a->models_gpu[idx]->impl.get();
    validate_layout(a, buffers);
    const uint32_t ni = a->num_inputs, no = a->num_outputs;
    const void* in[SPI_MAX_INPUTS] = {};
    void* out[SPI_MAX_OUTPUTS] = {};
    size_t in_bytes[SPI_MAX_INPUTS] = {}, out_bytes[SPI_MAX_OUTPUTS] = {};
    for (uint32_t i = 0; i < ni; ++i) {
      in_bytes[i] = byte_size_or_throw(buffers[i]);
      in[i] = reinterpret_cast<const void*>(buffer_ptr(buffers[i]));
    }
    for (uint32_t i = 0; i < no; ++i) {
      out_bytes[i] = byte_size_or_throw(buffers[ni + i]);
      out[i] = reinterpret_cast<void*>(buffer_ptr(buffers[ni + i]));
      if (!out[i]) throw CodeletError(SPI_ERR_INVALID_ARGUMENT, "[ERROR] Output buffer pointer is null");
    }
    try {
      m->check_io(*a, in_bytes, out_bytes);
    } catch (const std::exception& e) {
      const std::string msg = e.what();
      throw CodeletError(msg.find("Output buffer size") != std::string::npos ? SPI_ERR_OUTPUT_MISMATCH
                                                                              : SPI_ERR_INVALID_ARGUMENT,
                         msg);
    }
    a->executed_on = SPI_DEVICE_GPU;
    a->worker_id = worker;
    a->device_id = device;
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != m->device()) (void)hipSetDevice(m->device());
    a->inference_start_ns = now_ns();
    size_t n_aff = 0;
    if (m->family() == SPI_FAMILY_AFFINE) {
      int64_t e = 1;
      for (int d = 0; d < a->num_dims[0]; ++d) e *= a->dims[0][d];
      n_aff = (size_t)e;
    }
    const int S = a->num_dims[0] >= 2 ? (int)a->dims[0][1] : 0;
    m->forward(stream, (int)a->dims[0][0], S, n_aff, in, out);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) throw CodeletError(SPI_ERR_DEVICE, std::string("HIP error: ") + hipGetErrorString(err));
  } catch (const CodeletError& e) {
    set_error(a, e.status, std::string("[ERROR] Codelet failure: ") + e.what());
  } catch (const std::exception& e) {
    set_error(a, SPI_ERR_DEVICE, std::string("[ERROR] Codelet failure: ") + e.what());
  } catch (...) {
    set_error(a, SPI_ERR_DEVICE, "[ERROR] Codelet failure: unknown error");
  }
  a->codelet_end_ns = now_ns();
}

// cpu_inference_func (starpu_setup.cpp:784-801) with copy_output_to_buffer's
// checks (tensor_builder.cpp:162-190); the forward itself is the host's CPU
// model (LibTorch in the reference), bound through args->cpu_forward.
void spi_cpu_inference_func(void** buffers, void* cl_arg) {
  auto* a = static_cast<spi_codelet_args*>(cl_arg);
  if (a == nullptr) return;
  a->codelet_start_ns = now_ns();
  a->status = SPI_OK;
  a->error[0] = '\0';
  try {
    if (!a->cpu_forward || !a->model_cpu)
      throw CodeletError(SPI_ERR_NO_REPLICA, "[ERROR] No CPU model available");
    validate_layout(a, buffers);
    int32_t worker = -1, device = -1;
    hipStream_t stream = nullptr;
    current_worker(&worker, &device, &stream);
    a->executed_on = SPI_DEVICE_CPU;
    a->worker_id = worker;
    a->device_id = device;
    spi_tensor_view in[SPI_MAX_INPUTS] = {}, out[SPI_MAX_OUTPUTS] = {};
    for (uint32_t i = 0; i < a->num_inputs; ++i) {
      in[i].data = reinterpret_cast<void*>(buffer_ptr(buffers[i]));
      in[i].dtype = a->input_types[i];
      in[i].ndim = (int32_t)a->num_dims[i];
      for (int d = 0; d < in[i].ndim; ++d) in[i].shape[d] = a->dims[i][d];
    }
    size_t out_bytes[SPI_MAX_OUTPUTS] = {};
    for (uint32_t i = 0; i < a->num_outputs; ++i) {
      out_bytes[i] = byte_size_or_throw(buffers[a->num_inputs + i]);
      out[i].data = reinterpret_cast<void*>(buffer_ptr(buffers[a->num_inputs + i]));
      if (!out[i].data) throw CodeletError(SPI_ERR_INVALID_ARGUMENT, "[ERROR] Output buffer pointer is null");
      out[i].dtype = a->output_types[i];
      out[i].ndim = 1;
      const size_t es = spi_dtype_size(out[i].dtype);
      out[i].shape[0] = es ? (int64_t)(out_bytes[i] / es) : 0;
      if (es == 0 || out_bytes[i] % es != 0)
        throw CodeletError(SPI_ERR_OUTPUT_MISMATCH, "Output buffer size mismatch in bytes");
    }
    a->inference_start_ns = now_ns();
    char err[SPI_ERROR_LEN] = {};
    const int rc = a->cpu_forward(a->model_cpu, in, (int)a->num_inputs, out, (int)a->num_outputs, err, sizeof(err));
    if (rc != 0) {
      const std::string msg(err);
      throw CodeletError(msg.find("mismatch") != std::string::npos ? SPI_ERR_OUTPUT_MISMATCH : SPI_ERR_CPU_FORWARD,
                         msg.empty() ? "cpu forward failed" : msg);
    }
  } catch (const CodeletError& e) {
    set_error(a, e.status, std::string("[ERROR] Codelet failure: ") + e.what());
  } catch (const std::exception& e) {
    set_error(a, SPI_ERR_CPU_FORWARD, std::string("[ERROR] Codelet failure: ") + e.what());
  }
  a->codelet_end_ns = now_ns();
}

// spi_codelet_init: spi_starpu_adapter.cpp (the StarPU descriptor + layout static_asserts).

// ---------------------------------------------------------------------------
// Model replicas
// ---------------------------------------------------------------------------
spi_model* spi_model_create(int32_t device_id, const spi_model_config* config, const spi_named_tensor* params,
                            int32_t num_params, char* err, size_t errlen) {
  try {
    if (!config) throw std::runtime_error("null config");
    auto* m = new spi_model;
    try {
      m->impl = std::make_unique<spi::Model>(device_id, *config, params, num_params);
    } catch (...) {
      delete m;
      throw;
    }
    return m;
  } catch (const std::exception& e) {
    tl_last_error = e.what();
    if (err && errlen) std::snprintf(err, errlen, "%s", e.what());
    return nullptr;
  }
}

void spi_model_destroy(spi_model* m) { delete m; }
size_t spi_model_weight_bytes(const spi_model* m) { return m ? m->impl->weight_bytes() : 0; }
uint64_t spi_model_weight_digest(const spi_model* m) { return m ? m->impl->weight_digest() : 0; }
double spi_model_flops(const spi_model* m, int64_t b) { return m ? m->impl->flops(b) : 0.0; }
const char* spi_model_describe(const spi_model* m) { return m ? m->impl->describe().c_str() : ""; }
int spi_model_profile(spi_model* m, void* stream, int64_t batch, int64_t seq, const void* const* inputs,
                      void* const* outputs, float* op_ms, double* op_flops, double* op_bytes, char* op_names,
                      int32_t name_len, int32_t max_ops) {
  if (!m) return -1;
  try {
    return m->impl->profile(static_cast<hipStream_t>(stream), (int)batch, (int)seq, inputs, outputs, op_ms, op_flops,
                            op_bytes, op_names, name_len, max_ops);
  } catch (const std::exception& e) {
    tl_last_error = e.what();
    return -1;
  }
}

int spi_model_profile_op(spi_model* m, void* stream, int64_t batch, int64_t seq, const void* const* inputs,
                         void* const* outputs, const char* op_name, int32_t reps, float* ms, double* flops,
                         double* bytes) {
  if (!m) return -1;
  try {
    return m->impl->profile_op(static_cast<hipStream_t>(stream), (int)batch, (int)seq, inputs, outputs, op_name,
                               (int)reps, ms, flops, bytes);
  } catch (const std::exception& e) {
    tl_last_error = e.what();
    return -1;
  }
}

int64_t spi_model_launch_table(spi_model* m, void* stream, int64_t batch, int64_t seq, const void* const* inputs,
                               void* const* outputs, char* buf, size_t buflen) {
  if (!m) return -1;
  try {
    const std::string t =
        m->impl->launch_table(static_cast<hipStream_t>(stream), (int)batch, (int)seq, inputs, outputs);
    if (buf && buflen > 0) std::snprintf(buf, buflen, "%s", t.c_str());
    return (int64_t)t.size();
  } catch (const std::exception& e) {
    tl_last_error = e.what();
    return -1;
  }
}

void spi_model_set_graphs(spi_model* m, int32_t on) {
  if (m) m->impl->set_graphs(on != 0);
}

int spi_model_warmup(spi_model* m, void* stream, int64_t batch, int64_t seq, int32_t with_mask) {
  if (!m) return SPI_ERR_INVALID_ARGUMENT;
  try {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != m->impl->device()) (void)hipSetDevice(m->impl->device());
    m->impl->warmup(static_cast<hipStream_t>(stream), (int)batch, (int)seq, with_mask != 0);
    return SPI_OK;
  } catch (const std::exception& e) {
    tl_last_error = e.what();
    return SPI_ERR_DEVICE;
  }
}

// ---------------------------------------------------------------------------
// Device utilities
// ---------------------------------------------------------------------------
static int ret(hipError_t e) {
  if (e != hipSuccess) {
    tl_last_error = hipGetErrorString(e);
    return SPI_ERR_DEVICE;
  }
  return SPI_OK;
}

int spi_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
int spi_set_device(int32_t d) { return ret(hipSetDevice(d)); }
void* spi_device_malloc(size_t bytes) {
  void* p = nullptr;
  if (ret(hipMalloc(&p, bytes ? bytes : 1)) != SPI_OK) return nullptr;
  return p;
}
void spi_device_free(void* p) {
  if (p) (void)hipFree(p);
}
void* spi_host_malloc(size_t bytes) {
  void* p = nullptr;
  if (ret(hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocPortable)) != SPI_OK) return nullptr;
  return p;
}
void spi_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}
int spi_memcpy_h2d(void* dst, const void* src, size_t n, void* s) {
  return ret(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, static_cast<hipStream_t>(s)));
}
int spi_memcpy_d2h(void* dst, const void* src, size_t n, void* s) {
  return ret(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, static_cast<hipStream_t>(s)));
}
int spi_memset_d(void* dst, int v, size_t n, void* s) {
  return ret(hipMemsetAsync(dst, v, n, static_cast<hipStream_t>(s)));
}
void* spi_stream_create(void) {
  hipStream_t s = nullptr;
  if (ret(hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) != SPI_OK) return nullptr;
  return s;
}
void spi_stream_destroy(void* s) {
  if (s) (void)hipStreamDestroy(static_cast<hipStream_t>(s));
}
int spi_stream_synchronize(void* s) { return ret(hipStreamSynchronize(static_cast<hipStream_t>(s))); }

}  // extern "C"
