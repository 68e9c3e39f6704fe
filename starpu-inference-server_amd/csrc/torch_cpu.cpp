// LibTorch side of the boundary (include/spi_torch.h): TorchScript loading,
// the CPU codelet's forward (the reference's LibTorch CPU path, the timed host
// baseline), the C++ weight extractor feeding spi_model_create, and a closed
// loop of CPU-codelet tasks for the baseline measurement.
//
// The views, stamps, layout checks and output byte-size checks stay in
// spi_cpu_inference_func (codelet.cpp); this file supplies what LibTorch does
// inside it: forward under c10::InferenceMode (starpu_setup.cpp:784-801,
// 594-624), append_ivalue flattening (:496-513) and
// TensorBuilder::copy_output_to_buffer (tensor_builder.cpp:162-190).
#include <time.h>
#include <torch/script.h>
#include <ATen/Parallel.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#include "../../include/spi_torch.h"

struct spi_torch_module {
  torch::jit::script::Module module;
  // Owned fp32 copies handed out by spi_torch_named_tensors.
  std::vector<std::string> names;
  std::vector<at::Tensor> tensors;
  std::vector<spi_named_tensor> views;
};

namespace {

void put_err(char* err, size_t errlen, const std::string& msg) {
  if (err && errlen) std::snprintf(err, errlen, "%s", msg.c_str());
}

int64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

at::ScalarType to_scalar(int32_t dt) {
  // spi_dtype codes are at::ScalarType codes (spi_codelet.h).
  switch (dt) {
    case SPI_DTYPE_U8: return at::kByte;
    case SPI_DTYPE_I8: return at::kChar;
    case SPI_DTYPE_I16: return at::kShort;
    case SPI_DTYPE_I32: return at::kInt;
    case SPI_DTYPE_I64: return at::kLong;
    case SPI_DTYPE_F16: return at::kHalf;
    case SPI_DTYPE_F32: return at::kFloat;
    case SPI_DTYPE_F64: return at::kDouble;
    case SPI_DTYPE_BOOL: return at::kBool;
    case SPI_DTYPE_BF16: return at::kBFloat16;
    default: throw std::runtime_error("[ERROR] Unsupported input dtype " + std::to_string(dt));
  }
}

// append_ivalue (starpu_setup.cpp:496-513): depth-first, insertion order.
void append_ivalue(const c10::IValue& v, std::vector<at::Tensor>& out) {
  if (v.isTensor()) {
    out.push_back(v.toTensor());
  } else if (v.isTensorList()) {
    for (const at::Tensor& t : v.toTensorList()) out.push_back(t);
  } else if (v.isTuple()) {
    for (const auto& e : v.toTupleRef().elements()) append_ivalue(e, out);
  } else if (v.isList()) {
    for (const auto& e : v.toList()) append_ivalue(e, out);
  } else if (v.isGenericDict()) {
    for (const auto& kv : v.toGenericDict()) append_ivalue(kv.value(), out);
  } else {
    throw std::runtime_error("Unsupported model output type");
  }
}

double percentile(std::vector<double> xs, double p) {
  if (xs.empty()) return NAN;
  std::sort(xs.begin(), xs.end());
  if (xs.size() == 1) return xs[0];
  const double pos = p / 100.0 * (double)(xs.size() - 1);
  const size_t lo = (size_t)std::floor(pos);
  const size_t hi = std::min(lo + 1, xs.size() - 1);
  return xs[lo] + (xs[hi] - xs[lo]) * (pos - (double)lo);
}

}  // namespace

extern "C" {

spi_torch_module* spi_torch_load(const char* path, char* err, size_t errlen) {
  try {
    if (!path) throw std::runtime_error("null path");
    auto* m = new spi_torch_module;
    try {
      m->module = torch::jit::load(path, torch::kCPU);
      m->module.eval();
    } catch (...) {
      delete m;
      throw;
    }
    return m;
  } catch (const std::exception& e) {
    put_err(err, errlen, std::string("failed to load TorchScript model: ") + e.what());
    return nullptr;
  }
}

void spi_torch_free(spi_torch_module* m) { delete m; }

void spi_torch_set_num_threads(int32_t n) {
  if (n > 0) at::set_num_threads(n);
}
int32_t spi_torch_get_num_threads(void) { return (int32_t)at::get_num_threads(); }

int spi_torch_cpu_forward(void* model_cpu, const spi_tensor_view* inputs, int ni, spi_tensor_view* outputs, int no,
                          char* err, size_t errlen) {
  try {
    auto* m = static_cast<spi_torch_module*>(model_cpu);
    if (!m) throw std::runtime_error("[ERROR] No CPU model available");
    const c10::InferenceMode no_autograd;
    std::vector<c10::IValue> args;
    args.reserve(ni);
    for (int i = 0; i < ni; ++i) {
      // assign_tensor_view: non-owning row-major view, dims from the layout
      std::vector<int64_t> dims(inputs[i].shape, inputs[i].shape + inputs[i].ndim);
      args.emplace_back(torch::from_blob(inputs[i].data, dims, torch::TensorOptions().dtype(to_scalar(inputs[i].dtype))));
    }
    const c10::IValue result = m->module.forward(args);
    std::vector<at::Tensor> outs;
    append_ivalue(result, outs);
    if ((int)outs.size() != no) throw std::runtime_error("Mismatch between model outputs and StarPU buffers");
    for (int i = 0; i < no; ++i) {
      const at::Tensor& t = outs[i];
      spi_tensor_view& buf = outputs[i];
      // copy_output_to_buffer (tensor_builder.cpp:162-190); the CPU codelet
      // passes the output's own numel / scalar type as the expectation, so the
      // byte count against the W buffer is the binding check.
      if (!buf.data) throw std::runtime_error("[ERROR] Output buffer pointer is null");
      if (!t.is_contiguous()) throw std::runtime_error("[ERROR] Output tensor must be contiguous");
      const size_t es = spi_dtype_size(buf.dtype);
      const size_t buf_bytes = (size_t)buf.shape[0] * es;
      if (buf_bytes != t.nbytes()) throw std::runtime_error("[ERROR] Output buffer size mismatch in bytes");
      std::memcpy(buf.data, t.data_ptr(), t.nbytes());
    }
    return 0;
  } catch (const std::exception& e) {
    // c10::Error carries a backtrace after the first line; keep the message.
    std::string msg = e.what();
    const size_t nl = msg.find('\n');
    if (nl != std::string::npos) msg.resize(nl);
    put_err(err, errlen, msg);
    return 1;
  }
}

int32_t spi_torch_named_tensors(spi_torch_module* m, const spi_named_tensor** out) {
  if (!m || !out) return -1;
  try {
    if (m->views.empty()) {
      std::unordered_set<std::string> seen;
      auto add = [&](const std::string& name, const at::Tensor& t) {
        if (!t.is_floating_point() || !seen.insert(name).second) return;
        m->names.push_back(name);
        m->tensors.push_back(t.detach().to(at::kFloat).contiguous());
      };
      for (const auto& p : m->module.named_parameters(/*recurse=*/true)) add(p.name, p.value);
      for (const auto& b : m->module.named_buffers(/*recurse=*/true)) add(b.name, b.value);
      m->views.resize(m->names.size());
      for (size_t i = 0; i < m->names.size(); ++i) {
        spi_named_tensor& v = m->views[i];
        std::memset(&v, 0, sizeof(v));
        v.name = m->names[i].c_str();
        v.data = m->tensors[i].data_ptr();
        v.dtype = SPI_DTYPE_F32;
        v.ndim = (int32_t)m->tensors[i].dim();
        if (v.ndim > SPI_MAX_DIMS) throw std::runtime_error("parameter " + m->names[i] + " has too many dims");
        for (int d = 0; d < v.ndim; ++d) v.shape[d] = m->tensors[i].size(d);
      }
    }
    *out = m->views.data();
    return (int32_t)m->views.size();
  } catch (const std::exception&) {
    return -1;
  }
}

spi_model* spi_torch_create_replica(spi_torch_module* m, int32_t device_id, const spi_model_config* cfg, char* err,
                                    size_t errlen) {
  const spi_named_tensor* ts = nullptr;
  const int32_t n = spi_torch_named_tensors(m, &ts);
  if (n < 0) {
    put_err(err, errlen, "weight extraction failed");
    return nullptr;
  }
  return spi_model_create(device_id, cfg, ts, n, err, errlen);
}

int spi_torch_cpu_bench(spi_torch_module* m, const spi_tensor_view* inputs, int32_t ni, const size_t* out_bytes,
                        const int32_t* out_types, int32_t no, int32_t workers, int32_t threads, double seconds,
                        int64_t max_tasks, spi_cpu_bench_result* res) {
  if (!m || !res || ni < 1 || ni > SPI_MAX_INPUTS || no < 1 || no > SPI_MAX_OUTPUTS || workers < 1) return SPI_ERR_INVALID_ARGUMENT;
  std::memset(res, 0, sizeof(*res));
  std::mutex mu;
  std::vector<double> lat_ms;
  int64_t first = INT64_MAX, last = 0, tasks = 0;
  int32_t failed = 0;
  std::string first_err;
  std::atomic<int64_t> issued{0};
  const int64_t deadline = now_ns() + (int64_t)(seconds * 1e9);
  const int64_t batch = inputs[0].ndim > 0 ? inputs[0].shape[0] : 1;
  auto worker = [&](int wid) {
    if (threads > 0) at::set_num_threads(threads);
    // Per-worker copies of the inputs and its own output buffers (its slot).
    std::vector<std::vector<char>> in_data(ni), out_data(no);
    std::vector<spi_vector_interface> ifaces(ni + no);
    std::vector<void*> bufs(ni + no);
    spi_codelet_args a;
    spi_args_init(&a);
    a.num_inputs = ni;
    a.num_outputs = no;
    a.batch_size = batch;
    a.model_cpu = m;
    a.cpu_forward = &spi_torch_cpu_forward;
    for (int i = 0; i < ni; ++i) {
      size_t n = spi_dtype_size(inputs[i].dtype);
      for (int d = 0; d < inputs[i].ndim; ++d) n *= (size_t)inputs[i].shape[d];
      in_data[i].assign(static_cast<const char*>(inputs[i].data), static_cast<const char*>(inputs[i].data) + n);
      const size_t es = spi_dtype_size(inputs[i].dtype);
      ifaces[i] = spi_vector_interface{SPI_STARPU_VECTOR_INTERFACE_ID, (uintptr_t)in_data[i].data(), 0, 0, n / es, es, 0, n};
      a.num_dims[i] = inputs[i].ndim;
      for (int d = 0; d < inputs[i].ndim; ++d) a.dims[i][d] = inputs[i].shape[d];
      a.input_types[i] = inputs[i].dtype;
    }
    for (int i = 0; i < no; ++i) {
      out_data[i].assign(out_bytes[i], 0);
      const size_t es = spi_dtype_size(out_types[i]);
      ifaces[ni + i] = spi_vector_interface{SPI_STARPU_VECTOR_INTERFACE_ID, (uintptr_t)out_data[i].data(), 0, 0,
                                            out_bytes[i] / es, es, 0, out_bytes[i]};
      a.output_types[i] = out_types[i];
    }
    for (int i = 0; i < ni + no; ++i) bufs[i] = &ifaces[i];
    spi_set_worker_context(wid, -1, nullptr);
    std::vector<double> mine;
    int64_t my_first = INT64_MAX, my_last = 0;
    int32_t my_failed = 0;
    std::string my_err;
    for (;;) {
      if (now_ns() >= deadline) break;
      if (max_tasks > 0 && issued.fetch_add(1) >= max_tasks) break;
      a.request_id = (int32_t)mine.size();
      const int64_t t0 = now_ns();
      spi_cpu_inference_func(bufs.data(), &a);
      const int64_t t1 = now_ns();
      if (a.status != SPI_OK) {
        ++my_failed;
        if (my_err.empty()) my_err = a.error;
        break;
      }
      my_first = std::min(my_first, t0);
      my_last = std::max(my_last, t1);
      mine.push_back((t1 - t0) * 1e-6);
    }
    spi_clear_worker_context();
    std::lock_guard<std::mutex> lk(mu);
    lat_ms.insert(lat_ms.end(), mine.begin(), mine.end());
    tasks += (int64_t)mine.size();
    first = std::min(first, my_first);
    last = std::max(last, my_last);
    failed += my_failed;
    if (first_err.empty()) first_err = my_err;
  };
  std::vector<std::thread> ts;
  for (int w = 0; w < workers; ++w) ts.emplace_back(worker, w);
  for (auto& t : ts) t.join();
  res->tasks = tasks;
  res->inferences = tasks * batch;
  res->seconds = tasks > 0 ? (last - first) * 1e-9 : 0.0;
  res->inferences_per_s = res->seconds > 0 ? res->inferences / res->seconds : 0.0;
  res->p50_ms = percentile(lat_ms, 50);
  res->p95_ms = percentile(lat_ms, 95);
  res->failed = failed;
  std::snprintf(res->error, SPI_ERROR_LEN, "%s", first_err.c_str());
  return failed ? SPI_ERR_CPU_FORWARD : SPI_OK;
}

}  // extern "C"
