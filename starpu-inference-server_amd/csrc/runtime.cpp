// Mini-runtime: eager queue + per-device HIP workers + pinned slot staging
// around spi_hip_inference_func (include/spi_runtime.h).
#include <hip/hip_runtime.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/spi_runtime.h"

extern "C" void spi_set_last_error(const char* msg);

namespace {

int64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

struct Job {
  int32_t request_id;
  int64_t batch;
  std::vector<const void*> in;
  std::vector<void*> out;
  spi_job_done_fn done;
  void* user;
  int64_t submit_ns;
};

// One worker = one HIP stream + one pinned input/output slot + device buffers
// (slot count per device = workers: the reference's default pool size
// max(2, workers), slot_pool_buffer_utils.hpp:192-196, with one slot in use per
// in-flight task).
struct Worker {
  int32_t worker_id = 0;
  int32_t device = 0;
  spi_model* model = nullptr;
  hipStream_t stream = nullptr;
  std::vector<void*> h_in, h_out, d_in, d_out;  // pinned host slots / HBM buffers
  std::thread thread;
};

}  // namespace

struct spi_runtime {
  spi_runtime_config cfg{};
  std::vector<size_t> in_sample_bytes, out_sample_bytes;
  std::vector<std::unique_ptr<Worker>> workers;
  std::mutex mu;
  std::condition_variable cv_job, cv_idle;
  std::deque<Job> queue;
  int64_t inflight = 0;
  bool stop = false;
  std::atomic<int64_t> completed{0}, failed{0};

  void run(Worker* w);
  void free_worker(Worker* w);
};

void spi_runtime::free_worker(Worker* w) {
  (void)hipSetDevice(w->device);
  for (void* p : w->h_in) (void)hipHostFree(p);
  for (void* p : w->h_out) (void)hipHostFree(p);
  for (void* p : w->d_in) (void)hipFree(p);
  for (void* p : w->d_out) (void)hipFree(p);
  if (w->stream) (void)hipStreamDestroy(w->stream);
}

void spi_runtime::run(Worker* w) {
  (void)hipSetDevice(w->device);
  spi_set_worker_context(w->worker_id, w->device, w->stream);
  const int ni = cfg.num_inputs, no = cfg.num_outputs;
  const int max_jobs = std::max(1, cfg.coalesce_max_jobs);
  for (;;) {
    // ---- batch composition: the queue head, then queued jobs while their samples
    // fit max_batch (TensorBatchCompositionPolicy; the per-sample shapes are fixed
    // by the runtime config, so every pair of jobs is mergeable)
    std::vector<Job> jobs;
    int64_t total = 0;
    {
      std::unique_lock<std::mutex> lk(mu);
      cv_job.wait(lk, [&] { return stop || !queue.empty(); });
      if (stop && queue.empty()) break;
      auto take_fitting = [&] {
        while (!queue.empty() && (int)jobs.size() < max_jobs && total + queue.front().batch <= cfg.max_batch) {
          total += queue.front().batch;
          jobs.push_back(std::move(queue.front()));
          queue.pop_front();
        }
      };
      take_fitting();
      if (max_jobs > 1 && cfg.coalesce_delay_us > 0) {
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(cfg.coalesce_delay_us);
        while (!stop && (int)jobs.size() < max_jobs && total < cfg.max_batch && queue.empty()) {
          if (cv_job.wait_until(lk, deadline) == std::cv_status::timeout) break;
          take_fitting();
        }
        take_fitting();
      }
      if (!queue.empty()) cv_job.notify_one();  // leftovers belong to another worker
    }
    const int64_t dequeue_ns = now_ns();
    int status = SPI_OK;
    std::string err;
    // copy_job_inputs_to_slot: each job's samples at its offset in the pinned slot,
    // then one H2D per input on the worker stream
    std::vector<int64_t> offs;
    int64_t off = 0;
    for (const Job& j : jobs) {
      offs.push_back(off);
      for (int i = 0; i < ni; ++i)
        std::memcpy(static_cast<char*>(w->h_in[i]) + off * in_sample_bytes[i], j.in[i],
                    (size_t)j.batch * in_sample_bytes[i]);
      off += j.batch;
    }
    for (int i = 0; i < ni; ++i)
      if (hipMemcpyAsync(w->d_in[i], w->h_in[i], (size_t)total * in_sample_bytes[i], hipMemcpyHostToDevice,
                         w->stream) != hipSuccess) {
        status = SPI_ERR_DEVICE;
        err = "H2D copy failed";
      }
    spi_codelet_args args;
    spi_args_init(&args);
    args.num_inputs = ni;
    args.num_outputs = no;
    args.request_id = jobs.front().request_id;
    args.batch_size = total;
    for (int i = 0; i < ni; ++i) {
      args.num_dims[i] = cfg.input_ndims[i] + 1;
      args.dims[i][0] = total;
      for (int d = 0; d < cfg.input_ndims[i]; ++d) args.dims[i][d + 1] = cfg.input_dims[i][d];
      args.input_types[i] = cfg.input_types[i];
    }
    for (int i = 0; i < no; ++i) args.output_types[i] = cfg.output_types[i];
    args.num_replicas = 1;
    args.models_gpu[0] = w->model;
    args.num_device_ids = 1;
    args.device_ids[0] = w->device;
    // vector interfaces resized to this task's payload (resize_starpu_vector_interface)
    std::vector<spi_vector_interface> ifaces(ni + no);
    std::vector<void*> buffers(ni + no);
    for (int i = 0; i < ni; ++i) {
      const size_t es = spi_dtype_size(cfg.input_types[i]);
      ifaces[i] = spi_vector_interface{SPI_STARPU_VECTOR_INTERFACE_ID, (uintptr_t)w->d_in[i], 0, 0,
                                       (size_t)(total * in_sample_bytes[i] / es), es, 0,
                                       (size_t)cfg.max_batch * in_sample_bytes[i]};
      buffers[i] = &ifaces[i];
    }
    for (int i = 0; i < no; ++i) {
      const size_t es = spi_dtype_size(cfg.output_types[i]);
      ifaces[ni + i] = spi_vector_interface{SPI_STARPU_VECTOR_INTERFACE_ID, (uintptr_t)w->d_out[i], 0, 0,
                                            (size_t)(total * out_sample_bytes[i] / es), es, 0,
                                            (size_t)cfg.max_batch * out_sample_bytes[i]};
      buffers[ni + i] = &ifaces[ni + i];
    }
    int64_t cs = 0, ce = 0;
    if (status == SPI_OK) {
      spi_hip_inference_func(buffers.data(), &args);
      cs = args.codelet_start_ns;
      ce = args.codelet_end_ns;
      if (args.status != SPI_OK) {
        status = args.status;
        err = args.error;
      }
    }
    if (status == SPI_OK) {
      for (int i = 0; i < no; ++i)
        if (hipMemcpyAsync(w->h_out[i], w->d_out[i], (size_t)total * out_sample_bytes[i], hipMemcpyDeviceToHost,
                           w->stream) != hipSuccess) {
          status = SPI_ERR_DEVICE;
          err = "D2H copy failed";
        }
    }
    if (hipStreamSynchronize(w->stream) != hipSuccess && status == SPI_OK) {
      status = SPI_ERR_DEVICE;
      err = "stream synchronisation failed";
    }
    // output split: job k gets rows [offs[k], offs[k] + batch) of every output
    // (slice_outputs_for_sub_job), then its own completion callback
    for (size_t k = 0; k < jobs.size(); ++k) {
      const Job& j = jobs[k];
      if (status == SPI_OK)
        for (int i = 0; i < no; ++i)
          std::memcpy(j.out[i], static_cast<const char*>(w->h_out[i]) + offs[k] * out_sample_bytes[i],
                      (size_t)j.batch * out_sample_bytes[i]);
      spi_job_timing t{};
      t.submit_ns = j.submit_ns;
      t.dequeue_ns = dequeue_ns;
      t.codelet_start_ns = cs;
      t.codelet_end_ns = ce;
      t.device_id = w->device;
      t.worker_id = w->worker_id;
      t.task_batch = (int32_t)total;
      t.task_jobs = (int32_t)jobs.size();
      t.complete_ns = now_ns();
      (status == SPI_OK ? completed : failed).fetch_add(1);
      if (j.done) j.done(j.user, j.request_id, status, status == SPI_OK ? "" : err.c_str(), &t);
    }
    {
      std::lock_guard<std::mutex> lk(mu);
      inflight -= (int64_t)jobs.size();
      if (inflight == 0) cv_idle.notify_all();
    }
  }
  spi_clear_worker_context();
}

extern "C" {

spi_runtime* spi_runtime_create(const spi_runtime_config* c, char* err, size_t errlen) {
  auto fail = [&](const std::string& m) -> spi_runtime* {
    spi_set_last_error(m.c_str());
    if (err && errlen) std::snprintf(err, errlen, "%s", m.c_str());
    return nullptr;
  };
  if (!c || c->num_devices < 1 || c->num_devices > SPI_MAX_REPLICAS || c->max_batch < 1 || c->num_inputs < 1 ||
      c->num_inputs > SPI_MAX_INPUTS || c->num_outputs < 1 || c->num_outputs > SPI_MAX_OUTPUTS)
    return fail("invalid runtime configuration");
  auto rt = std::make_unique<spi_runtime>();
  rt->cfg = *c;
  if (rt->cfg.workers_per_device <= 0) rt->cfg.workers_per_device = 4;
  {
    // HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (default 4)
    // round-robin; worker streams sharing a queue run serially.
    const char* q = std::getenv("GPU_MAX_HW_QUEUES");
    const int queues = q ? std::atoi(q) : 4;
    if (queues < rt->cfg.workers_per_device + 1)
      std::fprintf(stderr,
                   "spi_runtime: GPU_MAX_HW_QUEUES=%d < workers_per_device+1=%d; worker streams will share "
                   "hardware queues and serialize (set it before the first HIP call)\n",
                   queues, rt->cfg.workers_per_device + 1);
  }
  for (int i = 0; i < c->num_inputs; ++i) {
    size_t n = spi_dtype_size(c->input_types[i]);
    if (!n || c->input_ndims[i] < 0 || c->input_ndims[i] >= SPI_MAX_DIMS) return fail("invalid input spec");
    for (int d = 0; d < c->input_ndims[i]; ++d) n *= (size_t)c->input_dims[i][d];
    rt->in_sample_bytes.push_back(n);
  }
  for (int i = 0; i < c->num_outputs; ++i) {
    const size_t es = spi_dtype_size(c->output_types[i]);
    if (!es || c->output_elems[i] <= 0) return fail("invalid output spec");
    rt->out_sample_bytes.push_back(es * (size_t)c->output_elems[i]);
  }
  int32_t wid = 0;
  for (int dv = 0; dv < c->num_devices; ++dv) {
    if (!c->models[dv]) return fail("missing replica for device " + std::to_string(c->device_ids[dv]));
    for (int k = 0; k < rt->cfg.workers_per_device; ++k) {
      auto w = std::make_unique<Worker>();
      w->worker_id = wid++;
      w->device = c->device_ids[dv];
      w->model = c->models[dv];
      bool ok = hipSetDevice(w->device) == hipSuccess &&
                hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking) == hipSuccess;
      for (size_t b : rt->in_sample_bytes) {
        void *h = nullptr, *d = nullptr;
        ok = ok && hipHostMalloc(&h, b * c->max_batch, hipHostMallocPortable) == hipSuccess;
        w->h_in.push_back(h);
        ok = ok && hipMalloc(&d, b * c->max_batch) == hipSuccess;
        w->d_in.push_back(d);
      }
      for (size_t b : rt->out_sample_bytes) {
        void *h = nullptr, *d = nullptr;
        ok = ok && hipHostMalloc(&h, b * c->max_batch, hipHostMallocPortable) == hipSuccess;
        w->h_out.push_back(h);
        ok = ok && hipMalloc(&d, b * c->max_batch) == hipSuccess;
        w->d_out.push_back(d);
      }
      if (!ok) {
        rt->free_worker(w.get());
        for (auto& x : rt->workers) rt->free_worker(x.get());
        return fail("device allocation failed for worker " + std::to_string(w->worker_id));
      }
      rt->workers.push_back(std::move(w));
    }
  }
  for (auto& w : rt->workers) w->thread = std::thread(&spi_runtime::run, rt.get(), w.get());
  return rt.release();
}

int spi_runtime_submit(spi_runtime* rt, int32_t request_id, int64_t batch, const void* const* inputs,
                       void* const* outputs, spi_job_done_fn done, void* user) {
  if (!rt || !inputs || !outputs || batch < 1 || batch > rt->cfg.max_batch) return SPI_ERR_INVALID_ARGUMENT;
  Job j;
  j.request_id = request_id;
  j.batch = batch;
  j.in.assign(inputs, inputs + rt->cfg.num_inputs);
  j.out.assign(outputs, outputs + rt->cfg.num_outputs);
  j.done = done;
  j.user = user;
  j.submit_ns = now_ns();
  {
    std::lock_guard<std::mutex> lk(rt->mu);
    if (rt->stop) return SPI_ERR_INVALID_ARGUMENT;
    if (rt->cfg.max_queue > 0 && (int64_t)rt->queue.size() >= rt->cfg.max_queue) return SPI_ERR_QUEUE_FULL;
    rt->queue.push_back(std::move(j));
    ++rt->inflight;
  }
  rt->cv_job.notify_one();
  return SPI_OK;
}

int spi_runtime_drain(spi_runtime* rt) {
  if (!rt) return SPI_ERR_INVALID_ARGUMENT;
  std::unique_lock<std::mutex> lk(rt->mu);
  rt->cv_idle.wait(lk, [&] { return rt->inflight == 0; });
  return SPI_OK;
}

void spi_runtime_stats(const spi_runtime* rt, int64_t* completed, int64_t* failed) {
  if (completed) *completed = rt ? rt->completed.load() : 0;
  if (failed) *failed = rt ? rt->failed.load() : 0;
}

void spi_runtime_destroy(spi_runtime* rt) {
  if (!rt) return;
  spi_runtime_drain(rt);
  {
    std::lock_guard<std::mutex> lk(rt->mu);
    rt->stop = true;
  }
  rt->cv_job.notify_all();
  for (auto& w : rt->workers)
    if (w->thread.joinable()) w->thread.join();
  for (auto& w : rt->workers) rt->free_worker(w.get());
  delete rt;
}

}  // extern "C"
