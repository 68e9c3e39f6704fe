// Mini-runtime around spi_hip_inference_func (include/spi_runtime.h): eager
// priority queue, per-device workers with a pipeline of tasks in flight,
// per-device pinned slot pools, parallel host staging, H2D on a copy stream
// joined by events, batching strategies, and the client load generator.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
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

// ---------------------------------------------------------------------------
// AdaptiveBatchingStrategy (batching_strategy.cpp:195-360), runtime-pressure
// path (no congestion monitor): queue fill + internal backlog pressure.
// ---------------------------------------------------------------------------
constexpr double kInternalHigh = 0.75, kInternalLow = 0.25, kInternalSevere = 0.95;
constexpr double kPreparedHigh = 1.0, kPreparedSevere = 2.0;

struct Pressure {
  bool congested = false, high = false, low = false, severe = false;
};

Pressure resolve_pressure(const spi_batching_config& c, const spi_batching_pressure& p) {
  Pressure r;
  if (!c.congestion_enabled) return r;
  const double fill_high = std::clamp(c.fill_high, 0.0, 1.0);
  const double fill_low = std::clamp(std::min(c.fill_low, c.fill_high), 0.0, fill_high);
  // sample_internal_pressure
  bool ih = false, il = false, is = false;
  const int64_t backlog = p.prepared_depth + p.inflight_tasks;
  if (p.max_inflight_tasks > 0) {
    const double inflight = (double)p.inflight_tasks / (double)p.max_inflight_tasks;
    const double back = (double)backlog / (double)p.max_inflight_tasks;
    ih = inflight >= kInternalHigh || back >= kInternalHigh;
    il = inflight <= kInternalLow && back <= kInternalLow;
    is = inflight >= kInternalSevere || back >= kInternalSevere;
  } else {
    const double ref = std::max(1, c.batch_limit);
    const double prepared = (double)p.prepared_depth / ref;
    ih = prepared >= kPreparedHigh;
    il = p.prepared_depth == 0;
    is = prepared >= kPreparedSevere;
  }
  // resolve_runtime_pressure
  const double fill = p.queue_capacity > 0 ? (double)p.queue_size / (double)p.queue_capacity : 0.0;
  r.congested = p.congested != 0;
  r.high = fill >= fill_high || ih;
  r.low = !r.congested && fill <= fill_low && il;
  r.severe = r.congested || is;
  return r;
}

int low_streak_threshold(const spi_batching_config& c) {
  if (!c.congestion_enabled) return 1;
  const int tick = std::max(1, c.tick_interval_us);
  return std::max(1, std::max(tick, c.exit_horizon_us) / tick);
}

int high_step(const spi_batching_config& c, int limit, bool severe) {
  if (limit <= 1 || !c.congestion_enabled) return 1;
  const int tick = std::max(1, c.tick_interval_us);
  const int entry_ticks = std::max(1, std::max(tick, c.entry_horizon_us) / tick);
  const int base = std::max(1, limit / entry_ticks);
  if (!severe) return base;
  return std::max(base, std::max(1, limit / std::max(1, low_streak_threshold(c))));
}

int coalesce_timeout(const spi_batching_config& c, bool congested, int target) {
  const int configured = std::max(0, c.coalesce_timeout_us);
  if (!c.congestion_enabled || !congested) return configured;
  const int tick = std::max(1, c.tick_interval_us);
  return std::max(configured, std::max(1, tick / std::max(1, target)));
}

// ---------------------------------------------------------------------------
// Host staging: a pool of copy threads shared by the workers.  A worker splits
// its copies into chunks, queues them, works on the queue itself and waits for
// its own chunks (parallel_for_each_index, slot_manager_component.cpp:56-95).
// ---------------------------------------------------------------------------
class CopyPool {
 public:
  struct Batch {
    std::atomic<int> remaining{0};
  };
  struct Chunk {
    char* dst;
    const char* src;
    size_t bytes;
    Batch* batch;
  };

  explicit CopyPool(int helpers) {
    for (int i = 0; i < helpers; ++i) threads_.emplace_back([this] { loop(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }

  // Copies every (dst, src, bytes) and returns when all are done.
  void copy(const std::vector<Chunk>& ops) {
    constexpr size_t kChunk = 1 << 20;
    std::vector<Chunk> chunks;
    Batch batch;
    for (const Chunk& op : ops)
      for (size_t off = 0; off < op.bytes; off += kChunk)
        chunks.push_back(Chunk{op.dst + off, op.src + off, std::min(kChunk, op.bytes - off), &batch});
    if (chunks.empty()) return;
    if (threads_.empty() || chunks.size() == 1) {
      for (const Chunk& c : chunks) std::memcpy(c.dst, c.src, c.bytes);
      return;
    }
    batch.remaining.store((int)chunks.size());
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (const Chunk& c : chunks) q_.push_back(c);
    }
    cv_.notify_all();
    // help: drain the queue (any worker's chunks) until ours are all done
    while (batch.remaining.load(std::memory_order_acquire) > 0) {
      Chunk c{};
      bool got = false;
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (!q_.empty()) {
          c = q_.front();
          q_.pop_front();
          got = true;
        }
      }
      if (got) {
        run(c);
      } else {
        std::this_thread::yield();
      }
    }
  }

 private:
  static void run(const Chunk& c) {
    std::memcpy(c.dst, c.src, c.bytes);
    c.batch->remaining.fetch_sub(1, std::memory_order_acq_rel);
  }
  void loop() {
    for (;;) {
      Chunk c{};
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        c = q_.front();
        q_.pop_front();
      }
      run(c);
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Chunk> q_;
  bool stop_ = false;
  std::vector<std::thread> threads_;
};

struct Job {
  int32_t request_id;
  int32_t fixed_worker;
  int32_t priority;
  int64_t batch;
  std::vector<const void*> in;
  std::vector<void*> out;
  spi_job_done_fn done;
  void* user;
  int64_t submit_ns;
  int64_t dequeue_ns = 0;
};

// One slot: pinned host staging for inputs/outputs and their HBM buffers.
struct Slot {
  std::vector<void*> h_in, h_out, d_in, d_out;
  hipEvent_t h2d = nullptr, done = nullptr;
  // SPI_H2D_WORKER_SDMA: completion signal of this slot's SDMA copies (value = copies in flight)
  hsa_signal_t sig{};
};

// SlotPoolBase::acquire / try_acquire / release (slot_pool_base.hpp:32-75).
struct SlotPool {
  int device = 0;
  std::vector<Slot> slots;
  std::vector<int> free_list;
  std::mutex mu;
  std::condition_variable cv;
  hipStream_t copy_stream = nullptr;  // SPI_H2D_DEVICE_STREAM
  hsa_agent_t gpu_agent{}, cpu_agent{};  // SPI_H2D_WORKER_SDMA

  int acquire() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return !free_list.empty(); });
    const int s = free_list.back();
    free_list.pop_back();
    return s;
  }
  int try_acquire() {
    std::lock_guard<std::mutex> lk(mu);
    if (free_list.empty()) return -1;
    const int s = free_list.back();
    free_list.pop_back();
    return s;
  }
  void release(int s) {
    {
      std::lock_guard<std::mutex> lk(mu);
      free_list.push_back(s);
    }
    cv.notify_one();
  }
};

struct Task {
  std::vector<Job> jobs;
  std::vector<int64_t> offs;
  int64_t total = 0;
  int slot = -1;
  int status = SPI_OK;
  std::string err;
  int64_t cs = 0, ce = 0;
};

struct Worker {
  int32_t worker_id = 0;
  int32_t device = 0;
  int pool = 0;  // index into the runtime's pools
  spi_model* model = nullptr;
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;  // H2D stream (may be the pool's shared one)
  bool own_copy_stream = false;
  std::deque<Task> inflight;
  std::deque<Job> fixed;  // jobs pinned to this worker (under the runtime mutex)
  std::thread thread;
  // where the worker thread's time goes (spi_runtime_worker_times): tasks, slot wait,
  // host staging, H2D + codelet + D2H enqueue, completion-event wait (ns)
  std::atomic<int64_t> t_tasks{0}, t_slot{0}, t_stage{0}, t_enqueue{0}, t_event{0};
};

using QueueKey = std::pair<int64_t, uint64_t>;  // (-priority, submission sequence)

// HIP device -> its HSA GPU agent and the first CPU agent, for
// SPI_H2D_WORKER_SDMA.  Matched by the agent UUID (hipDeviceGetUuid carries the
// 16 hex digits of HSA_AMD_AGENT_INFO_UUID's body), so partitions of one GPU
// that share a PCI bus / device (CPX / TPX modes) are told apart; without a
// UUID, by PCI domain / bus / device / function, accepted only when exactly one
// agent matches.  Resolved once per device and cached.  hsa_init / hsa_shut_down
// are paired around the enumeration: HIP holds its own reference, which keeps
// the agent handles valid for the process.
bool resolve_hsa_agents(int device, hsa_agent_t& gpu, hsa_agent_t& cpu) {
  hipUUID uuid{};
  const bool have_uuid = hipDeviceGetUuid(&uuid, device) == hipSuccess;
  int bus = 0, dev = 0, dom = 0;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainId, device) != hipSuccess)
    return false;
  struct Find {
    char uuid[16];
    bool have_uuid;
    uint32_t bdf, dom;
    hsa_agent_t by_uuid{}, by_bdf{}, cpu{};
    int n_uuid = 0, n_bdf = 0;
    bool c = false;
  } f{};
  std::memcpy(f.uuid, uuid.bytes, 16);
  f.have_uuid = have_uuid;
  f.bdf = (uint32_t)((bus << 8) | (dev << 3));
  f.dom = (uint32_t)dom;
  if (hsa_init() != HSA_STATUS_SUCCESS) return false;
  hsa_iterate_agents(
      [](hsa_agent_t a, void* u) {
        Find& f = *static_cast<Find*>(u);
        hsa_device_type_t t;
        if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
        if (t == HSA_DEVICE_TYPE_CPU && !f.c) {
          f.cpu = a;
          f.c = true;
        } else if (t == HSA_DEVICE_TYPE_GPU) {
          char id[32] = {};
          if (f.have_uuid && hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_UUID, id) == HSA_STATUS_SUCCESS &&
              std::strncmp(id, "GPU-", 4) == 0 && std::strlen(id) >= 20 && std::memcmp(id + 4, f.uuid, 16) == 0) {
            f.by_uuid = a;
            ++f.n_uuid;
          }
          uint32_t bdf = 0, dom = 0;
          hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
          hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
          if ((bdf & ~7u) == f.bdf && dom == f.dom) {
            f.by_bdf = a;
            ++f.n_bdf;
          }
        }
        return HSA_STATUS_SUCCESS;
      },
      &f);
  (void)hsa_shut_down();
  cpu = f.cpu;
  if (f.n_uuid == 1) {
    gpu = f.by_uuid;
  } else if (f.n_uuid == 0 && f.n_bdf == 1) {
    gpu = f.by_bdf;
  } else {
    return false;  // ambiguous (partitioned GPU without UUIDs): the stream H2D modes
  }
  return f.c;
}

bool find_hsa_agents(int device, hsa_agent_t& gpu, hsa_agent_t& cpu) {
  struct Entry {
    bool ok;
    hsa_agent_t gpu, cpu;
  };
  static std::mutex mu;
  static std::map<int, Entry> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(device);
  if (it == cache.end()) {
    Entry e{};
    e.ok = resolve_hsa_agents(device, e.gpu, e.cpu);
    it = cache.emplace(device, e).first;
  }
  gpu = it->second.gpu;
  cpu = it->second.cpu;
  return it->second.ok;
}

// One host -> device SDMA copy on the engine ROCr assigns (pinning one engine measured no
// different, round 3).
hsa_status_t sdma_h2d(const SlotPool& pl, void* dst, const void* src, size_t bytes, hsa_signal_t sig) {
  return hsa_amd_memory_async_copy(dst, pl.gpu_agent, src, pl.cpu_agent, bytes, 0, nullptr, sig);
}

}  // namespace

struct spi_runtime {
  spi_runtime_config cfg{};
  std::vector<size_t> in_sample_bytes, out_sample_bytes;
  std::vector<std::unique_ptr<SlotPool>> pools;
  std::vector<std::unique_ptr<Worker>> workers;
  std::unique_ptr<CopyPool> copier;
  std::mutex mu;
  std::condition_variable cv_job, cv_idle;
  std::map<QueueKey, Job> queue;
  uint64_t seq = 0;
  int64_t inflight_jobs = 0;   // submitted, not completed
  int64_t inflight_tasks = 0;  // codelet calls enqueued, not finalized
  bool stop = false;
  bool congested = false;      // a submission was rejected since the last decision
  spi_batching_state bstate{};
  int32_t last_target = 0;
  double warmup_s = 0.0;  // spi_runtime_create's per-worker warm-up
  std::atomic<int64_t> completed{0}, failed{0};

  void run(Worker* w);
  bool compose(Worker* w, std::unique_lock<std::mutex>& lk, std::vector<Job>& jobs);
  void launch(Worker* w, std::vector<Job>&& jobs);
  void finalize_oldest(Worker* w);
  void destroy_resources();
  size_t queued_for(const Worker* w) const { return queue.size() + w->fixed.size(); }
};

// Batch composition under the batching strategy (caller holds mu, and w has
// work).  Takes the worker's pinned jobs first, then the queue head in
// priority order, while the samples fit the target (merge_input_tensors needs
// equal per-sample shapes, which the runtime config fixes).
bool spi_runtime::compose(Worker* w, std::unique_lock<std::mutex>& lk, std::vector<Job>& jobs) {
  const spi_batching_config& bc = cfg.batching;
  int target = cfg.max_batch, max_jobs = 1, timeout_us = 0;
  if (bc.kind == SPI_BATCHING_ADAPTIVE) {
    spi_batching_pressure p{};
    p.queue_size = (int64_t)queue.size();
    p.queue_capacity = cfg.max_queue;
    p.prepared_depth = 0;
    p.inflight_tasks = inflight_tasks;
    p.max_inflight_tasks = (int64_t)workers.size() * cfg.pipeline_depth;
    p.congested = congested ? 1 : 0;
    congested = false;
    spi_batching_decide(&bstate, &bc, &p, now_ns(), &target, &timeout_us);
    target = std::clamp(target, 1, cfg.max_batch);
    max_jobs = INT_MAX;
  } else if (bc.kind == SPI_BATCHING_FIXED) {
    max_jobs = std::max(1, cfg.coalesce_max_jobs);
    timeout_us = max_jobs > 1 ? cfg.coalesce_delay_us : 0;
  }
  last_target = target;
  int64_t total = 0;
  auto take = [&] {
    while ((int)jobs.size() < max_jobs && !w->fixed.empty() && total + w->fixed.front().batch <= target) {
      total += w->fixed.front().batch;
      jobs.push_back(std::move(w->fixed.front()));
      w->fixed.pop_front();
    }
    while ((int)jobs.size() < max_jobs && !queue.empty() && total + queue.begin()->second.batch <= target) {
      total += queue.begin()->second.batch;
      jobs.push_back(std::move(queue.begin()->second));
      queue.erase(queue.begin());
    }
  };
  take();
  if (jobs.empty()) {  // the head alone exceeds an adaptive target: run it alone
    if (!w->fixed.empty()) {
      jobs.push_back(std::move(w->fixed.front()));
      w->fixed.pop_front();
    } else {
      jobs.push_back(std::move(queue.begin()->second));
      queue.erase(queue.begin());
    }
    total = jobs.back().batch;
  }
  // Coalescing wait only when this worker has nothing in flight: with tasks in
  // flight the GPU is busy anyway and their completions must not be delayed.
  // idle_dispatch (this build's tuning): an idle worker does not wait at all -- on the
  // reference's CI workload the 10 ms coalescer held requests while the GPU sat idle
  // (p50 queue 8.25 of 11.2 ms); under load the queue fills while every worker is busy
  // and the next free worker takes a batch of it anyway.  The adaptive strategy's option only:
  // the FIXED kind keeps its coalesce_max_jobs / coalesce_delay_us merging.
  const bool idle_now = bc.idle_dispatch && bc.kind == SPI_BATCHING_ADAPTIVE;
  if (timeout_us > 0 && w->inflight.empty() && !idle_now) {
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(timeout_us);
    while (!stop && (int)jobs.size() < max_jobs && total < target) {
      if (cv_job.wait_until(lk, deadline) == std::cv_status::timeout) {
        take();
        break;
      }
      take();
    }
  }
  if (!queue.empty()) cv_job.notify_one();  // leftovers belong to another worker
  return !jobs.empty();
}

void spi_runtime::launch(Worker* w, std::vector<Job>&& jobs) {
  const int ni = cfg.num_inputs, no = cfg.num_outputs;
  SlotPool& pool = *pools[w->pool];
  Task t;
  t.jobs = std::move(jobs);
  const int64_t c0 = now_ns();
  // a free slot: never block while this worker still holds finished work
  int s = pool.try_acquire();
  while (s < 0 && !w->inflight.empty()) {
    finalize_oldest(w);
    s = pool.try_acquire();
  }
  if (s < 0) s = pool.acquire();
  t.slot = s;
  Slot& slot = pool.slots[s];
  const int64_t c1 = now_ns();
  // copy_job_inputs_to_slot: every job's samples at its row offset
  std::vector<CopyPool::Chunk> ops;
  for (const Job& j : t.jobs) {
    t.offs.push_back(t.total);
    for (int i = 0; i < ni; ++i)
      ops.push_back(CopyPool::Chunk{static_cast<char*>(slot.h_in[i]) + t.total * in_sample_bytes[i],
                                    static_cast<const char*>(j.in[i]), (size_t)j.batch * in_sample_bytes[i],
                                    nullptr});
    t.total += j.batch;
  }
  copier->copy(ops);
  const int64_t c2 = now_ns();
  // H2D into the slot's HBM buffers (StarPU's fetch of the R handles)
  hipStream_t h2d = w->copy_stream ? w->copy_stream : w->stream;
  if (cfg.h2d_mode == SPI_H2D_WORKER_SDMA) {
    // SDMA engine copies (HIP's own hipMemcpyAsync takes a shader copy kernel for a
    // share of these 4.8 MB copies, 256 workgroups for ~120 us each, competing with
    // the forwards: DESIGN.md 5.1); the slot's HBM buffers are free (the slot was
    // released after its last task's completion event), so is its signal
    const SlotPool& pl = *pools[w->pool];
    hsa_signal_store_screlease(slot.sig, ni);
    for (int i = 0; i < ni; ++i)
      if (sdma_h2d(pl, slot.d_in[i], slot.h_in[i], (size_t)t.total * in_sample_bytes[i], slot.sig) !=
          HSA_STATUS_SUCCESS) {
        t.status = SPI_ERR_DEVICE;
        t.err = "SDMA H2D copy failed";
        hsa_signal_subtract_screlease(slot.sig, ni - i);
        break;
      }
    // The worker thread waits (round 4 measured the alternative -- the worker stream waiting on
    // the signal's value word with hipStreamWaitValue64 -- releasing 46-55 ms after the copy on
    // this stack, tools/sdma_streamwait.cpp).  A wait may return before the
    // condition holds (the HSA spec allows it; ROCclr loops too): wait until the value drops
    // below 1.  Each completed copy decrements it; a failed copy leaves it negative.
    hsa_signal_value_t v = hsa_signal_load_scacquire(slot.sig);
    while (v >= 1)
      v = hsa_signal_wait_scacquire(slot.sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
    if (v < 0 && t.status == SPI_OK) {
      t.status = SPI_ERR_DEVICE;
      t.err = "SDMA H2D failed";
    }
  }
  for (int i = 0; i < ni && t.status == SPI_OK && cfg.h2d_mode != SPI_H2D_WORKER_SDMA; ++i)
    if (hipMemcpyAsync(slot.d_in[i], slot.h_in[i], (size_t)t.total * in_sample_bytes[i], hipMemcpyHostToDevice,
                       h2d) != hipSuccess) {
      t.status = SPI_ERR_DEVICE;
      t.err = "H2D copy failed";
    }
  if (h2d != w->stream && t.status == SPI_OK) {
    if (hipEventRecord(slot.h2d, h2d) != hipSuccess || hipStreamWaitEvent(w->stream, slot.h2d, 0) != hipSuccess) {
      t.status = SPI_ERR_DEVICE;
      t.err = "H2D event join failed";
    }
  }
  // the codelet over vector interfaces resized to this task's payload
  spi_codelet_args args;
  spi_args_init(&args);
  args.num_inputs = ni;
  args.num_outputs = no;
  args.request_id = t.jobs.front().request_id;
  args.batch_size = t.total;
  for (int i = 0; i < ni; ++i) {
    args.num_dims[i] = cfg.input_ndims[i] + 1;
    args.dims[i][0] = t.total;
    for (int d = 0; d < cfg.input_ndims[i]; ++d) args.dims[i][d + 1] = cfg.input_dims[i][d];
    args.input_types[i] = cfg.input_types[i];
  }
  for (int i = 0; i < no; ++i) args.output_types[i] = cfg.output_types[i];
  args.num_replicas = 1;
  args.models_gpu[0] = w->model;
  args.num_device_ids = 1;
  args.device_ids[0] = w->device;
  spi_vector_interface ifaces[SPI_MAX_INPUTS + SPI_MAX_OUTPUTS];
  void* buffers[SPI_MAX_INPUTS + SPI_MAX_OUTPUTS];
  for (int i = 0; i < ni; ++i) {
    const size_t es = spi_dtype_size(cfg.input_types[i]);
    ifaces[i] = spi_vector_interface{SPI_STARPU_VECTOR_INTERFACE_ID, (uintptr_t)slot.d_in[i], 0, 0,
                                     t.total * in_sample_bytes[i] / es, es, 0,
                                     (size_t)cfg.max_batch * in_sample_bytes[i]};
    buffers[i] = &ifaces[i];
  }
  for (int i = 0; i < no; ++i) {
    const size_t es = spi_dtype_size(cfg.output_types[i]);
    ifaces[ni + i] = spi_vector_interface{SPI_STARPU_VECTOR_INTERFACE_ID, (uintptr_t)slot.d_out[i], 0, 0,
                                          t.total * out_sample_bytes[i] / es, es, 0,
                                          (size_t)cfg.max_batch * out_sample_bytes[i]};
    buffers[ni + i] = &ifaces[ni + i];
  }
  if (t.status == SPI_OK) {
    spi_hip_inference_func(buffers, &args);
    t.cs = args.codelet_start_ns;
    t.ce = args.codelet_end_ns;
    if (args.status != SPI_OK) {
      t.status = args.status;
      t.err = args.error;
    }
  }
  if (t.status == SPI_OK)
    for (int i = 0; i < no; ++i)
      if (hipMemcpyAsync(slot.h_out[i], slot.d_out[i], (size_t)t.total * out_sample_bytes[i],
                         hipMemcpyDeviceToHost, w->stream) != hipSuccess) {
        t.status = SPI_ERR_DEVICE;
        t.err = "D2H copy failed";
      }
  if (hipEventRecord(slot.done, w->stream) != hipSuccess && t.status == SPI_OK) {
    t.status = SPI_ERR_DEVICE;
    t.err = "completion event failed";
  }
  {
    std::lock_guard<std::mutex> lk(mu);
    ++inflight_tasks;
  }
  w->inflight.push_back(std::move(t));
  const int64_t c3 = now_ns();
  w->t_tasks += 1;
  w->t_slot += c1 - c0;
  w->t_stage += c2 - c1;
  w->t_enqueue += c3 - c2;
}

// starpu_output_callback: wait for the task's completion event, hand each job
// its rows of every output (slice_outputs_for_sub_job), run its callback,
// release the slot.
void spi_runtime::finalize_oldest(Worker* w) {
  Task t = std::move(w->inflight.front());
  w->inflight.pop_front();
  SlotPool& pool = *pools[w->pool];
  Slot& slot = pool.slots[t.slot];
  const int64_t e0 = now_ns();
  const hipError_t se = hipEventSynchronize(slot.done);
  if (se != hipSuccess && t.status == SPI_OK) {
    t.status = SPI_ERR_DEVICE;
    t.err = "stream synchronisation failed";
  }
  w->t_event += now_ns() - e0;
  const int no = cfg.num_outputs;
  for (size_t k = 0; k < t.jobs.size(); ++k) {
    const Job& j = t.jobs[k];
    if (t.status == SPI_OK)
      for (int i = 0; i < no; ++i)
        std::memcpy(j.out[i], static_cast<const char*>(slot.h_out[i]) + t.offs[k] * out_sample_bytes[i],
                    (size_t)j.batch * out_sample_bytes[i]);
    spi_job_timing tm{};
    tm.submit_ns = j.submit_ns;
    tm.dequeue_ns = j.dequeue_ns;
    tm.codelet_start_ns = t.cs;
    tm.codelet_end_ns = t.ce;
    tm.device_id = w->device;
    tm.worker_id = w->worker_id;
    tm.task_batch = (int32_t)t.total;
    tm.task_jobs = (int32_t)t.jobs.size();
    tm.complete_ns = now_ns();
    (t.status == SPI_OK ? completed : failed).fetch_add(1);
    if (j.done) j.done(j.user, j.request_id, t.status, t.status == SPI_OK ? "" : t.err.c_str(), &tm);
  }
  pool.release(t.slot);
  {
    std::lock_guard<std::mutex> lk(mu);
    --inflight_tasks;
    inflight_jobs -= (int64_t)t.jobs.size();
    if (inflight_jobs == 0) cv_idle.notify_all();
  }
}

void spi_runtime::run(Worker* w) {
  (void)hipSetDevice(w->device);
  spi_set_worker_context(w->worker_id, w->device, w->stream);
  const size_t depth = (size_t)std::max(1, cfg.pipeline_depth);
  for (;;) {
    // deliver whatever already finished
    while (!w->inflight.empty() && hipEventQuery(pools[w->pool]->slots[w->inflight.front().slot].done) == hipSuccess)
      finalize_oldest(w);
    // a full pipeline takes no new work: jobs stay in the shared queue for
    // workers that can start them now (eager scheduling)
    if (w->inflight.size() >= depth) {
      finalize_oldest(w);
      continue;
    }
    std::vector<Job> jobs;
    bool quit = false;
    {
      std::unique_lock<std::mutex> lk(mu);
      cv_job.wait(lk, [&] { return stop || queued_for(w) > 0 || !w->inflight.empty(); });
      if (queued_for(w) > 0) {
        compose(w, lk, jobs);
        const int64_t t = now_ns();
        for (Job& j : jobs) j.dequeue_ns = t;
      } else if (stop && w->inflight.empty()) {
        quit = true;
      }
    }
    if (quit) break;
    if (jobs.empty()) {  // nothing new: wait for the oldest task in flight
      finalize_oldest(w);
      continue;
    }
    launch(w, std::move(jobs));
  }
  while (!w->inflight.empty()) finalize_oldest(w);
  spi_clear_worker_context();
}

void spi_runtime::destroy_resources() {
  for (auto& w : workers) {
    (void)hipSetDevice(w->device);
    if (w->own_copy_stream && w->copy_stream) (void)hipStreamDestroy(w->copy_stream);

    if (w->stream) (void)hipStreamDestroy(w->stream);
  }
  for (auto& p : pools) {
    (void)hipSetDevice(p->device);
    for (Slot& s : p->slots) {
      for (void* x : s.h_in) (void)hipHostFree(x);
      for (void* x : s.h_out) (void)hipHostFree(x);
      for (void* x : s.d_in) (void)hipFree(x);
      for (void* x : s.d_out) (void)hipFree(x);
      if (s.h2d) (void)hipEventDestroy(s.h2d);
      if (s.done) (void)hipEventDestroy(s.done);
      if (s.sig.handle) (void)hsa_signal_destroy(s.sig);
    }
    if (p->copy_stream) (void)hipStreamDestroy(p->copy_stream);
  }
}

extern "C" {

int spi_batching_decide(spi_batching_state* st, const spi_batching_config* c, const spi_batching_pressure* p,
                        int64_t now, int32_t* out_target, int32_t* out_timeout_us) {
  if (!st || !c || !p || !out_target || !out_timeout_us) return SPI_ERR_INVALID_ARGUMENT;
  const Pressure pr = resolve_pressure(*c, *p);
  const int limit = std::max(1, c->batch_limit);
  const int min_limit = std::clamp(c->min_batch_limit, 1, limit);
  if (c->kind == SPI_BATCHING_DISABLED) {
    *out_target = 1;
    *out_timeout_us = 0;
    return SPI_OK;
  }
  if (c->kind == SPI_BATCHING_FIXED) {
    *out_target = limit;
    *out_timeout_us = std::max(0, c->coalesce_timeout_us);
    return SPI_OK;
  }
  if (limit <= min_limit) {
    st->target = min_limit;
    st->initialized = 1;
    st->low_streak = 0;
    *out_target = min_limit;
    *out_timeout_us = coalesce_timeout(*c, pr.congested, min_limit);
    return SPI_OK;
  }
  if (!c->congestion_enabled) {
    st->low_streak = 0;
    *out_target = limit;
    *out_timeout_us = std::max(0, c->coalesce_timeout_us);
    return SPI_OK;
  }
  if (!st->initialized) {
    st->target = limit;
    st->initialized = 1;
  }
  // update_target_batch_limit
  st->target = std::clamp(st->target, min_limit, limit);
  bool refresh = true;
  const int64_t tick_ns = (int64_t)std::max(1, c->tick_interval_us) * 1000;
  if (st->has_marker && now - st->last_update_ns < tick_ns) refresh = false;
  if (refresh) {
    st->has_marker = 1;
    st->last_update_ns = now;
    if (pr.congested) {
      st->target = limit;
      st->low_streak = 0;
    } else if (pr.high) {
      st->low_streak = 0;
      st->target = std::min(limit, st->target + high_step(*c, limit, pr.severe));
    } else if (pr.low) {
      if (st->low_streak < INT_MAX) ++st->low_streak;
      if (st->low_streak >= low_streak_threshold(*c)) {
        st->target = std::max(min_limit, st->target - 1);
        st->low_streak = 0;
      }
    } else {
      st->low_streak = 0;
    }
  }
  const int target = std::clamp(st->target, 1, limit);
  *out_target = target;
  *out_timeout_us = coalesce_timeout(*c, pr.congested, target);
  return SPI_OK;
}

void spi_runtime_config_init(spi_runtime_config* c) {
  if (!c) return;
  std::memset(c, 0, sizeof(*c));
  c->workers_per_device = 4;
  c->coalesce_max_jobs = 1;
  c->pipeline_depth = 2;
  c->copy_threads = 4;
  c->h2d_mode = SPI_H2D_AUTO;
  c->batching.kind = SPI_BATCHING_FIXED;
}

spi_runtime* spi_runtime_create(const spi_runtime_config* c, char* err, size_t errlen) {
  auto fail = [&](const std::string& m) -> spi_runtime* {
    spi_set_last_error(m.c_str());
    if (err && errlen) std::snprintf(err, errlen, "%s", m.c_str());
    return nullptr;
  };
  if (!c || c->num_devices < 1 || c->num_devices > SPI_MAX_REPLICAS || c->max_batch < 1 || c->num_inputs < 1 ||
      c->num_inputs > SPI_MAX_INPUTS || c->num_outputs < 1 || c->num_outputs > SPI_MAX_OUTPUTS ||
      c->h2d_mode < 0 || c->h2d_mode > SPI_H2D_WORKER_SDMA || c->batching.kind < 0 ||
      c->batching.kind > SPI_BATCHING_ADAPTIVE)
    return fail("invalid runtime configuration");
  auto rt = std::make_unique<spi_runtime>();
  rt->cfg = *c;
  spi_runtime_config& cfg = rt->cfg;
  if (cfg.workers_per_device <= 0) cfg.workers_per_device = 4;
  if (cfg.pipeline_depth <= 0) cfg.pipeline_depth = 2;
  if (cfg.copy_threads <= 0) cfg.copy_threads = 4;
  if (cfg.slots_per_device <= 0) cfg.slots_per_device = std::max(2, cfg.workers_per_device * cfg.pipeline_depth);
  if (cfg.batching.batch_limit <= 0 || cfg.batching.batch_limit > cfg.max_batch) cfg.batching.batch_limit = cfg.max_batch;
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
  if (cfg.h2d_mode == SPI_H2D_AUTO) {
    // SDMA-engine copies when the task's input keeps the PCIe link busy: at least 120 KiB of
    // input per GFLOP of the forward.  The threshold sits on a measured crossover
    // (tools/sdma_crossover.py, bs8, 4 workers, 32 in flight, profiles/r03/sdma_crossover.log):
    // SDMA / stream e2e = 1.116 for ResNet-18 (162 KiB/GFLOP), 0.952 ResNet-34 (80), 0.930
    // ResNet-50 (72), 0.949 ResNet-101 (38), 0.950 ResNet-152 (26); ViT-L (5) and BERT (0.1)
    // lose too.  The compute-bound side loses because the device's kernels run slower beside
    // the SDMA traffic, not because the worker waits for the copy: pinning the copies to a
    // free engine (a round-3 option, since removed) cut ResNet-152's per-task copy wait from ~7 ms
    // to ~1 ms and the rate still fell (9.2k vs 10.6k inf/s on the streams); round 4 re-measured
    // C4 / C5 at 10.1k / 4.56k on SDMA against 11.2k / 4.79k on the streams (tools/sdma_ab.py).
    // Below the threshold: a shared copy stream for <= 3 workers, the worker streams beyond
    // (four busy streams per device)
    size_t task_in = 0;
    for (size_t b : rt->in_sample_bytes) task_in += b * (size_t)cfg.max_batch;
    const double gflop = c->models[0] ? spi_model_flops(c->models[0], cfg.max_batch) * 1e-9 : 0.0;
    bool sdma = gflop > 0.0 && (double)task_in / gflop >= 120.0 * 1024.0;
    for (int dv = 0; dv < c->num_devices && sdma; ++dv) {
      hsa_agent_t g{}, h{};
      sdma = find_hsa_agents(c->device_ids[dv], g, h);
    }
    cfg.h2d_mode = sdma ? SPI_H2D_WORKER_SDMA
                        : cfg.workers_per_device <= 3 ? SPI_H2D_DEVICE_STREAM : SPI_H2D_WORKER_STREAM;
  }
  {
    // HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (default 4)
    // round-robin; worker streams sharing a queue run serially.
    const char* q = std::getenv("GPU_MAX_HW_QUEUES");
    const int queues = q ? std::atoi(q) : 4;
    const int need = cfg.workers_per_device + (cfg.h2d_mode == SPI_H2D_DEVICE_STREAM ? 1
                                               : cfg.h2d_mode == SPI_H2D_WORKER_COPY ? cfg.workers_per_device : 0);
    if (queues < need + 1)
      std::fprintf(stderr,
                   "spi_runtime: GPU_MAX_HW_QUEUES=%d < %d streams + 1; streams will share hardware queues and "
                   "serialize (set it before the first HIP call)\n",
                   queues, need);
  }
  for (int dv = 0; dv < c->num_devices; ++dv)
    if (!c->models[dv]) return fail("missing replica for device " + std::to_string(c->device_ids[dv]));
  auto cleanup_fail = [&](const std::string& m) {
    rt->destroy_resources();
    return fail(m);
  };
  int32_t wid = 0;
  for (int dv = 0; dv < c->num_devices; ++dv) {
    auto pool = std::make_unique<SlotPool>();
    pool->device = c->device_ids[dv];
    if (hipSetDevice(pool->device) != hipSuccess) return cleanup_fail("hipSetDevice failed");
    pool->slots.resize(cfg.slots_per_device);
    bool ok = true;
    for (int s = 0; s < cfg.slots_per_device && ok; ++s) {
      Slot& sl = pool->slots[s];
      for (size_t b : rt->in_sample_bytes) {
        void *h = nullptr, *d = nullptr;
        ok = ok && hipHostMalloc(&h, b * cfg.max_batch, hipHostMallocPortable) == hipSuccess;
        sl.h_in.push_back(h);
        ok = ok && hipMalloc(&d, b * cfg.max_batch) == hipSuccess;
        sl.d_in.push_back(d);
      }
      for (size_t b : rt->out_sample_bytes) {
        void *h = nullptr, *d = nullptr;
        ok = ok && hipHostMalloc(&h, b * cfg.max_batch, hipHostMallocPortable) == hipSuccess;
        sl.h_out.push_back(h);
        ok = ok && hipMalloc(&d, b * cfg.max_batch) == hipSuccess;
        sl.d_out.push_back(d);
      }
      ok = ok && hipEventCreateWithFlags(&sl.h2d, hipEventDisableTiming) == hipSuccess;
      ok = ok && hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) == hipSuccess;
      pool->free_list.push_back(cfg.slots_per_device - 1 - s);
    }
    if (ok && cfg.h2d_mode == SPI_H2D_DEVICE_STREAM)
      ok = hipStreamCreateWithFlags(&pool->copy_stream, hipStreamNonBlocking) == hipSuccess;
    if (ok && cfg.h2d_mode == SPI_H2D_WORKER_SDMA && !find_hsa_agents(pool->device, pool->gpu_agent, pool->cpu_agent)) {
      rt->pools.push_back(std::move(pool));
      return cleanup_fail("no HSA agents for device " + std::to_string(c->device_ids[dv]));
    }
    if (ok && cfg.h2d_mode == SPI_H2D_WORKER_SDMA)
      for (Slot& sl : pool->slots)
        ok = ok && hsa_signal_create(0, 0, nullptr, &sl.sig) == HSA_STATUS_SUCCESS;
    rt->pools.push_back(std::move(pool));
    if (!ok) return cleanup_fail("slot pool allocation failed on device " + std::to_string(c->device_ids[dv]));
    for (int k = 0; k < cfg.workers_per_device; ++k) {
      auto w = std::make_unique<Worker>();
      w->worker_id = wid++;
      w->device = c->device_ids[dv];
      w->pool = dv;
      w->model = c->models[dv];
      bool wok = hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking) == hipSuccess;
      if (cfg.h2d_mode == SPI_H2D_DEVICE_STREAM) {
        w->copy_stream = rt->pools.back()->copy_stream;
      } else if (cfg.h2d_mode == SPI_H2D_WORKER_COPY) {
        wok = wok && hipStreamCreateWithFlags(&w->copy_stream, hipStreamNonBlocking) == hipSuccess;
        w->own_copy_stream = true;
      }
      rt->workers.push_back(std::move(w));
      if (!wok) return cleanup_fail("stream creation failed for worker " + std::to_string(wid - 1));
    }
  }
  // Every slot's transfer path exercised once before serving: the first SDMA copy from a
  // pinned buffer (or the first copy on a stream) costs far more than the steady state --
  // the first measured requests of a fresh runtime had shown 10-19 ms latencies beside a
  // 3 ms p50 (tools/e2e_tail.py) -- so the copy engines, queues and mappings are set up now.
  for (size_t dv = 0; dv < rt->pools.size(); ++dv) {
    SlotPool& pl = *rt->pools[dv];
    (void)hipSetDevice(pl.device);
    Worker* w0 = nullptr;
    for (auto& w : rt->workers)
      if (w->pool == (int)dv) {
        w0 = w.get();
        break;
      }
    hipStream_t st = pl.copy_stream ? pl.copy_stream : w0->stream;
    for (Slot& sl : pl.slots) {
      for (size_t i = 0; i < sl.h_in.size(); ++i) {
        const size_t bytes = rt->in_sample_bytes[i] * (size_t)cfg.max_batch;
        std::memset(sl.h_in[i], 0, bytes);
        if (cfg.h2d_mode == SPI_H2D_WORKER_SDMA) {
          hsa_signal_store_screlease(sl.sig, 1);
          if (sdma_h2d(pl, sl.d_in[i], sl.h_in[i], bytes, sl.sig) != HSA_STATUS_SUCCESS)
            return cleanup_fail("SDMA warm-up copy failed on device " + std::to_string(pl.device));
          hsa_signal_value_t v = hsa_signal_load_scacquire(sl.sig);
          while (v >= 1)
            v = hsa_signal_wait_scacquire(sl.sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
          if (v < 0) return cleanup_fail("SDMA warm-up copy failed on device " + std::to_string(pl.device));
        } else if (hipMemcpyAsync(sl.d_in[i], sl.h_in[i], bytes, hipMemcpyHostToDevice, st) != hipSuccess) {
          return cleanup_fail("H2D warm-up copy failed on device " + std::to_string(pl.device));
        }
      }
      for (size_t i = 0; i < sl.h_out.size(); ++i)
        if (hipMemcpyAsync(sl.h_out[i], sl.d_out[i], rt->out_sample_bytes[i] * (size_t)cfg.max_batch,
                           hipMemcpyDeviceToHost, w0->stream) != hipSuccess)
          return cleanup_fail("D2H warm-up copy failed on device " + std::to_string(pl.device));
    }
    if (hipStreamSynchronize(st) != hipSuccess || hipStreamSynchronize(w0->stream) != hipSuccess)
      return cleanup_fail("transfer warm-up failed on device " + std::to_string(pl.device));
  }
  // Per-worker warm-up before serving (the reference warms every worker through the
  // pipeline, inference_runner.cpp:507-560): the workspace and the graph of every batch
  // size the batchers can compose, so no capture (serialised process-wide) or workspace
  // allocation ever lands on a live request.
  const int64_t seq = cfg.input_ndims[0] >= 1 ? cfg.input_dims[0][0] : 0;
  std::vector<int> warm;
  if (cfg.warmup_batches >= 0) {
    const int upto = cfg.warmup_batches == 0 ? cfg.max_batch : std::min(cfg.warmup_batches, cfg.max_batch);
    for (int b = 1; b <= upto; ++b) warm.push_back(b);
  }
  if (warm.empty() || warm.back() != cfg.max_batch) warm.push_back(cfg.max_batch);
  const auto warm_t0 = std::chrono::steady_clock::now();
  for (auto& w : rt->workers) {
    (void)hipSetDevice(w->device);
    for (int b : warm)
      if (spi_model_warmup(w->model, w->stream, b, seq, cfg.num_inputs >= 2) != SPI_OK)
        return cleanup_fail(std::string("warm-up failed for worker ") + std::to_string(w->worker_id) + " batch " +
                            std::to_string(b) + ": " + spi_last_error());
  }
  rt->warmup_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - warm_t0).count();
  rt->copier = std::make_unique<CopyPool>(cfg.copy_threads - 1);
  rt->last_target = cfg.max_batch;
  for (auto& w : rt->workers) w->thread = std::thread(&spi_runtime::run, rt.get(), w.get());
  return rt.release();
}

int spi_runtime_submit_job(spi_runtime* rt, const spi_job_desc* d) {
  if (!rt || !d || !d->inputs || !d->outputs || d->batch < 1 || d->batch > rt->cfg.max_batch)
    return SPI_ERR_INVALID_ARGUMENT;
  if (d->fixed_worker >= (int32_t)rt->workers.size()) return SPI_ERR_INVALID_ARGUMENT;
  Job j;
  j.request_id = d->request_id;
  j.fixed_worker = d->fixed_worker;
  // InferenceTask::create_task: priority = max(min_prio, max_prio - request_id)
  j.priority = d->has_priority ? d->priority
                               : (int32_t)std::max<int64_t>(rt->cfg.min_priority,
                                                            (int64_t)rt->cfg.max_priority - d->request_id);
  j.batch = d->batch;
  j.in.assign(d->inputs, d->inputs + rt->cfg.num_inputs);
  j.out.assign(d->outputs, d->outputs + rt->cfg.num_outputs);
  j.done = d->done;
  j.user = d->user;
  j.submit_ns = now_ns();
  {
    std::lock_guard<std::mutex> lk(rt->mu);
    if (rt->stop) return SPI_ERR_INVALID_ARGUMENT;
    if (rt->cfg.max_queue > 0 && (int64_t)rt->queue.size() >= rt->cfg.max_queue) {
      rt->congested = true;
      return SPI_ERR_QUEUE_FULL;
    }
    if (j.fixed_worker >= 0) {
      rt->workers[j.fixed_worker]->fixed.push_back(std::move(j));
    } else {
      rt->queue.emplace(QueueKey{-(int64_t)j.priority, rt->seq++}, std::move(j));
    }
    ++rt->inflight_jobs;
  }
  if (d->fixed_worker >= 0)
    rt->cv_job.notify_all();  // the pinned worker must see it
  else
    rt->cv_job.notify_one();
  return SPI_OK;
}

int spi_runtime_submit(spi_runtime* rt, int32_t request_id, int64_t batch, const void* const* inputs,
                       void* const* outputs, spi_job_done_fn done, void* user) {
  spi_job_desc d{};
  d.request_id = request_id;
  d.fixed_worker = -1;
  d.batch = batch;
  d.inputs = inputs;
  d.outputs = outputs;
  d.done = done;
  d.user = user;
  return spi_runtime_submit_job(rt, &d);
}

int spi_runtime_drain(spi_runtime* rt) {
  if (!rt) return SPI_ERR_INVALID_ARGUMENT;
  std::unique_lock<std::mutex> lk(rt->mu);
  rt->cv_idle.wait(lk, [&] { return rt->inflight_jobs == 0; });
  return SPI_OK;
}

void spi_runtime_stats(const spi_runtime* rt, int64_t* completed, int64_t* failed) {
  if (completed) *completed = rt ? rt->completed.load() : 0;
  if (failed) *failed = rt ? rt->failed.load() : 0;
}

int32_t spi_runtime_num_workers(const spi_runtime* rt) { return rt ? (int32_t)rt->workers.size() : 0; }

int spi_runtime_worker_times(const spi_runtime* rt, int32_t worker, int64_t* out) {
  if (!rt || !out || worker < 0 || worker >= (int32_t)rt->workers.size()) return SPI_ERR_INVALID_ARGUMENT;
  const auto& w = *rt->workers[worker];
  out[0] = w.t_tasks.load();
  out[1] = w.t_slot.load();
  out[2] = w.t_stage.load();
  out[3] = w.t_enqueue.load();
  out[4] = w.t_event.load();
  return SPI_OK;
}

int32_t spi_runtime_h2d_mode(const spi_runtime* rt) { return rt ? rt->cfg.h2d_mode : -1; }

double spi_runtime_warmup_seconds(const spi_runtime* rt) { return rt ? rt->warmup_s : 0.0; }



int32_t spi_runtime_batch_target(const spi_runtime* rt) {
  if (!rt) return 0;
  std::lock_guard<std::mutex> lk(const_cast<spi_runtime*>(rt)->mu);
  return rt->last_target;
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
  rt->copier.reset();
  rt->destroy_resources();
  delete rt;
}

// ---------------------------------------------------------------------------
// Load generator
// ---------------------------------------------------------------------------
namespace {
struct LoadGen {
  struct Req {
    int64_t submit = 0, complete = 0, dequeue = 0, cstart = 0;
    int32_t status = -1, jobs = 0, batch = 0;
    int buf = -1;
    LoadGen* gen = nullptr;
  };
  std::vector<Req> reqs;
  std::vector<std::vector<std::vector<char>>> out_bufs;  // [buffer][output]
  std::vector<int> free_bufs;
  std::mutex mu;
  std::condition_variable cv;
  int64_t outstanding = 0;
  std::string first_err;

  static void done(void* user, int32_t, int32_t status, const char* error, const spi_job_timing* t) {
    Req* r = static_cast<Req*>(user);
    LoadGen* g = r->gen;
    r->complete = t->complete_ns;
    r->dequeue = t->dequeue_ns;
    r->cstart = t->codelet_start_ns;
    r->status = status;
    r->jobs = t->task_jobs;
    r->batch = t->task_batch;
    {
      std::lock_guard<std::mutex> lk(g->mu);
      if (status != SPI_OK && g->first_err.empty()) g->first_err = error ? error : "";
      g->free_bufs.push_back(r->buf);
      --g->outstanding;
    }
    g->cv.notify_all();
  }
};

double pct(std::vector<double>& xs, double p) {  // latency_statistics.hpp:52-93
  if (xs.empty()) return NAN;
  if (xs.size() == 1) return xs[0];
  const double pos = p / 100.0 * (double)(xs.size() - 1);
  const size_t lo = (size_t)std::floor(pos), hi = std::min(lo + 1, xs.size() - 1);
  return xs[lo] + (xs[hi] - xs[lo]) * (pos - (double)lo);
}

void sleep_until_ns(int64_t t) {
  for (;;) {
    const int64_t now = now_ns();
    if (now >= t) return;
    const int64_t left = t - now;
    if (left > 200000) {
      timespec ts{0, (long)(left - 100000)};
      nanosleep(&ts, nullptr);
    } else {
      std::this_thread::yield();
    }
  }
}
}  // namespace

int spi_runtime_loadgen(spi_runtime* rt, const spi_loadgen_config* c, const void* const* inputs,
                        spi_loadgen_result* res) {
  if (!rt || !c || !inputs || !res || c->request_batch < 1 || c->request_batch > rt->cfg.max_batch)
    return SPI_ERR_INVALID_ARGUMENT;
  std::memset(res, 0, sizeof(*res));
  const bool open = c->num_segments > 0;
  int64_t n = c->requests;
  if (open) {
    n = 0;
    for (int i = 0; i < c->num_segments; ++i) n += std::max<int64_t>(0, c->segments[i].repeat);
  }
  const int nbuf = std::max(1, open ? std::max(c->inflight, 256) : c->inflight);
  LoadGen g;
  g.out_bufs.resize(nbuf);
  for (auto& b : g.out_bufs)
    for (size_t bytes : rt->out_sample_bytes) b.emplace_back(bytes * c->request_batch);
  for (int i = nbuf - 1; i >= 0; --i) g.free_bufs.push_back(i);
  auto submit = [&](LoadGen::Req& r, int32_t id) -> int {
    int buf;
    {
      std::unique_lock<std::mutex> lk(g.mu);
      g.cv.wait(lk, [&] { return !g.free_bufs.empty() && (open || g.outstanding < c->inflight); });
      buf = g.free_bufs.back();
      g.free_bufs.pop_back();
      ++g.outstanding;
    }
    r.buf = buf;
    r.gen = &g;
    void* outs[SPI_MAX_OUTPUTS];
    for (int i = 0; i < rt->cfg.num_outputs; ++i) outs[i] = g.out_bufs[buf][i].data();
    r.submit = now_ns();
    const int rc = spi_runtime_submit(rt, id, c->request_batch, inputs, outs, &LoadGen::done, &r);
    if (rc != SPI_OK) {
      std::lock_guard<std::mutex> lk(g.mu);
      g.free_bufs.push_back(buf);
      --g.outstanding;
    }
    return rc;
  };
  // warm-up (not measured)
  if (c->warmup_requests > 0) {
    std::vector<LoadGen::Req> warm(c->warmup_requests);
    for (int i = 0; i < c->warmup_requests; ++i)
      while (submit(warm[i], -1 - i) == SPI_ERR_QUEUE_FULL) std::this_thread::yield();
    spi_runtime_drain(rt);
  }
  g.reqs.resize(n);
  int64_t rejected = 0;
  if (!open) {
    for (int64_t i = 0; i < n; ++i) {
      int rc;
      while ((rc = submit(g.reqs[i], (int32_t)i)) == SPI_ERR_QUEUE_FULL) std::this_thread::yield();
      if (rc != SPI_OK) {
        std::snprintf(res->error, SPI_ERROR_LEN, "submit failed (%d)", rc);
        spi_runtime_drain(rt);
        return rc;
      }
    }
  } else {
    int64_t t = now_ns(), i = 0;
    for (int s = 0; s < c->num_segments; ++s)
      for (int64_t k = 0; k < c->segments[s].repeat; ++k, ++i) {
        t += c->segments[s].delta_us * 1000;
        sleep_until_ns(t);
        const int rc = submit(g.reqs[i], (int32_t)i);
        if (rc == SPI_ERR_QUEUE_FULL) {
          ++rejected;
          g.reqs[i].status = SPI_ERR_QUEUE_FULL;
        }
      }
  }
  spi_runtime_drain(rt);
  std::vector<double> lat, qlat, slat, dlat;
  int64_t first = INT64_MAX, last = 0, ok = 0, bad = 0, worst_submit = 0;
  double jobs = 0, batch = 0, sum = 0, mx = 0;
  for (auto& r : g.reqs) {
    if (r.status == SPI_ERR_QUEUE_FULL) continue;
    if (r.status != SPI_OK) {
      ++bad;
      continue;
    }
    ++ok;
    first = std::min(first, r.submit);
    last = std::max(last, r.complete);
    const double ms = (r.complete - r.submit) * 1e-6;
    lat.push_back(ms);
    qlat.push_back((r.dequeue - r.submit) * 1e-6);
    slat.push_back((r.cstart - r.dequeue) * 1e-6);
    dlat.push_back((r.complete - r.cstart) * 1e-6);
    sum += ms;
    if (ms > mx) worst_submit = r.submit;
    mx = std::max(mx, ms);
    jobs += r.jobs;
    batch += r.batch;
  }
  std::sort(lat.begin(), lat.end());
  std::sort(qlat.begin(), qlat.end());
  std::sort(slat.begin(), slat.end());
  std::sort(dlat.begin(), dlat.end());
  res->completed = ok;
  res->failed = bad;
  res->rejected = rejected;
  res->inferences = ok * c->request_batch;
  res->seconds = ok ? (last - first) * 1e-9 : 0.0;
  res->inferences_per_s = res->seconds > 0 ? res->inferences / res->seconds : 0.0;
  res->p50_ms = pct(lat, 50);
  res->p95_ms = pct(lat, 95);
  res->p99_ms = pct(lat, 99);
  res->mean_ms = ok ? sum / ok : NAN;
  res->max_ms = mx;
  res->mean_jobs_per_task = ok ? jobs / ok : 0;
  res->mean_task_batch = ok ? batch / ok : 0;
  res->p50_queue_ms = pct(qlat, 50);
  res->p99_queue_ms = pct(qlat, 99);
  res->p50_stage_ms = pct(slat, 50);
  res->p99_stage_ms = pct(slat, 99);
  res->p50_device_ms = pct(dlat, 50);
  res->p99_device_ms = pct(dlat, 99);
  res->worst_at_frac = ok && last > first ? (double)(worst_submit - first) / (double)(last - first) : 0.0;
  std::snprintf(res->error, SPI_ERROR_LEN, "%s", g.first_err.c_str());
  return bad ? SPI_ERR_DEVICE : SPI_OK;
}

}  // extern "C"
