/*
 * spi_runtime.h — a StarPU stand-in that drives the HIP codelet, plus the
 * client-side load generator used to measure it.
 *
 * Reproduces the task path around the codelet:
 *   submit        SlotManager::submit_inference_task   slot_manager_component.cpp:517-647
 *   priority      priority = max(min_prio, max_prio - request_id)
 *                 (InferenceTask::create_task, inference_task.cpp:690-753)
 *   fixed worker  a job pinned to one worker (assign_fixed_worker_if_needed,
 *                 inference_task.cpp:824-842; the per-worker warm-up jobs)
 *   eager queue   STARPU_SCHED=eager: one shared queue   models/resnet18.yml:3
 *   workers       STARPU_NWORKER_PER_CUDA workers per device, one HIP stream each
 *   pipeline      up to `pipeline_depth` tasks in flight per worker (STARPU_CUDA_PIPELINE,
 *                 ci/perf/resnet152_ci_perf.yml): task n+1 is staged and its H2D
 *                 enqueued while task n computes
 *   slot pools    InputSlotPool / OutputSlotPool: per device `slots_per_device` slots of
 *                 pinned host memory (hipHostMalloc portable, max_batch x per-sample
 *                 bytes) + their HBM buffers, acquire / try_acquire / release
 *                 (input_slot_pool.cpp:77-215, output_slot_pool.cpp:287-330,
 *                 slot_pool_base.hpp:32-75; default max(2, workers),
 *                 slot_pool_buffer_utils.hpp:192-196 -- here workers x depth so a
 *                 full pipeline never waits for a slot)
 *   staging       copy_job_inputs_to_slot: each job's samples at its row offset in the
 *                 pinned slot, chunks spread over `copy_threads` host threads
 *                 (parallel_for_each_index + CudaCopyBatch,
 *                 slot_manager_component.cpp:56-95,222-293, 649-727), then hipMemcpyAsync
 *                 H2D into the slot's HBM buffer on a copy stream joined to the worker
 *                 stream by an event (h2d_mode)
 *   resize        nx = batch x per-sample (starpu_vector_resize_utils.hpp:19-89)
 *   codelet       spi_hip_inference_func with the worker context set
 *   output        hipMemcpyAsync D2H on the worker stream + completion event
 *                 (starpu_data_acquire_cb(R), inference_task.cpp:907-935), rows sliced
 *                 back per job (slice_outputs_for_sub_job, batching_helpers.hpp:75-125;
 *                 propagate_completion_to_sub_jobs, result_dispatcher_component.cpp:678-740),
 *                 completion callback with the latency breakdown
 *   queue full    SPI_ERR_QUEUE_FULL (RESOURCE_EXHAUSTED, docs/server_guide.md:120)
 *   batching      batch composition (merge_input_tensors, batch_composition_policy.cpp:
 *                 153-193) under a batching strategy: disabled, fixed (coalesce_max_jobs /
 *                 coalesce_delay_us) or adaptive (AdaptiveBatchingStrategy::decide /
 *                 update_target_batch_limit, batching_strategy.cpp:195-360)
 */
#ifndef SPI_RUNTIME_H
#define SPI_RUNTIME_H

#include "spi_codelet.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SPI_ERR_QUEUE_FULL 8

/* ---------------------------------------------------------------------------
 * Batching strategy (batching_strategy.hpp / .cpp).  Times are microseconds
 * where the reference uses milliseconds: a ResNet-18 bs8 task takes ~0.3 ms
 * on one MI355X, so millisecond ticks would be coarser than a task.
 * ------------------------------------------------------------------------- */
enum spi_batching_kind {
  SPI_BATCHING_FIXED = 0,    /* coalesce_max_jobs / coalesce_delay_us (the round-1 rule) */
  SPI_BATCHING_DISABLED = 1, /* one job per task */
  SPI_BATCHING_ADAPTIVE = 2  /* AdaptiveBatchingStrategy */
};

typedef struct spi_batching_config {
  int32_t kind;                /* enum spi_batching_kind */
  int32_t min_batch_limit;     /* samples */
  int32_t batch_limit;         /* samples (<= runtime max_batch; 0 -> max_batch) */
  int32_t coalesce_timeout_us; /* wait for more jobs while under the target */
  int32_t congestion_enabled;
  int32_t tick_interval_us;    /* congestion_tick_interval_ms */
  int32_t entry_horizon_us;    /* congestion_entry_horizon_ms */
  int32_t exit_horizon_us;     /* congestion_exit_horizon_ms */
  double fill_high, fill_low;  /* queue fill thresholds */
  double rho_high, rho_low;    /* kept for the monitor path; unused without a monitor */
  /* This build's MI355X tuning (not in the reference): a worker with no task in flight
   * dispatches what the queue holds at once (up to the strategy's target) instead of
   * waiting up to coalesce_timeout_us for more jobs; batches still form from the jobs
   * that queue while every worker is busy.  0 = the reference's collector.  Applies to
   * SPI_BATCHING_ADAPTIVE only: the FIXED kind ignores it and keeps coalesce_max_jobs /
   * coalesce_delay_us. */
  int32_t idle_dispatch;
  int32_t _pad1;
} spi_batching_config;

/* BatchingStrategyRuntimeState + the `congested` flag. */
typedef struct spi_batching_pressure {
  int64_t queue_size;
  int64_t queue_capacity;
  int64_t prepared_depth;
  int64_t inflight_tasks;
  int64_t max_inflight_tasks;
  int32_t congested;
  int32_t _pad;
} spi_batching_pressure;

/* AdaptiveBatchingStrategy's members; zero-initialise before first use. */
typedef struct spi_batching_state {
  int32_t target;
  int32_t initialized;
  int32_t low_streak;
  int32_t has_marker;
  int64_t last_update_ns;
} spi_batching_state;

/* One decision (decide()): target batch limit in samples and the coalescing timeout. */
int spi_batching_decide(spi_batching_state* state, const spi_batching_config* config,
                        const spi_batching_pressure* pressure, int64_t now_ns, int32_t* target_batch_limit,
                        int32_t* coalesce_timeout_us);

/* ---------------------------------------------------------------------------
 * Runtime
 * ------------------------------------------------------------------------- */
typedef struct spi_runtime spi_runtime;

/* CLOCK_MONOTONIC nanoseconds. */
typedef struct spi_job_timing {
  int64_t submit_ns;         /* spi_runtime_submit entered */
  int64_t dequeue_ns;        /* a worker popped the job */
  int64_t codelet_start_ns;  /* after host->slot copy and H2D enqueue */
  int64_t codelet_end_ns;    /* codelet returned (kernels enqueued) */
  int64_t complete_ns;       /* outputs in the caller's buffers */
  int32_t device_id;
  int32_t worker_id;
  int32_t task_batch;        /* samples in the codelet call that ran this job */
  int32_t task_jobs;         /* jobs merged into that call */
} spi_job_timing;

/* Called on a runtime worker thread after the job's outputs were written (or
 * it failed: status != SPI_OK, error set). */
typedef void (*spi_job_done_fn)(void* user, int32_t request_id, int32_t status, const char* error,
                                const spi_job_timing* timing);

/* A device serves about four busy streams at once: with a fifth (four workers +
 * a copy stream, or five workers) one or two of them get a third of the others'
 * tasks.  SPI_H2D_AUTO takes the SDMA engines directly (no stream,
 * and no H2D turned into a shader copy kernel beside the forwards); without HSA
 * agents it keeps a device at <= 4 busy streams: a shared copy stream for <= 3
 * workers, the H2D on the worker stream beyond. */
enum spi_h2d_mode {
  SPI_H2D_DEVICE_STREAM = 0, /* one copy stream per device, event-joined */
  SPI_H2D_WORKER_STREAM = 1, /* H2D on the worker's own stream */
  SPI_H2D_WORKER_COPY = 2,   /* one copy stream per worker, event-joined */
  SPI_H2D_AUTO = 3,          /* default: WORKER_SDMA when the task input is >= 120 KiB per GFLOP of the
                                forward (link-bound serving); otherwise (or without HSA agents)
                                DEVICE_STREAM for <= 3 workers per device, else WORKER_STREAM */
  SPI_H2D_WORKER_SDMA = 4    /* H2D on an SDMA engine (hsa_amd_memory_async_copy), waited by the worker
                                thread before the codelet is enqueued: no stream, no shader copy kernel */
};

typedef struct spi_runtime_config {
  int32_t num_devices;
  int32_t device_ids[SPI_MAX_REPLICAS];
  spi_model* models[SPI_MAX_REPLICAS]; /* replica for device_ids[i] */
  int32_t workers_per_device;          /* STARPU_NWORKER_PER_CUDA (0 -> 4) */
  int32_t max_batch;
  int32_t max_queue;                   /* 0 = unbounded */
  int32_t num_inputs;
  int32_t input_types[SPI_MAX_INPUTS];
  int32_t input_ndims[SPI_MAX_INPUTS];               /* per-sample dims (batch excluded) */
  int64_t input_dims[SPI_MAX_INPUTS][SPI_MAX_DIMS];
  int32_t num_outputs;
  int32_t output_types[SPI_MAX_OUTPUTS];
  int64_t output_elems[SPI_MAX_OUTPUTS];             /* per-sample element count */
  int32_t coalesce_max_jobs;  /* FIXED: <= 1 one job per call; N: merge up to N queued jobs */
  int32_t coalesce_delay_us;  /* FIXED: how long a worker waits for more jobs to fill max_batch */
  int32_t pipeline_depth;     /* tasks in flight per worker (0 -> 2) */
  int32_t slots_per_device;   /* slot pool size per device (0 -> workers x depth) */
  int32_t copy_threads;       /* host staging threads incl. the worker (0 -> 4) */
  int32_t h2d_mode;           /* enum spi_h2d_mode: spi_runtime_config_init sets SPI_H2D_AUTO; a
                                 zeroed struct means SPI_H2D_DEVICE_STREAM (value 0) */
  int32_t min_priority;       /* starpu_sched_get_min_priority (0 with eager) */
  int32_t max_priority;       /* starpu_sched_get_max_priority (0 with eager) */
  spi_batching_config batching;
  int32_t warmup_batches;     /* per-worker warm-up at create (inference_runner.cpp:507-560):
                                 0 = every batch size 1..max_batch captured before serving (no
                                 capture on a live request), k > 0 = batch sizes 1..k and max_batch,
                                 -1 = max_batch only.  Cost: one hipGraph capture per (worker,
                                 batch size), serialised process-wide -- e.g. 4 workers x 32 sizes
                                 per device for ResNet-152 bs32; a zeroed struct asks for all of
                                 them.  spi_runtime_warmup_seconds() reports what it took. */
  int32_t _pad0;
} spi_runtime_config;

/* Fills the defaults above (FIXED batching, one job per task, SPI_H2D_AUTO,
 * every batch size warmed up).  A zeroed struct means the same, except the H2D
 * mode: 0 is SPI_H2D_DEVICE_STREAM, only spi_runtime_config_init selects AUTO. */
void spi_runtime_config_init(spi_runtime_config* config);

spi_runtime* spi_runtime_create(const spi_runtime_config* config, char* err, size_t errlen);

typedef struct spi_job_desc {
  int32_t request_id;
  int32_t fixed_worker;   /* -1: any worker; else a global worker index */
  int32_t has_priority;   /* 0: priority = max(min_prio, max_prio - request_id) */
  int32_t priority;
  int64_t batch;
  const void* const* inputs;  /* host, valid until the callback */
  void* const* outputs;       /* host, valid until the callback */
  spi_job_done_fn done;
  void* user;
} spi_job_desc;

int spi_runtime_submit_job(spi_runtime* rt, const spi_job_desc* job);
/* Shorthand: any worker, default priority. */
int spi_runtime_submit(spi_runtime* rt, int32_t request_id, int64_t batch, const void* const* inputs,
                       void* const* outputs, spi_job_done_fn done, void* user);
/* Block until every submitted job has completed. */
int spi_runtime_drain(spi_runtime* rt);
void spi_runtime_stats(const spi_runtime* rt, int64_t* completed, int64_t* failed);
int32_t spi_runtime_num_workers(const spi_runtime* rt);
/* Measurement hook: where worker `worker`'s thread spent its time so far --
 * out[0] tasks launched, out[1] ns waiting for a free slot, out[2] ns of host
 * staging (copy_job_inputs_to_slot), out[3] ns enqueueing H2D + codelet + D2H,
 * out[4] ns waiting on completion events.  Returns SPI_OK or an error status. */
int spi_runtime_worker_times(const spi_runtime* rt, int32_t worker, int64_t* out);
/* The H2D mode the runtime resolved (SPI_H2D_AUTO -> one of the concrete modes). */
int32_t spi_runtime_h2d_mode(const spi_runtime* rt);
/* Current adaptive target batch limit (samples); the fixed limit otherwise. */
int32_t spi_runtime_batch_target(const spi_runtime* rt);
/* Wall time spi_runtime_create spent in the per-worker warm-up (graph captures, workspaces). */
double spi_runtime_warmup_seconds(const spi_runtime* rt);
void spi_runtime_destroy(spi_runtime* rt);

/* ---------------------------------------------------------------------------
 * Load generator: the reference client's measurement loop
 * (src/grpc/client/inference_client.cpp:259-270, client_main.cpp schedules,
 * src/core/latency_statistics.hpp:52-93), in C++ so no interpreter sits on
 * the measured path.  Every request is `request_batch` samples read from the
 * same caller-owned host inputs (pageable, like a received request).
 *   closed loop (num_segments == 0): keep `inflight` requests outstanding;
 *   open loop: send requests on the schedule (delta_us, repeat) segments
 *   (ci/perf/ci_perf_resnet.csv), rejections (queue full) counted.
 * ------------------------------------------------------------------------- */
typedef struct spi_schedule_segment {
  int64_t delta_us;
  int64_t repeat;
} spi_schedule_segment;

typedef struct spi_loadgen_config {
  int64_t requests;        /* closed loop: requests to complete */
  int32_t inflight;        /* closed loop: outstanding requests */
  int32_t num_segments;    /* 0 = closed loop */
  const spi_schedule_segment* segments;
  int64_t request_batch;   /* samples per request */
  int32_t warmup_requests; /* sent and drained first, not measured */
  int32_t _pad;
} spi_loadgen_config;

typedef struct spi_loadgen_result {
  int64_t completed, failed, rejected;
  int64_t inferences;
  double seconds;            /* last response - first request */
  double inferences_per_s;
  double p50_ms, p95_ms, p99_ms, mean_ms, max_ms;
  double mean_jobs_per_task, mean_task_batch;
  double p50_queue_ms;       /* submit -> dequeue */
  /* latency breakdown (CLOCK_MONOTONIC stamps of spi_job_timing): queue = submit -> dequeue,
     stage = dequeue -> codelet start (slot, host staging, H2D), device = codelet start ->
     outputs in the caller's buffers (kernels, D2H, completion wait, slicing) */
  double p99_queue_ms, p50_stage_ms, p99_stage_ms, p50_device_ms, p99_device_ms;
  double worst_at_frac;      /* submit time of the slowest request, as a fraction of the run */
  char error[SPI_ERROR_LEN];
} spi_loadgen_result;

int spi_runtime_loadgen(spi_runtime* rt, const spi_loadgen_config* config, const void* const* inputs,
                        spi_loadgen_result* result);

#ifdef __cplusplus
}
#endif
#endif /* SPI_RUNTIME_H */
