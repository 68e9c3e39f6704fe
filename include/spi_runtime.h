/*
 * spi_runtime.h — a minimal StarPU stand-in that drives the HIP codelet.
 *
 * Reproduces the task path around the codelet:
 *   submit        SlotManager::submit_inference_task   slot_manager_component.cpp:517-647
 *   eager queue   STARPU_SCHED=eager, one shared queue  models/resnet18.yml:3
 *   workers       STARPU_NWORKER_PER_CUDA workers per device, one HIP stream each
 *   slots         InputSlotPool / OutputSlotPool: pinned (hipHostMalloc portable)
 *                 host buffers sized max_batch x per-sample bytes
 *                 (input_slot_pool.cpp:77-215, output_slot_pool.cpp:287-330)
 *   staging       copy_job_inputs_to_slot (memcpy into the pinned slot, :649-727),
 *                 then hipMemcpyAsync H2D on the worker stream (StarPU's R fetch)
 *   resize        nx = batch x per-sample (starpu_vector_resize_utils.hpp:66-89)
 *   codelet       spi_hip_inference_func with the worker context set
 *   output        hipMemcpyAsync D2H + stream sync (starpu_data_acquire_cb(R),
 *                 inference_task.cpp:907-935), copy to the caller's buffer,
 *                 completion callback with the latency breakdown
 *   queue full    SPI_ERR_QUEUE_FULL (RESOURCE_EXHAUSTED, docs/server_guide.md:120)
 *   batching      (coalesce_max_jobs > 1) a worker merges queued jobs into one task
 *                 while the samples fit max_batch: inputs concatenated along
 *                 dim 0 into the slot (TensorBatchCompositionPolicy::
 *                 merge_input_tensors, batch_composition_policy.cpp:153-193),
 *                 one codelet call, outputs sliced back per job
 *                 (slice_outputs_for_sub_job, batching_helpers.hpp:75-125;
 *                 ResultDispatcher::propagate_completion_to_sub_jobs,
 *                 result_dispatcher_component.cpp:678-740)
 */
#ifndef SPI_RUNTIME_H
#define SPI_RUNTIME_H

#include "spi_codelet.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SPI_ERR_QUEUE_FULL 8

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
  int32_t coalesce_max_jobs;  /* <= 1: one job per codelet call; N: merge up to N queued jobs */
  int32_t coalesce_delay_us;  /* how long a worker waits for more jobs to fill max_batch */
} spi_runtime_config;

spi_runtime* spi_runtime_create(const spi_runtime_config* config, char* err, size_t errlen);
/* Host input/output pointers must stay valid until the callback runs. */
int spi_runtime_submit(spi_runtime* rt, int32_t request_id, int64_t batch, const void* const* inputs,
                       void* const* outputs, spi_job_done_fn done, void* user);
/* Block until every submitted job has completed. */
int spi_runtime_drain(spi_runtime* rt);
void spi_runtime_stats(const spi_runtime* rt, int64_t* completed, int64_t* failed);
void spi_runtime_destroy(spi_runtime* rt);

#ifdef __cplusplus
}
#endif
#endif /* SPI_RUNTIME_H */
