/*
 * spi_torch.h — the LibTorch side of the boundary: TorchScript loading, the
 * CPU codelet's forward, and the C++ weight extractor that feeds
 * spi_model_create.  Built as libspi_torch.so (links libtorch_cpu + libspi_hip),
 * so libspi_hip.so itself never depends on LibTorch.
 *
 * Reference interfaces each entry point replaces:
 *
 *   spi_torch_load            <- load_model (torch::jit::load + eval)
 *                                src/core/inference_runner.cpp:243-249
 *   spi_torch_cpu_forward     <- the body of run_inference on the CPU codelet:
 *                                forward under c10::InferenceMode, IValue
 *                                flattening (append_ivalue), output-count check
 *                                and TensorBuilder::copy_output_to_buffer
 *                                src/core/starpu_setup.cpp:594-624, 784-801,
 *                                496-513; src/core/tensor_builder.cpp:162-190.
 *                                It is an spi_cpu_forward_fn: the host puts it in
 *                                spi_codelet_args.cpu_forward with model_cpu =
 *                                the spi_torch_module*, and spi_cpu_inference_func
 *                                does the views, stamps and buffer checks.
 *   spi_torch_named_tensors   <- named_parameters()/named_buffers() of the
 *                                loaded module (what clone_model_to_gpus copies,
 *                                inference_runner.cpp:251-275), as fp32 arrays
 *   spi_torch_create_replica  <- clone_model_to_gpus for one device: extract +
 *                                spi_model_create (BN-fold, pack, upload)
 *   spi_torch_cpu_bench       <- N StarPU CPU workers draining a closed loop of
 *                                CPU-codelet tasks; inf/s = inferences /
 *                                (last response - first request)
 *                                (src/grpc/client/inference_client.cpp:259-270),
 *                                linear-interpolated percentiles
 *                                (src/core/latency_statistics.hpp:52-93).
 *                                Worker layouts: one worker with all cores as
 *                                intra-op threads (group_cpu_by_numa,
 *                                starpu_setup.cpp:299-385) or one per NUMA node.
 */
#ifndef SPI_TORCH_H
#define SPI_TORCH_H

#include "spi_codelet.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct spi_torch_module spi_torch_module;

spi_torch_module* spi_torch_load(const char* path, char* err, size_t errlen);
void spi_torch_free(spi_torch_module* module);

/* spi_cpu_forward_fn over a spi_torch_module* (see above). */
int spi_torch_cpu_forward(void* model_cpu, const spi_tensor_view* inputs, int num_inputs,
                          spi_tensor_view* outputs, int num_outputs, char* err, size_t errlen);

/* Floating named_parameters() then named_buffers() (first occurrence of a name
 * wins), each copied to contiguous fp32 and owned by the module handle.
 * Returns the count, or -1 on error. */
int32_t spi_torch_named_tensors(spi_torch_module* module, const spi_named_tensor** out);

spi_model* spi_torch_create_replica(spi_torch_module* module, int32_t device_id,
                                    const spi_model_config* config, char* err, size_t errlen);

/* at::set_num_threads / at::get_num_threads for the calling thread. */
void spi_torch_set_num_threads(int32_t n);
int32_t spi_torch_get_num_threads(void);

typedef struct spi_cpu_bench_result {
  int64_t tasks;            /* codelet calls completed */
  int64_t inferences;       /* tasks x batch */
  double seconds;           /* last response - first request */
  double inferences_per_s;
  double p50_ms, p95_ms;    /* per-task codelet latency */
  int32_t failed;
  char error[SPI_ERROR_LEN];
} spi_cpu_bench_result;

/* Closed loop through spi_cpu_inference_func: `workers` threads, each with
 * `threads_per_worker` intra-op threads and its own copy of the inputs
 * (host views, dims from the layout), run tasks until `seconds` have passed
 * or `max_tasks` tasks completed (0 = no cap).  `inputs` describe one batch;
 * outputs are sized from output_bytes. */
int spi_torch_cpu_bench(spi_torch_module* module, const spi_tensor_view* inputs, int32_t num_inputs,
                        const size_t* output_bytes, const int32_t* output_types, int32_t num_outputs,
                        int32_t workers, int32_t threads_per_worker, double seconds, int64_t max_tasks,
                        spi_cpu_bench_result* result);

#ifdef __cplusplus
}
#endif
#endif /* SPI_TORCH_H */
