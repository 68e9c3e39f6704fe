/*
 * spi_codelet.h — C-ABI drop-in boundary of the MI355X inference codelet.
 *
 * This header is the whole contract between a StarPU-Inference-Server style
 * host (task submission, slot pools, StarPU workers) and the HIP/CDNA4
 * forward pass.  It carries no C++ and no torch types: plain pointers, sizes,
 * fixed-size arrays and C function pointers.
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference repository daxmawal/StarPU-Inference-Server):
 *
 *   spi_hip_inference_func   <- InferenceCodelet::cuda_inference_func
 *                               src/core/starpu_setup.cpp:807-846
 *   spi_cpu_inference_func   <- InferenceCodelet::cpu_inference_func
 *                               src/core/starpu_setup.cpp:784-801
 *   spi_codelet_init         <- InferenceCodelet::InferenceCodelet
 *                               src/core/starpu_setup.cpp:559-568
 *   spi_codelet_args         <- struct InferenceParams
 *                               src/core/inference_params.hpp:20-92
 *   spi_buffer_byte_size     <- starpu_setup_detail::buffer_byte_size
 *                               src/core/starpu_setup.cpp:515-542
 *   spi_select_replica       <- select_gpu_module
 *                               src/core/starpu_setup.cpp:725-778
 *   spi_model_create         <- clone_model_to_gpus / load_model
 *                               src/core/inference_runner.cpp:243-275
 *                               (one device-resident weight replica per device)
 *
 * Buffer convention (src/core/inference_task.cpp:802-822): buffers[0..ni) are
 * the inputs (STARPU_R), buffers[ni..ni+no) the outputs (STARPU_W); each
 * buffers[i] points at a StarPU vector or variable interface whose layout is
 * mirrored below.  On a GPU worker `ptr` is a device (HBM) address.
 *
 * Errors never cross this ABI as exceptions (the reference throws
 * StarPUCodeletException through StarPU's C frames, starpu_setup.cpp:710-716):
 * they are returned in args->status / args->error, and the host adapter turns
 * them into its own exception type.
 */
#ifndef SPI_CODELET_H
#define SPI_CODELET_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPI_ABI_VERSION 1u

/* src/utils/inference_limits.hpp:6-8 */
#define SPI_MAX_INPUTS 16
#define SPI_MAX_OUTPUTS 16
#define SPI_MAX_DIMS 8
#define SPI_MAX_REPLICAS 32
#define SPI_ERROR_LEN 256

/* ---------------------------------------------------------------------------
 * StarPU 1.4 data-interface layouts (starpu_data_interfaces.h).  The codelet
 * reads only id, ptr, nx and elemsize, exactly like the reference
 * (starpu_setup.cpp:515-542, tensor_builder.cpp:120).  The id values follow
 * StarPU 1.4's enum starpu_data_interface_id; a build against the real
 * <starpu.h> static_asserts them (csrc/spi_starpu_adapter.cpp, -DSPI_WITH_STARPU).
 * ------------------------------------------------------------------------- */
enum spi_interface_id {
  SPI_STARPU_MATRIX_INTERFACE_ID = 0,
  SPI_STARPU_BLOCK_INTERFACE_ID = 1,
  SPI_STARPU_VECTOR_INTERFACE_ID = 2,
  SPI_STARPU_CSR_INTERFACE_ID = 3,
  SPI_STARPU_BCSR_INTERFACE_ID = 4,
  SPI_STARPU_VARIABLE_INTERFACE_ID = 5
};

/* Field widths: StarPU 1.4 declares the vector's nx (and slice_base) size_t --
 * its register call takes `size_t nx`, which the reference's own link-time
 * override of starpu_vector_data_register has to match exactly
 * (tests/support/starpu_task_submit_override.cpp:117-119; the Dockerfile pins
 * StarPU 1.4.8, Dockerfile:58).  A resize writes the full 8 bytes
 * (resize_starpu_vector_interface, starpu_vector_resize_utils.hpp:19-64). */
typedef struct spi_vector_interface {
  int32_t id; /* enum starpu_data_interface_id */
  uintptr_t ptr;
  uintptr_t dev_handle;
  size_t offset;
  size_t nx;
  size_t elemsize;
  size_t slice_base;
  size_t allocsize;
} spi_vector_interface;

typedef struct spi_variable_interface {
  int32_t id;
  uintptr_t ptr;
  uintptr_t dev_handle;
  size_t offset;
  size_t elemsize;
} spi_variable_interface;

/* Element types use at::ScalarType's numeric codes, so a LibTorch caller can
 * pass static_cast<int>(scalar_type) (datatype_utils.hpp:20-46). */
enum spi_dtype {
  SPI_DTYPE_U8 = 0,
  SPI_DTYPE_I8 = 1,
  SPI_DTYPE_I16 = 2,
  SPI_DTYPE_I32 = 3,
  SPI_DTYPE_I64 = 4,
  SPI_DTYPE_F16 = 5,
  SPI_DTYPE_F32 = 6,
  SPI_DTYPE_F64 = 7,
  SPI_DTYPE_BOOL = 11,
  SPI_DTYPE_BF16 = 15
};

/* DeviceType (src/core/device_type.hpp) */
enum spi_device_type { SPI_DEVICE_UNKNOWN = 0, SPI_DEVICE_CPU = 1, SPI_DEVICE_GPU = 2 };

/* Status codes mirroring the reference exception taxonomy
 * (src/utils/exceptions.hpp:11-157). */
enum spi_status {
  SPI_OK = 0,
  SPI_ERR_INVALID_ARGUMENT = 1,   /* InferenceExecutionException (layout/limits) */
  SPI_ERR_NO_REPLICA = 2,         /* "No GPU model replica available ..." */
  SPI_ERR_OUTPUT_MISMATCH = 3,    /* "Output buffer size mismatch in bytes" */
  SPI_ERR_UNSUPPORTED = 4,        /* unsupported interface id / dtype / model */
  SPI_ERR_DEVICE = 5,             /* HIP runtime error */
  SPI_ERR_MODEL = 6,              /* model recognition / weight packing */
  SPI_ERR_CPU_FORWARD = 7         /* host forward callback failed */
};

/* Opaque per-device weight replica (BN-folded, MFMA-packed, in HBM). */
typedef struct spi_model spi_model;

/* One host-side view handed to the CPU forward callback. */
typedef struct spi_tensor_view {
  void* data;
  int32_t dtype;
  int32_t ndim;
  int64_t shape[SPI_MAX_DIMS];
} spi_tensor_view;

/* CPU forward (the reference's LibTorch model_cpu->forward): the host binds
 * its own CPU model here; the codelet does views, stamps and checked copies.
 * Returns 0 on success; on failure writes a message into err. */
typedef int (*spi_cpu_forward_fn)(void* model_cpu, const spi_tensor_view* inputs,
                                  int num_inputs, spi_tensor_view* outputs,
                                  int num_outputs, char* err, size_t errlen);

/* The cl_arg block (InferenceParams, inference_params.hpp:77-92), as POD.
 * The caller owns it for the task's lifetime (inference_task.hpp:41-64). */
typedef struct spi_codelet_args {
  uint32_t abi_version; /* = SPI_ABI_VERSION */
  uint32_t num_inputs;
  uint32_t num_outputs;
  int32_t request_id;
  int64_t batch_size;
  int32_t verbosity;
  int32_t _pad0;

  /* TensorLayout: dims[i][0] is the effective batch
   * (inference_task.cpp:606-613). */
  int64_t dims[SPI_MAX_INPUTS][SPI_MAX_DIMS];
  int64_t num_dims[SPI_MAX_INPUTS];
  int32_t input_types[SPI_MAX_INPUTS];
  /* expected output element types (copy_output_to_buffer's expected_type) */
  int32_t output_types[SPI_MAX_OUTPUTS];

  /* Limits */
  uint64_t max_inputs;
  uint64_t max_dims;

  /* ModelPointers: replica i serves device_ids[i] (or worker_ids[i]). */
  void* model_cpu;
  spi_cpu_forward_fn cpu_forward;
  int32_t num_replicas;
  int32_t num_device_ids;
  int32_t num_worker_ids;
  int32_t _pad1;
  int32_t device_ids[SPI_MAX_REPLICAS];
  int32_t worker_ids[SPI_MAX_REPLICAS];
  spi_model* models_gpu[SPI_MAX_REPLICAS];

  /* Timing out-fields: CLOCK_MONOTONIC nanoseconds (MonotonicClock). */
  int64_t codelet_start_ns;
  int64_t codelet_end_ns;
  int64_t inference_start_ns;

  /* DeviceInfo out-fields */
  int32_t executed_on; /* enum spi_device_type */
  int32_t worker_id;
  int32_t device_id;

  /* Result */
  int32_t status;
  char error[SPI_ERROR_LEN];
} spi_codelet_args;

/* ---------------------------------------------------------------------------
 * Codelet entry points (starpu_cpu_func_t / starpu_hip_func_t signature).
 * ------------------------------------------------------------------------- */

/* GPU codelet: enqueues the whole forward pass on the worker's HIP stream and
 * returns without synchronising (STARPU_HIP_ASYNC).  Outputs are written by the
 * last kernel straight into the W buffers. */
void spi_hip_inference_func(void** buffers, void* cl_arg);

/* CPU codelet: views over host buffers -> args->cpu_forward -> checked memcpy
 * (tensor_builder.cpp:162-190). */
void spi_cpu_inference_func(void** buffers, void* cl_arg);

/* Fills a `struct starpu_codelet` (passed as void*) when the library is built
 * with <starpu.h> (SPI_WITH_STARPU); returns SPI_ERR_UNSUPPORTED otherwise. */
int spi_codelet_init(void* starpu_codelet);

/* Worker context for the calling thread: what starpu_worker_get_id(),
 * starpu_worker_get_devid() and starpu_hip_get_local_stream() return inside a
 * StarPU worker.  The mini-runtime and tests set it; with SPI_WITH_STARPU the
 * codelet queries StarPU instead when no context was set. */
void spi_set_worker_context(int32_t worker_id, int32_t device_id, void* hip_stream);
void spi_clear_worker_context(void);

/* Helpers that mirror reference utilities (exposed for host-side tests). */
int spi_buffer_byte_size(const void* buffer_iface, size_t* out_bytes);
int spi_select_replica(const spi_codelet_args* args, int32_t worker_id,
                       int32_t device_id, int32_t* out_index);
size_t spi_dtype_size(int32_t dtype);
void spi_args_init(spi_codelet_args* args);

/* ---------------------------------------------------------------------------
 * Model replicas.
 * ------------------------------------------------------------------------- */
enum spi_family {
  SPI_FAMILY_AUTO = 0,   /* recognise from parameter names */
  SPI_FAMILY_RESNET = 1, /* torchvision resnet18/34/50/101/152 naming */
  SPI_FAMILY_BERT = 2,   /* HF BertModel naming, returns last_hidden_state */
  SPI_FAMILY_VIT = 3,    /* torchvision vit_*_16 naming */
  SPI_FAMILY_AFFINE = 4  /* y = x * scale + shift (toy models of the reference tests) */
};

/* SPI_PREC_F16X3: split fp16 -- fp32 activations, each MFMA operand split into
 * hi + lo fp16 halves, hi*hi + hi*lo + lo*hi per fragment (fp32-grade
 * results at the fp16 MFMA rate).
 * SPI_PREC_F16M, ResNet: fp16 activations and fp16 MFMA operands everywhere except
 * the precision-critical layers -- the stem (the image rounded to fp16 x hi + lo
 * weights, fp16 out) and the downsample 1x1 convs (fp16 activations x hi + lo weights,
 * fp16 out); the FC runs on plain fp16 weights (round 5: CPU emulation worst case
 * 0.74e-3 over 8 input seeds against the 1e-3 bar, GPU 0.60-0.69e-3).  BERT / ViT: the
 * F16 path with hi + lo weights on every GEMM (two fp16 MFMAs per fragment pair: the
 * weights' rounding is the largest of the fp16 path's error sites,
 * tools/prec_emulate_bert.py). */
enum spi_precision { SPI_PREC_F32 = 0, SPI_PREC_F16 = 1, SPI_PREC_F16X3 = 2, SPI_PREC_F16M = 3 };

typedef struct spi_named_tensor {
  const char* name; /* parameter/buffer name as in named_parameters() */
  const void* data; /* host pointer, fp32, contiguous */
  int32_t dtype;    /* SPI_DTYPE_F32 */
  int32_t ndim;
  int64_t shape[SPI_MAX_DIMS];
} spi_named_tensor;

typedef struct spi_model_config {
  int32_t family;     /* enum spi_family */
  int32_t precision;  /* enum spi_precision: MFMA operand type */
  int32_t max_batch;  /* largest dims[0] the replica will see */
  int32_t num_heads;  /* transformers: attention heads (0 = default for family) */
  int32_t seq_len;    /* BERT: max sequence length (0 = from position table) */
  int32_t image_size; /* ResNet/ViT: input H = W (0 = 224) */
  float eps;          /* norm epsilon (0 = family default) */
  float affine_scale; /* AFFINE only */
  float affine_shift; /* AFFINE only */
  int32_t _pad;
} spi_model_config;

spi_model* spi_model_create(int32_t device_id, const spi_model_config* config,
                            const spi_named_tensor* params, int32_t num_params,
                            char* err, size_t errlen);
void spi_model_destroy(spi_model* model);
/* Device bytes of the packed weight blob. */
size_t spi_model_weight_bytes(const spi_model* model);
/* FNV-1a 64 digest of the packed weight blob (computed on the host at build
 * time): identical inputs give identical digests, whichever thread built it. */
uint64_t spi_model_weight_digest(const spi_model* model);
/* Algorithmic FLOPs of one forward at the given batch (roofline numerator). */
double spi_model_flops(const spi_model* model, int64_t batch);
/* Short description ("resnet[2,2,2,2] basic f16 ..."). */
const char* spi_model_describe(const spi_model* model);
/* Measurement hook (not on the task path): runs one forward on `stream` with
 * every kernel launch bracketed by hipEvents, synchronises, and returns the
 * number of ops; per op: device milliseconds, algorithmic FLOPs, algorithmic
 * HBM bytes and a name (name_len bytes each).  Returns -1 on error. */
int spi_model_profile(spi_model* model, void* stream, int64_t batch, int64_t seq,
                      const void* const* inputs, void* const* outputs, float* op_ms,
                      double* op_flops, double* op_bytes, char* op_names, int32_t name_len,
                      int32_t max_ops);
/* Measurement hook: the same eager forward with the op named `op_name` (its
 * first occurrence) launched `reps` times back to back between one pair of
 * hipEvents; returns its device milliseconds per launch and its algorithmic
 * FLOPs / HBM bytes per launch.  Returns 0, or -1 (unknown op, bad arguments). */
int spi_model_profile_op(spi_model* model, void* stream, int64_t batch, int64_t seq,
                         const void* const* inputs, void* const* outputs, const char* op_name,
                         int32_t reps, float* ms_per_launch, double* flops, double* bytes);
/* Measurement hook: one eager forward on `stream` with every kernel launch recorded,
 * as text, one line per launch: "op_index\top_name\tkernel\tgrid_x\tgrid_y\tgrid_z\tblock\n"
 * (grid in workgroups).  It maps a rocprofv3 kernel trace of graph-replayed forwards,
 * which names kernels and grids only, back to ops (tools/trace_ops.py --launches).
 * Writes at most buflen - 1 bytes plus a NUL; returns the full length, or -1 on error. */
int64_t spi_model_launch_table(spi_model* model, void* stream, int64_t batch, int64_t seq,
                               const void* const* inputs, void* const* outputs, char* buf, size_t buflen);
/* Capture launch-bound forwards into hipGraphs (per stream, per batch). */
void spi_model_set_graphs(spi_model* model, int32_t enable);
/* Per-worker warm-up (inference_runner.cpp:507-560): allocate `stream`'s
 * workspace and, with graphs on, capture the forward body for (batch, seq,
 * with_mask) now rather than inside a live request.  Enqueues no work.
 * seq / with_mask matter for BERT only.  Returns SPI_OK or an error status
 * (message in spi_last_error()). */
int spi_model_warmup(spi_model* model, void* stream, int64_t batch, int64_t seq, int32_t with_mask);

/* ---------------------------------------------------------------------------
 * Small device utilities so hosts without a HIP runtime binding (ctypes,
 * cgo, JNI) can allocate and move buffers.
 * ------------------------------------------------------------------------- */
int spi_device_count(void);
int spi_set_device(int32_t device_id);
void* spi_device_malloc(size_t bytes);
void spi_device_free(void* ptr);
void* spi_host_malloc(size_t bytes); /* pinned (hipHostMalloc portable) */
void spi_host_free(void* ptr);
int spi_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream);
int spi_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream);
int spi_memset_d(void* dst, int value, size_t bytes, void* stream);
void* spi_stream_create(void);
void spi_stream_destroy(void* stream);
int spi_stream_synchronize(void* stream);
const char* spi_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* SPI_CODELET_H */
