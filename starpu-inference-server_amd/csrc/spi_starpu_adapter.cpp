// StarPU adapter: the codelet descriptor and the layout contract between the
// vendored interface structs (include/spi_codelet.h) and StarPU 1.4's own.
//
// Reference: InferenceCodelet::InferenceCodelet (src/core/starpu_setup.cpp:559-568)
// fills nbuffers = STARPU_VARIABLE_NBUFFERS, type = STARPU_FORKJOIN,
// max_parallelism = INT_MAX, cpu_funcs[0], cuda_funcs[0] and cuda_flags[0] = 1
// (async).  The MI355X build registers the same CPU function and the HIP codelet
// in hip_funcs[0] with STARPU_HIP_ASYNC: the codelet only enqueues on the
// worker's stream and StarPU synchronises it before the task's callback.
//
// Built two ways:
//   * default (no StarPU on this image or the GPU box): spi_codelet_init()
//     reports SPI_ERR_UNSUPPORTED; the mini-runtime (runtime.cpp) stands in for
//     StarPU and hands the codelet its buffers the same way.
//   * -DSPI_WITH_STARPU with <starpu.h> on the include path: the static_asserts
//     below pin every field the codelet reads (id, ptr, nx, elemsize) and the
//     interface-id values against StarPU's real declarations, so a layout drift
//     is a compile error instead of a silent misread at run time.
#include <climits>
#include <cstddef>

#include "../../include/spi_codelet.h"

#ifdef SPI_WITH_STARPU
#if !__has_include(<starpu.h>)
#error "SPI_WITH_STARPU needs <starpu.h> on the include path (StarPU 1.4, Dockerfile:58 pins 1.4.8)"
#endif
#include <starpu.h>

// starpu_data_interfaces.h: enum starpu_data_interface_id
static_assert((int)STARPU_VECTOR_INTERFACE_ID == SPI_STARPU_VECTOR_INTERFACE_ID, "vector interface id");
static_assert((int)STARPU_VARIABLE_INTERFACE_ID == SPI_STARPU_VARIABLE_INTERFACE_ID, "variable interface id");
static_assert((int)STARPU_MATRIX_INTERFACE_ID == SPI_STARPU_MATRIX_INTERFACE_ID, "matrix interface id");

// struct starpu_vector_interface {id, ptr, dev_handle, offset, nx, elemsize, slice_base, allocsize}
#define SPI_SAME_FIELD(S, T, f) \
  static_assert(offsetof(S, f) == offsetof(T, f) && sizeof(((S*)0)->f) == sizeof(((T*)0)->f), #f)
SPI_SAME_FIELD(struct starpu_vector_interface, spi_vector_interface, id);
SPI_SAME_FIELD(struct starpu_vector_interface, spi_vector_interface, ptr);
SPI_SAME_FIELD(struct starpu_vector_interface, spi_vector_interface, dev_handle);
SPI_SAME_FIELD(struct starpu_vector_interface, spi_vector_interface, offset);
SPI_SAME_FIELD(struct starpu_vector_interface, spi_vector_interface, nx);
SPI_SAME_FIELD(struct starpu_vector_interface, spi_vector_interface, elemsize);
SPI_SAME_FIELD(struct starpu_vector_interface, spi_vector_interface, slice_base);
SPI_SAME_FIELD(struct starpu_vector_interface, spi_vector_interface, allocsize);
// struct starpu_variable_interface {id, ptr, dev_handle, offset, elemsize}
SPI_SAME_FIELD(struct starpu_variable_interface, spi_variable_interface, id);
SPI_SAME_FIELD(struct starpu_variable_interface, spi_variable_interface, ptr);
SPI_SAME_FIELD(struct starpu_variable_interface, spi_variable_interface, dev_handle);
SPI_SAME_FIELD(struct starpu_variable_interface, spi_variable_interface, offset);
SPI_SAME_FIELD(struct starpu_variable_interface, spi_variable_interface, elemsize);
#undef SPI_SAME_FIELD

// The codelet's C signature is exactly StarPU's function-pointer types.
static_assert(sizeof(starpu_cpu_func_t) == sizeof(&spi_cpu_inference_func), "cpu func");
#endif

extern "C" int spi_codelet_init(void* starpu_codelet) {
#ifdef SPI_WITH_STARPU
  auto* cl = static_cast<struct starpu_codelet*>(starpu_codelet);
  if (!cl) return SPI_ERR_INVALID_ARGUMENT;
  starpu_codelet_init(cl);
  cl->nbuffers = STARPU_VARIABLE_NBUFFERS;
  cl->type = STARPU_FORKJOIN;
  cl->max_parallelism = INT_MAX;
  cl->cpu_funcs[0] = &spi_cpu_inference_func;
  cl->hip_funcs[0] = &spi_hip_inference_func;
  cl->hip_flags[0] = STARPU_HIP_ASYNC;
  cl->name = "spi_inference_codelet";
  return SPI_OK;
#else
  (void)starpu_codelet;
  return SPI_ERR_UNSUPPORTED;
#endif
}
