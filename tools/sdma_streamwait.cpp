// Probe (round 4): can a HIP stream wait on the device for an HSA SDMA copy's completion
// signal, instead of the worker thread waiting on the host (runtime.cpp SPI_H2D_WORKER_SDMA)?
// hipStreamWaitValue64 on the signal's value word (hsa_amd_signal_value_pointer), then a
// kernel that reads the copied bytes.  Prints whether the API accepts the pointer, whether
// the kernel is held back until the signal drops, and whether it sees the copied data.
// Every wait on the host is bounded; the signal is always released before exit.
//   hipcc --offload-arch=gfx950 -O2 tools/sdma_streamwait.cpp -o tools/sdma_streamwait -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

__global__ void check_kernel(const int* data, int n, int* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    int ok = 1;
    for (int i = 0; i < n; ++i) ok &= data[i] == i * 7 + 1;
    out[0] = ok ? 1 : 2;
  }
}

struct Agents {
  hsa_agent_t gpu{}, cpu{};
  bool have_gpu = false, have_cpu = false;
};

int main(int argc, char** argv) {
  int can = 0;
  (void)hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0);
  std::printf("CanUseStreamWaitValue=%d\n", can);
  if (hsa_init() != HSA_STATUS_SUCCESS) return 1;
  Agents ag;
  hsa_iterate_agents(
      [](hsa_agent_t a, void* u) {
        auto* g = static_cast<Agents*>(u);
        hsa_device_type_t t;
        hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
        if (t == HSA_DEVICE_TYPE_GPU && !g->have_gpu) {
          g->gpu = a;
          g->have_gpu = true;
        }
        if (t == HSA_DEVICE_TYPE_CPU && !g->have_cpu) {
          g->cpu = a;
          g->have_cpu = true;
        }
        return HSA_STATUS_SUCCESS;
      },
      &ag);
  if (!ag.have_gpu || !ag.have_cpu) return 2;
  const int n = 1 << 20;  // 4 MiB
  int *h = nullptr, *d = nullptr, *flag = nullptr;
  (void)hipHostMalloc((void**)&h, n * sizeof(int), hipHostMallocPortable);
  (void)hipMalloc((void**)&d, n * sizeof(int));
  (void)hipHostMalloc((void**)&flag, sizeof(int), hipHostMallocPortable);
  for (int i = 0; i < n; ++i) h[i] = i * 7 + 1;
  (void)hipMemset(d, 0, n * sizeof(int));
  *flag = 0;
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  (void)hipDeviceSynchronize();

  // hsa_amd_signal_value_pointer needs an HSA_AMD_SIGNAL_AMD_GPU_ONLY or _IPC signal (a plain
  // hsa_signal_create one returns INVALID_ARGUMENT): argv[1] = attribute bits (default 1)
  const uint64_t attr = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : 1;
  hsa_signal_t sig;
  const hsa_status_t cs0 = hsa_amd_signal_create(1, 0, nullptr, attr, &sig);
  volatile hsa_signal_value_t* vp = nullptr;
  const hsa_status_t ps = hsa_amd_signal_value_pointer(sig, &vp);
  std::printf("attributes=%llu create status=%d signal_value_pointer status=%d ptr=%p\n", (unsigned long long)attr,
              (int)cs0, (int)ps, (void*)vp);
  if (ps != HSA_STATUS_SUCCESS) return 0;  // not usable: reported above
  const hipError_t we = hipStreamWaitValue64(s, (void*)vp, 0, hipStreamWaitValueEq, ~0ull);
  std::printf("hipStreamWaitValue64 -> %s\n", hipGetErrorString(we));
  hipLaunchKernelGGL(check_kernel, dim3(1), dim3(64), 0, s, d, n, flag);
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  std::printf("before copy: kernel ran=%d (stream query %s)\n", *flag, hipGetErrorString(hipStreamQuery(s)));
  const auto t0 = std::chrono::steady_clock::now();
  const hsa_status_t cs = hsa_amd_memory_async_copy(d, ag.gpu, h, ag.cpu, n * sizeof(int), 0, nullptr, sig);
  std::printf("async_copy status=%d\n", (int)cs);
  bool done = false;
  for (int i = 0; i < 2000 && !done; ++i) {  // bounded: 2 s
    done = hipStreamQuery(s) == hipSuccess;
    if (!done) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  std::printf("after copy: stream done=%d flag=%d (1 = data seen) in %.0f us, signal=%ld\n", done, *flag, us,
              (long)hsa_signal_load_scacquire(sig));
  if (!done) {
    hsa_signal_store_screlease(sig, 0);  // never leave the queue waiting
    for (int i = 0; i < 2000 && hipStreamQuery(s) != hipSuccess; ++i)
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    std::printf("released by host: flag=%d\n", *flag);
  }
  // latency: copy issued while the kernel is already queued behind the wait, repeated
  double tot = 0;
  int good = 0;
  for (int r = 0; r < 20; ++r) {
    hsa_signal_store_screlease(sig, 1);
    *flag = 0;
    (void)hipMemsetAsync(d, 0, n * sizeof(int), s);
    (void)hipStreamSynchronize(s);
    (void)hipStreamWaitValue64(s, (void*)vp, 0, hipStreamWaitValueEq, ~0ull);
    hipLaunchKernelGGL(check_kernel, dim3(1), dim3(64), 0, s, d, n, flag);
    const auto a = std::chrono::steady_clock::now();
    hsa_amd_memory_async_copy(d, ag.gpu, h, ag.cpu, n * sizeof(int), 0, nullptr, sig);
    bool ok = false;
    for (int i = 0; i < 20000 && !ok; ++i) ok = hipStreamQuery(s) == hipSuccess;
    if (!ok) {
      hsa_signal_store_screlease(sig, 0);
      (void)hipStreamSynchronize(s);
    }
    tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    good += ok && *flag == 1;
  }
  std::printf("20 rounds: %d correct, mean copy+kernel %.0f us\n", good, tot / 20);
  hsa_signal_store_screlease(sig, 0);
  (void)hipStreamSynchronize(s);
  hsa_signal_destroy(sig);
  (void)hipStreamDestroy(s);
  (void)hipFree(d);
  (void)hipHostFree(h);
  (void)hipHostFree(flag);
  return 0;
}
