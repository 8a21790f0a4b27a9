// queue_probe.hip -- measurement tool (not product code): do kernels on N
// separate HIP streams run concurrently, or do streams share a hardware queue
// and serialise?  Each stream gets one bounded spin kernel (one wave, spins on
// s_memrealtime for a fixed tick count, then exits); the kernels' own start /
// end ticks give the overlap.  Streams are made the way gevws_ctx_create makes
// its stream (non-blocking, default priority), or with priorities cycling
// over the device's range.  Run once per GPU_MAX_HW_QUEUES setting.
//   hipcc --offload-arch=gfx950 -O2 -o tools/queue_probe tools/queue_probe.hip && tools/queue_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                        \
  do {                                                               \
    if ((x) != hipSuccess) {                                         \
      fprintf(stderr, "%s failed at line %d\n", #x, __LINE__);       \
      exit(1);                                                       \
    }                                                                \
  } while (0)

__global__ void k_spin(uint64_t ticks, uint64_t* out) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t t = t0;
  for (int i = 0; i < (1 << 22) && t - t0 < ticks; ++i) {  // bounded either way
    __builtin_amdgcn_s_sleep(4);
    t = __builtin_amdgcn_s_memrealtime();
  }
  if (threadIdx.x == 0) {
    out[0] = t0;
    out[1] = t;
  }
}

int main() {
  const uint64_t spin = 20000;  // s_memrealtime runs at 100 MHz: 200 us
  const int counts[] = {1, 2, 4, 8, 16};
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  uint64_t* d = nullptr;
  CK(hipMalloc(&d, 2 * 16 * sizeof(uint64_t)));
  const char* q = getenv("GPU_MAX_HW_QUEUES");
  for (int mode = 0; mode < 2; ++mode) {
    for (int n : counts) {
      std::vector<hipStream_t> s(n);
      for (int i = 0; i < n; ++i) {
        if (mode == 0) {
          CK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
        } else {
          const int span = lo - hi + 1;  // hi is the greatest (most negative) priority
          CK(hipStreamCreateWithPriority(&s[i], hipStreamNonBlocking, hi + i % span));
        }
      }
      for (int i = 0; i < n; ++i) k_spin<<<1, 64, 0, s[i]>>>(1, d + 2 * i);  // the queues exist from here
      CK(hipDeviceSynchronize());
      for (int i = 0; i < n; ++i) k_spin<<<1, 64, 0, s[i]>>>(spin, d + 2 * i);
      CK(hipDeviceSynchronize());
      std::vector<uint64_t> h(2 * n);
      CK(hipMemcpy(h.data(), d, 2 * n * sizeof(uint64_t), hipMemcpyDeviceToHost));
      uint64_t first = ~0ull, last = 0;
      for (int i = 0; i < n; ++i) {
        first = std::min(first, h[2 * i]);
        last = std::max(last, h[2 * i + 1]);
      }
      int concurrent = 0;  // most kernels running at one kernel's start
      for (int i = 0; i < n; ++i) {
        int c = 0;
        for (int j = 0; j < n; ++j) c += h[2 * j] <= h[2 * i] && h[2 * i] < h[2 * j + 1];
        concurrent = std::max(concurrent, c);
      }
      printf("{\"gpu_max_hw_queues\": \"%s\", \"streams\": %d, \"priorities\": \"%s\", \"span_us\": %.1f, "
             "\"serial_us\": %.1f, \"max_concurrent\": %d}\n",
             q ? q : "default", n, mode ? "cycling" : "same (as gevws_ctx_create)", (last - first) / 100.0,
             n * spin / 100.0, concurrent);
      for (auto& x : s) CK(hipStreamDestroy(x));
    }
  }
  CK(hipFree(d));
  return 0;
}
