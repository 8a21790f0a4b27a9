// queue_probe.hip -- measurement tool (not product code): do kernels on N
// separate HIP streams run concurrently, or do streams share a hardware queue
// and serialise?  Each stream gets one bounded spin kernel (one wave, spins on
// s_memrealtime for a fixed tick count, then exits); the kernels' own start /
// end ticks give the overlap.  Streams are made the way gevws_ctx_create makes
// its stream (non-blocking, default priority), or with priorities cycling
// over the device's range.  Run once per GPU_MAX_HW_QUEUES setting.
// Second experiment ("pairs"): one host thread per stream makes R passes of
// two dependent kernels (10 us each) and waits for each pass, as the live
// server's loops do with the decode and handler launches; the gap between
// the first kernel's end and the second's start is reported, with the second
// launched normally and with hipExtAnyOrderLaunch (no barrier: the kernels
// are independent here).
//   hipcc --offload-arch=gfx950 -O2 -o tools/queue_probe tools/queue_probe.hip && tools/queue_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <thread>
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
  // ---- pairs
  const uint64_t pspin = 1000;  // 10 us
  const int R = 200;
  for (int any = 0; any < 2; ++any) {
    for (int n : {1, 4, 8, 16}) {
      std::vector<hipStream_t> s(n);
      const int span = lo - hi + 1;
      for (int i = 0; i < n; ++i) CK(hipStreamCreateWithPriority(&s[i], hipStreamNonBlocking, hi + i % span));
      uint64_t* t = nullptr;
      CK(hipMalloc(&t, (size_t)n * R * 4 * sizeof(uint64_t)));
      std::vector<std::thread> th;
      for (int i = 0; i < n; ++i)
        th.emplace_back([&, i]() {
          for (int r = 0; r < R; ++r) {
            uint64_t* o = t + ((size_t)i * R + r) * 4;
            k_spin<<<1, 64, 0, s[i]>>>(pspin, o);
            if (any)
              hipExtLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s[i], nullptr, nullptr, hipExtAnyOrderLaunch, pspin,
                                    o + 2);
            else
              k_spin<<<1, 64, 0, s[i]>>>(pspin, o + 2);
            CK(hipStreamSynchronize(s[i]));
          }
        });
      for (auto& x : th) x.join();
      std::vector<uint64_t> h((size_t)n * R * 4);
      CK(hipMemcpy(h.data(), t, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
      std::vector<double> gaps;
      for (size_t k = 0; k < (size_t)n * R; ++k)
        gaps.push_back(((double)h[4 * k + 2] - (double)h[4 * k + 1]) / 100.0);  // us; < 0: overlapped
      std::sort(gaps.begin(), gaps.end());
      double mean = 0;
      for (double g : gaps) mean += g;
      mean /= gaps.size();
      printf("{\"gpu_max_hw_queues\": \"%s\", \"pairs_streams\": %d, \"second_launch\": \"%s\", "
             "\"gap_us_mean\": %.1f, \"gap_us_p50\": %.1f, \"gap_us_p90\": %.1f}\n",
             q ? q : "default", n, any ? "hipExtAnyOrderLaunch" : "ordered", mean, gaps[gaps.size() / 2],
             gaps[gaps.size() * 9 / 10]);
      CK(hipFree(t));
      for (auto& x : s) CK(hipStreamDestroy(x));
    }
  }
  CK(hipFree(d));
  return 0;
}
