// gevws_device.hip -- the context and the device half of the C ABI declared
// in include/gevws.h (the host mirror of the websocket plugin is
// gevws_host.cpp), plus the synthetic-batch generator / verifier the bench
// and the full-size parity tests use.  The kernels of the hot path live in
// gevws_walk.hip (header walk, records), gevws_unmask.hip (payload unmask)
// and gevws_encode.hip (encode, control-frame dispatch); gevws_kernels.hpp
// holds what they share.
#include <atomic>
#include <cstdlib>
#include <cstring>

#include "gevws_internal.hpp"

namespace {

// ------------------------------------------------------------------ synthetic frames
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ u32x4 plain16(uint64_t seed, uint64_t g, uint64_t i) {
  const uint64_t b = seed ^ (g * 0x9E3779B97F4A7C15ull);
  const uint64_t w0 = splitmix64(b + (i >> 3));
  const uint64_t w1 = splitmix64(b + (i >> 3) + 1);
  return u32x4{(uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)};
}

__device__ __forceinline__ uint32_t synth_hlen(const gevws_synth_desc& d) {
  return 2 + (d.len_form == 7 ? 0 : (d.len_form == 16 ? 2 : 8)) + (d.masked ? 4 : 0);
}

__global__ __launch_bounds__(256) void k_synth(uint8_t* __restrict__ in,
                                               const gevws_synth_desc* __restrict__ desc,
                                               uint64_t n_frames, uint64_t seed) {
  for (uint64_t g = blockIdx.x; g < n_frames; g += gridDim.x) {
    const gevws_synth_desc d = desc[g];
    const uint32_t hlen = synth_hlen(d);
    uint8_t* h = in + d.hdr_off;
    if (threadIdx.x == 0) {
      h[0] = d.b0;
      const uint8_t mbit = d.masked ? 0x80 : 0;
      uint32_t e = 2;
      if (d.len_form == 7) {
        h[1] = mbit | (uint8_t)d.length;
      } else if (d.len_form == 16) {
        h[1] = mbit | 126;
        h[2] = (uint8_t)(d.length >> 8);
        h[3] = (uint8_t)d.length;
        e = 4;
      } else {
        h[1] = mbit | 127;
        for (int k = 0; k < 8; ++k) h[2 + k] = (uint8_t)(d.length >> (56 - 8 * k));
        e = 10;
      }
      if (d.masked)
        for (int k = 0; k < 4; ++k) h[e + k] = (uint8_t)(d.mask >> (8 * k));
    }
    uint8_t* pl = h + hlen;
    const uint32_t key = d.masked ? d.mask : 0u;
    for (uint64_t i = (uint64_t)threadIdx.x * 16; i < d.length; i += 256 * 16) {
      const u32x4 x = plain16(seed, g, i) ^ key;
      if (i + 16 <= d.length) {
        __builtin_memcpy(pl + i, &x, 16);
      } else {
        for (uint32_t b = 0; b < d.length - i; ++b) pl[i + b] = (uint8_t)(x[b >> 2] >> (8 * (b & 3)));
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_synth_verify(const gevws_synth_desc* __restrict__ desc,
                                                      uint64_t n_frames, uint64_t seed,
                                                      const gevws_frame* __restrict__ frames,
                                                      const uint8_t* __restrict__ payload,
                                                      uint64_t payload_cap,
                                                      unsigned long long* __restrict__ mismatch) {
  uint64_t bad = 0;
  for (uint64_t g = blockIdx.x; g < n_frames; g += gridDim.x) {
    const gevws_synth_desc d = desc[g];
    const gevws_frame fr = frames[g];
    if (fr.payload_off > payload_cap || round16(d.length) > payload_cap - fr.payload_off) {
      bad += threadIdx.x == 0 ? d.length + 1 : 0;  // record out of range: never dereferenced
      continue;
    }
    if (threadIdx.x == 0) {
      uint32_t k;
      memcpy(&k, fr.hdr.mask, 4);
      bad += fr.hdr.fin != (d.b0 >> 7);
      bad += fr.hdr.rsv != ((d.b0 & 0x70) >> 4);
      bad += fr.hdr.opcode != (d.b0 & 0x0f);
      bad += fr.hdr.masked != d.masked;
      bad += k != (d.masked ? d.mask : 0u);
      bad += (uint64_t)fr.hdr.length != d.length;
      bad += fr.src_off != d.hdr_off + synth_hlen(d);
      bad += (fr.payload_off & 15) != 0;
    }
    const uint64_t padded = round16(d.length);
    for (uint64_t i = (uint64_t)threadIdx.x * 16; i < padded; i += 256 * 16) {
      u32x4 want = plain16(seed, g, i);
      if (d.length - i < 16) want = keep_bytes(want, (int64_t)(d.length - i));
      const u32x4 got = *reinterpret_cast<const u32x4*>(payload + fr.payload_off + i);
      const u32x4 x = got ^ want;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        for (int b = 0; b < 4; ++b) bad += ((x[j] >> (8 * b)) & 0xff) != 0;
    }
  }
  const uint64_t w = wave_sum(bad);
  if ((threadIdx.x & 63) == 0 && w) atomicAdd(mismatch, (unsigned long long)w);
}

}  // namespace

using namespace gevws_impl;

extern "C" {

int gevws_abi_version(void) { return GEVWS_ABI_VERSION; }

const char* gevws_status_string(int s) {
  switch (s) {
    case GEVWS_OK: return "ok";
    case GEVWS_NEED_MORE: return "header error: not enough";  // ws.ErrHeaderNotReady text
    case GEVWS_ERR_LEN_MSB: return "header error: the most significant bit must be 0";
    case GEVWS_ERR_CAPACITY: return "output capacity exceeded";
    case GEVWS_ERR_INVALID: return "invalid argument";
    case GEVWS_ERR_DEVICE: return "HIP device error";
    case GEVWS_HANDSHAKE: return "handshake response";
    case GEVWS_ERR_NOT_UPGRADED: return "connection not upgraded and the protocol has no upgrader";
    case GEVWS_ERR_HANDSHAKE: return "websocket upgrade failed";
    default: return "unknown status";
  }
}

int gevws_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// The priority of the n-th context's stream on a device.  The HIP runtime
// gives each priority level its own hardware queues, and same-priority
// streams share that level's few (3 of the default GPU_MAX_HW_QUEUES = 4 on
// the box): eight event loops' contexts at one priority ran at most 3 loops'
// kernels at once, cycling the levels runs more (tools/queue_probe.hip,
// profiles/r05/r05u_queue_probe.jsonl).  By default the cycle is the normal
// level and the levels BELOW it (0, 1, ... inside the device's range): a
// context never outranks the application's own work on normal-priority
// streams, and no loop sits below another loop's level by more than the
// range allows.  GEVWS_STREAM_PRIORITIES=all adds the levels above
// normal (0, -1, 1, -2, 2, ...: the most queues, for a process whose only
// device work is its loops' passes); =normal keeps every context at 0.
static int ctx_stream_priority(int device) {
  static std::atomic<uint32_t> seq[64];
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess || least == greatest) return 0;
  const char* e = getenv("GEVWS_STREAM_PRIORITIES");
  const bool all = e && !strcmp(e, "all");
  if (e && !strcmp(e, "normal")) return 0;
  int levels[64];
  uint32_t nl = 0;
  levels[nl++] = 0;
  for (int i = 1; nl < 64 && (i <= least || -i >= greatest); ++i) {
    if (all && -i >= greatest) levels[nl++] = -i;
    if (i <= least && nl < 64) levels[nl++] = i;
  }
  return levels[seq[device & 63].fetch_add(1, std::memory_order_relaxed) % nl];
}

gevws_ctx* gevws_ctx_create(int device) {
  int n = gevws_device_count();
  if (device < 0 || device >= n) {
    fprintf(stderr, "[gevws] gevws_ctx_create: device %d not available (%d visible)\n", device, n);
    return nullptr;
  }
  DeviceGuard g(device);
  gevws_ctx* ctx = new gevws_ctx();
  ctx->device = device;
  if (hipStreamCreateWithPriority(&ctx->stream, hipStreamNonBlocking, ctx_stream_priority(device)) != hipSuccess) {
    delete ctx;
    return nullptr;
  }
  if (hipEventCreateWithFlags(&ctx->last_done, hipEventDisableTiming) != hipSuccess) {
    gevws_ctx_destroy(ctx);
    return nullptr;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    ctx->num_cus = prop.multiProcessorCount;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && khz > 0)
    ctx->wall_khz = (uint64_t)khz;
  if (hipMalloc(reinterpret_cast<void**>(&ctx->d_sum), sizeof(gevws_summary)) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&ctx->d_done), 256) != hipSuccess ||
      hipMemset(ctx->d_done, 0, 256) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&ctx->d_walk_part), kWalkPartBytes) != hipSuccess ||
      hipMemset(ctx->d_walk_part, 0, kWalkPartBytes) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&ctx->h_stats), 64, hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->d_stats), ctx->h_stats, 0) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    gevws_ctx_destroy(ctx);
    return nullptr;
  }
  return ctx;
}

void gevws_ctx_destroy(gevws_ctx* ctx) {
  if (!ctx) return;
  DeviceGuard g(ctx->device);
  service_stop(ctx);  // (its instance returns at once: the stream drains)
  direct_close(ctx);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  // the last call may have run on another stream (a caller's): its kernels
  // still read the scratch freed below
  if (ctx->has_last && ctx->last_done && last_event(ctx) == GEVWS_OK) (void)hipEventSynchronize(ctx->last_done);
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->d_sum) (void)hipFree(ctx->d_sum);
  if (ctx->d_done) (void)hipFree(ctx->d_done);
  if (ctx->d_small_stage) (void)hipFree(ctx->d_small_stage);
  if (ctx->d_walk_part) (void)hipFree(ctx->d_walk_part);
  if (ctx->h_stats) (void)hipHostFree(ctx->h_stats);
  if (ctx->svc_box) (void)hipHostFree(ctx->svc_box);
  if (ctx->d_svc_ctl) (void)hipFree(ctx->d_svc_ctl);
  if (ctx->last_done) (void)hipEventDestroy(ctx->last_done);
  for (auto& set : ctx->evs)
    for (auto& e : set.e) (void)hipEventDestroy(e);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

int gevws_ctx_device(const gevws_ctx* ctx) { return ctx ? ctx->device : -1; }

void* gevws_ctx_stream(const gevws_ctx* ctx) { return ctx ? reinterpret_cast<void*>(ctx->stream) : nullptr; }

// (also used by the multi-GPU count reduce, gevws_comm.cpp)
int gevws_ctx_order_after_last(gevws_ctx* ctx, void* stream) {
  if (!ctx) return GEVWS_ERR_INVALID;
  DeviceGuard g(ctx->device);
  return order_after_last(ctx, reinterpret_cast<hipStream_t>(stream));
}

int gevws_ctx_set_tuning(gevws_ctx* ctx, int key, int64_t value) {
  if (!ctx) return GEVWS_ERR_INVALID;
  switch (key) {
    case GEVWS_TUNE_UNMASK_VARIANT:
      if (value < 0 || value >= unmask_variant_count()) return GEVWS_ERR_INVALID;
      ctx->unmask_variant = (int)value;
      return GEVWS_OK;
    case GEVWS_TUNE_UNMASK_GRID:
      if (value < 0 || value > (1 << 20)) return GEVWS_ERR_INVALID;
      ctx->unmask_grid = (int)value;
      return GEVWS_OK;
    case GEVWS_TUNE_ENCODE_VARIANT:
      if (value < 0 || value >= encode_variant_count()) return GEVWS_ERR_INVALID;
      ctx->encode_variant = (int)value;
      return GEVWS_OK;
    case GEVWS_TUNE_SMALL_BATCH:
      if (value < 0 || (uint64_t)value > kOneLaunchBytes) return GEVWS_ERR_INVALID;
      ctx->small_bytes = (uint64_t)value;
      return GEVWS_OK;
    case GEVWS_TUNE_SPLIT_LANES:
      if (value < 0 || value > kSplitMaxLanes || (value > 1 && (value & (value - 1)))) return GEVWS_ERR_INVALID;
      ctx->split_lanes = (uint32_t)value;
      return GEVWS_OK;
    case GEVWS_TUNE_WALK_VARIANT:
      if (value < 0 || value >= walk_variant_count()) return GEVWS_ERR_INVALID;
      ctx->walk_variant = (int)value;
      return GEVWS_OK;
    case GEVWS_TUNE_SPLIT_MIN_BYTES:
      if (value < 1024 || value > (1ll << 30)) return GEVWS_ERR_INVALID;
      ctx->split_min_bytes = (uint64_t)value;
      return GEVWS_OK;
    case GEVWS_TUNE_SPLIT_LANES_PER_CU:
      if (value < 64 || value > 4096) return GEVWS_ERR_INVALID;
      ctx->split_lanes_per_cu = (uint64_t)value;
      return GEVWS_OK;
    default:
      return GEVWS_ERR_INVALID;
  }
}

const char* gevws_tuning_name(int key, int64_t value) {
  if (value < 0 || value > 1024) return nullptr;
  if (key == GEVWS_TUNE_UNMASK_VARIANT) return unmask_variant_name((int)value);
  if (key == GEVWS_TUNE_WALK_VARIANT) return walk_variant_name((int)value);
  return nullptr;
}

int gevws_ctx_last_split_lanes(const gevws_ctx* ctx) { return ctx ? (int)ctx->last_ks : -1; }

int64_t gevws_ctx_last_split_fallbacks(gevws_ctx* ctx) {
  if (!ctx) return -1;
  if (ctx->last_ks <= 1) return 0;
  DeviceGuard g(ctx->device);
  uint32_t n = 0;
  if ((ctx->has_last && (last_event(ctx) != GEVWS_OK || hipEventSynchronize(ctx->last_done) != hipSuccess)) ||
      hipMemcpy(&n, ctx->d_done + split_fallback_counter(), sizeof(n), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return (int64_t)n;
}

int gevws_ctx_set_completion_flag(gevws_ctx* ctx, uint32_t* d_flag) {
  if (!ctx) return GEVWS_ERR_INVALID;
  if (d_flag != ctx->done_flag) direct_forget_flag(ctx);
  ctx->done_flag = d_flag;
  ctx->last_signal = -1;
  return GEVWS_OK;
}

int64_t gevws_ctx_completion_seq(const gevws_ctx* ctx) { return ctx ? ctx->last_signal : -1; }

int gevws_ctx_set_timeline_ticks(gevws_ctx* ctx, uint64_t* d_ticks) {
  if (!ctx) return GEVWS_ERR_INVALID;
  ctx->ticks = d_ticks;
  return GEVWS_OK;
}

int gevws_ctx_last_unmask_grid(const gevws_ctx* ctx) { return ctx ? (int)ctx->last_unmask_grid : -1; }

int gevws_ctx_set_timing(gevws_ctx* ctx, int enable) {
  if (!ctx) return GEVWS_ERR_INVALID;
  ctx->timing = enable != 0;
  return GEVWS_OK;
}

int gevws_ctx_timing(gevws_ctx* ctx, float ms_sum[4], uint32_t* calls) {
  if (!ctx || !ms_sum || !calls) return GEVWS_ERR_INVALID;
  DeviceGuard g(ctx->device);
  float acc[4] = {0, 0, 0, 0};
  for (size_t k = 0; k < ctx->evs_used; ++k) {
    auto& set = ctx->evs[k];
    GEVWS_HIP(hipEventSynchronize(set.e[4]));
    for (int i = 0; i < 4; ++i) {
      float t = 0;
      GEVWS_HIP(hipEventElapsedTime(&t, set.e[i], set.e[i + 1]));
      acc[i] += t;
    }
  }
  for (int i = 0; i < 4; ++i) ms_sum[i] = acc[i];
  *calls = (uint32_t)ctx->evs_used;
  ctx->evs_used = 0;
  return GEVWS_OK;
}

int gevws_decode_batch_async(gevws_ctx* ctx, void* stream, const uint8_t* d_in, uint64_t in_bytes,
                             const gevws_conn_in* d_conns, uint32_t n_conns, gevws_frame* d_frames,
                             uint64_t max_frames, uint8_t* d_payload, uint64_t payload_cap,
                             gevws_conn_out* d_conn_out, gevws_summary* d_summary) {
  if (!ctx || !d_summary) return GEVWS_ERR_INVALID;
  if (n_conns && (!d_in || !d_conns || !d_conn_out)) return GEVWS_ERR_INVALID;
  if (max_frames > 0xFFFFFFFFull) return GEVWS_ERR_INVALID;  // tile map holds 32-bit frame ids
  DeviceGuard g(ctx->device);
  hipStream_t st = pick_stream(ctx, stream);
  // a small batch with the default kernels: the whole decode in one launch
  // (per-phase timing and the variant knobs keep the multi-kernel path)
  if (n_conns <= kOneLaunchConns && in_bytes <= ctx->small_bytes && !ctx->timing && ctx->walk_variant == 0 &&
      ctx->unmask_variant == 0 && ctx->unmask_grid == 0)
    return decode_small(ctx, st, d_in, in_bytes, d_conns, n_conns, d_frames, max_frames, d_payload, payload_cap,
                        d_conn_out, d_summary);
  hipEvent_t* ev = nullptr;
  if (ctx->timing) {
    if (ctx->evs_used == ctx->evs.size()) {
      gevws_ctx::EventSet set;
      for (auto& e : set.e) GEVWS_HIP(hipEventCreate(&e));
      ctx->evs.push_back(set);
    }
    ev = ctx->evs[ctx->evs_used++].e;
  }
  // walk, scan, bases, record pass (gevws_walk.hip)
  uint32_t* tile_first = nullptr;
  int r = decode_front(ctx, st, d_in, in_bytes, d_conns, n_conns, d_frames, max_frames, payload_cap, d_conn_out,
                       d_summary, ev, &tile_first);
  if (r != GEVWS_OK) return r;
  if (ev) GEVWS_HIP(hipEventRecord(ev[3], st));
  r = launch_unmask(ctx, st, payload_cap, d_in, d_frames, tile_first, d_summary, d_payload);
  if (r != GEVWS_OK) return r;
  if (ev) GEVWS_HIP(hipEventRecord(ev[4], st));
  GEVWS_HIP(hipGetLastError());
  return mark_last(ctx, st);
}

int gevws_ctx_set_service(gevws_ctx* ctx, int enable) {
  if (!ctx) return GEVWS_ERR_INVALID;
  DeviceGuard g(ctx->device);
  if (!enable) {
    service_stop(ctx);
    ctx->svc_enabled = false;
    return GEVWS_OK;
  }
  if (!ctx->svc_box) {
    void* h = nullptr;
    void* d = nullptr;
    if (hipHostMalloc(&h, 4096, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess || !h)
      return GEVWS_ERR_DEVICE;
    memset(h, 0, 4096);
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d) {
      (void)hipHostFree(h);
      return GEVWS_ERR_DEVICE;
    }
    ctx->svc_box = static_cast<ServiceBox*>(h);
    ctx->svc_box_dev = static_cast<ServiceBox*>(d);
  }
  ctx->svc_enabled = true;
  return GEVWS_OK;
}

int gevws_ctx_service_stop(gevws_ctx* ctx) {
  if (!ctx) return GEVWS_ERR_INVALID;
  service_stop(ctx);
  return GEVWS_OK;
}

int gevws_ctx_set_direct(gevws_ctx* ctx, int enable) {
  if (!ctx) return GEVWS_ERR_INVALID;
  DeviceGuard g(ctx->device);
  if (!enable) direct_forget_flag(ctx);
  ctx->direct_enabled = enable != 0;
  return GEVWS_OK;
}

int64_t gevws_ctx_direct_dispatches(const gevws_ctx* ctx) { return ctx ? ctx->direct_dispatches : -1; }

int gevws_ctx_synchronize(gevws_ctx* ctx) {
  if (!ctx) return GEVWS_ERR_INVALID;
  DeviceGuard g(ctx->device);
  service_stop(ctx);
  if (ctx->last_direct) {
    const int r = direct_drain(ctx);
    if (r != GEVWS_OK) return r;
    ctx->last_direct = false;
  }
  GEVWS_HIP(hipStreamSynchronize(ctx->stream));
  if (ctx->has_last && ctx->last_stream != ctx->stream) {
    const int r = last_event(ctx);
    if (r != GEVWS_OK) return r;
    GEVWS_HIP(hipEventSynchronize(ctx->last_done));
  }
  return GEVWS_OK;
}

int gevws_ctx_service_stats(const gevws_ctx* ctx, int64_t* launches, int64_t* posts) {
  if (!ctx) return GEVWS_ERR_INVALID;
  if (launches) *launches = ctx->svc_launches;
  if (posts) *posts = ctx->svc_posts;
  return GEVWS_OK;
}

int gevws_decode_batch_post(gevws_ctx* ctx, const uint8_t* d_in, uint64_t in_bytes, const gevws_conn_in* d_conns,
                            uint32_t n_conns, gevws_frame* d_frames, uint64_t max_frames, uint8_t* d_payload,
                            uint64_t payload_cap, gevws_conn_out* d_conn_out, gevws_summary* d_summary) {
  if (!ctx || !d_summary) return GEVWS_ERR_INVALID;
  if (n_conns && (!d_in || !d_conns || !d_conn_out)) return GEVWS_ERR_INVALID;
  if (max_frames > 0xFFFFFFFFull) return GEVWS_ERR_INVALID;
  DeviceGuard g(ctx->device);
  if (!ctx->timing && ctx->walk_variant == 0 && ctx->unmask_variant == 0 && ctx->unmask_grid == 0 &&
      in_bytes <= ctx->small_bytes &&
      direct_post(ctx, d_in, in_bytes, d_conns, n_conns, d_frames, max_frames, d_payload, payload_cap, d_conn_out,
                  d_summary))
    return GEVWS_OK;
  if (!ctx->timing && ctx->walk_variant == 0 && ctx->unmask_variant == 0 && ctx->unmask_grid == 0 &&
      in_bytes <= ctx->small_bytes &&
      service_post(ctx, ctx->stream, d_in, in_bytes, d_conns, n_conns, d_frames, max_frames, d_payload, payload_cap,
                   d_conn_out, d_summary))
    return GEVWS_OK;
  return gevws_decode_batch_async(ctx, ctx->stream, d_in, in_bytes, d_conns, n_conns, d_frames, max_frames, d_payload,
                                  payload_cap, d_conn_out, d_summary);
}

int gevws_decode_batch(gevws_ctx* ctx, void* stream, const uint8_t* d_in, uint64_t in_bytes,
                       const gevws_conn_in* d_conns, uint32_t n_conns, gevws_frame* d_frames,
                       uint64_t max_frames, uint8_t* d_payload, uint64_t payload_cap,
                       gevws_conn_out* d_conn_out, gevws_summary* h_summary) {
  if (!ctx || !h_summary) return GEVWS_ERR_INVALID;
  DeviceGuard g(ctx->device);
  hipStream_t st = pick_stream(ctx, stream);
  gevws_summary* d_sum = ctx->d_sum;
  int r = gevws_decode_batch_async(ctx, stream, d_in, in_bytes, d_conns, n_conns, d_frames, max_frames,
                                   d_payload, payload_cap, d_conn_out, d_sum);
  if (r == GEVWS_OK) {
    GEVWS_HIP(hipMemcpyAsync(h_summary, d_sum, sizeof(gevws_summary), hipMemcpyDeviceToHost, st));
    GEVWS_HIP(hipStreamSynchronize(st));
    r = h_summary->status;
  }
  return r;
}

int gevws_pinned_alloc(uint64_t bytes, void** host_ptr, void** dev_ptr) {
  if (!host_ptr || !dev_ptr || bytes == 0) return GEVWS_ERR_INVALID;
  *host_ptr = nullptr;
  *dev_ptr = nullptr;
  void* h = nullptr;
  if (hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess || !h)
    return GEVWS_ERR_DEVICE;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d) {
    (void)hipHostFree(h);
    return GEVWS_ERR_DEVICE;
  }
  *host_ptr = h;
  *dev_ptr = d;
  return GEVWS_OK;
}

int gevws_device_alloc(int device, uint64_t bytes, int kind, void** ptr) {
  if (!ptr || bytes == 0 || device < 0 || device >= gevws_device_count()) return GEVWS_ERR_INVALID;
  if (kind < GEVWS_MEM_DEFAULT || kind > GEVWS_MEM_UNCACHED) return GEVWS_ERR_INVALID;
  *ptr = nullptr;
  DeviceGuard g(device);
  void* p = nullptr;
  if (kind == GEVWS_MEM_DEFAULT) {
    GEVWS_HIP(hipMalloc(&p, bytes));
  } else {
    GEVWS_HIP(hipExtMallocWithFlags(&p, bytes, kind == GEVWS_MEM_FINE ? hipDeviceMallocFinegrained
                                                                     : hipDeviceMallocUncached));
  }
  if (hipMemset(p, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    (void)hipFree(p);
    return GEVWS_ERR_DEVICE;
  }
  *ptr = p;
  return GEVWS_OK;
}

int gevws_device_free(int device, void* ptr) {
  if (!ptr) return GEVWS_OK;
  DeviceGuard g(device);
  return hipFree(ptr) == hipSuccess ? GEVWS_OK : GEVWS_ERR_DEVICE;
}

int gevws_pinned_free(void* host_ptr) {
  if (!host_ptr) return GEVWS_OK;
  return hipHostFree(host_ptr) == hipSuccess ? GEVWS_OK : GEVWS_ERR_DEVICE;
}

int gevws_synth_async(gevws_ctx* ctx, void* stream, uint8_t* d_in, const gevws_synth_desc* d_desc,
                      uint64_t n_frames, uint64_t seed) {
  if (!ctx || (n_frames && (!d_in || !d_desc))) return GEVWS_ERR_INVALID;
  if (n_frames == 0) return GEVWS_OK;
  DeviceGuard g(ctx->device);
  hipStream_t st = pick_stream(ctx, stream);
  uint64_t grid = n_frames < (1u << 20) ? n_frames : (1u << 20);
  k_synth<<<(uint32_t)grid, 256, 0, st>>>(d_in, d_desc, n_frames, seed);
  GEVWS_HIP(hipGetLastError());
  return GEVWS_OK;
}

int gevws_synth_verify_async(gevws_ctx* ctx, void* stream, const gevws_synth_desc* d_desc,
                             uint64_t n_frames, uint64_t seed, const gevws_frame* d_frames,
                             const uint8_t* d_payload, uint64_t payload_cap, uint64_t* d_mismatch) {
  if (!ctx || !d_mismatch || (n_frames && (!d_desc || !d_frames || !d_payload))) return GEVWS_ERR_INVALID;
  if (n_frames == 0) return GEVWS_OK;
  DeviceGuard g(ctx->device);
  hipStream_t st = pick_stream(ctx, stream);
  uint64_t grid = n_frames < (1u << 16) ? n_frames : (1u << 16);
  k_synth_verify<<<(uint32_t)grid, 256, 0, st>>>(d_desc, n_frames, seed, d_frames, d_payload, payload_cap,
                                                  reinterpret_cast<unsigned long long*>(d_mismatch));
  GEVWS_HIP(hipGetLastError());
  return GEVWS_OK;
}

}  // extern "C"
