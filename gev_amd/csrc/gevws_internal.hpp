// gevws_internal.hpp -- the host side shared by the files of libgevws.so: the
// context behind gevws_ctx (include/gevws.h), stream / scratch helpers, and
// the launchers one file provides to another.  Nothing here is exported
// (-fvisibility=hidden; the C ABI is declared in gevws.h only).
#pragma once

#include <vector>

#include "gevws_kernels.hpp"

// The resident decode service's mailbox (k_decode_service, gevws_walk.hip):
// mapped, coherent host memory written by the host, read by the kernel.
constexpr int kServiceArgs = 10;  // in, in_bytes, conns, n, frames, max_frames, payload, payload_cap, cout, sum
struct ServiceBox {
  uint64_t req;                 // the posted pass: {its generation << 32 | its number}, stored last (release)
  uint32_t gen;                 // the live generation: an instance of another one returns once no pass of
                                //   its own is pending
  uint32_t ack;                 // (written by the kernel) the number of the last pass taken
  uint64_t args[kServiceArgs];  // the posted pass's arguments (device addresses and sizes)
};

// The one-launch decode's arguments as one by-value kernel argument, so a
// dispatch written straight into an AQL queue (gevws_direct.cpp) lays out the
// kernarg segment exactly as the kernel reads it (k_decode_small_direct).
struct DirectDecodeArgs {
  const uint8_t* in;
  uint64_t in_bytes;
  const gevws_conn_in* conns;
  gevws_frame* frames;
  uint64_t max_frames;
  uint8_t* payload;
  uint64_t payload_cap;
  gevws_conn_out* cout;
  gevws_summary* sum;
  uint32_t* done;
  uint64_t* ticks;
  uint64_t* stage_buf;
  uint32_t* stage_done;
  uint32_t n, seq, tag, nwg;
  uint64_t* phase;  // (measurement: GEVWS_PHASE_TICKS)
};
struct DirectQueue;  // gevws_direct.cpp

struct gevws_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  bool timing = false;
  struct EventSet {
    hipEvent_t e[5];
  };
  std::vector<EventSet> evs;  // one set per timed call since the last gevws_ctx_timing
  size_t evs_used = 0;
  gevws_summary* d_sum = nullptr;  // summary slot of the synchronous entry point
  int unmask_variant = 0;  // GEVWS_TUNE_UNMASK_VARIANT (kUnmaskVariants)
  int unmask_grid = 0;     // 0 = auto
  int encode_variant = 0;  // GEVWS_TUNE_ENCODE_VARIANT (kNumEncodeVariants)
  uint64_t small_bytes = kOneLaunchBytes;  // one-launch decode (k_decode_small) up to this many input bytes
  uint32_t* done_flag = nullptr;  // mapped host word the one-launch kernels signal (gevws_ctx_set_completion_flag)
  uint32_t done_seq = 0;
  uint64_t* ticks = nullptr;  // mapped host u64[4]: the one-launch kernels' start / end ticks (gevws_ctx_set_timeline_ticks)
  int64_t last_signal = -1;  // the value the last call's last kernel stores there, -1: none
  // the context's history: the last multi-kernel decode's frame / payload /
  // equal-size-run totals (written by k_walk_bases into mapped host memory)
  // and its connection count, read once that decode has finished; it picks
  // the split walk, the walk's speculation and the unmask's wide grid
  uint64_t* h_stats = nullptr;
  uint64_t* d_stats = nullptr;
  bool stats_pending = false, stats_known = false;
  uint64_t stats_conns = 0, prev_frames_per_conn = 0, prev_frame_bytes = 0;
  bool prev_mixed = false;
  uint32_t last_unmask_grid = 0;  // workgroups of the last decode's unmask launch
  uint32_t* unmask_runs = nullptr;  // the unmask v5 path's per-XCD run counters (decode scratch)
  uint32_t last_ks = 1;    // lanes per connection of the last multi-kernel decode's walk
  uint32_t split_lanes = 0;  // lanes per connection (k_walk_split); 0 = auto, 1 = off
  uint64_t split_min_bytes = kSplitMinBytes;        // split walk: bytes per segment at least
  uint64_t split_lanes_per_cu = kSplitLanesPerCU;   // split walk auto: lanes per CU at most
  int walk_variant = 0;    // 0 = speculation (D = 8) unless the history is mixed, 1 = plain chain walk
                           // (D = 0), 2 = no entry table (the record pass re-walks every chain), 3 =
                           // the writer wave whatever the batch size
  // Scratch is per context: calls on a different stream than the previous one
  // first wait for it (one in-flight batch per context; use one context per
  // stream for concurrency).
  hipEvent_t last_done = nullptr;
  hipStream_t last_stream = nullptr;
  bool has_last = false;
  bool last_recorded = true;  // last_done marks the last call (else: recorded when first needed)
  bool prev_small_decode = false;  // the last call was a one-launch decode (mark_last_lazy)
  int num_cus = 256;
  uint32_t* d_done = nullptr;  // 256 B: the decode walk's finished-workgroup counter ([0], zero between calls)
                               // and the one-launch decode's staging counter ([kSmallStageCounter])
  // The in-launch cross-workgroup hand-offs' tagged granules (gevws_walk.hip,
  // "hand-offs"), zeroed at allocation, and the number that tags the next
  // launch's (never 0):
  uint64_t* d_walk_part = nullptr;    // the walk's block partials (kFusedScanMaxBlocks x kDecFields x 2)
  uint64_t* d_small_stage = nullptr;  // a live pass's staged input (k_decode_small; 4 granules a 16-byte chunk)
  uint32_t hand_seq = 0;
  // the resident decode service (gevws_ctx_set_service)
  bool svc_enabled = false;      // posting allowed
  bool svc_live = false;         // an instance of this generation is on the stream
  ServiceBox* svc_box = nullptr;  // mapped host memory (host address = device address on ROCm, checked)
  ServiceBox* svc_box_dev = nullptr;
  uint32_t svc_gen = 0, svc_last = 0;  // generation; the last pass number posted
  uint32_t* svc_flag = nullptr;   // the completion word / ticks the live instance signals
  const uint32_t* svc_flag_host = nullptr;  // (the word's host address)
  uint64_t* svc_ticks = nullptr;
  int64_t svc_t_launch_ns = 0;    // host clock at the live instance's launch
  uint64_t* d_svc_ctl = nullptr;  // the instance's broadcast granules (k_decode_service), zeroed at allocation
  uint32_t svc_t0 = 0, svc_passes = 0;  // the live instance's tags [t0, t0 + kServiceMaxPasses); passes posted
  int64_t svc_launches = 0, svc_posts = 0;  // (gevws_ctx_service_stats)
  uint64_t wall_khz = 100000;     // the GPU's constant-rate clock (hipDeviceAttributeWallClockRate)
  // direct dispatch (gevws_ctx_set_direct): live passes written into the
  // context's own AQL queue instead of launched through the HIP runtime
  bool direct_enabled = false;
  DirectQueue* direct = nullptr;
  bool last_direct = false;  // the last call went to that queue (not the stream)
  int64_t direct_dispatches = 0;
};

// The tag of a launch's hand-offs.
inline uint32_t next_hand_tag(gevws_ctx* ctx) {
  if (++ctx->hand_seq == 0) ctx->hand_seq = 1;
  return ctx->hand_seq;
}
// n consecutive tags, none 0: the first.
inline uint32_t reserve_hand_tags(gevws_ctx* ctx, uint32_t n) {
  if ((uint64_t)ctx->hand_seq + n > 0xFFFFFFFFull) ctx->hand_seq = 0;
  const uint32_t t0 = ctx->hand_seq + 1;
  ctx->hand_seq += n;
  return t0;
}

namespace gevws_impl {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

#define GEVWS_HIP(call)                                                                \
  do {                                                                                  \
    hipError_t e_ = (call);                                                             \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "[gevws] %s failed: %s\n", #call, hipGetErrorString(e_));          \
      return GEVWS_ERR_DEVICE;                                                          \
    }                                                                                   \
  } while (0)

// NULL = the HIP default (null) stream, as in every HIP/CUDA API; callers
// that want the context's own stream pass gevws_ctx_stream(ctx).
inline hipStream_t pick_stream(gevws_ctx* ctx, void* stream) {
  (void)ctx;
  return reinterpret_cast<hipStream_t>(stream);
}

// Ends the live service instance (if any): bumping the mailbox's generation
// makes it return within a poll once the pass posted to it (if any) is done,
// so work enqueued behind it on the stream runs after that pass, at once.
inline void service_stop(gevws_ctx* ctx) {
  if (!ctx->svc_live) return;
  __atomic_store_n(&ctx->svc_box->gen, ++ctx->svc_gen, __ATOMIC_RELEASE);
  ctx->svc_live = false;
}

// last_done, recorded now if the last call left it to its first use.
inline int last_event(gevws_ctx* ctx) {
  if (ctx->has_last && !ctx->last_recorded) {
    GEVWS_HIP(hipEventRecord(ctx->last_done, ctx->last_stream));
    ctx->last_recorded = true;
  }
  return GEVWS_OK;
}

// gevws_direct.cpp: waits until every pass dispatched to the context's own
// queue has signalled (GEVWS_ERR_DEVICE past 10 s).
int direct_drain(gevws_ctx* ctx);

// Orders this call after the context's previous one when the stream changes
// or the previous one went to the context's own queue (and ends the service
// instance first: every launcher calls this).
inline int order_after_last(gevws_ctx* ctx, hipStream_t st) {
  service_stop(ctx);
  if (ctx->last_direct) {
    const int r = direct_drain(ctx);
    if (r != GEVWS_OK) return r;
    ctx->last_direct = false;
  }
  if (ctx->has_last && ctx->last_stream != st) {
    const int r = last_event(ctx);
    if (r != GEVWS_OK) return r;
    GEVWS_HIP(hipStreamWaitEvent(st, ctx->last_done, 0));
  }
  return GEVWS_OK;
}

inline int mark_last(gevws_ctx* ctx, hipStream_t st) {
  ctx->last_signal = -1;  // (the one-launch paths set it after this)
  GEVWS_HIP(hipEventRecord(ctx->last_done, st));
  ctx->last_stream = st;
  ctx->has_last = true;
  ctx->last_recorded = true;
  ctx->prev_small_decode = false;
  return GEVWS_OK;
}

// A one-launch call on the context's own stream, where only this context
// enqueues work: its event is recorded only when something needs it (another
// stream's call, a synchronisation, destroy) -- an event recorded later on
// that stream marks this call and nothing foreign.  Saves a live pass the
// hipEventRecord call (C1's launch phase 4.7-5.5 -> 3.4-3.9 us,
// profiles/r06/r06n_lb_ab.jsonl).  Only a one-launch decode that follows
// another: with the handler step chained behind it lazy too the wsserver
// shape lost 25 % (r06m_lb_ab.jsonl: launch 13-15 -> 21-24 us, its decode
// kernel 9.4 -> 11 us), and with the decode alone lazy behind a recorded
// handler step 10-20 % on another box (r06t_lb_ab.jsonl); so passes that
// chain anything behind the decode keep every record.
inline int mark_last_lazy(gevws_ctx* ctx, hipStream_t st) {
  if (st != ctx->stream) return mark_last(ctx, st);
  ctx->last_signal = -1;
  ctx->last_stream = st;
  ctx->has_last = true;
  ctx->last_recorded = false;
  return GEVWS_OK;
}

inline int ensure_scratch(gevws_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->scratch_bytes) return GEVWS_OK;
  if (ctx->scratch) {
    GEVWS_HIP(hipDeviceSynchronize());
    GEVWS_HIP(hipFree(ctx->scratch));
    ctx->scratch = nullptr;
    ctx->scratch_bytes = 0;
  }
  size_t want = bytes + bytes / 4 + 4096;
  GEVWS_HIP(hipMalloc(&ctx->scratch, want));
  ctx->scratch_bytes = want;
  return GEVWS_OK;
}

// ---- gevws_walk.hip: the decode up to the unmask
// the one-launch decode of a small batch (k_decode_small)
int decode_small(gevws_ctx* ctx, hipStream_t st, const uint8_t* d_in, uint64_t in_bytes,
                 const gevws_conn_in* d_conns, uint32_t n_conns, gevws_frame* d_frames, uint64_t max_frames,
                 uint8_t* d_payload, uint64_t payload_cap, gevws_conn_out* d_conn_out, gevws_summary* d_summary);
// a live pass written into the context's own AQL queue, or false (gevws_direct.cpp)
bool direct_dispatch(gevws_ctx* ctx, int wide, const DirectDecodeArgs& a);
void direct_close(gevws_ctx* ctx);
// drains the direct passes and drops the completion word they signal (it is being replaced or freed)
void direct_forget_flag(gevws_ctx* ctx);
bool direct_post(gevws_ctx* ctx, const uint8_t* d_in, uint64_t in_bytes, const gevws_conn_in* d_conns,
                 uint32_t n_conns, gevws_frame* d_frames, uint64_t max_frames, uint8_t* d_payload,
                 uint64_t payload_cap, gevws_conn_out* d_conn_out, gevws_summary* d_summary);
// a narrow-shape live pass posted to the context's resident decode service
// (launched first if none is live), or false (gevws_decode_batch_post)
bool service_post(gevws_ctx* ctx, hipStream_t st, const uint8_t* d_in, uint64_t in_bytes,
                  const gevws_conn_in* d_conns, uint32_t n_conns, gevws_frame* d_frames, uint64_t max_frames,
                  uint8_t* d_payload, uint64_t payload_cap, gevws_conn_out* d_conn_out, gevws_summary* d_summary);
// header walk, scan, bases and record pass into the context's scratch; the
// output-tile -> frame map for the unmask in *tile_first.  ev: the timing
// events 0..2 (walk start, walk end, scan end) or null.
int decode_front(gevws_ctx* ctx, hipStream_t st, const uint8_t* d_in, uint64_t in_bytes,
                 const gevws_conn_in* d_conns, uint32_t n_conns, gevws_frame* d_frames, uint64_t max_frames,
                 uint64_t payload_cap, gevws_conn_out* d_conn_out, gevws_summary* d_summary, hipEvent_t* ev,
                 uint32_t** tile_first);
int walk_variant_count();
uint32_t split_fallback_counter();  // the word of ctx->d_done the split walk counts its serial re-walks in
const char* walk_variant_name(int i);

// ---- gevws_unmask.hip
int launch_unmask(gevws_ctx* ctx, hipStream_t st, uint64_t payload_cap, const uint8_t* d_in,
                  const gevws_frame* d_frames, const uint32_t* tile_first, const gevws_summary* d_summary,
                  uint8_t* d_payload);
int unmask_variant_count();
const char* unmask_variant_name(int i);

// ---- gevws_encode.hip
int encode_variant_count();

}  // namespace gevws_impl
