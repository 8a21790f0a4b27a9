// gevws_host.cpp -- C++ host side above the device ABI, mirroring the
// reference's plugin surface for the decode path (Go is absent from this image,
// so the host side is C++; INTEGRATION.md shows the cgo binding):
//
//   RingBuffer  ~ github.com/Allenxuxu/ringbuffer v0.0.11 as gev uses it
//                 (Write / Length / PeekAll / Retrieve; virtual cursor calls at
//                 read.go:20,27,63 and protocol.go:47-60 are replaced by the
//                 device header walk).  Growable circular buffer.
//   Connection  ~ gev.Connection's KeyValueContext entries the websocket plugin
//                 keeps (protocol.go:11-14, 28-39) plus the queue of frames
//                 decoded for it and not yet delivered.
//   Protocol    ~ websocket.Protocol (plugins/websocket/protocol.go:16-69):
//                 UnPacket returns one frame per call exactly like the
//                 reference; its decode runs on the device, batched across
//                 every connection handed to UnPacketBatch.  Before the
//                 upgrade it runs the HTTP handshake (handshake.cpp, host).
//
// The decode itself is never done on the host: this file only stages bytes,
// launches gevws_decode_batch and hands out the device's results.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <vector>

#include "gevws.h"
#include "handshake.hpp"
#include "ringbuffer.hpp"

namespace gevws {

// ------------------------------------------------------------------ logging (gev/log)
// log.Error prints with the "[Gev]" prefix unless GEV_LOG_LEVEL silences it
// (log/log.go:51-62).
static bool log_errors_enabled() {
  static int level = [] {
    const char* s = std::getenv("GEV_LOG_LEVEL");
    if (!s) return 2;
    if (!strcmp(s, "FATAL") || !strcmp(s, "fatal")) return 0;
    if (!strcmp(s, "INFO") || !strcmp(s, "info")) return 1;
    return 2;
  }();
  return level >= 1;
}
static void log_error(const char* what, int status) {
  if (log_errors_enabled()) fprintf(stderr, "[Gev] ERROR %s%s\n", what, gevws_status_string(status));
}
static void log_error_text(const char* what, const std::string& text) {
  if (log_errors_enabled()) fprintf(stderr, "[Gev] ERROR %s%s\n", what, text.c_str());
}

// ------------------------------------------------------------------ pinned arenas
// The payload arena of a device pass is copied D2H straight into page-locked
// host memory and handed out from there: every frame a pass delivers holds a
// reference to its arena, which goes back to the protocol's pool when the last
// of them is released (no second host copy).  Thread-confined like the
// protocol (one per event loop); the mutex only guards a release that happens
// after the protocol is gone.
// Page-locked host memory mapped into the device address space and coherent
// (fine-grained: device accesses go to host memory, never stale in a device
// cache), so a small pass's kernels can read the staged input and write their
// results in place (Protocol::kZeroCopyMax).
constexpr unsigned kHostFlags = hipHostMallocMapped | hipHostMallocCoherent;

// The device address of mapped host memory (this file's hipHostMalloc
// buffers only), or nullptr.  ROCm maps such memory at its host address (one
// address space): checked once per process on a mapped allocation, after
// which no runtime lookup is made -- hipHostGetDevicePointer takes the
// runtime's memory-map lock and a search per call, and a live pass makes
// 4-11 of them on the loop's critical path (launch phase 5.2-6.5 -> 4.5-4.9
// us a pass, profiles/r05/r05f_loopback_timeline.jsonl).
inline void* device_of(void* h) {
  static const bool same_address = [] {
    void* p = nullptr;
    void* d = nullptr;
    if (hipHostMalloc(&p, 64, kHostFlags) != hipSuccess || !p) return false;
    const bool same = hipHostGetDevicePointer(&d, p, 0) == hipSuccess && d == p;
    (void)hipHostFree(p);
    return same;
  }();
  if (same_address) return h;
  void* d = nullptr;
  return hipHostGetDevicePointer(&d, h, 0) == hipSuccess ? d : nullptr;
}

class PinnedPool : public std::enable_shared_from_this<PinnedPool> {
 public:
  ~PinnedPool() {
    for (auto& b : free_) (void)hipHostFree(b.p);
  }
  // A buffer of at least `need` bytes, or nullptr.
  std::shared_ptr<uint8_t> Acquire(uint64_t need) {
    need = std::max<uint64_t>(need, 16);
    Buf b{nullptr, 0};
    {
      // the smallest kept buffer that fits (first-fit let one big
      // pass's arena serve every later tiny one)
      std::lock_guard<std::mutex> g(mu_);
      size_t best = free_.size();
      for (size_t i = 0; i < free_.size(); ++i)
        if (free_[i].cap >= need && (best == free_.size() || free_[i].cap < free_[best].cap)) best = i;
      if (best < free_.size()) {
        b = free_[best];
        free_.erase(free_.begin() + (long)best);
      }
    }
    if (!b.p) {
      const uint64_t want = std::max<uint64_t>(need + need / 2, 1 << 16);
      if (hipHostMalloc((void**)&b.p, want, kHostFlags) != hipSuccess) return nullptr;
      b.cap = want;
    }
    std::weak_ptr<PinnedPool> pool = shared_from_this();
    return std::shared_ptr<uint8_t>(b.p, [pool, b](uint8_t*) {
      if (auto pp = pool.lock()) pp->Release(b);
      else (void)hipHostFree(b.p);
    });
  }
 private:
  struct Buf {
    uint8_t* p;
    uint64_t cap;
  };
  void Release(Buf b) {
    std::lock_guard<std::mutex> g(mu_);
    if (free_.size() < kKeep && b.cap <= kKeepMaxBytes) {
      free_.push_back(b);
      return;
    }
    (void)hipHostFree(b.p);
  }
  static constexpr size_t kKeep = 8;  // arenas kept for reuse
  // page-locked memory is a system-wide resource: an arena bigger than this
  // (a bulk pass's) goes back to the OS instead of staying pinned for the
  // protocol's life
  static constexpr uint64_t kKeepMaxBytes = 64ull << 20;
  std::mutex mu_;
  std::vector<Buf> free_;
};

// ------------------------------------------------------------------ connection
struct Delivered {
  gevws_header hdr;
  uint64_t frame_bytes;  // h + L, consumed from the ring on delivery
  uint64_t payload_off;  // into the pass's pinned arena
  std::shared_ptr<uint8_t> arena;
  // the device handler's answer (HandlerWrap.OnMessage, wrap.go:38-90): the
  // wire bytes of the reply frame (none: len 0) in the pass's reply buffer and
  // whether the frame was a close (c.ShutdownWrite(), wrap.go:56)
  std::shared_ptr<uint8_t> replies;
  uint64_t reply_off = 0, reply_len = 0;
  bool shutdown = false;
  bool handled = false;  // the frame's pass ran the handler (its reply fields are the answer)
};

struct Connection {
  bool upgraded = false;                 // "gev_ws_upgraded" (protocol.go:12, 36)
  int poisoned = GEVWS_OK;               // sticky ERR_LEN_MSB (Appendix A P9/U3)
  std::deque<Delivered> queue;           // decoded, not yet returned by UnPacket
  std::shared_ptr<uint8_t> current;      // keeps the last payload's arena alive
  std::shared_ptr<uint8_t> current_replies;  // ... and its reply buffer (device handler)
  uint64_t reply_off = 0, reply_len = 0;
  bool reply_valid = false, shutdown = false;
  HandshakeResult hs;                    // last Upgrade's response + Handshake
  // Completeness carry (protocol.go:47, 59-61): ring bytes, counted from the
  // ring's read position, that must be buffered before a device pass can
  // decode anything this connection has not queued yet -- h + L of its first
  // incomplete frame once its header is known, 6 before that (read.go:20-23).
  // Valid only while the ring's read position is the one it was derived at
  // (need_ring / need_at): bytes consumed by anyone else invalidate it.
  uint64_t need = 0;
  const RingBuffer* need_ring = nullptr;
  uint64_t need_at = 0;
  uint64_t epoch = 0;                    // last UnPacketBatch that took this connection
};

// ------------------------------------------------------------------ protocol
class Protocol {
  struct Staged;  // a pass in flight (below)

 public:
  explicit Protocol(gevws_ctx* ctx) : ctx_(ctx), pool_(std::make_shared<PinnedPool>()) {}
  void SetUpgrader(const Upgrader* u) { upgrader_ = u; }
  ~Protocol() { release(); }

  int UnPacket(Connection* c, RingBuffer* ring, gevws_header* hdr, const uint8_t** out,
               uint64_t* out_len) {
    *out = nullptr;
    *out_len = 0;
    if (!c->upgraded) {  // protocol.go:28-37: the handshake path
      if (!upgrader_) {
        log_error("Websocket Upgrade :", GEVWS_ERR_NOT_UPGRADED);
        return GEVWS_ERR_NOT_UPGRADED;
      }
      upgrader_->Upgrade(static_cast<gevws_conn*>(static_cast<void*>(c)), ring, &c->hs);
      *out = c->hs.out.empty() ? nullptr : (const uint8_t*)c->hs.out.data();
      *out_len = c->hs.out.size();
      if (c->hs.error != GEVWS_HS_OK) {  // (nil, error response or nil), logged
        log_error_text("Websocket Upgrade :", c->hs.reason);
        return GEVWS_ERR_HANDSHAKE;
      }
      c->upgraded = true;
      return GEVWS_HANDSHAKE;
    }
    if (pend_.active) {  // a pass begun by BeginBatch finishes first
      const int64_t r = EndBatch();
      if (r < 0) return (int)r;
    }
    if (c->queue.empty() && c->poisoned == GEVWS_OK) {
      if (Ready(c, ring)) {
        Connection* cs[1] = {c};
        RingBuffer* rs[1] = {ring};
        int64_t r = UnPacketBatch(cs, rs, 1);
        if (r < 0) return (int)r;
      } else {
        ++stats_.gated;
      }
    }
    if (c->queue.empty()) {
      if (c->poisoned != GEVWS_OK) {  // protocol.go:41-45: log and return (nil, nil)
        log_error("", c->poisoned);
        return c->poisoned;
      }
      return GEVWS_NEED_MORE;  // ErrHeaderNotReady / gate: silent (nil, nil)
    }
    Delivered d = std::move(c->queue.front());
    c->queue.pop_front();
    const bool carried = c->need_ring == ring && c->need_at == ring->Retrieved();
    ring->Retrieve(d.frame_bytes);  // VirtualFlush + Read (protocol.go:48-51)
    if (carried) {
      c->need = c->need > d.frame_bytes ? c->need - d.frame_bytes : 0;
      c->need_at = ring->Retrieved();
    }
    c->current = std::move(d.arena);
    c->current_replies = std::move(d.replies);
    c->reply_off = d.reply_off;
    c->reply_len = d.reply_len;
    c->shutdown = d.shutdown;
    // (from the frame's own pass: a frame queued before set_handler() has no
    // answer, one queued before the handler was turned off keeps its answer)
    c->reply_valid = d.handled;
    *hdr = d.hdr;
    *out = c->current.get() + d.payload_off;
    *out_len = (uint64_t)d.hdr.length;
    return GEVWS_OK;
  }

  // One device pass over every listed connection that can make progress.
  int64_t UnPacketBatch(Connection* const* conns, RingBuffer* const* rings, uint32_t n) {
    if (pend_.active) {  // a pass begun by BeginBatch finishes first, as in UnPacket
      const int64_t e = EndBatch();
      if (e < 0) return e;
    }
    const int64_t r = BeginBatch(conns, rings, n);
    if (r <= 0) return r;
    return EndBatch();
  }

  // The pass of UnPacketBatch in two halves, so an event loop can read its
  // sockets while the device decodes: BeginBatch selects, stages and enqueues
  // the pass and its copies (no synchronisation) and returns the number of
  // connections in it (0: nothing to do); EndBatch waits for it and queues the
  // frames on their connections.  One pass in flight per protocol; between
  // the two, the rings may take new bytes (the pass decodes its staged copy)
  // but are not read; UnPacket ends a pass in flight first.
  int64_t BeginBatch(Connection* const* conns, RingBuffer* const* rings, uint32_t n) {
    if (pend_.active) return GEVWS_ERR_INVALID;
    const auto tb0 = std::chrono::steady_clock::now();
    // Skipped: connections that still hold undelivered frames (their ring
    // prefix is decoded already), poisoned ones, ones whose first undecoded
    // frame is not complete yet (the carried gate), and repeats of a
    // connection already taken by this call.
    ++epoch_;
    std::vector<uint32_t>& sel = pend_.sel;
    std::vector<gevws_host_conn> segs;
    sel.clear();
    sel.reserve(n);
    for (uint32_t i = 0; i < n; ++i) {
      Connection* c = conns[i];
      if (c->epoch == epoch_ || !c->upgraded || !c->queue.empty() || c->poisoned != GEVWS_OK) continue;
      if (!Ready(c, rings[i])) continue;
      c->epoch = epoch_;
      gevws_host_conn h;
      rings[i]->PeekAll(&h.seg0, &h.n0, &h.seg1, &h.n1);
      sel.push_back(i);
      segs.push_back(h);
    }
    if (sel.empty()) return 0;
    const uint32_t m = (uint32_t)sel.size();
    DeviceScope scope(gevws_ctx_device(ctx_));
    pend_.sg = Staged{};
    Staged& sg = pend_.sg;
    const auto tb1 = std::chrono::steady_clock::now();
    tl_.ns_select += ns_since(tb0, tb1);
    int64_t r = StageDecode(segs.data(), m, &sg, true);
    if (r < 0) return r;
    pend_.conns.assign(conns, conns + n);
    pend_.rings.assign(rings, rings + n);
    if (sg.zc) {
      if (handler_ >= 0 && (r = ChainHandler(&sg)) < 0) return r;
      pend_.arena = sg.arena;
    } else {
      // frames + payload land in pinned memory with the summary: one
      // synchronisation for a pass whose output fits the first estimate
      hipStream_t st = (hipStream_t)gevws_ctx_stream(ctx_);
      pend_.est_f = std::min<uint64_t>(sg.max_frames, sg.total / 48 + 2ull * m + 16);
      pend_.est_p = std::min<uint64_t>(sg.payload_cap, sg.total + 16 * pend_.est_f + 16);
      if (!grow_host(&h_out_, &h_out_cap_, pend_.est_f * sizeof(gevws_frame))) return fail();
      pend_.arena = pool_->Acquire(pend_.est_p);
      if (!pend_.arena) return fail();
      if (hipMemcpyAsync(h_out_, d_frames_, pend_.est_f * sizeof(gevws_frame), hipMemcpyDeviceToHost, st) !=
              hipSuccess ||
          hipMemcpyAsync(pend_.arena.get(), d_payload_, pend_.est_p, hipMemcpyDeviceToHost, st) != hipSuccess)
        return fail();
    }
    pend_.active = true;
    const auto tb2 = std::chrono::steady_clock::now();
    tl_.ns_stage += ns_since(stage_begin_, stage_end_);
    tl_.ns_launch += ns_since(stage_end_, tb2);
    return (int64_t)m;
  }

  int64_t EndBatch() {
    if (!pend_.active) return 0;
    pend_.active = false;
    DeviceScope scope(gevws_ctx_device(ctx_));
    Staged& sg = pend_.sg;
    std::shared_ptr<uint8_t> arena = std::move(pend_.arena);
    const auto te0 = std::chrono::steady_clock::now();
    int64_t r = Finish(&sg);
    if (r < 0) return r;
    const auto te1 = std::chrono::steady_clock::now();
    ++tl_.passes;
    tl_.ns_wait += ns_since(te0, te1);
    if (last_signalled_ && h_ticks_ && !sg.retried) {
      const uint64_t d0 = __atomic_load_n(h_ticks_ + 0, __ATOMIC_ACQUIRE), d1 = h_ticks_[1];
      const uint64_t k0 = h_ticks_[2], k1 = h_ticks_[3];
      ++tl_.signalled;
      if (d1 > d0 && d0) tl_.ns_gpu_decode += (uint64_t)((double)(d1 - d0) * ns_per_tick_);
      if (k1 > k0 && k0) tl_.ns_gpu_handler += (uint64_t)((double)(k1 - k0) * ns_per_tick_);
      if (k0 > d1 && d1 && k0) tl_.ns_gpu_gap += (uint64_t)((double)(k0 - d1) * ns_per_tick_);
      memset(h_ticks_, 0, 32);
    }
    struct DeliverTimer {  // the rest of EndBatch: queueing the frames on their connections
      gevws_protocol_timeline& tl;
      std::chrono::steady_clock::time_point t;
      ~DeliverTimer() { tl.ns_deliver += ns_since(t, std::chrono::steady_clock::now()); }
    } deliver_timer{tl_, te1};
    if (sg.zc) {
      arena = sg.arena;
    } else {
      hipStream_t st = (hipStream_t)gevws_ctx_stream(ctx_);
      const gevws_summary& sum = sg.sum;
      const uint64_t fb = sum.frames * sizeof(gevws_frame);
      if (sg.retried || sum.frames > pend_.est_f || sum.payload_bytes > pend_.est_p) {  // more than estimated
        if (sum.payload_bytes > pend_.est_p && !(arena = pool_->Acquire(sum.payload_bytes))) return fail();
        if (!grow_host(&h_out_, &h_out_cap_, fb)) return fail();
        if ((fb && hipMemcpyAsync(h_out_, d_frames_, fb, hipMemcpyDeviceToHost, st) != hipSuccess) ||
            (sum.payload_bytes &&
             hipMemcpyAsync(arena.get(), d_payload_, sum.payload_bytes, hipMemcpyDeviceToHost, st) != hipSuccess) ||
            hipStreamSynchronize(st) != hipSuccess)
          return fail();
      }
    }
    if (handler_ >= 0 && !ChainedDone(&sg)) {
      const int64_t h = RunHandler(&sg, arena);
      if (h < 0) return h;
    }
    return Deliver(pend_.conns.data(), pend_.rings.data(), pend_.sel, sg, arena);
  }

  // Hands a finished pass's frames to their connections in stream order and
  // carries each connection's completeness gate to the next pass.
  int64_t Deliver(Connection* const* conns, RingBuffer* const* rings, const std::vector<uint32_t>& sel,
                  const Staged& sg, const std::shared_ptr<uint8_t>& arena) {
    const uint32_t m = (uint32_t)sel.size();
    const gevws_summary& sum = sg.sum;
    const gevws_conn_out* cout = reinterpret_cast<const gevws_conn_out*>(h_res_ + sizeof(gevws_summary));
    const gevws_frame* fr = reinterpret_cast<const gevws_frame*>(h_out_);
    const uint8_t* hin = h_in_ + sg.coff;
    const bool handled = handler_ >= 0 && sg.hd.done;
    const int64_t* rof = reinterpret_cast<const int64_t*>(h_rof_);
    const uint64_t* roff = reinterpret_cast<const uint64_t*>(h_roff_);
    const uint64_t nrep = handled ? sg.hd.disp.frames : 0, wire = handled ? sg.hd.enc.payload_bytes : 0;
    // hand the frames to their connections in stream order
    for (uint32_t j = 0; j < m; ++j) {
      Connection* c = conns[sel[j]];
      const gevws_conn_out& o = cout[j];
      uint64_t prev_end = sg.cin[j].off;
      for (uint32_t k = 0; k < o.nframes; ++k) {
        const gevws_frame& f = fr[o.first_frame + k];
        Delivered d;
        d.hdr = f.hdr;
        d.frame_bytes = f.src_off + (uint64_t)f.hdr.length - prev_end;
        d.payload_off = f.payload_off;
        d.arena = arena;
        d.handled = handled;
        if (handled) {
          const int64_t r = rof[o.first_frame + k];
          if (r >= 0) {
            d.replies = sg.hd.rbuf;
            d.reply_off = roff[r];
            d.reply_len = ((uint64_t)r + 1 < nrep ? roff[r + 1] : wire) - roff[r];
          }
          d.shutdown = f.hdr.opcode == 0x8;  // ws.OpClose: ShutdownWrite after the reply (wrap.go:52-56)
        }
        prev_end = f.src_off + (uint64_t)f.hdr.length;
        c->queue.push_back(std::move(d));
      }
      if (o.status < 0) {
        c->poisoned = o.status;
        continue;
      }
      // the gate for the next pass: the frame at the end of what was decoded,
      // read from the staged copy of the ring (still in pinned memory)
      c->need = o.consumed + Need(hin + sg.cin[j].off + o.consumed, sg.cin[j].len - o.consumed);
      c->need_ring = rings[sel[j]];
      c->need_at = rings[sel[j]]->Retrieved();
    }
    return (int64_t)sum.frames;
  }

  // Host segments in, caller buffers out (gevws_decode_host_batch).
  int64_t DecodeHost(const gevws_host_conn* segs, uint32_t n, gevws_frame* frames, uint64_t max_frames,
                     uint8_t* payload, uint64_t payload_cap, gevws_conn_out* conn_out, gevws_summary* sum_out) {
    gevws_summary zero{};
    *sum_out = zero;
    if (pend_.active) {  // the pass in flight shares the staging buffers: deliver it first
      const int64_t e = EndBatch();
      if (e < 0) return e;
    }
    if (n == 0) return 0;
    DeviceScope scope(gevws_ctx_device(ctx_));
    Staged sg;
    int64_t r = StageDecode(segs, n, &sg, true);
    if (r < 0) return r;
    r = Finish(&sg);
    if (r < 0) return r;
    const gevws_summary& sum = sg.sum;
    // src_off is reported relative to each connection's own stream
    *sum_out = sum;
    if (sum.frames > max_frames || sum.payload_bytes > payload_cap) {
      sum_out->status = GEVWS_ERR_CAPACITY;
      return GEVWS_ERR_CAPACITY;
    }
    memcpy(conn_out, h_res_ + sizeof(gevws_summary), n * sizeof(gevws_conn_out));
    if (sg.zc) {  // the results are in mapped host memory already: the caller's buffers are host memory too
      if (sum.frames) memcpy(frames, h_out_, sum.frames * sizeof(gevws_frame));
      if (sum.payload_bytes) memcpy(payload, sg.arena.get(), sum.payload_bytes);
    } else {
      hipStream_t st = (hipStream_t)gevws_ctx_stream(ctx_);
      if ((sum.frames && hipMemcpyAsync(frames, d_frames_, sum.frames * sizeof(gevws_frame),
                                        hipMemcpyDeviceToHost, st) != hipSuccess) ||
          (sum.payload_bytes &&
           hipMemcpyAsync(payload, d_payload_, sum.payload_bytes, hipMemcpyDeviceToHost, st) != hipSuccess) ||
          hipStreamSynchronize(st) != hipSuccess)
        return fail();
    }
    for (uint32_t j = 0; j < n; ++j)
      for (uint32_t k = 0; k < conn_out[j].nframes; ++k) frames[conn_out[j].first_frame + k].src_off -= sg.cin[j].off;
    return (int64_t)sum.frames;
  }

  void GetStats(gevws_protocol_stats* out) const { *out = stats_; }
  void GetTimeline(gevws_protocol_timeline* out) const { *out = tl_; }
  int SetHandler(int policy) {
    if (policy < -1 || policy > GEVWS_HANDLER_ECHO_TEXT) return GEVWS_ERR_INVALID;
    handler_ = policy;
    return GEVWS_OK;
  }
  // The device handler's answer for the frame UnPacket last returned on c.
  int Reply(Connection* c, const uint8_t** reply, uint64_t* len, int* shutdown) const {
    *reply = nullptr;
    *len = 0;
    *shutdown = 0;
    if (!c->reply_valid) return GEVWS_ERR_INVALID;
    if (c->reply_len) *reply = c->current_replies.get() + c->reply_off;
    *len = c->reply_len;
    *shutdown = c->shutdown ? 1 : 0;
    return GEVWS_OK;
  }
  void SetZeroCopyMax(uint64_t bytes) { zc_max_ = bytes; }
  // The context's resident decode service for this protocol's zero-copy
  // passes without a handler step (gevws_ctx_set_service).
  int SetService(int on) {
    const int r = gevws_ctx_set_service(ctx_, on);
    if (r == GEVWS_OK) service_ = on != 0;
    return r;
  }
  int SetDirect(int on) {
    const int r = gevws_ctx_set_direct(ctx_, on);
    if (r == GEVWS_OK) direct_ = on != 0;
    return r;
  }

 private:
  struct DeviceScope {
    int prev = -1, dev;
    explicit DeviceScope(int d) : dev(d) {
      if (hipGetDevice(&prev) != hipSuccess) prev = -1;
      if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceScope() {
      if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
    }
  };

  // A zero-copy pass with the handler on: the handler step (dispatch +
  // FrameToBytes, counts read on the device from the decode's summary) is
  // enqueued right behind the decode, sized for the most the staged bytes can
  // hold -- <= max_frames frames, payload <= the staged bytes, the close
  // bodies' aux region after payload_cap in the pass's mapped arena -- so the
  // pass has ONE synchronisation instead of two.  When the decode had to be
  // re-run (capacity) or the step reports a capacity miss, RunHandler runs it
  // again with the exact sizes.
  static uint64_t ChainAuxSlots(const Staged& sg) { return std::min<uint64_t>(std::max<uint64_t>(sg.max_frames, 1), 4096); }
  static uint64_t ChainArenaBytes(const Staged& sg) {
    return ((sg.payload_cap + 15) & ~15ull) + 128 * ChainAuxSlots(sg) + 32;
  }
  int64_t ChainHandler(Staged* sg) {
    const uint64_t n = std::max<uint64_t>(sg->max_frames, 1);
    hipStream_t st = (hipStream_t)gevws_ctx_stream(ctx_);
    const uint64_t aux_off = (sg->payload_cap + 15) & ~15ull;
    const uint64_t rcap = sg->total + 141 * n + 16;
    if (!grow_host(&h_rof_, &h_rof_cap_, 8 * n) || !grow_host(&h_roff_, &h_roff_cap_, 8 * n) ||
        !grow_host(&h_hs_, &h_hs_cap_, 2 * sizeof(gevws_summary)) || !grow_dev(&d_rep_, &d_rep_cap_, 32 * n))
      return fail();
    sg->hd = Handled{};
    sg->hd.rbuf = pool_->Acquire(rcap + GEVWS_OUT_PAD);
    if (!sg->hd.rbuf || sg->arena_cap < ChainArenaBytes(*sg)) return fail();
    const gevws_frame* dfr = (const gevws_frame*)device_of(h_out_);
    const gevws_summary* dsum = (const gevws_summary*)device_of(h_res_);
    uint8_t* dpay = (uint8_t*)device_of(sg->arena.get());
    gevws_summary* dhs = (gevws_summary*)device_of(h_hs_);
    int64_t* drof = (int64_t*)device_of(h_rof_);
    uint64_t* droff = (uint64_t*)device_of(h_roff_);
    uint8_t* drb = (uint8_t*)device_of(sg->hd.rbuf.get());
    if (!dfr || !dsum || !dpay || !dhs || !drof || !droff || !drb) return fail();
    if (gevws_handle_decoded_async(ctx_, st, dfr, n, dsum, handler_, dpay, aux_off, 128 * ChainAuxSlots(*sg),
                                   (gevws_out_frame*)d_rep_, drof, dhs, drb, rcap, droff, dhs + 1) != GEVWS_OK)
      return fail();
    sg->hd.chained = true;
    sg->seq = gevws_ctx_completion_seq(ctx_);  // the handler step is the pass's last launch
    ++stats_.chained_handler_passes;
    return 0;
  }
  // After Finish: did the chained step answer this pass?
  bool ChainedDone(Staged* sg) {
    if (!sg->hd.chained || sg->retried) return false;
    memcpy(&sg->hd.disp, h_hs_, sizeof(gevws_summary));
    memcpy(&sg->hd.enc, h_hs_ + sizeof(gevws_summary), sizeof(gevws_summary));
    if (sg->hd.disp.status != GEVWS_OK || sg->hd.enc.status != GEVWS_OK) return false;
    sg->hd.done = true;
    ++stats_.handler_passes;
    return true;
  }

  // After the decode of sg finished (its frames in the pass's outputs: device
  // memory, or mapped host memory for a zero-copy pass): the handler step,
  // sized exactly from the decode's summary, then one synchronisation.  The
  // close bodies go to an aux region behind the payloads in the pass's
  // payload arena; a capacity miss (more closes than the first guess of aux
  // slots) re-runs the step once with the exact count.
  int64_t RunHandler(Staged* sg, std::shared_ptr<uint8_t>& arena) {
    const uint64_t n = sg->sum.frames;
    sg->hd = Handled{};
    sg->hd.done = true;
    if (n == 0) return 0;
    hipStream_t st = (hipStream_t)gevws_ctx_stream(ctx_);
    const uint64_t aux_off = (sg->sum.payload_bytes + 15) & ~15ull;
    uint64_t aux_slots = std::min<uint64_t>(n, 4096);
    // reply wire bytes: <= L + 10 per echo / pong / ping, <= 131 per close
    const uint64_t rcap = sg->sum.payload_len + 141 * n + 16;
    if (!grow_host(&h_rof_, &h_rof_cap_, 8 * n) || !grow_host(&h_roff_, &h_roff_cap_, 8 * n) ||
        !grow_host(&h_hs_, &h_hs_cap_, 2 * sizeof(gevws_summary)) || !grow_dev(&d_rep_, &d_rep_cap_, 32 * n))
      return fail();
    sg->hd.rbuf = pool_->Acquire(rcap + GEVWS_OUT_PAD);
    if (!sg->hd.rbuf) return fail();
    for (int attempt = 0; attempt < 2; ++attempt) {
      // the aux region lives in the payload arena the decode wrote
      uint8_t* dpay = nullptr;
      const uint64_t need = aux_off + 128 * aux_slots + 32;
      if (sg->zc) {
        if (sg->arena_cap < need) {  // a bigger mapped arena holding the decoded payloads
          std::shared_ptr<uint8_t> a = pool_->Acquire(need);
          if (!a) return fail();
          memcpy(a.get(), sg->arena.get(), sg->sum.payload_bytes);
          sg->arena = a;
          sg->arena_cap = need;
          arena = a;
        }
        dpay = (uint8_t*)device_of(sg->arena.get());
      } else {
        if (d_payload_cap_ < need) {  // keep the decoded payloads while growing
          void* np = nullptr;
          if (hipStreamSynchronize(st) != hipSuccess || hipMalloc(&np, need + need / 2) != hipSuccess ||
              hipMemcpy(np, d_payload_, sg->sum.payload_bytes, hipMemcpyDeviceToDevice) != hipSuccess)
            return fail();
          (void)hipFree(d_payload_);
          d_payload_ = np;
          d_payload_cap_ = need + need / 2;
        }
        dpay = (uint8_t*)d_payload_;
      }
      const gevws_frame* dfr = sg->zc ? (const gevws_frame*)device_of(h_out_) : (const gevws_frame*)d_frames_;
      gevws_summary* dhs = (gevws_summary*)device_of(h_hs_);
      int64_t* drof = (int64_t*)device_of(h_rof_);
      uint64_t* droff = (uint64_t*)device_of(h_roff_);
      uint8_t* drb = (uint8_t*)device_of(sg->hd.rbuf.get());
      if (!dpay || !dfr || !dhs || !drof || !droff || !drb) return fail();
      if (gevws_dispatch_async(ctx_, st, dfr, n, handler_, dpay, aux_off, 128 * aux_slots, (gevws_out_frame*)d_rep_,
                               drof, dhs) != GEVWS_OK ||
          gevws_encode_replies_async(ctx_, st, (const gevws_out_frame*)d_rep_, n, dhs, dpay, drb, rcap, droff,
                                     dhs + 1) != GEVWS_OK ||
          hipStreamSynchronize(st) != hipSuccess)
        return fail();
      memcpy(&sg->hd.disp, h_hs_, sizeof(gevws_summary));
      memcpy(&sg->hd.enc, h_hs_ + sizeof(gevws_summary), sizeof(gevws_summary));
      if (sg->hd.disp.status == GEVWS_ERR_CAPACITY && attempt == 0) {
        aux_slots = std::max<uint64_t>(sg->hd.disp.payload_bytes, 1);  // aux slots the closes need
        continue;
      }
      break;
    }
    if (sg->hd.disp.status != GEVWS_OK || sg->hd.enc.status != GEVWS_OK) {
      log_error("handler: ", sg->hd.disp.status != GEVWS_OK ? sg->hd.disp.status : sg->hd.enc.status);
      return GEVWS_ERR_DEVICE;
    }
    ++stats_.handler_passes;
    return 0;
  }

  // Bytes that must be buffered at p for its first frame to be complete
  // (read.go:20-23, U1 and the protocol.go:47 gate); 0 when the header is
  // unreadable (ErrHeaderLengthMSB: a pass reports it).
  static uint64_t Need(const uint8_t* p, uint64_t avail) {
    gevws_header h;
    uint32_t hl = 0;
    const int r = gevws_parse_header(p, avail, &h, &hl);
    if (r == GEVWS_OK) return (uint64_t)hl + (uint64_t)h.length;
    if (r == GEVWS_NEED_MORE) return std::max<uint64_t>(6, hl);
    return 0;
  }

  // May a device pass decode anything new for this connection (whose queue is
  // empty, so the ring's read position is its first undecoded frame)?  The
  // carried count answers most calls; otherwise the frame's header is parsed
  // on the host, 14 bytes at most.
  bool Ready(Connection* c, RingBuffer* ring) {
    const uint64_t len = ring->Length();
    if (len < 6) return false;  // read.go:20-23
    if (c->need_ring == ring && c->need_at == ring->Retrieved() && len < c->need) return false;
    const uint8_t *a, *b;
    uint64_t na, nb;
    ring->PeekAll(&a, &na, &b, &nb);
    gevws_header h;
    uint32_t hl = 0;
    const int r = gevws_parse_header_ring(a, na, b, nb, &h, &hl);
    if (r == GEVWS_OK) c->need = (uint64_t)hl + (uint64_t)h.length;
    else if (r == GEVWS_NEED_MORE) c->need = std::max<uint64_t>(6, hl);
    else c->need = 0;  // ErrHeaderLengthMSB: the pass reports and poisons
    c->need_ring = ring;
    c->need_at = ring->Retrieved();
    return len >= c->need;
  }

  // The device handler's step of a pass: HandlerWrap.OnMessage over every
  // decoded frame (gevws_dispatch_decoded_async: close -> HandleClose reply,
  // ping -> pong, pong -> ping, data -> the policy's echo) and FrameToBytes of
  // the replies (gevws_encode_replies_async), written into mapped pinned host
  // memory -- reply_of / wire offsets / summaries in the protocol's buffers,
  // the reply bytes in a pool buffer the delivered frames hold.
  struct Handled {
    bool done = false;
    bool chained = false;  // enqueued behind the decode (ChainHandler)
    gevws_summary disp{}, enc{};
    std::shared_ptr<uint8_t> rbuf;
  };
  struct Staged {
    Handled hd;
    std::vector<gevws_conn_in> cin;
    uint64_t coff = 0, total = 0, res = 0, max_frames = 0, payload_cap = 0;
    bool retried = false;  // Finish re-ran the pass: copies enqueued before it are stale
    bool zc = false;       // zero-copy pass: kernels on the pinned buffers themselves
    bool flagged = false;  // its one-launch kernels signal the protocol's flag word
    int64_t seq = -1;      // ... with this number (taken right after its launches)
    bool posted = false;   // posted to the context's resident decode service
    std::shared_ptr<uint8_t> arena;  // zero-copy: the payload arena the kernels write
    uint64_t arena_cap = 0;
    gevws_summary sum{};
  };

  // Join each connection's segments into pinned staging behind the connection
  // table, ONE H2D, enqueue the decode on the context's stream and the D2H of
  // {summary, conn_out} into pinned h_res_ (no synchronisation yet: the caller
  // adds its own copies, then Finish waits).
  // (stage_begin_ / stage_end_: the staging phase of the pass timeline; a
  // path that returns before the launch books no staging time)
  int64_t StageDecode(const gevws_host_conn* segs, uint32_t m, Staged* sg, bool allow_zc = false) {
    stage_begin_ = stage_end_ = std::chrono::steady_clock::now();
    uint64_t total = 0;
    for (uint32_t j = 0; j < m; ++j) total += segs[j].n0 + segs[j].n1;
    sg->cin.resize(m);
    sg->total = total;
    sg->coff = ((uint64_t)m * sizeof(gevws_conn_in) + 255) & ~255ull;  // input starts here
    const uint64_t stage = sg->coff + total + GEVWS_IN_PAD;
    if (!grow_host(&h_in_, &h_in_cap_, stage)) return fail();
    uint8_t* hin = h_in_ + sg->coff;
    uint64_t off = 0;
    for (uint32_t j = 0; j < m; ++j) {
      if (segs[j].n0) memcpy(hin + off, segs[j].seg0, segs[j].n0);
      if (segs[j].n1) memcpy(hin + off + segs[j].n0, segs[j].seg1, segs[j].n1);
      sg->cin[j] = {off, segs[j].n0 + segs[j].n1};
      off += sg->cin[j].len;
    }
    memcpy(h_in_, sg->cin.data(), m * sizeof(gevws_conn_in));
    memset(hin + off, 0, GEVWS_IN_PAD);
    sg->res = sizeof(gevws_summary) + (uint64_t)m * sizeof(gevws_conn_out);
    if (!grow_host(&h_res_, &h_res_cap_, sg->res)) return fail();
    // every frame is >= 2 bytes; the arena bound covers frames of >= 64 bytes
    // (Finish retries with the exact sizes on GEVWS_ERR_CAPACITY)
    sg->max_frames = std::min<uint64_t>(total / 2 + 1, 0xFFFFFFFFull);
    sg->payload_cap = total + 16 * std::min<uint64_t>(sg->max_frames, total / 64 + 64) + 64;
    hipStream_t st = (hipStream_t)gevws_ctx_stream(ctx_);
    sg->zc = allow_zc && total <= zc_max_;
    if (sg->zc) {
      sg->flagged = EnsureFlag();  // (without it the pass synchronises the stream)
      // small pass: no copies -- the kernels read the staged bytes and write
      // records, payload and results into mapped host memory (a pass is then
      // its launches and one synchronisation, no H2D / D2H on the way)
      sg->max_frames = std::min<uint64_t>(sg->max_frames, total / 48 + 2ull * m + 16);
      sg->payload_cap = std::min<uint64_t>(sg->payload_cap, total + 16 * sg->max_frames + 16);
      ++stats_.zero_copy_passes;
    } else if (!grow_dev(&d_in_, &d_in_cap_, stage) || !grow_dev(&d_res_, &d_res_cap_, sg->res) ||
               hipMemcpyAsync(d_in_, h_in_, stage, hipMemcpyHostToDevice, st) != hipSuccess) {
      return fail();
    }
    ++stats_.device_passes;
    stats_.conns_staged += m;
    stats_.bytes_staged += stage;
    stage_end_ = std::chrono::steady_clock::now();
    return Launch(sg);
  }

  int64_t Launch(Staged* sg, bool may_post = true) {
    hipStream_t st = (hipStream_t)gevws_ctx_stream(ctx_);
    sg->posted = false;
    if (sg->zc) {
      const uint32_t m = (uint32_t)sg->cin.size();
      if (!grow_host(&h_out_, &h_out_cap_, std::max<uint64_t>(sg->max_frames, 1) * sizeof(gevws_frame)))
        return fail();
      const uint64_t abytes = handler_ >= 0 ? ChainArenaBytes(*sg) : sg->payload_cap + 16;
      if (!sg->arena || sg->arena_cap < abytes) {
        sg->arena = pool_->Acquire(abytes);
        sg->arena_cap = abytes;
      }
      uint8_t* din = (uint8_t*)device_of(h_in_);
      uint8_t* dres = (uint8_t*)device_of(h_res_);
      void* dfr = sg->arena ? device_of(h_out_) : nullptr;
      void* dpay = sg->arena ? device_of(sg->arena.get()) : nullptr;
      if (!din || !dres || !dfr || !dpay) return fail();
      // (with the resident service on and no handler chained behind, the
      // pass is posted to it instead of launched: gevws_decode_batch_post)
      const bool post = may_post && (service_ || direct_) && handler_ < 0 && sg->flagged;
      int64_t posts0 = 0, posts1 = 0;
      if (post) (void)gevws_ctx_service_stats(ctx_, nullptr, &posts0);
      const int r = post
                        ? gevws_decode_batch_post(ctx_, din + sg->coff, sg->total, (gevws_conn_in*)din, m,
                                                  (gevws_frame*)dfr, sg->max_frames, (uint8_t*)dpay, sg->payload_cap,
                                                  (gevws_conn_out*)(dres + sizeof(gevws_summary)), (gevws_summary*)dres)
                        : gevws_decode_batch_async(ctx_, st, din + sg->coff, sg->total, (gevws_conn_in*)din, m,
                                                   (gevws_frame*)dfr, sg->max_frames, (uint8_t*)dpay, sg->payload_cap,
                                                   (gevws_conn_out*)(dres + sizeof(gevws_summary)),
                                                   (gevws_summary*)dres);
      sg->seq = gevws_ctx_completion_seq(ctx_);
      if (post) (void)gevws_ctx_service_stats(ctx_, nullptr, &posts1);
      sg->posted = posts1 > posts0;  // (else launched)
      if (sg->posted) ++stats_.service_passes;
      return r;
    }
    if (!grow_dev(&d_frames_, &d_frames_cap_, sg->max_frames * sizeof(gevws_frame)) ||
        !grow_dev(&d_payload_, &d_payload_cap_, sg->payload_cap + 16))
      return fail();
    const uint32_t m = (uint32_t)sg->cin.size();
    gevws_summary* d_sum = (gevws_summary*)d_res_;
    gevws_conn_out* d_cout = (gevws_conn_out*)((uint8_t*)d_res_ + sizeof(gevws_summary));
    int r = gevws_decode_batch_async(ctx_, st, (const uint8_t*)d_in_ + sg->coff, sg->total, (gevws_conn_in*)d_in_, m,
                                     (gevws_frame*)d_frames_, sg->max_frames, (uint8_t*)d_payload_, sg->payload_cap,
                                     d_cout, d_sum);
    if (r != GEVWS_OK) return r;
    if (hipMemcpyAsync(h_res_, d_res_, sg->res, hipMemcpyDeviceToHost, st) != hipSuccess) return fail();
    return GEVWS_OK;
  }

  // A zero-copy pass's launches end with a one-launch kernel that signals
  // the protocol's mapped flag word (gevws_ctx_set_completion_flag): the host
  // spins on it (~1 us after the kernel's last write) instead of sleeping in
  // hipStreamSynchronize.  Passes with copies behind the kernels, or whose
  // last launch does not signal, synchronise the stream.
  // (set on the context for every zero-copy pass: another protocol on the
  // same context may have pointed it elsewhere since)
  bool EnsureFlag() {
    if (!h_flag_) {
      if (hipHostMalloc((void**)&h_flag_, 64, kHostFlags) != hipSuccess) {
        h_flag_ = nullptr;
        return false;
      }
      __atomic_store_n(h_flag_, 0u, __ATOMIC_RELEASE);
    }
    uint32_t* d = (uint32_t*)device_of(h_flag_);
    if (!d || gevws_ctx_set_completion_flag(ctx_, d) != GEVWS_OK) {
      (void)hipHostFree(h_flag_);
      h_flag_ = nullptr;
      return false;
    }
    if (!h_ticks_ && hipHostMalloc((void**)&h_ticks_, 64, kHostFlags) == hipSuccess) {
      int khz = 0;
      if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, gevws_ctx_device(ctx_)) == hipSuccess &&
          khz > 0)
        ns_per_tick_ = 1e6 / khz;
    }
    if (h_ticks_) {
      memset(h_ticks_, 0, 32);  // a kernel of this pass that stamps sets its end tick
      (void)gevws_ctx_set_timeline_ticks(ctx_, (uint64_t*)device_of(h_ticks_));
    }
    return true;
  }
  int64_t Wait(Staged* sg) {
    last_signalled_ = false;
    const int64_t seq = (sg->zc && sg->flagged) ? sg->seq : -1;
    if (seq >= 0) {
      const auto t0 = std::chrono::steady_clock::now();
      for (uint64_t i = 1;; ++i) {
        if (__atomic_load_n(h_flag_, __ATOMIC_ACQUIRE) == (uint32_t)seq) {
          ++stats_.signalled_passes;
          last_signalled_ = true;
          return 0;
        }
        // a pass takes tens of us: past 50 ms, wait for the stream instead
        if ((i & 4095) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) break;
        __builtin_ia32_pause();
      }
    }
    // (the stream, a live service instance -- stopped first -- and direct passes)
    if (gevws_ctx_synchronize(ctx_) != GEVWS_OK) return fail();
    if (seq >= 0 && __atomic_load_n(h_flag_, __ATOMIC_ACQUIRE) == (uint32_t)seq) {
      last_signalled_ = true;
    } else if (sg->posted) {
      // the service's instance ended without the pass (not seen): launch it
      ++stats_.service_misses;
      if (Launch(sg, false) < 0 || gevws_ctx_synchronize(ctx_) != GEVWS_OK) return fail();
    }
    return 0;
  }

  // Waits for the pass (and whatever the caller enqueued after it); on
  // GEVWS_ERR_CAPACITY runs it once more with the exact sizes.
  int64_t Finish(Staged* sg) {
    if (Wait(sg) < 0) return GEVWS_ERR_DEVICE;
    memcpy(&sg->sum, h_res_, sizeof(gevws_summary));
    if (sg->sum.status == GEVWS_ERR_CAPACITY) {
      sg->max_frames = std::max<uint64_t>(sg->sum.frames, 1);
      sg->payload_cap = std::max<uint64_t>(sg->sum.payload_bytes, 16);
      sg->retried = true;
      int64_t r = Launch(sg);
      if (r < 0) return r;
      if (Wait(sg) < 0) return GEVWS_ERR_DEVICE;
      memcpy(&sg->sum, h_res_, sizeof(gevws_summary));
    }
    return sg->sum.status == GEVWS_OK ? (int64_t)sg->sum.frames : (int64_t)sg->sum.status;
  }

  // Every failure waits for the context's stream first: a failing step may
  // follow an enqueued H2D copy or a zero-copy kernel still reading the
  // pinned staging, which the next pass would overwrite.
  int64_t fail() {
    if (ctx_) (void)gevws_ctx_synchronize(ctx_);  // (a service instance stopped, direct passes drained too)
    log_error("device: ", GEVWS_ERR_DEVICE);
    return GEVWS_ERR_DEVICE;
  }
  static bool grow_host(uint8_t** p, uint64_t* cap, uint64_t need) {
    if (need <= *cap) return true;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    uint64_t want = std::max<uint64_t>(need + need / 2, 1 << 16);
    if (hipHostMalloc((void**)p, want, kHostFlags) != hipSuccess) {
      *cap = 0;
      return false;
    }
    *cap = want;
    return true;
  }
  static bool grow_dev(void** p, uint64_t* cap, uint64_t need) {
    if (need <= *cap && *p) return true;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    uint64_t want = std::max<uint64_t>(need + need / 2, 4096);
    if (hipMalloc(p, want) != hipSuccess) {
      *cap = 0;
      return false;
    }
    *cap = want;
    return true;
  }
  void release() {
    if (ctx_ && service_) (void)gevws_ctx_set_service(ctx_, 0);
    if (ctx_ && direct_) (void)gevws_ctx_set_direct(ctx_, 0);
    if (ctx_) (void)gevws_ctx_synchronize(ctx_);
    if (h_flag_) {
      if (ctx_) (void)gevws_ctx_set_completion_flag(ctx_, nullptr);
      (void)hipHostFree(h_flag_);
      h_flag_ = nullptr;
    }
    if (h_ticks_) {
      if (ctx_) (void)gevws_ctx_set_timeline_ticks(ctx_, nullptr);
      (void)hipHostFree(h_ticks_);
      h_ticks_ = nullptr;
    }
    for (uint8_t* p : {h_in_, h_res_, h_out_, h_rof_, h_roff_, h_hs_})
      if (p) (void)hipHostFree(p);
    for (void* p : {d_in_, d_res_, d_frames_, d_payload_, d_rep_})
      if (p) (void)hipFree(p);
  }

  gevws_ctx* ctx_;
  uint32_t* h_flag_ = nullptr;  // completion word of the one-launch kernels (mapped pinned)
  struct Pending {  // the pass between BeginBatch and EndBatch
    bool active = false;
    std::vector<Connection*> conns;
    std::vector<RingBuffer*> rings;
    std::vector<uint32_t> sel;
    Staged sg;
    std::shared_ptr<uint8_t> arena;
    uint64_t est_f = 0, est_p = 0;
  };
  Pending pend_;
  const Upgrader* upgrader_ = nullptr;
  std::shared_ptr<PinnedPool> pool_;   // payload arenas handed out with the frames
  uint8_t *h_in_ = nullptr, *h_res_ = nullptr, *h_out_ = nullptr;  // pinned staging
  uint64_t h_in_cap_ = 0, h_res_cap_ = 0, h_out_cap_ = 0;
  void *d_in_ = nullptr, *d_res_ = nullptr, *d_frames_ = nullptr, *d_payload_ = nullptr;
  uint64_t d_in_cap_ = 0, d_res_cap_ = 0, d_frames_cap_ = 0, d_payload_cap_ = 0;
  uint64_t epoch_ = 0;
  uint64_t zc_max_ = GEVWS_ZERO_COPY_MAX_DEFAULT;
  int handler_ = -1;  // device handler policy (GEVWS_HANDLER_*), -1 = none
  bool service_ = false;  // passes posted to the context's resident decode service
  bool direct_ = false;   // passes written into the context's own queue (gevws_ctx_set_direct)
  uint8_t *h_rof_ = nullptr, *h_roff_ = nullptr, *h_hs_ = nullptr;  // handler outputs (mapped pinned)
  uint64_t h_rof_cap_ = 0, h_roff_cap_ = 0, h_hs_cap_ = 0;
  void* d_rep_ = nullptr;  // reply records (gevws_out_frame)
  uint64_t d_rep_cap_ = 0;
  gevws_protocol_stats stats_{};
  // per-pass timeline (gevws_protocol_get_timeline): host phases and, via the
  // one-launch kernels' tick stamps in h_ticks_ (mapped pinned u64[4]), GPU time
  gevws_protocol_timeline tl_{};
  uint64_t* h_ticks_ = nullptr;
  double ns_per_tick_ = 10.0;  // 100 MHz unless the device says otherwise
  std::chrono::steady_clock::time_point stage_begin_, stage_end_;
  bool last_signalled_ = false;
  static uint64_t ns_since(std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
  }
};

}  // namespace gevws

struct gevws_ring : gevws::RingBuffer {
  using gevws::RingBuffer::RingBuffer;
};
struct gevws_conn : gevws::Connection {};
struct gevws_upgrader : gevws::Upgrader {};
struct gevws_protocol : gevws::Protocol {
  using gevws::Protocol::Protocol;
};

extern "C" {

gevws_ring* gevws_ring_new(uint64_t size) { return new gevws_ring(size); }
void gevws_ring_free(gevws_ring* r) { delete r; }
uint64_t gevws_ring_write(gevws_ring* r, const uint8_t* p, uint64_t n) { return r->Write(p, n); }
uint64_t gevws_ring_length(const gevws_ring* r) { return r->Length(); }
uint64_t gevws_ring_capacity(const gevws_ring* r) { return r->Capacity(); }
void gevws_ring_peek_all(const gevws_ring* r, const uint8_t** first, uint64_t* n_first, const uint8_t** end,
                         uint64_t* n_end) {
  r->PeekAll(first, n_first, end, n_end);
}
void gevws_ring_retrieve(gevws_ring* r, uint64_t n) { r->Retrieve(n); }

gevws_conn* gevws_conn_new(void) { return new gevws_conn(); }
void gevws_conn_free(gevws_conn* c) { delete c; }
void gevws_conn_set_upgraded(gevws_conn* c, int upgraded) { c->upgraded = upgraded != 0; }
int gevws_conn_upgraded(const gevws_conn* c) { return c->upgraded ? 1 : 0; }
uint64_t gevws_conn_pending(const gevws_conn* c) { return c->queue.size(); }

gevws_protocol* gevws_protocol_new(gevws_ctx* ctx) { return ctx ? new gevws_protocol(ctx) : nullptr; }
void gevws_protocol_free(gevws_protocol* p) { delete p; }

int gevws_protocol_unpacket(gevws_protocol* p, gevws_conn* c, gevws_ring* ring, gevws_header* ctx_out,
                            const uint8_t** out, uint64_t* out_len) {
  if (!p || !c || !ring || !ctx_out || !out || !out_len) return GEVWS_ERR_INVALID;
  return p->UnPacket(c, ring, ctx_out, out, out_len);
}

int64_t gevws_protocol_unpacket_batch(gevws_protocol* p, gevws_conn* const* conns, gevws_ring* const* rings,
                                      uint32_t n) {
  if (!p || (n && (!conns || !rings))) return GEVWS_ERR_INVALID;
  std::vector<gevws::Connection*> cs(n);
  std::vector<gevws::RingBuffer*> rs(n);
  for (uint32_t i = 0; i < n; ++i) {
    cs[i] = conns[i];
    rs[i] = rings[i];
  }
  return p->UnPacketBatch(cs.data(), rs.data(), n);
}

int64_t gevws_protocol_unpacket_batch_begin(gevws_protocol* p, gevws_conn* const* conns, gevws_ring* const* rings,
                                            uint32_t n) {
  if (!p || (n && (!conns || !rings))) return GEVWS_ERR_INVALID;
  std::vector<gevws::Connection*> cs(n);
  std::vector<gevws::RingBuffer*> rs(n);
  for (uint32_t i = 0; i < n; ++i) {
    cs[i] = conns[i];
    rs[i] = rings[i];
  }
  return p->BeginBatch(cs.data(), rs.data(), n);
}

int64_t gevws_protocol_unpacket_batch_end(gevws_protocol* p) {
  if (!p) return GEVWS_ERR_INVALID;
  return p->EndBatch();
}

void gevws_protocol_get_timeline(const gevws_protocol* p, gevws_protocol_timeline* out) {
  if (p && out) p->GetTimeline(out);
}

void gevws_protocol_get_stats(const gevws_protocol* p, gevws_protocol_stats* out) {
  if (!out) return;
  if (!p) {
    *out = gevws_protocol_stats{};
    return;
  }
  p->GetStats(out);
}

void gevws_protocol_set_zero_copy_max(gevws_protocol* p, uint64_t bytes) {
  if (p) p->SetZeroCopyMax(bytes);
}

int gevws_protocol_set_service(gevws_protocol* p, int on) {
  if (!p) return GEVWS_ERR_INVALID;
  return p->SetService(on);
}

int gevws_protocol_set_direct(gevws_protocol* p, int on) {
  if (!p) return GEVWS_ERR_INVALID;
  return p->SetDirect(on);
}

int gevws_protocol_set_handler(gevws_protocol* p, int policy) {
  if (!p) return GEVWS_ERR_INVALID;
  return p->SetHandler(policy);
}

int gevws_protocol_reply(const gevws_protocol* p, const gevws_conn* c, const uint8_t** reply, uint64_t* len,
                         int* shutdown_write) {
  if (!p || !c || !reply || !len || !shutdown_write) return GEVWS_ERR_INVALID;
  return p->Reply(const_cast<gevws_conn*>(c), reply, len, shutdown_write);
}

int64_t gevws_decode_host_batch(gevws_protocol* p, const gevws_host_conn* conns, uint32_t n,
                                gevws_frame* frames, uint64_t max_frames, uint8_t* payload, uint64_t payload_cap,
                                gevws_conn_out* conn_out, gevws_summary* summary) {
  if (!p || !summary || (n && (!conns || !conn_out))) return GEVWS_ERR_INVALID;
  return p->DecodeHost(conns, n, frames, max_frames, payload, payload_cap, conn_out, summary);
}

int64_t gevws_decode_host_stream(gevws_protocol* p, const uint8_t* seg0, uint64_t n0, const uint8_t* seg1,
                                 uint64_t n1, gevws_frame* frames, uint64_t max_frames, uint8_t* payload,
                                 uint64_t payload_cap, gevws_conn_out* conn_out, gevws_summary* summary) {
  const gevws_host_conn hc = {seg0, n0, seg1, n1};
  return gevws_decode_host_batch(p, &hc, 1, frames, max_frames, payload, payload_cap, conn_out, summary);
}

gevws_upgrader* gevws_upgrader_new(void) { return new gevws_upgrader(); }
void gevws_upgrader_free(gevws_upgrader* u) { delete u; }
void gevws_upgrader_set_header(gevws_upgrader* u, const uint8_t* hdr, uint64_t n) {
  if (u) u->header = hdr ? std::string((const char*)hdr, n) : std::string();
}
void gevws_upgrader_set_hooks(gevws_upgrader* u, const gevws_upgrader_hooks* hooks) {
  if (u) u->hooks = hooks ? *hooks : gevws_upgrader_hooks{};
}

static void fill_handshake(const gevws::HandshakeResult& r, gevws_handshake* hs) {
  hs->protocol = (const uint8_t*)r.protocol.data();
  hs->protocol_len = r.protocol.size();
  hs->extensions = (const uint8_t*)r.extensions.data();
  hs->extensions_len = r.extensions.size();
  hs->error = r.error;
  hs->http_code = r.http_code;
  hs->reason = r.reason.c_str();
}

int gevws_upgrader_upgrade(const gevws_upgrader* u, gevws_conn* c, gevws_ring* in, const uint8_t** out,
                           uint64_t* out_len, gevws_handshake* hs) {
  if (!u || !c || !in || !out || !out_len) return GEVWS_ERR_INVALID;
  u->Upgrade(c, in, &c->hs);
  *out = c->hs.out.empty() ? nullptr : (const uint8_t*)c->hs.out.data();
  *out_len = c->hs.out.size();
  if (hs) fill_handshake(c->hs, hs);
  return c->hs.error == GEVWS_HS_OK ? GEVWS_OK : GEVWS_ERR_HANDSHAKE;
}

int gevws_conn_handshake(const gevws_conn* c, gevws_handshake* hs) {
  if (!c || !hs) return GEVWS_ERR_INVALID;
  fill_handshake(c->hs, hs);
  return GEVWS_OK;
}

const char* gevws_handshake_error_string(int e) {
  switch (e) {
    case GEVWS_HS_OK: return "";
    case GEVWS_HS_MALFORMED_REQUEST: return "malformed HTTP request";
    case GEVWS_HS_BAD_PROTOCOL: return "handshake error: bad HTTP protocol version";
    case GEVWS_HS_BAD_METHOD: return "handshake error: bad HTTP request method";
    case GEVWS_HS_BAD_HOST: return "handshake error: bad \"Host\" header";
    case GEVWS_HS_BAD_UPGRADE: return "handshake error: bad \"Upgrade\" header";
    case GEVWS_HS_BAD_CONNECTION: return "handshake error: bad \"Connection\" header";
    case GEVWS_HS_BAD_SEC_ACCEPT: return "handshake error: bad \"Sec-WebSocket-Accept\" header";
    case GEVWS_HS_BAD_SEC_KEY: return "handshake error: bad \"Sec-WebSocket-Key\" header";
    case GEVWS_HS_BAD_SEC_VERSION:
    case GEVWS_HS_UPGRADE_REQUIRED: return "handshake error: bad \"Sec-WebSocket-Version\" header";
    case GEVWS_HS_HOOK: return "rejected by an Upgrader hook";
    default: return "unknown handshake error";
  }
}

void gevws_accept_key(const uint8_t nonce[24], char accept[28]) {
  const std::string a = gevws::AcceptFromNonce(nonce);
  memcpy(accept, a.data(), 28);
}

void gevws_protocol_set_upgrader(gevws_protocol* p, const gevws_upgrader* u) {
  if (p) p->SetUpgrader(u);
}

const uint8_t* gevws_protocol_packet(gevws_protocol* p, gevws_conn* c, const uint8_t* data, uint64_t n,
                                     uint64_t* out_len) {
  (void)p;
  (void)c;
  if (out_len) *out_len = n;
  return data;  // protocol.go:67-69: Packet returns data unchanged
}

}  // extern "C"
