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
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
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

// ------------------------------------------------------------------ connection
struct Delivered {
  gevws_header hdr;
  uint64_t frame_bytes;  // h + L, consumed from the ring on delivery
  uint64_t payload_off;  // into the batch's host arena
  std::shared_ptr<std::vector<uint8_t>> arena;
};

struct Connection {
  bool upgraded = false;                 // "gev_ws_upgraded" (protocol.go:12, 36)
  int poisoned = GEVWS_OK;               // sticky ERR_LEN_MSB (Appendix A P9/U3)
  std::deque<Delivered> queue;           // decoded, not yet returned by UnPacket
  std::shared_ptr<std::vector<uint8_t>> current;  // keeps the last payload alive
  HandshakeResult hs;                    // last Upgrade's response + Handshake
  uint64_t tail_len = ~0ull;             // undecodable ring bytes after the last device pass
};

// ------------------------------------------------------------------ protocol
class Protocol {
 public:
  explicit Protocol(gevws_ctx* ctx) : ctx_(ctx) {}
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
    if (c->queue.empty() && c->poisoned == GEVWS_OK && ring->Length() != c->tail_len) {
      Connection* cs[1] = {c};
      RingBuffer* rs[1] = {ring};
      int64_t r = UnPacketBatch(cs, rs, 1);
      if (r < 0) return (int)r;
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
    ring->Retrieve(d.frame_bytes);  // VirtualFlush + Read (protocol.go:48-51)
    c->current = d.arena;
    *hdr = d.hdr;
    *out = d.arena->data() + d.payload_off;
    *out_len = (uint64_t)d.hdr.length;
    return GEVWS_OK;
  }

  // One device pass over every listed connection's buffered bytes.
  int64_t UnPacketBatch(Connection* const* conns, RingBuffer* const* rings, uint32_t n) {
    // Connections that already hold undelivered frames (or are poisoned) are
    // skipped: their ring prefix is already decoded.
    std::vector<uint32_t> sel;
    std::vector<gevws_host_conn> segs;
    sel.reserve(n);
    for (uint32_t i = 0; i < n; ++i) {
      if (!conns[i]->upgraded || !conns[i]->queue.empty() || conns[i]->poisoned != GEVWS_OK) continue;
      if (rings[i]->Length() < 6) continue;  // read.go:20-23: nothing can be decoded
      if (rings[i]->Length() == conns[i]->tail_len) continue;  // no new bytes since the last pass
      gevws_host_conn h;
      rings[i]->PeekAll(&h.seg0, &h.n0, &h.seg1, &h.n1);
      sel.push_back(i);
      segs.push_back(h);
    }
    if (sel.empty()) return 0;
    const uint32_t m = (uint32_t)sel.size();
    gevws_summary sum{};
    std::vector<gevws_conn_in> cin;
    DeviceScope scope(gevws_ctx_device(ctx_));
    int64_t r = StageDecode(segs.data(), m, &sum, cin);
    if (r < 0) return r;
    // frames + payload back in one round trip through pinned memory
    const uint64_t fb = sum.frames * sizeof(gevws_frame);
    if (!grow_host(&h_out_, &h_out_cap_, fb + sum.payload_bytes + 16)) return fail();
    hipStream_t st = (hipStream_t)gevws_ctx_stream(ctx_);
    if ((fb && hipMemcpyAsync(h_out_, d_frames_, fb, hipMemcpyDeviceToHost, st) != hipSuccess) ||
        (sum.payload_bytes &&
         hipMemcpyAsync(h_out_ + fb, d_payload_, sum.payload_bytes, hipMemcpyDeviceToHost, st) != hipSuccess) ||
        hipStreamSynchronize(st) != hipSuccess)
      return fail();
    const gevws_conn_out* cout = reinterpret_cast<const gevws_conn_out*>(h_res_ + sizeof(gevws_summary));
    const gevws_frame* fr = reinterpret_cast<const gevws_frame*>(h_out_);
    auto arena = std::make_shared<std::vector<uint8_t>>(h_out_ + fb, h_out_ + fb + sum.payload_bytes);
    if (arena->empty()) arena->resize(1);
    // hand the frames to their connections in stream order
    for (uint32_t j = 0; j < m; ++j) {
      Connection* c = conns[sel[j]];
      const gevws_conn_out& o = cout[j];
      c->tail_len = cin[j].len - o.consumed;
      uint64_t prev_end = cin[j].off;
      for (uint32_t k = 0; k < o.nframes; ++k) {
        const gevws_frame& f = fr[o.first_frame + k];
        Delivered d;
        d.hdr = f.hdr;
        d.frame_bytes = f.src_off + (uint64_t)f.hdr.length - prev_end;
        d.payload_off = f.payload_off;
        d.arena = arena;
        prev_end = f.src_off + (uint64_t)f.hdr.length;
        c->queue.push_back(std::move(d));
      }
      if (o.status < 0) c->poisoned = o.status;
    }
    return (int64_t)sum.frames;
  }

  // Host segments in, caller buffers out (gevws_decode_host_batch).
  int64_t DecodeHost(const gevws_host_conn* segs, uint32_t n, gevws_frame* frames, uint64_t max_frames,
                     uint8_t* payload, uint64_t payload_cap, gevws_conn_out* conn_out, gevws_summary* sum_out) {
    gevws_summary sum{};
    *sum_out = sum;
    if (n == 0) return 0;
    std::vector<gevws_conn_in> cin;
    DeviceScope scope(gevws_ctx_device(ctx_));
    int64_t r = StageDecode(segs, n, &sum, cin);
    if (r < 0) return r;
    // src_off is reported relative to each connection's own stream
    *sum_out = sum;
    if (sum.frames > max_frames || sum.payload_bytes > payload_cap) {
      sum_out->status = GEVWS_ERR_CAPACITY;
      return GEVWS_ERR_CAPACITY;
    }
    memcpy(conn_out, h_res_ + sizeof(gevws_summary), n * sizeof(gevws_conn_out));
    hipStream_t st = (hipStream_t)gevws_ctx_stream(ctx_);
    if ((sum.frames && hipMemcpyAsync(frames, d_frames_, sum.frames * sizeof(gevws_frame), hipMemcpyDeviceToHost,
                                      st) != hipSuccess) ||
        (sum.payload_bytes &&
         hipMemcpyAsync(payload, d_payload_, sum.payload_bytes, hipMemcpyDeviceToHost, st) != hipSuccess) ||
        hipStreamSynchronize(st) != hipSuccess)
      return fail();
    for (uint32_t j = 0; j < n; ++j)
      for (uint32_t k = 0; k < conn_out[j].nframes; ++k) frames[conn_out[j].first_frame + k].src_off -= cin[j].off;
    return (int64_t)sum.frames;
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

  // Join each connection's segments into pinned staging behind the connection
  // table, ONE H2D, decode on the context's stream, ONE D2H of {summary,
  // conn_out} into pinned h_res_ and one sync.  Frames and payload stay in
  // the device buffers.  Retries once with the exact sizes on ERR_CAPACITY.
  int64_t StageDecode(const gevws_host_conn* segs, uint32_t m, gevws_summary* sum,
                      std::vector<gevws_conn_in>& cin) {
    uint64_t total = 0;
    for (uint32_t j = 0; j < m; ++j) total += segs[j].n0 + segs[j].n1;
    cin.resize(m);
    const uint64_t coff = ((uint64_t)m * sizeof(gevws_conn_in) + 255) & ~255ull;  // input starts here
    const uint64_t stage = coff + total + GEVWS_IN_PAD;
    if (!grow_host(&h_in_, &h_in_cap_, stage)) return fail();
    uint8_t* hin = h_in_ + coff;
    uint64_t off = 0;
    for (uint32_t j = 0; j < m; ++j) {
      if (segs[j].n0) memcpy(hin + off, segs[j].seg0, segs[j].n0);
      if (segs[j].n1) memcpy(hin + off + segs[j].n0, segs[j].seg1, segs[j].n1);
      cin[j] = {off, segs[j].n0 + segs[j].n1};
      off += cin[j].len;
    }
    memcpy(h_in_, cin.data(), m * sizeof(gevws_conn_in));
    memset(hin + off, 0, GEVWS_IN_PAD);
    const uint64_t res = sizeof(gevws_summary) + (uint64_t)m * sizeof(gevws_conn_out);
    if (!grow_host(&h_res_, &h_res_cap_, res)) return fail();
    uint64_t max_frames = std::min<uint64_t>(total / 2 + 1, 0xFFFFFFFFull);
    uint64_t payload_cap = total + 16 * std::min<uint64_t>(max_frames, total / 64 + 64) + 64;
    hipStream_t st = (hipStream_t)gevws_ctx_stream(ctx_);
    if (!grow_dev(&d_in_, &d_in_cap_, stage) || !grow_dev(&d_res_, &d_res_cap_, res) ||
        hipMemcpyAsync(d_in_, h_in_, stage, hipMemcpyHostToDevice, st) != hipSuccess)
      return fail();
    gevws_summary* d_sum = (gevws_summary*)d_res_;
    gevws_conn_out* d_cout = (gevws_conn_out*)((uint8_t*)d_res_ + sizeof(gevws_summary));
    for (int attempt = 0; attempt < 2; ++attempt) {
      if (!grow_dev(&d_frames_, &d_frames_cap_, max_frames * sizeof(gevws_frame)) ||
          !grow_dev(&d_payload_, &d_payload_cap_, payload_cap + 16))
        return fail();
      int r = gevws_decode_batch_async(ctx_, st, (const uint8_t*)d_in_ + coff, total, (gevws_conn_in*)d_in_, m,
                                       (gevws_frame*)d_frames_, max_frames, (uint8_t*)d_payload_, payload_cap,
                                       d_cout, d_sum);
      if (r != GEVWS_OK) return r;
      if (hipMemcpyAsync(h_res_, d_res_, res, hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess)
        return fail();
      memcpy(sum, h_res_, sizeof(gevws_summary));
      r = sum->status;
      if (r == GEVWS_ERR_CAPACITY && attempt == 0) {
        max_frames = std::max<uint64_t>(sum->frames, 1);
        payload_cap = std::max<uint64_t>(sum->payload_bytes, 16);
        continue;
      }
      return r == GEVWS_OK ? (int64_t)sum->frames : (int64_t)r;
    }
    return GEVWS_ERR_CAPACITY;
  }

  int64_t fail() {
    log_error("device: ", GEVWS_ERR_DEVICE);
    return GEVWS_ERR_DEVICE;
  }
  static bool grow_host(uint8_t** p, uint64_t* cap, uint64_t need) {
    if (need <= *cap) return true;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    uint64_t want = std::max<uint64_t>(need + need / 2, 1 << 16);
    if (hipHostMalloc((void**)p, want, hipHostMallocDefault) != hipSuccess) {
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
    for (uint8_t* p : {h_in_, h_res_, h_out_})
      if (p) (void)hipHostFree(p);
    for (void* p : {d_in_, d_res_, d_frames_, d_payload_})
      if (p) (void)hipFree(p);
  }

  gevws_ctx* ctx_;
  const Upgrader* upgrader_ = nullptr;
  uint8_t *h_in_ = nullptr, *h_res_ = nullptr, *h_out_ = nullptr;  // pinned staging
  uint64_t h_in_cap_ = 0, h_res_cap_ = 0, h_out_cap_ = 0;
  void *d_in_ = nullptr, *d_res_ = nullptr, *d_frames_ = nullptr, *d_payload_ = nullptr;
  uint64_t d_in_cap_ = 0, d_res_cap_ = 0, d_frames_cap_ = 0, d_payload_cap_ = 0;
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
