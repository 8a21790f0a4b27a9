// ws_loopback.cpp -- the live loopback echo server over the C ABI with the
// device decode (host ingress; C1's plumbing shape).
// Server/client skeleton: ws_loopback.hpp.  Per loop iteration ONE device pass
// over every readable upgraded connection (gevws_protocol_unpacket_batch:
// PeekAll segments gathered into pinned staging, H2D, decode, D2H), then
// websocket.(*Protocol).UnPacket per connection hands the frames out.  Small
// passes run zero-copy on mapped host memory (gevws_protocol_set_zero_copy_max;
// env GEVWS_LB_ZERO_COPY_MAX overrides the default for an A/B); with
// GEVWS_LB_SERVICE=1 they are posted to the context's resident decode service
// (gevws_protocol_set_service), with GEVWS_LB_DIRECT=1 written into the
// context's own AQL queue (gevws_protocol_set_direct), instead of launched.
#include "ws_loopback.hpp"

namespace {

struct DeviceDecoder {
  gevws_ctx* ctx;
  gevws_protocol* p;
  gevws_upgrader* u;
  std::vector<gevws_conn*> bc;
  std::vector<gevws_ring*> br;

  explicit DeviceDecoder(int device) {
    ctx = gevws_ctx_create(device);
    if (!ctx) {
      fprintf(stderr, "ws_loopback: no device %d\n", device);
      exit(2);
    }
    p = gevws_protocol_new(ctx);
    if (const char* zc = getenv("GEVWS_LB_ZERO_COPY_MAX"))  // A/B: 0 = copy every pass in and out
      gevws_protocol_set_zero_copy_max(p, strtoull(zc, nullptr, 10));
    if (const char* sb = getenv("GEVWS_LB_SMALL_BATCH"))  // A/B: 0 = multi-kernel decode for small passes
      gevws_ctx_set_tuning(ctx, GEVWS_TUNE_SMALL_BATCH, (int64_t)strtoll(sb, nullptr, 10));
    if (const char* sv = getenv("GEVWS_LB_SERVICE"))  // 1: passes posted to a resident decode service
      if (atoi(sv) == 1 && gevws_protocol_set_service(p, 1) != GEVWS_OK) {
        fprintf(stderr, "ws_loopback: gevws_protocol_set_service failed\n");
        exit(2);
      }
    if (const char* dd = getenv("GEVWS_LB_DIRECT"))  // 1: passes written into the context's own AQL queue
      if (atoi(dd) == 1 && gevws_protocol_set_direct(p, 1) != GEVWS_OK) {
        fprintf(stderr, "ws_loopback: gevws_protocol_set_direct failed\n");
        exit(2);
      }
    u = gevws_upgrader_new();  // &ws.Upgrader{} as benchmarks/websocket/server.go:52
    gevws_protocol_set_upgrader(p, u);
  }
  ~DeviceDecoder() {
    gevws_protocol_free(p);
    gevws_upgrader_free(u);
    gevws_ctx_destroy(ctx);
  }
  int64_t pass(wslb::ServerConn* const* conns, uint32_t n) {
    bc.clear();
    br.clear();
    for (uint32_t i = 0; i < n; ++i) {
      bc.push_back(conns[i]->c);
      br.push_back(conns[i]->r);
    }
    return gevws_protocol_unpacket_batch(p, bc.data(), br.data(), n);
  }
  // the pass in two halves (gevws_protocol_unpacket_batch_begin / _end)
  static constexpr bool kPipelined = true;
  int64_t begin(wslb::ServerConn* const* conns, uint32_t n) {
    bc.clear();
    br.clear();
    for (uint32_t i = 0; i < n; ++i) {
      bc.push_back(conns[i]->c);
      br.push_back(conns[i]->r);
    }
    return gevws_protocol_unpacket_batch_begin(p, bc.data(), br.data(), n);
  }
  int64_t end() { return gevws_protocol_unpacket_batch_end(p); }
  int unpacket(wslb::ServerConn* s, gevws_header* h, const uint8_t** data, uint64_t* len) {
    return gevws_protocol_unpacket(p, s->c, s->r, h, data, len);
  }
  // HandlerWrap.OnMessage on the device (the protocol's handler step)
  static constexpr bool kHandler = true;
  void set_handler(int policy) { gevws_protocol_set_handler(p, policy); }
  int reply(wslb::ServerConn* s, const uint8_t** out, uint64_t* len, int* shutdown_write) {
    return gevws_protocol_reply(p, s->c, out, len, shutdown_write);
  }
  static constexpr bool kTimeline = true;
  void timeline(gevws_protocol_timeline* t) const {
    gevws_protocol_get_timeline(p, t);
    gevws_protocol_stats s;
    gevws_protocol_get_stats(p, &s);
    wslb::g_service_passes += s.service_passes;
    wslb::g_direct_passes += gevws_ctx_direct_dispatches(ctx);
  }
  static const char* name() { return "device"; }
  static const char* path() { return "batched device decode (gevws_protocol_unpacket_batch) -> UnPacket"; }
};

}  // namespace

int main(int argc, char** argv) { return wslb::loopback_main<DeviceDecoder>(argc, argv); }
