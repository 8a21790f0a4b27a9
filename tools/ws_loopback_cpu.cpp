// ws_loopback_cpu.cpp -- CPU baseline for C1 (plumbing): the same loopback echo
// server and ping-pong client as gev_amd/ws_loopback (ws_loopback.hpp), but each
// frame is decoded on the loop's own core by the reference's per-frame
// UnPacket pipeline as restated in oracle/ws_ref.c (TEST / MEASUREMENT
// INFRASTRUCTURE, never part of libgevws.so or gev_amd/ws_loopback):
//
//   ws.VirtualReadHeader (read.go:19-84) over the ring's first bytes ->
//   completeness gate (protocol.go:47) -> payload := make([]byte, L) ->
//   ring Read (protocol.go:48-51) -> ws.Cipher (cipher.go:14-53).
//
// The handshake goes through the library's host upgrader (once per connection,
// outside the measured steady state), so the two binaries differ only in the
// frame decode.
#include <cstdlib>

#include "ws_loopback.hpp"

extern "C" {
// oracle/ws_ref.c
typedef struct {
  uint8_t fin, rsv, opcode, masked;
  uint8_t mask[4];
  int64_t length;
} wsref_header;
int wsref_read_header(const uint8_t* p, uint64_t avail, wsref_header* h, uint32_t* hlen);
void wsref_cipher(uint8_t* p, size_t n, const uint8_t mask[4], size_t offset);
}

namespace {

struct CpuDecoder {
  gevws_upgrader* u;
  explicit CpuDecoder(int) { u = gevws_upgrader_new(); }
  ~CpuDecoder() { gevws_upgrader_free(u); }
  int64_t pass(wslb::ServerConn* const*, uint32_t) { return 0; }  // per-frame decode happens in unpacket
  static constexpr bool kPipelined = false;  // nothing to overlap: the decode runs in unpacket
  static constexpr bool kTimeline = false;    // no device passes
  void timeline(gevws_protocol_timeline*) const {}
  int64_t begin(wslb::ServerConn* const*, uint32_t) { return 0; }
  int64_t end() { return 0; }
  // no device handler: the wsserver mode's text echo is framed on the host
  static constexpr bool kHandler = false;
  void set_handler(int) {}
  int reply(wslb::ServerConn*, const uint8_t**, uint64_t*, int*) { return GEVWS_ERR_INVALID; }

  int unpacket(wslb::ServerConn* s, gevws_header* h, const uint8_t** data, uint64_t* len) {
    *data = nullptr;
    *len = 0;
    if (!gevws_conn_upgraded(s->c)) {  // protocol.go:28-37
      const int r = gevws_upgrader_upgrade(u, s->c, s->r, data, len, nullptr);
      if (r == GEVWS_OK) {
        gevws_conn_set_upgraded(s->c, 1);
        return GEVWS_HANDSHAKE;
      }
      return GEVWS_ERR_HANDSHAKE;
    }
    if (s->poisoned) return GEVWS_ERR_LEN_MSB;
    const uint8_t *a, *b;
    uint64_t na, nb;
    gevws_ring_peek_all(s->r, &a, &na, &b, &nb);
    // the virtual reads of read.go:27,63 across the ring's wrap
    uint8_t hb[14];
    const uint64_t ca = na < 14 ? na : 14, cb = nb < 14 - ca ? nb : 14 - ca;
    memcpy(hb, a, ca);
    if (cb) memcpy(hb + ca, b, cb);
    wsref_header wh;
    uint32_t hl = 0;
    const int r = wsref_read_header(hb, na + nb, &wh, &hl);
    if (r < 0) {
      s->poisoned = 1;
      return GEVWS_ERR_LEN_MSB;
    }
    if (r != 0 || na + nb - hl < (uint64_t)wh.length) return GEVWS_NEED_MORE;  // protocol.go:47, 59-61
    const uint64_t L = (uint64_t)wh.length;
    s->frame.assign(L ? L : 1, 0);  // make([]byte, L): zero-filled (protocol.go:50)
    // buffer.Read(payload) after the header (protocol.go:48-51)
    uint64_t skip = hl, got = 0;
    const uint8_t* segs[2] = {a, b};
    const uint64_t lens[2] = {na, nb};
    for (int k = 0; k < 2 && got < L; ++k) {
      if (skip >= lens[k]) {
        skip -= lens[k];
        continue;
      }
      const uint64_t c = std::min<uint64_t>(lens[k] - skip, L - got);
      memcpy(s->frame.data() + got, segs[k] + skip, c);
      got += c;
      skip = 0;
    }
    gevws_ring_retrieve(s->r, hl + L);
    if (wh.masked) wsref_cipher(s->frame.data(), L, wh.mask, 0);  // protocol.go:53-55
    static_assert(sizeof(wsref_header) == sizeof(gevws_header), "ws.Header layout");
    memcpy(h, &wh, sizeof(*h));
    *data = s->frame.data();
    *len = L;
    return GEVWS_OK;
  }
  static const char* name() { return "cpu (oracle/ws_ref.c per-frame UnPacket pipeline)"; }
  static const char* path() { return "per-frame UnPacket on the loop core (reference pipeline restated)"; }
};

}  // namespace

int main(int argc, char** argv) { return wslb::loopback_main<CpuDecoder>(argc, argv); }
