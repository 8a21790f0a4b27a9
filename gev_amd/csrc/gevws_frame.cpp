// gevws_frame.cpp -- the per-frame host exports of the C ABI (SURVEY.md §8b
// items 1 and 2): what a cgo / C++ host calls on ONE frame at the ring head,
// e.g. to apply the reference's completeness gate (protocol.go:47) before it
// decides to hand a connection's bytes to a device pass.  The batch decode
// never comes here: it runs on the device (gevws_device.hip).
//
//   gevws_parse_header       ws.VirtualReadHeader, plugins/websocket/ws/read.go:19-84
//   gevws_parse_header_ring  the same over ringbuffer.PeekAll()'s two segments
//                            (the header may straddle the wrap, as the virtual
//                            reads of read.go:27,63 do)
//   gevws_cipher             ws.Cipher, plugins/websocket/ws/cipher.go:14-53
#include <cstring>

#include "gevws.h"

namespace {

// remain, cipher.go:56: bytes to the next 4-byte key boundary for offset % 4.
constexpr unsigned kRemain[4] = {0, 3, 2, 1};

}  // namespace

extern "C" {

int gevws_parse_header(const uint8_t* p, uint64_t avail, gevws_header* out, uint32_t* hdr_len) {
  if (hdr_len) *hdr_len = 0;
  if (!out || (avail && !p)) return GEVWS_ERR_INVALID;
  static_assert(sizeof(gevws_header) == 16, "ws.Header layout");
  // read.go:20-23: fewer than 6 bytes buffered -> ErrHeaderNotReady, even for a
  // complete 2..5-byte unmasked frame (Appendix A P1)
  if (avail >= 2 && hdr_len) {
    const uint32_t len7 = p[1] & 0x7fu;
    *hdr_len = 2 + (len7 < 126 ? 0u : (len7 == 126 ? 2u : 8u)) + ((p[1] & 0x80u) ? 4u : 0u);
  }
  if (avail < 6) return GEVWS_NEED_MORE;
  const uint8_t b0 = p[0], b1 = p[1];
  gevws_header h;
  std::memset(&h, 0, sizeof(h));
  h.fin = (b0 & 0x80) ? 1 : 0;                 // read.go:29
  h.rsv = (uint8_t)((b0 & 0x70) >> 4);         // read.go:30
  h.opcode = b0 & 0x0f;                        // read.go:31
  h.masked = (b1 & 0x80) ? 1 : 0;              // read.go:35-37
  const uint32_t len7 = b1 & 0x7fu;            // read.go:39
  const uint32_t ext = len7 < 126 ? 0u : (len7 == 126 ? 2u : 8u);  // read.go:41-49
  const uint32_t hl = 2 + ext + (h.masked ? 4u : 0u);
  // Appendix A U1: the extended header is not complete yet.  The reference's
  // outcome depends on ringbuffer internals (read.go:63 ignores the short
  // read); this build answers NEED_MORE, the RFC-correct choice.
  if (avail < hl) return GEVWS_NEED_MORE;
  const uint8_t* e = p + 2;
  if (len7 < 126) {
    h.length = (int64_t)len7;
  } else if (len7 == 126) {  // BE16, read.go:65-67
    h.length = ((int64_t)e[0] << 8) | e[1];
    e += 2;
  } else {  // BE64, read.go:69-76
    if (e[0] & 0x80) return GEVWS_ERR_LEN_MSB;  // ErrHeaderLengthMSB, read.go:71-73
    uint64_t L = 0;
    for (int i = 0; i < 8; ++i) L = (L << 8) | e[i];
    h.length = (int64_t)L;
    e += 8;
  }
  if (h.masked) std::memcpy(h.mask, e, 4);  // read.go:78-81
  *out = h;
  return GEVWS_OK;
}

int gevws_parse_header_ring(const uint8_t* seg0, uint64_t n0, const uint8_t* seg1, uint64_t n1,
                            gevws_header* out, uint32_t* hdr_len) {
  if ((n0 && !seg0) || (n1 && !seg1)) {
    if (hdr_len) *hdr_len = 0;
    return GEVWS_ERR_INVALID;
  }
  // a header is at most 14 bytes (write.go:9): gather them across the wrap
  uint8_t w[14];
  const uint64_t a = n0 < 14 ? n0 : 14;
  const uint64_t b = (n1 < 14 - a) ? n1 : 14 - a;
  if (a) std::memcpy(w, seg0, a);
  if (b) std::memcpy(w + a, seg1, b);
  // the availability checks (in.Length(), read.go:20) only ever compare with
  // 6 and the header length (<= 14), so min(buffered, 14) decides them alike
  return gevws_parse_header(w, a + b, out, hdr_len);
}

void gevws_cipher(uint8_t* p, uint64_t n, const uint8_t mask[4], uint64_t offset) {
  if (!p || !mask || n == 0) return;
  // cipher.go:16-21: short payloads bytewise
  if (n < 8) {
    for (uint64_t i = 0; i < n; ++i) p[i] ^= mask[(offset + i) & 3];
    return;
  }
  // cipher.go:24-51: head bytes up to the key boundary, tail bytes, and a
  // native-endian 64-bit body XOR with m || m (the compiler widens the body
  // loop to vector registers; the result is the byte definition either way)
  const uint64_t mpos = offset & 3;
  const uint64_t ln = kRemain[mpos];
  const uint64_t rn = (n - ln) & 7;
  for (uint64_t i = 0; i < ln; ++i) p[i] ^= mask[(mpos + i) & 3];
  for (uint64_t i = n - rn; i < n; ++i) p[i] ^= mask[(mpos + i) & 3];
  uint32_t m;
  std::memcpy(&m, mask, 4);
  const uint64_t m2 = ((uint64_t)m << 32) | m;
  uint8_t* body = p + ln;
  const uint64_t words = (n - ln - rn) >> 3;
  for (uint64_t i = 0; i < words; ++i) {
    uint64_t v;
    std::memcpy(&v, body + 8 * i, 8);
    v ^= m2;
    std::memcpy(body + 8 * i, &v, 8);
  }
}

}  // extern "C"
