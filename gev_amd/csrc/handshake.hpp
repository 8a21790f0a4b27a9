// handshake.hpp -- the websocket HTTP upgrade: a C++
// restatement of ws.Upgrader.Upgrade (plugins/websocket/ws/ws.go:158-343) and
// its helpers (http.go, nonce.go, util.go, errors.go).  Once per connection and
// byte-serial, so it runs on the host; no HIP here (fuzzed under ASan/UBSan by
// tests/cpp/handshake_fuzz.cpp).
#pragma once

#include <cstdint>
#include <string>

#include "gevws.h"
#include "ringbuffer.hpp"

namespace gevws {

// SHA-1 (FIPS 180-4) of `n` bytes -> 20 bytes; base64 (RFC 4648 std, padded).
void Sha1(const uint8_t* p, uint64_t n, uint8_t out[20]);
std::string Base64Std(const uint8_t* p, uint64_t n);
// initAcceptFromNonce (nonce.go:23-39): base64(sha1(nonce || magic)), 28 chars.
std::string AcceptFromNonce(const uint8_t nonce[24]);

// net/http.StatusText (Go) for the codes the handshake can emit; "" otherwise.
const char* StatusText(int code);

struct HandshakeResult {
  std::string out;          // response bytes (101 or error response); may be empty
  std::string protocol;     // Handshake.Protocol
  std::string extensions;   // Handshake.Extensions as written in the response
  std::string reason;       // err.Error(), "" on success
  int error = GEVWS_HS_OK;  // GEVWS_HS_*
  int http_code = 0;        // status of `out`, 0 when nothing was written
};

class Upgrader {
 public:
  gevws_upgrader_hooks hooks{};
  std::string header;  // Upgrader.Header (ws.go:88-95), raw "Key: value\r\n" lines

  // ws.go:158-343.  Consumes the request head from `in` when it is complete
  // (and only then); fills `r`.  `conn` is handed to the hooks unchanged.
  void Upgrade(gevws_conn* conn, RingBuffer* in, HandshakeResult* r) const;
};

}  // namespace gevws
