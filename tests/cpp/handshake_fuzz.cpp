// Mutated upgrade requests through gevws::Upgrader::Upgrade
// (gev_amd/csrc/handshake.cpp) under ASan/UBSan, over ring buffers whose
// contents wrap: no out-of-bounds access, and the ring only ever loses the
// bytes of one complete head.  Built by tests/test_host_sanitizers.py.
#include <cstdio>
#include <random>
#include <string>

#include "../../gev_amd/csrc/handshake.hpp"

static int hook_proto(void*, const uint8_t* t, uint64_t n) { return n == 4 && t[0] == 'c'; }
static int hook_ext(void*, const uint8_t*, uint64_t n, const gevws_ext_param* ps, uint32_t np) {
  for (uint32_t i = 0; i < np; ++i)
    if (ps[i].key_len == 0) return 0;
  return n % 2;
}

int main() {
  std::mt19937_64 rng(7);
  const std::string base =
      "GET /chat HTTP/1.1\r\nHost: h\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
      "Sec-WebSocket-Key: dGhlIHNhbXBsZSBub25jZQ==\r\nSec-WebSocket-Protocol: chat, cxyz\r\n"
      "Sec-WebSocket-Extensions: permessage-deflate; a=\"q\\\"x\"; b, x-y\r\n"
      "Sec-WebSocket-Version: 13\r\n\r\n";
  gevws::Upgrader u;
  u.hooks.protocol = hook_proto;
  u.hooks.extension = hook_ext;
  u.header = "X-A: b\r\n";
  int ok = 0;
  for (int it = 0; it < 20000; ++it) {
    std::string req = base;
    const int muts = rng() % 6;
    for (int m = 0; m < muts && !req.empty(); ++m) {
      const size_t pos = rng() % req.size();
      switch (rng() % 4) {
        case 0: req[pos] = (char)(rng() % 256); break;
        case 1: req.erase(pos, 1 + rng() % 8); break;
        case 2: req.insert(pos, std::string(1 + rng() % 4, "\r\n:; ,=\"\\"[rng() % 9])); break;
        default: req.resize(pos); break;
      }
    }
    const uint64_t wrap = rng() % (req.size() + 1);
    gevws::RingBuffer r(req.size() + 3);
    const uint64_t pre = req.size() + 3 - wrap;
    std::string pad(pre, 'z');
    r.Write((const uint8_t*)pad.data(), pad.size());
    r.Retrieve(pre ? pre - 1 : 0);
    r.Write((const uint8_t*)req.data(), req.size());
    r.Retrieve(pre ? 1 : 0);
    const uint64_t before = r.Length();
    gevws::HandshakeResult res;
    u.Upgrade(nullptr, &r, &res);
    const uint64_t used = before - r.Length();
    if (used > before || (used != 0 && used < 4)) {
      fprintf(stderr, "bad consumption %llu of %llu\n", (unsigned long long)used, (unsigned long long)before);
      return 1;
    }
    ok += res.error == GEVWS_HS_OK;
  }
  printf("handshake_fuzz ok (%d upgrades)\n", ok);
  return 0;
}
