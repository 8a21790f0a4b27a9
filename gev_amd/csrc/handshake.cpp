// handshake.cpp -- host-side websocket upgrade (see handshake.hpp).
//
// Follows plugins/websocket/ws/ws.go:158-343 (Upgrader.Upgrade), http.go
// (request-line / header-line parsing, response writers), nonce.go:23-39
// (accept key), util.go (asciiToInt, bsplit3, btrim, canonicalizeHeaderKey),
// errors.go (error texts and status codes).  Sec-WebSocket-Protocol /
// -Extensions token and option scanning is github.com/gobwas/httphead
// v0.0.0-20180130184737-2c6c146eadee (go.mod:10), not vendored: restated from
// its RFC 7230 list grammar -- parity unpinned.
#include "handshake.hpp"

#include <cstring>
#include <vector>

namespace gevws {

// ------------------------------------------------------------------ SHA-1 / base64
namespace {
inline uint32_t rol(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }

void sha1_block(uint32_t h[5], const uint8_t* b) {
  uint32_t w[80];
  for (int i = 0; i < 16; ++i)
    w[i] = (uint32_t)b[4 * i] << 24 | (uint32_t)b[4 * i + 1] << 16 | (uint32_t)b[4 * i + 2] << 8 | b[4 * i + 3];
  for (int i = 16; i < 80; ++i) w[i] = rol(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
  uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4];
  for (int i = 0; i < 80; ++i) {
    uint32_t f, k;
    if (i < 20) {
      f = (bb & c) | (~bb & d);
      k = 0x5A827999u;
    } else if (i < 40) {
      f = bb ^ c ^ d;
      k = 0x6ED9EBA1u;
    } else if (i < 60) {
      f = (bb & c) | (bb & d) | (c & d);
      k = 0x8F1BBCDCu;
    } else {
      f = bb ^ c ^ d;
      k = 0xCA62C1D6u;
    }
    const uint32_t t = rol(a, 5) + f + e + k + w[i];
    e = d;
    d = c;
    c = rol(bb, 30);
    bb = a;
    a = t;
  }
  h[0] += a;
  h[1] += bb;
  h[2] += c;
  h[3] += d;
  h[4] += e;
}
}  // namespace

void Sha1(const uint8_t* p, uint64_t n, uint8_t out[20]) {
  uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  uint64_t i = 0;
  for (; i + 64 <= n; i += 64) sha1_block(h, p + i);
  uint8_t tail[128] = {0};
  const uint64_t r = n - i;
  if (r) memcpy(tail, p + i, r);
  tail[r] = 0x80;
  const uint64_t tl = r < 56 ? 64 : 128;
  const uint64_t bits = n * 8;
  for (int k = 0; k < 8; ++k) tail[tl - 1 - k] = (uint8_t)(bits >> (8 * k));
  sha1_block(h, tail);
  if (tl == 128) sha1_block(h, tail + 64);
  for (int k = 0; k < 5; ++k)
    for (int j = 0; j < 4; ++j) out[4 * k + j] = (uint8_t)(h[k] >> (24 - 8 * j));
}

std::string Base64Std(const uint8_t* p, uint64_t n) {
  static const char A[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string s;
  s.reserve((n + 2) / 3 * 4);
  uint64_t i = 0;
  for (; i + 3 <= n; i += 3) {
    const uint32_t v = (uint32_t)p[i] << 16 | (uint32_t)p[i + 1] << 8 | p[i + 2];
    s += A[v >> 18];
    s += A[(v >> 12) & 63];
    s += A[(v >> 6) & 63];
    s += A[v & 63];
  }
  if (n - i == 1) {
    const uint32_t v = (uint32_t)p[i] << 16;
    s += A[v >> 18];
    s += A[(v >> 12) & 63];
    s += "==";
  } else if (n - i == 2) {
    const uint32_t v = (uint32_t)p[i] << 16 | (uint32_t)p[i + 1] << 8;
    s += A[v >> 18];
    s += A[(v >> 12) & 63];
    s += A[(v >> 6) & 63];
    s += '=';
  }
  return s;
}

std::string AcceptFromNonce(const uint8_t nonce[24]) {
  static const char magic[] = "258EAFA5-E914-47DA-95CA-C5AB0DC85B11";  // nonce.go:24 (RFC 6455 §1.3)
  uint8_t buf[24 + sizeof(magic) - 1];
  memcpy(buf, nonce, 24);
  memcpy(buf + 24, magic, sizeof(magic) - 1);
  uint8_t sum[20];
  Sha1(buf, sizeof(buf), sum);
  return Base64Std(sum, 20);
}

const char* StatusText(int code) {
  switch (code) {  // Go net/http status.go
    case 100: return "Continue";
    case 101: return "Switching Protocols";
    case 102: return "Processing";
    case 103: return "Early Hints";
    case 200: return "OK";
    case 201: return "Created";
    case 202: return "Accepted";
    case 203: return "Non-Authoritative Information";
    case 204: return "No Content";
    case 205: return "Reset Content";
    case 206: return "Partial Content";
    case 300: return "Multiple Choices";
    case 301: return "Moved Permanently";
    case 302: return "Found";
    case 303: return "See Other";
    case 304: return "Not Modified";
    case 307: return "Temporary Redirect";
    case 308: return "Permanent Redirect";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 402: return "Payment Required";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 406: return "Not Acceptable";
    case 407: return "Proxy Authentication Required";
    case 408: return "Request Timeout";
    case 409: return "Conflict";
    case 410: return "Gone";
    case 411: return "Length Required";
    case 412: return "Precondition Failed";
    case 414: return "Request URI Too Long";
    case 415: return "Unsupported Media Type";
    case 417: return "Expectation Failed";
    case 418: return "I'm a teapot";
    case 421: return "Misdirected Request";
    case 422: return "Unprocessable Entity";
    case 423: return "Locked";
    case 424: return "Failed Dependency";
    case 425: return "Too Early";
    case 426: return "Upgrade Required";
    case 428: return "Precondition Required";
    case 429: return "Too Many Requests";
    case 431: return "Request Header Fields Too Large";
    case 451: return "Unavailable For Legal Reasons";
    case 500: return "Internal Server Error";
    case 501: return "Not Implemented";
    case 502: return "Bad Gateway";
    case 503: return "Service Unavailable";
    case 504: return "Gateway Timeout";
    case 505: return "HTTP Version Not Supported";
    case 511: return "Network Authentication Required";
    default: return "";
  }
}

// ------------------------------------------------------------------ Go helpers
namespace {
struct Bytes {  // a Go []byte view
  const uint8_t* p = nullptr;
  uint64_t n = 0;
  bool eq(const char* s) const {
    const uint64_t l = strlen(s);
    return l == n && (n == 0 || memcmp(p, s, n) == 0);
  }
  Bytes sub(uint64_t a, uint64_t b) const { return {p + a, b - a}; }
  int64_t index_byte(uint8_t c) const {
    for (uint64_t i = 0; i < n; ++i)
      if (p[i] == c) return (int64_t)i;
    return -1;
  }
  std::string str() const { return std::string((const char*)p, n); }
};

int64_t index_of(const uint8_t* p, uint64_t n, const char* pat, uint64_t m) {
  if (m > n) return -1;
  for (uint64_t i = 0; i + m <= n; ++i)
    if (memcmp(p + i, pat, m) == 0) return (int64_t)i;
  return -1;
}

// util.go asciiToInt: bytes with high nibble 0x3 count as digits (so ':'..'?'
// are 10..15); Go int arithmetic wraps at 64 bits.
bool ascii_to_int(Bytes b, int64_t* ret) {
  if (b.n < 1) return false;
  uint64_t r = 0;
  for (uint64_t i = 0; i < b.n; ++i) {
    if ((b.p[i] & 0xf0) != 0x30) return false;
    uint64_t pw = 1, a = 10, e = b.n - i - 1;  // util.go pow: square-and-multiply
    while (e > 0) {
      if (e & 1) pw *= a;
      e >>= 1;
      a *= a;
    }
    r += (uint64_t)(b.p[i] & 0xf) * pw;
  }
  *ret = (int64_t)r;
  return true;
}

// util.go bsplit3
void bsplit3(Bytes b, uint8_t sep, Bytes* b1, Bytes* b2, Bytes* b3) {
  const int64_t a = b.index_byte(sep);
  const Bytes rest = b.sub((uint64_t)(a + 1), b.n);
  int64_t c = rest.index_byte(sep);
  if (a == -1 || c == -1) {
    *b1 = b;
    *b2 = Bytes{};
    *b3 = Bytes{};
    return;
  }
  c += a + 1;
  *b1 = b.sub(0, (uint64_t)a);
  *b2 = b.sub((uint64_t)a + 1, (uint64_t)c);
  *b3 = b.sub((uint64_t)c + 1, b.n);
}

// util.go btrim: spaces and tabs
Bytes btrim(Bytes b) {
  uint64_t i = 0, j = b.n;
  while (i < b.n && (b.p[i] == ' ' || b.p[i] == '\t')) ++i;
  while (j > i && (b.p[j - 1] == ' ' || b.p[j - 1] == '\t')) --j;
  return b.sub(i, j);
}

// util.go canonicalizeHeaderKey (in place)
void canonicalize(uint8_t* k, uint64_t n) {
  bool upper = true;
  for (uint64_t i = 0; i < n; ++i) {
    const uint8_t c = k[i];
    if (upper && c >= 'a' && c <= 'z')
      k[i] = c & (uint8_t)~0x20;
    else if (!upper && c >= 'A' && c <= 'Z')
      k[i] = c | 0x20;
    upper = c == '-';
  }
}

// http.go httpParseVersion
bool parse_version(Bytes b, int64_t* major, int64_t* minor) {
  if (b.eq("HTTP/1.0")) {
    *major = 1;
    *minor = 0;
    return true;
  }
  if (b.eq("HTTP/1.1")) {
    *major = 1;
    *minor = 1;
    return true;
  }
  if (b.n < 8 || memcmp(b.p, "HTTP/", 5) != 0) return false;
  const Bytes v = b.sub(5, b.n);
  const int64_t dot = v.index_byte('.');
  if (dot == -1) return false;
  return ascii_to_int(v.sub(0, (uint64_t)dot), major) && ascii_to_int(v.sub((uint64_t)dot + 1, v.n), minor);
}

// ---- httphead list scanning (RFC 7230 §3.2.6, §7): parity unpinned
bool is_tchar(uint8_t c) {
  if (c <= 32 || c >= 127) return false;
  return !strchr("()<>@,;:\\\"/[]?={}", c);
}
bool is_ws(uint8_t c) { return c == ' ' || c == '\t'; }

// ScanTokens: 1#token.  Calls it(token) until it returns false; false when
// the list is malformed or holds no token.
template <class F>
bool scan_tokens(Bytes h, F it) {
  uint64_t i = 0;
  bool any = false;
  while (i < h.n) {
    while (i < h.n && is_ws(h.p[i])) ++i;
    if (i >= h.n) break;
    if (h.p[i] == ',') {
      ++i;
      continue;
    }
    if (!is_tchar(h.p[i])) return false;
    const uint64_t s = i;
    while (i < h.n && is_tchar(h.p[i])) ++i;
    any = true;
    if (!it(h.sub(s, i))) return true;
    while (i < h.n && is_ws(h.p[i])) ++i;
    if (i < h.n && h.p[i] != ',') return false;
  }
  return any;
}

struct ExtOption {
  std::string name;
  std::vector<std::pair<std::string, std::pair<bool, std::string>>> params;  // key -> (has value, value)
};

// extension-list = 1#( token *( OWS ";" OWS token [ "=" ( token / quoted-string ) ] ) )
bool scan_options(Bytes h, std::vector<ExtOption>* out) {
  uint64_t i = 0;
  auto skip = [&] {
    while (i < h.n && is_ws(h.p[i])) ++i;
  };
  auto token = [&](std::string* t) {
    const uint64_t s = i;
    while (i < h.n && is_tchar(h.p[i])) ++i;
    if (i == s) return false;
    t->assign((const char*)h.p + s, i - s);
    return true;
  };
  while (true) {
    skip();
    if (i >= h.n) break;
    if (h.p[i] == ',') {
      ++i;
      continue;
    }
    ExtOption o;
    if (!token(&o.name)) return false;
    skip();
    while (i < h.n && h.p[i] == ';') {
      ++i;
      skip();
      std::string k, v;
      if (!token(&k)) return false;
      skip();
      bool has = false;
      if (i < h.n && h.p[i] == '=') {
        ++i;
        skip();
        has = true;
        if (i < h.n && h.p[i] == '"') {
          ++i;
          bool closed = false;
          while (i < h.n) {
            if (h.p[i] == '\\' && i + 1 < h.n) {
              v += (char)h.p[i + 1];
              i += 2;
            } else if (h.p[i] == '"') {
              ++i;
              closed = true;
              break;
            } else {
              v += (char)h.p[i++];
            }
          }
          if (!closed) return false;
        } else if (!token(&v)) {
          return false;
        }
        skip();
      }
      o.params.push_back({k, {has, v}});
    }
    out->push_back(std::move(o));
    if (i < h.n && h.p[i] != ',') return false;
  }
  return !out->empty();
}

// httphead.WriteOptions: "name;key=value;key, name2" (values quoted when not tokens)
void write_option(std::string* s, const ExtOption& o) {
  if (!s->empty()) *s += ", ";
  *s += o.name;
  for (const auto& kv : o.params) {
    *s += ';';
    *s += kv.first;
    if (kv.second.first) {
      *s += '=';
      const std::string& v = kv.second.second;
      bool tok = !v.empty();
      for (unsigned char c : v) tok = tok && is_tchar(c);
      if (tok) {
        *s += v;
      } else {
        *s += '"';
        for (char c : v) {
          if (c == '"' || c == '\\') *s += '\\';
          *s += c;
        }
        *s += '"';
      }
    }
  }
}

// The error of a handshake: which Go error value, its reply status and header.
struct HsErr {
  int kind = GEVWS_HS_OK;
  std::string reason;
  int code = 0;           // rejectConnectionError.code (0 -> 500)
  bool reject = true;     // *rejectConnectionError (vs a plain error)
  std::string header;     // rejectConnectionError.header
};

HsErr std_err(int kind) {
  HsErr e;
  e.kind = kind;
  switch (kind) {  // errors.go:25-79
    case GEVWS_HS_MALFORMED_REQUEST: e.code = 400; e.reason = "malformed HTTP request"; break;
    case GEVWS_HS_BAD_PROTOCOL: e.code = 505; e.reason = "handshake error: bad HTTP protocol version"; break;
    case GEVWS_HS_BAD_METHOD: e.code = 405; e.reason = "handshake error: bad HTTP request method"; break;
    case GEVWS_HS_BAD_HOST: e.code = 400; e.reason = "handshake error: bad \"Host\" header"; break;
    case GEVWS_HS_BAD_UPGRADE: e.code = 400; e.reason = "handshake error: bad \"Upgrade\" header"; break;
    case GEVWS_HS_BAD_CONNECTION: e.code = 400; e.reason = "handshake error: bad \"Connection\" header"; break;
    case GEVWS_HS_BAD_SEC_ACCEPT:
      e.code = 400;
      e.reason = "handshake error: bad \"Sec-WebSocket-Accept\" header";
      break;
    case GEVWS_HS_BAD_SEC_KEY: e.code = 400; e.reason = "handshake error: bad \"Sec-WebSocket-Key\" header"; break;
    case GEVWS_HS_BAD_SEC_VERSION:
      e.code = 400;
      e.reason = "handshake error: bad \"Sec-WebSocket-Version\" header";
      break;
    case GEVWS_HS_UPGRADE_REQUIRED:
      e.code = 426;
      e.header = "Sec-WebSocket-Version: 13\r\n";
      e.reason = "handshake error: bad \"Sec-WebSocket-Version\" header";
      break;
    default: break;
  }
  return e;
}

HsErr hook_err(const gevws_reject& r) {
  HsErr e;
  e.kind = GEVWS_HS_HOOK;
  e.reject = r.plain == 0;
  e.code = e.reject ? r.code : 0;
  if (r.reason) e.reason.assign(r.reason, r.reason_len);
  if (e.reject && r.header) e.header.assign((const char*)r.header, r.header_len);
  return e;
}

// http.go httpWriteResponseError: status line + Content-Type, custom headers,
// "Content-Length: n\r\n\r\n" + reason.
std::string write_error(const HsErr& e, int code, const std::string& hdr) {
  std::string s = "HTTP/1.1 " + std::to_string(code) + " " + StatusText(code) + "\r\n";
  s += "Content-Type: text/plain; charset=utf-8\r\n";
  s += hdr;
  s += "Content-Length: " + std::to_string(e.reason.size()) + "\r\n\r\n";
  s += e.reason;
  return s;
}
}  // namespace

void Upgrader::Upgrade(gevws_conn* conn, RingBuffer* in, HandshakeResult* r) const {
  *r = HandshakeResult{};
  enum { SeenHost = 1, SeenUpgrade = 2, SeenConnection = 4, SeenSecVersion = 8, SeenSecKey = 16, SeenAll = 31 };
  auto fail_silent = [&](const HsErr& e) {  // returned before any response is written
    r->error = e.kind;
    r->reason = e.reason;
  };

  // ws.go:178-192: the head must end in the first segment, or in the second
  // one alone (then index+4 bytes are read from the front of the ring).
  const uint8_t *first, *end;
  uint64_t n_first, n_end;
  in->PeekAll(&first, &n_first, &end, &n_end);
  std::vector<uint8_t> data;
  int64_t idx = index_of(first, n_first, "\r\n\r\n", 4);
  if (idx == -1 && n_end > 0) idx = index_of(end, n_end, "\r\n\r\n", 4);
  if (idx != -1) {
    data.resize((uint64_t)idx + 4);
    in->Read(data.data(), data.size());
  }

  // bytes.Split(data, "\r\n")
  std::vector<Bytes> lines;
  {
    uint64_t s = 0;
    for (uint64_t i = 0; i + 1 < data.size();) {
      if (data[i] == '\r' && data[i + 1] == '\n') {
        lines.push_back({data.data() + s, i - s});
        i += 2;
        s = i;
      } else {
        ++i;
      }
    }
    lines.push_back({data.data() + s, data.size() - s});
  }

  // http.go httpParseRequestLine
  Bytes method, uri, proto;
  bsplit3(lines[0], ' ', &method, &uri, &proto);
  int64_t major = 0, minor = 0;
  if (!parse_version(proto, &major, &minor)) return fail_silent(std_err(GEVWS_HS_MALFORMED_REQUEST));
  if (major != 1 || minor < 1) return fail_silent(std_err(GEVWS_HS_BAD_PROTOCOL));
  if (!method.eq("GET")) return fail_silent(std_err(GEVWS_HS_BAD_METHOD));
  if (hooks.on_request) {
    gevws_reject rej{};
    if (hooks.on_request(hooks.user, conn, uri.p, uri.n, &rej)) return fail_silent(hook_err(rej));
  }

  HsErr err;
  bool has_err = false;
  uint8_t seen = 0;
  uint8_t nonce[24] = {0};
  std::vector<ExtOption> exts;
  for (size_t i = 1; i < lines.size(); ++i) {
    if (has_err || lines[i].n == 0) break;
    // http.go httpParseHeaderLine (the key is canonicalized in place)
    const int64_t colon = lines[i].index_byte(':');
    if (colon == -1) {
      err = std_err(GEVWS_HS_MALFORMED_REQUEST);
      has_err = true;
      break;
    }
    Bytes k = btrim(lines[i].sub(0, (uint64_t)colon));
    canonicalize(const_cast<uint8_t*>(k.p), k.n);
    const Bytes v = btrim(lines[i].sub((uint64_t)colon + 1, lines[i].n));
    gevws_reject rej{};
    if (k.eq("Host")) {
      seen |= SeenHost;
      if (hooks.on_host && hooks.on_host(hooks.user, conn, v.p, v.n, &rej)) err = hook_err(rej), has_err = true;
    } else if (k.eq("Upgrade")) {
      seen |= SeenUpgrade;
      if (!v.eq("websocket")) err = std_err(GEVWS_HS_BAD_UPGRADE), has_err = true;
    } else if (k.eq("Connection")) {
      seen |= SeenConnection;
      if (!v.eq("Upgrade") && !v.eq("upgrade")) err = std_err(GEVWS_HS_BAD_CONNECTION), has_err = true;
    } else if (k.eq("Sec-Websocket-Version")) {
      seen |= SeenSecVersion;
      if (!v.eq("13")) err = std_err(GEVWS_HS_UPGRADE_REQUIRED), has_err = true;
    } else if (k.eq("Sec-Websocket-Key")) {
      seen |= SeenSecKey;
      if (v.n != 24)
        err = std_err(GEVWS_HS_BAD_SEC_KEY), has_err = true;
      else
        memcpy(nonce, v.p, 24);
    } else if (k.eq("Sec-Websocket-Protocol")) {
      if (r->protocol.empty() && (hooks.protocol_custom || hooks.protocol)) {
        bool ok;
        if (hooks.protocol_custom) {
          const uint8_t* sel = nullptr;
          uint64_t sn = 0;
          ok = hooks.protocol_custom(hooks.user, conn, v.p, v.n, &sel, &sn) != 0;
          r->protocol = sel ? std::string((const char*)sel, sn) : std::string();
        } else {
          Bytes selected;
          bool got = false;
          ok = scan_tokens(v, [&](Bytes t) {
            if (hooks.protocol(hooks.user, t.p, t.n)) {
              selected = t;
              got = true;
              return false;
            }
            return true;
          });
          if (ok && got) r->protocol = selected.str();
        }
        if (!ok) err = std_err(GEVWS_HS_MALFORMED_REQUEST), has_err = true;
      }
    } else if (k.eq("Sec-Websocket-Extensions")) {
      if (hooks.extension_custom || hooks.extension) {
        bool ok;
        if (hooks.extension_custom) {
          const uint8_t* sel = nullptr;
          uint64_t sn = 0;
          ok = hooks.extension_custom(hooks.user, conn, v.p, v.n, (const uint8_t*)r->extensions.data(),
                                      r->extensions.size(), &sel, &sn) != 0;
          r->extensions = sel ? std::string((const char*)sel, sn) : std::string();
        } else {  // OptionSelector{SelectUnique | SelectCopy}
          std::vector<ExtOption> offered;
          ok = scan_options(v, &offered);
          if (ok) {
            for (const ExtOption& o : offered) {
              bool dup = false;
              for (const ExtOption& s : exts) dup = dup || s.name == o.name;
              if (dup) continue;
              std::vector<gevws_ext_param> ps;
              for (const auto& kv : o.params)
                ps.push_back({(const uint8_t*)kv.first.data(), kv.first.size(),
                              kv.second.first ? (const uint8_t*)kv.second.second.data() : nullptr,
                              kv.second.second.size()});
              if (hooks.extension(hooks.user, (const uint8_t*)o.name.data(), o.name.size(), ps.data(),
                                  (uint32_t)ps.size()))
                exts.push_back(o);
            }
            r->extensions.clear();
            for (const ExtOption& o : exts) write_option(&r->extensions, o);
          }
        }
        if (!ok) err = std_err(GEVWS_HS_MALFORMED_REQUEST), has_err = true;
      }
    } else if (hooks.on_header) {
      if (hooks.on_header(hooks.user, conn, k.p, k.n, v.p, v.n, &rej)) err = hook_err(rej), has_err = true;
    }
  }

  std::string extra;  // header[1] (ws.go:201-203, 322, 328)
  if (!has_err && seen != SeenAll) {
    has_err = true;
    if (!(seen & SeenHost))
      err = std_err(GEVWS_HS_BAD_HOST);
    else if (!(seen & SeenUpgrade))
      err = std_err(GEVWS_HS_BAD_UPGRADE);
    else if (!(seen & SeenConnection))
      err = std_err(GEVWS_HS_BAD_CONNECTION);
    else if (!(seen & SeenSecVersion))
      err = std_err(GEVWS_HS_BAD_SEC_VERSION);
    else
      err = std_err(GEVWS_HS_BAD_SEC_KEY);
  } else if (!has_err && hooks.on_before_upgrade) {
    const uint8_t* h = nullptr;
    uint64_t hn = 0;
    gevws_reject rej{};
    if (hooks.on_before_upgrade(hooks.user, conn, &h, &hn, &rej)) {
      err = hook_err(rej);
      has_err = true;
    } else if (h) {
      extra.assign((const char*)h, hn);
    }
  }
  if (has_err) {
    if (err.reject) extra = err.header;
    const int code = err.reject && err.code != 0 ? err.code : 500;
    r->error = err.kind;
    r->reason = err.reason;
    r->http_code = code;
    r->out = write_error(err, code, header + extra);
    return;
  }
  // http.go httpWriteResponseUpgrade
  std::string& o = r->out;
  o = "HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n";
  o += "Sec-WebSocket-Accept: " + AcceptFromNonce(nonce) + "\r\n";
  if (!r->protocol.empty()) o += "Sec-WebSocket-Protocol: " + r->protocol + "\r\n";
  if (!r->extensions.empty()) o += "Sec-WebSocket-Extensions: " + r->extensions + "\r\n";
  o += header;
  o += extra;
  o += "\r\n";
  r->http_code = 101;
}

}  // namespace gevws
