// ringbuffer.hpp -- growable circular byte buffer, the part of
// github.com/Allenxuxu/ringbuffer v0.0.11 (go.mod:7) that gev's read path and
// the websocket plugin use: Write (connection.go:241-244), Length, PeekAll
// (connection.go:237-240, ws.go:176-192), Read (ws.go:180), Retrieve (consumption of a decoded
// frame, protocol.go:48-51).  The un-vendored library's virtual-cursor calls
// (read.go:20,27,63; protocol.go:47-60) are replaced by the device header walk.
// Host-only C++ (no HIP): fuzzed under ASan/UBSan by tests/cpp/ring_fuzz.cpp.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

namespace gevws {

class RingBuffer {
 public:
  explicit RingBuffer(uint64_t size) : buf_(size ? size : 1), size_(buf_.size()) {}

  uint64_t Length() const {
    if (empty_) return 0;
    return w_ > r_ ? w_ - r_ : size_ - r_ + w_;
  }
  uint64_t Capacity() const { return size_; }
  bool IsEmpty() const { return empty_; }

  uint64_t Write(const uint8_t* p, uint64_t n) {
    if (n == 0) return 0;
    const uint64_t free_bytes = size_ - Length();
    if (n > free_bytes) grow(Length() + n);
    uint64_t first = std::min<uint64_t>(n, size_ - w_);
    memcpy(buf_.data() + w_, p, first);
    if (n > first) memcpy(buf_.data(), p + first, n - first);
    w_ = (w_ + n) % size_;
    empty_ = false;
    return n;
  }

  void PeekAll(const uint8_t** first, uint64_t* n1, const uint8_t** end, uint64_t* n2) const {
    *first = *end = nullptr;
    *n1 = *n2 = 0;
    if (empty_) return;
    if (w_ > r_) {
      *first = buf_.data() + r_;
      *n1 = w_ - r_;
      return;
    }
    *first = buf_.data() + r_;
    *n1 = size_ - r_;
    if (w_ > 0) {
      *end = buf_.data();
      *n2 = w_;
    }
  }

  // Read(p): copies min(n, Length()) bytes from the front and consumes them
  // (ws.go:180, 186; protocol.go:51).
  uint64_t Read(uint8_t* p, uint64_t n) {
    const uint8_t *a, *b;
    uint64_t na, nb;
    PeekAll(&a, &na, &b, &nb);
    const uint64_t c1 = std::min(n, na), c2 = std::min(n - c1, nb);
    if (c1) memcpy(p, a, c1);
    if (c2) memcpy(p + c1, b, c2);
    Retrieve(c1 + c2);
    return c1 + c2;
  }

  // Bytes consumed since construction: identifies the read position, so a
  // value derived from the buffered bytes (the protocol's completeness carry)
  // can tell whether anyone consumed bytes since it was derived.
  uint64_t Retrieved() const { return retrieved_; }

  void Retrieve(uint64_t n) {
    const uint64_t len = Length();
    retrieved_ += n < len ? n : len;
    if (n >= len) {
      r_ = w_ = 0;
      empty_ = true;
      return;
    }
    r_ = (r_ + n) % size_;
  }

 private:
  void grow(uint64_t need) {
    uint64_t ns = size_;
    while (ns < need) ns *= 2;
    std::vector<uint8_t> nb(ns);
    const uint8_t *a, *b;
    uint64_t na, nb2;
    PeekAll(&a, &na, &b, &nb2);
    if (na) memcpy(nb.data(), a, na);
    if (nb2) memcpy(nb.data() + na, b, nb2);
    const uint64_t len = na + nb2;
    buf_.swap(nb);
    size_ = ns;
    r_ = 0;
    w_ = len % size_;
    empty_ = len == 0;
  }

  std::vector<uint8_t> buf_;
  uint64_t size_;
  uint64_t r_ = 0, w_ = 0;
  uint64_t retrieved_ = 0;
  bool empty_ = true;
};

}  // namespace gevws
