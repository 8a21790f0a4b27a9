// Differential fuzz of gevws::RingBuffer (gev_amd/csrc/ringbuffer.hpp) against
// a std::deque model, built with -fsanitize=address,undefined by
// tests/test_host_sanitizers.py.  Exit 0 = every operation matched.
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <random>

#include "../../gev_amd/csrc/ringbuffer.hpp"

int main(int argc, char** argv) {
  const unsigned seed = argc > 1 ? (unsigned)atoi(argv[1]) : 1u;
  std::mt19937_64 rng(seed);
  for (int round = 0; round < 200; ++round) {
    gevws::RingBuffer r(1 + rng() % 64);
    std::deque<uint8_t> model;
    for (int op = 0; op < 2000; ++op) {
      if (rng() % 100 < 55) {
        std::vector<uint8_t> d(rng() % 300);
        for (auto& b : d) b = (uint8_t)rng();
        r.Write(d.data(), d.size());
        model.insert(model.end(), d.begin(), d.end());
      } else if (rng() % 4 == 0) {
        std::vector<uint8_t> got(rng() % 300);
        const uint64_t k = r.Read(got.data(), got.size());
        if (k != std::min<uint64_t>(got.size(), model.size())) return 5;
        for (uint64_t i = 0; i < k; ++i)
          if (got[i] != model[i]) return 6;
        model.erase(model.begin(), model.begin() + k);
      } else {
        const uint64_t k = rng() % 400;
        r.Retrieve(k);
        model.erase(model.begin(), model.begin() + std::min<uint64_t>(k, model.size()));
      }
      if (r.Length() != model.size() || r.IsEmpty() != model.empty()) {
        fprintf(stderr, "length mismatch seed %u round %d op %d\n", seed, round, op);
        return 1;
      }
      const uint8_t *a, *b;
      uint64_t na, nb;
      r.PeekAll(&a, &na, &b, &nb);
      if (na + nb != model.size()) return 2;
      for (uint64_t i = 0; i < na; ++i)
        if (a[i] != model[i]) return 3;
      for (uint64_t i = 0; i < nb; ++i)
        if (b[i] != model[na + i]) return 4;
    }
  }
  puts("ring_fuzz ok");
  return 0;
}
