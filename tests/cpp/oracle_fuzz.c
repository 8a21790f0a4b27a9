/* Random byte streams through the C oracle's decode (oracle/ws_ref.c) under
 * ASan/UBSan: no out-of-bounds access on truncated / hostile input, and the
 * per-connection results are consistent (consumed <= len; payload arena
 * offsets increase).  Built by tests/test_host_sanitizers.py. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { uint8_t fin, rsv, opcode, masked; uint8_t mask[4]; int64_t length; } wsref_header;
typedef struct { wsref_header hdr; uint64_t payload_off; uint64_t src_off; } wsref_frame;
int64_t wsref_decode_batch(const uint8_t *in, const uint64_t *conn_off, const uint64_t *conn_len, uint32_t n,
                           wsref_frame *frames, uint64_t max_frames, uint8_t *payload, uint64_t payload_cap,
                           uint64_t *conn_first, uint32_t *conn_nframes, int32_t *conn_status,
                           uint64_t *conn_consumed, uint64_t *total_payload);

static uint64_t s = 88172645463325252ull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }

int main(void) {
  for (int it = 0; it < 3000; ++it) {
    uint32_t n = 1 + rnd() % 8;
    uint64_t off[8], len[8], tot = 0;
    for (uint32_t c = 0; c < n; ++c) { off[c] = tot; len[c] = rnd() % 400; tot += len[c]; }
    uint8_t *in = malloc(tot + 1);
    for (uint64_t i = 0; i < tot; ++i) {
      uint64_t r = rnd();
      /* bias towards plausible header bytes so frames actually parse */
      in[i] = (r & 3) == 0 ? (uint8_t)(0x80 | (r >> 8) % 16) : (r & 3) == 1 ? (uint8_t)((r >> 8) % 140) : (uint8_t)(r >> 16);
    }
    uint64_t mf = tot / 2 + 1, cap = tot + 16 * mf + 16;
    wsref_frame *fr = malloc(mf * sizeof(wsref_frame));
    uint8_t *pay = malloc(cap);
    uint64_t first[8], cons[8], tp;
    uint32_t nf[8];
    int32_t st[8];
    int64_t r = wsref_decode_batch(in, off, len, n, fr, mf, pay, cap, first, nf, st, cons, &tp);
    if (r < 0) { fprintf(stderr, "capacity error\n"); return 1; }
    for (uint32_t c = 0; c < n; ++c)
      if (cons[c] > len[c]) { fprintf(stderr, "consumed > len\n"); return 2; }
    for (int64_t k = 1; k < r; ++k)
      if (fr[k].payload_off < fr[k - 1].payload_off) { fprintf(stderr, "offsets\n"); return 3; }
    free(in); free(fr); free(pay);
  }
  puts("oracle_fuzz ok");
  return 0;
}
