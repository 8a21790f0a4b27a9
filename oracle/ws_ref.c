/*
 * ws_ref.c -- C restatement of the reference WebSocket decode path.
 *
 * TEST INFRASTRUCTURE ONLY (checker + CPU baseline).  Never linked into the
 * product library (gev_amd/libgevws.so); only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg load oracle/libwsref.so.
 *
 * Restated from the semantics of Allenxuxu/gev (Go); no reference source is
 * copied.  The reference cannot be built here (no Go toolchain), so this file
 * also serves as the CPU baseline ("kind": "port"): it mirrors the per-frame
 * work of websocket.(*Protocol).UnPacket -- header parse, zero-filled
 * make([]byte, L), ring Read (memcpy), Cipher word loop -- and is compiled
 * -O2 -fno-tree-vectorize to mirror Go gc's scalar code.
 *
 * Parity: pinned by RFC 6455 §5.7 KATs and cross-checked against the Python
 * oracle (oracle/ws_oracle.py); ringbuffer-dependent rows U1-U3 of SURVEY.md
 * Appendix A are unpinned (NEED_MORE chosen).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define WSREF_OK 0
#define WSREF_NEED_MORE 1
#define WSREF_ERR_LEN_MSB (-1)
#define WSREF_ERR_CAPACITY (-2)

typedef struct {
    uint8_t fin, rsv, opcode, masked;
    uint8_t mask[4];
    int64_t length;
} wsref_header; /* ws.Header, frame.go:169-176 */

typedef struct {
    wsref_header hdr;
    uint64_t payload_off;
    uint64_t src_off;
} wsref_frame;

/* remain, cipher.go:56 */
static const int k_remain[4] = {0, 3, 2, 1};

/* ws.Cipher, cipher.go:14-53: bytewise for n < 8; else head ln, tail rn
 * bytewise and a native-endian uint64 body XOR with m<<32|m. */
void wsref_cipher(uint8_t *p, size_t n, const uint8_t mask[4], size_t offset) {
    if (n < 8) {
        for (size_t i = 0; i < n; i++) p[i] ^= mask[(offset + i) & 3];
        return;
    }
    size_t mpos = offset & 3;
    size_t ln = (size_t)k_remain[mpos];
    size_t rn = (n - ln) & 7;
    for (size_t i = 0; i < ln; i++) p[i] ^= mask[(mpos + i) & 3];
    for (size_t i = n - rn; i < n; i++) p[i] ^= mask[(mpos + i) & 3];
    uint32_t m;
    memcpy(&m, mask, 4);
    uint64_t m2 = ((uint64_t)m << 32) | m;
    size_t words = (n - ln - rn) >> 3;
    for (size_t i = 0; i < words; i++) {
        uint64_t v;
        memcpy(&v, p + ln + (i << 3), 8);
        v ^= m2;
        memcpy(p + ln + (i << 3), &v, 8);
    }
}

/* ws.VirtualReadHeader, read.go:19-84, on a linear view (ring PeekAll joined). */
int wsref_read_header(const uint8_t *p, uint64_t avail, wsref_header *h, uint32_t *hlen) {
    if (avail < 6) return WSREF_NEED_MORE; /* read.go:20-23 */
    memset(h, 0, sizeof(*h));
    uint8_t b0 = p[0], b1 = p[1];
    h->fin = (b0 & 0x80) != 0;
    h->rsv = (uint8_t)((b0 & 0x70) >> 4);
    h->opcode = b0 & 0x0F;
    uint32_t extra = 0;
    if (b1 & 0x80) { h->masked = 1; extra += 4; }
    uint8_t len7 = b1 & 0x7F;
    if (len7 < 126) h->length = len7;
    else if (len7 == 126) extra += 2;
    else extra += 8;
    *hlen = 2 + extra;
    if (extra == 0) return WSREF_OK;
    if (avail < *hlen) return WSREF_NEED_MORE; /* U1: unpinned, RFC-correct choice */
    const uint8_t *e = p + 2;
    if (len7 == 126) {
        h->length = ((int64_t)e[0] << 8) | e[1];
        e += 2;
    } else if (len7 == 127) {
        if (e[0] & 0x80) return WSREF_ERR_LEN_MSB; /* read.go:71-73 */
        uint64_t L = 0;
        for (int i = 0; i < 8; i++) L = (L << 8) | e[i];
        h->length = (int64_t)L;
        e += 8;
    }
    if (h->masked) memcpy(h->mask, e, 4);
    return WSREF_OK;
}

/* Repeated UnPacket (protocol.go:38-62) driven like handlerProtocol
 * (connection.go:208-218) over every connection of a batch, writing into the
 * product's output layout (frames in connection order; payload offsets are the
 * running sum of 16-byte-rounded lengths; pad bytes zero) so the GPU result can
 * be compared byte for byte.  Returns total frames, or a negative status. */
int64_t wsref_decode_batch(const uint8_t *in, const uint64_t *conn_off, const uint64_t *conn_len,
                           uint32_t n_conns, wsref_frame *frames, uint64_t max_frames,
                           uint8_t *payload, uint64_t payload_cap, uint64_t *conn_first,
                           uint32_t *conn_nframes, int32_t *conn_status, uint64_t *conn_consumed,
                           uint64_t *total_payload) {
    uint64_t nf = 0, poff = 0;
    for (uint32_t c = 0; c < n_conns; c++) {
        const uint8_t *s = in + conn_off[c];
        uint64_t len = conn_len[c], pos = 0;
        uint32_t cnt = 0;
        int32_t st = WSREF_OK;
        conn_first[c] = nf;
        for (;;) {
            wsref_header h;
            uint32_t hl = 0;
            int r = wsref_read_header(s + pos, len - pos, &h, &hl);
            if (r != WSREF_OK) { st = (r == WSREF_NEED_MORE) ? WSREF_OK : r; break; }
            if (len - pos - hl < (uint64_t)h.length) break; /* protocol.go:47 gate */
            uint64_t L = (uint64_t)h.length;
            uint64_t padded = (L + 15) & ~(uint64_t)15;
            if (nf >= max_frames || poff + padded > payload_cap) return WSREF_ERR_CAPACITY;
            frames[nf].hdr = h;
            frames[nf].payload_off = poff;
            frames[nf].src_off = conn_off[c] + pos + hl;
            memcpy(payload + poff, s + pos + hl, L);
            memset(payload + poff + L, 0, padded - L);
            if (h.masked) wsref_cipher(payload + poff, L, h.mask, 0);
            poff += padded;
            nf++;
            cnt++;
            pos += hl + L;
        }
        conn_nframes[c] = cnt;
        conn_status[c] = st;
        conn_consumed[c] = pos;
    }
    *total_payload = poff;
    return (int64_t)nf;
}

/* ------------------------------------------------------------------ CPU baseline
 * The reference per-frame pipeline, as UnPacket does it for each frame:
 * header parse; payload := make([]byte, L) (zero-filled); ring.Read(payload)
 * (memcpy); Cipher if masked; the slice is handed to the handler and later
 * collected.  A checksum keeps the work observable.
 *
 * Where make's memory comes from (alloc_mode):
 *   WSREF_ALLOC_FRESH (the baseline): a per-thread bump arena, reset when it
 *     runs out, whose size keeps the threads' arenas together larger than the
 *     host's last-level cache -- each frame's destination is memory the loop
 *     has not touched for a while, as Go's make hands out spans the collector
 *     swept (protocol.go:50), zero-filled like make;
 *   WSREF_ALLOC_CACHE_HOT: calloc + free per frame -- glibc hands the same
 *     chunk back each time, so the destination stays in L1/L2 (flatters the
 *     CPU; kept as a second number). */
enum { WSREF_ALLOC_FRESH = 0, WSREF_ALLOC_CACHE_HOT = 1 };

typedef struct {
    uint8_t *base;
    uint64_t cap, top;
} bump_arena;

static uint8_t *arena_make(bump_arena *a, size_t L) {
    const uint64_t need = (L + 63) & ~(uint64_t)63;
    if (a->top + need > a->cap) a->top = 0;  /* the sweep starts over: the oldest memory */
    uint8_t *p = a->base + a->top;
    a->top += need;
    memset(p, 0, L);  /* make's zero fill */
    return p;
}

static uint64_t pipeline_stream(const uint8_t *s, uint64_t len, uint64_t *frames_out,
                                uint64_t *payload_out, bump_arena *arena) {
    uint64_t pos = 0, nf = 0, pb = 0, ck = 0;
    for (;;) {
        wsref_header h;
        uint32_t hl = 0;
        if (wsref_read_header(s + pos, len - pos, &h, &hl) != WSREF_OK) break;
        if (len - pos - hl < (uint64_t)h.length) break;
        size_t L = (size_t)h.length;
        uint8_t *payload = arena ? arena_make(arena, L) : (uint8_t *)calloc(L ? L : 1, 1);
        memcpy(payload, s + pos + hl, L);
        if (h.masked) wsref_cipher(payload, L, h.mask, 0);
        if (L) ck += payload[0] + payload[L - 1];
        if (!arena) free(payload);
        pos += hl + L;
        nf++;
        pb += L;
    }
    *frames_out += nf;
    *payload_out += pb;
    return ck;
}

typedef struct {
    const uint8_t *in;
    const uint64_t *conn_off, *conn_len;
    uint32_t n_conns, tid, nthreads;
    double min_seconds;
    uint64_t frames, payload, checksum;
    int iters;
    double seconds;
    bump_arena *arena;
} bench_arg;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void *bench_thread(void *p) {
    bench_arg *a = (bench_arg *)p;
    double t0 = now_s();
    a->iters = 0;
    do {
        /* connections assigned round-robin to loops, load_balance.go:7-14 */
        for (uint32_t c = a->tid; c < a->n_conns; c += a->nthreads)
            a->checksum += pipeline_stream(a->in + a->conn_off[c], a->conn_len[c], &a->frames,
                                           &a->payload, a->arena);
        a->iters++;
        a->seconds = now_s() - t0;
    } while (a->seconds < a->min_seconds);
    return NULL;
}

/* Runs the pipeline over the batch repeatedly (>= min_seconds) on `threads`
 * threads; returns wall seconds, total payload bytes and frames processed.
 * alloc_mode: WSREF_ALLOC_FRESH with arena_bytes per thread (its pages are
 * touched before the clock starts), or WSREF_ALLOC_CACHE_HOT.  -1 on an
 * arena allocation failure. */
double wsref_bench_pipeline_alloc(const uint8_t *in, const uint64_t *conn_off, const uint64_t *conn_len,
                                  uint32_t n_conns, int threads, double min_seconds, int alloc_mode,
                                  uint64_t arena_bytes, uint64_t *payload_bytes, uint64_t *frames,
                                  uint64_t *checksum) {
    if (threads < 1) threads = 1;
    bench_arg *args = (bench_arg *)calloc((size_t)threads, sizeof(bench_arg));
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    bump_arena *arenas = alloc_mode == WSREF_ALLOC_FRESH ? (bump_arena *)calloc((size_t)threads, sizeof(bump_arena))
                                                         : NULL;
    /* the largest frame must fit an arena */
    uint64_t maxf = 0;
    for (uint32_t c = 0; c < n_conns; c++) maxf = conn_len[c] > maxf ? conn_len[c] : maxf;
    if (arena_bytes < maxf + 64) arena_bytes = maxf + 64;
    double wall = -1;
    for (int i = 0; arenas && i < threads; i++) {
        arenas[i].base = (uint8_t *)malloc(arena_bytes);
        if (!arenas[i].base) goto out;
        memset(arenas[i].base, 1, arena_bytes);  /* fault the pages in before the clock */
        arenas[i].cap = arena_bytes;
    }
    double t0 = now_s();
    for (int i = 0; i < threads; i++) {
        args[i] = (bench_arg){in, conn_off, conn_len, n_conns, (uint32_t)i, (uint32_t)threads,
                              min_seconds, 0, 0, 0, 0, 0.0, arenas ? &arenas[i] : NULL};
        pthread_create(&th[i], NULL, bench_thread, &args[i]);
    }
    uint64_t pb = 0, nf = 0, ck = 0;
    for (int i = 0; i < threads; i++) {
        pthread_join(th[i], NULL);
        pb += args[i].payload;
        nf += args[i].frames;
        ck += args[i].checksum;
    }
    wall = now_s() - t0;
    *payload_bytes = pb;
    *frames = nf;
    *checksum = ck;
out:
    for (int i = 0; arenas && i < threads; i++) free(arenas[i].base);
    free(arenas);
    free(args);
    free(th);
    return wall;
}

double wsref_bench_pipeline(const uint8_t *in, const uint64_t *conn_off, const uint64_t *conn_len,
                            uint32_t n_conns, int threads, double min_seconds,
                            uint64_t *payload_bytes, uint64_t *frames, uint64_t *checksum) {
    return wsref_bench_pipeline_alloc(in, conn_off, conn_len, n_conns, threads, min_seconds,
                                      WSREF_ALLOC_CACHE_HOT, 0, payload_bytes, frames, checksum);
}

/* ------------------------------------------------------------------ outbound encode
 * ws.WriteHeader (write.go:48-84) with Go's byte arithmetic, and a batch of
 * ws.FrameToBytes (frame.go:274-278) written back to back. */
typedef struct {
    wsref_header hdr;
    uint64_t payload_off;
    uint64_t payload_len;
} wsref_out_frame;

uint32_t wsref_write_header(const wsref_header *h, uint8_t out[14]) {
    memset(out, 0, 14);
    if (h->fin) out[0] |= 0x80;
    out[0] |= (uint8_t)(h->rsv << 4);
    out[0] |= h->opcode;
    uint32_t n;
    if (h->length <= 125) {
        out[1] = (uint8_t)h->length;
        n = 2;
    } else if (h->length <= 0xFFFF) {
        out[1] = 126;
        out[2] = (uint8_t)(h->length >> 8);
        out[3] = (uint8_t)h->length;
        n = 4;
    } else {
        out[1] = 127;
        for (int i = 0; i < 8; i++) out[2 + i] = (uint8_t)((uint64_t)h->length >> (56 - 8 * i));
        n = 10;
    }
    if (h->masked) {
        out[1] |= 0x80;
        memcpy(out + n, h->mask, 4);
        n += 4;
    }
    return n;
}

/* Returns the wire total, or WSREF_ERR_CAPACITY. */
int64_t wsref_encode_batch(const wsref_out_frame *f, uint64_t n, const uint8_t *payload, uint8_t *out,
                           uint64_t out_cap, uint64_t *out_off) {
    uint64_t o = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint8_t h[14];
        uint32_t hl = wsref_write_header(&f[i].hdr, h);
        if (o + hl + f[i].payload_len > out_cap) return WSREF_ERR_CAPACITY;
        out_off[i] = o;
        memcpy(out + o, h, hl);
        memcpy(out + o + hl, payload + f[i].payload_off, f[i].payload_len);
        o += hl + f[i].payload_len;
    }
    return (int64_t)o;
}
