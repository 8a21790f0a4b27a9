// gevws_small.hpp -- the one-launch decode's body (decode_small_body), the
// cross-workgroup hand-off it stages a live pass's input with, and its
// staging rules: what k_decode_small, k_decode_small_direct and the resident
// service (gevws_walk.hip) share.  (A decode + handler step fused into one
// launch was built on it and measured 45 % slower on the wsserver shape,
// profiles/r06/r06aj_lb_ab.jsonl; not kept.)
#pragma once

#include "gevws_internal.hpp"

namespace {

// ------------------------------------------------------------------ hand-offs
// Two hand-offs cross workgroups inside one launch: the walk's block partials
// to its last workgroup (walk_block_done) and a live pass's input, staged by
// many workgroups, to the one-launch decode's last one (k_decode_small).
// Both move TAGGED GRANULES: 8 bytes {u32 data, u32 tag}, stored and loaded
// as agent-scope relaxed 64-bit atomics, the tag being the launch's number
// (next_hand_tag: never 0; the buffers start zeroed).  The last workgroup is
// elected by an agent-scope counter (relaxed: the read-modify-writes on it
// are totally ordered, so exactly one sees nwg - 1) and takes a granule's
// data only once it has loaded that granule carrying this launch's tag.  A
// load that returns the tag returns the data of the same store (an atomic
// is never torn; per-location coherence), so the hand-off rests neither on a
// release / acquire pair nor on cache behaviour.  On gfx950 the first load
// carries the tag (the writers' stores are write-through and drained by
// s_waitcnt before their counter add); the re-load loop is what the memory
// model guarantees, bounded: a granule that never shows its tag fails the
// launch (GEVWS_ERR_DEVICE).  A release (buffer_wbl2) in every workgroup and
// an acquire in the last cost ~1.7 us each on gfx950 (MI355X_MICROARCH.md,
// the fence rows) against a ~9 us live-pass kernel; the tags cost twice the
// bytes of a hand-off of a few KB.
constexpr uint32_t kHandSpin = 1u << 16;  // re-loads of one granule before the launch fails
__device__ __forceinline__ void put_granule(uint64_t* p, uint32_t v, uint32_t tag) {
  __hip_atomic_store(p, (uint64_t)v | ((uint64_t)tag << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t load_granule(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The data of the granule at p, loaded as g, once it carries `tag` (bad = 1 if it never did).
__device__ __forceinline__ uint32_t take_granule(const uint64_t* p, uint64_t g, uint32_t tag, uint32_t& bad) {
  for (uint32_t i = 0; (uint32_t)(g >> 32) != tag; ++i) {
    if (i == kHandSpin) {
      bad = 1;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
    g = load_granule(p);
  }
  return (uint32_t)g;
}

// ------------------------------------------------------------------ 3c. small batches, one launch
// A live server's pass is small (C1: ~100 connections x 136 B per loop
// iteration) and pays per launch, not per byte: four kernels cost ~5 us each
// of GPU time whatever their size (profiles/r02/r02_loopback_*), plus their host
// launch costs.  Batches of at most kOneLaunchConns connections and
// GEVWS_TUNE_SMALL_BATCH bytes (default kOneLaunchBytes) run the whole decode
// in ONE workgroup of NT lanes: each lane walks its connection (k_walk_count's
// rules), a block scan gives the bases and the summary, each lane re-walks its
// chain writing the records and unmasking payloads of up to kSmallLaneBytes
// itself (all its chunk loads at once), and the workgroup unmasks the larger
// ones together.  Output identical to the multi-kernel decode.
// The whole input (<= SB + the pad) is staged into LDS first, by independent
// coalesced 16-byte loads, and every header and payload read after that is an
// LDS read: a live pass's input sits in mapped pinned host memory, where each
// of the walk's and the record pass's DEPENDENT header loads was a PCIe round
// trip (the kernel took ~10 us for 100 connections of 1-2 frames,
// profiles/r05/r05_loopback_timeline.jsonl).
// Two shapes (SmallShape): <256 lanes, 64 KiB> for a loop's usual pass and
// <1 024 lanes, 128 KiB> above it -- 146 KB of LDS, one workgroup per CU --
// which takes the 4 000-connection live shape's passes (~500 connections,
// ~67 KB) that used to fall to the multi-kernel decode over mapped memory.
constexpr uint32_t kSmallLaneBytes = 256;

// 16 bytes at byte `off` of the staged input (any alignment: five aligned
// dword reads and a byte funnel shift)
__device__ __forceinline__ u32x4 lds16(const uint32_t* __restrict__ s, uint32_t off) {
  const uint32_t k = off >> 2, e = off & 3;
  const uint32_t w0 = s[k], w1 = s[k + 1], w2 = s[k + 2], w3 = s[k + 3], w4 = s[k + 4];
  return u32x4{__builtin_amdgcn_alignbyte(w1, w0, e), __builtin_amdgcn_alignbyte(w2, w1, e),
               __builtin_amdgcn_alignbyte(w3, w2, e), __builtin_amdgcn_alignbyte(w4, w3, e)};
}
__device__ __forceinline__ void lds_window(const uint32_t* __restrict__ s, uint32_t off, uint64_t& lo, uint64_t& hi) {
  const u32x4 v = lds16(s, off);
  lo = (uint64_t)v[0] | ((uint64_t)v[1] << 32);
  hi = (uint64_t)v[2] | ((uint64_t)v[3] << 32);
}

template <uint32_t NT_, uint64_t SB_>
struct SmallShape {
  static constexpr uint32_t NT = NT_;  // lanes = connections at most
  static constexpr uint64_t SB = SB_;  // input bytes at most
  static constexpr uint32_t kStage = (uint32_t)((SB + GEVWS_IN_PAD) / 16);  // 16-byte chunks of staged input
  static constexpr uint32_t kBig = (uint32_t)(SB / kSmallLaneBytes);  // larger payloads fit in the input at most this often
  // staging loads a thread keeps in flight (4 granules a chunk in the hand-off)
  static constexpr int kBatch = NT >= 1024 ? 4 : 8;
};
using SmallNarrow = SmallShape<kSmallConns, kSmallBytes>;
using SmallWide = SmallShape<kOneLaunchConns, kOneLaunchBytes>;

// A live pass's input is read by up to kSmallStageWGs workgroups, a slice of
// at least kSmallSliceChunks 16-byte chunks each (2 KiB)
constexpr uint32_t kSmallStageWGs = 32;
constexpr uint64_t kSmallSliceChunks = 128;
// their finished-workgroup counter: a word of ctx->d_done of its own (the
// walk's is d_done[0]), 128 bytes apart
constexpr uint32_t kSmallStageCounter = 32;
// ... and the split walk's count of connections re-walked serially after a
// missed guess (gevws_ctx_last_split_fallbacks), a word of its own too
constexpr uint32_t kSplitFallbackCounter = 48;

// The body of the one-launch decode (k_decode_small, and each pass of the
// resident service k_decode_service); every return is workgroup-uniform.
// With nwg > 1 the nwg workgroups (this one is wg) count themselves in on
// stage_done after staging their slice of the input (nslices of them, the
// rest empty); true for the workgroup that decoded (and signalled).
template <class S>
__device__ __forceinline__ bool decode_small_body(const uint8_t* __restrict__ in, uint64_t in_bytes,
                                                  const gevws_conn_in* __restrict__ conns, uint32_t n,
                                                  gevws_frame* __restrict__ frames, uint64_t max_frames,
                                                  uint8_t* __restrict__ payload, uint64_t payload_cap,
                                                  gevws_conn_out* __restrict__ cout, gevws_summary* __restrict__ sum,
                                                  uint32_t* __restrict__ done, uint32_t seq,
                                                  uint64_t* __restrict__ ticks, uint64_t* __restrict__ stage_buf,
                                                  uint32_t* __restrict__ stage_done, uint32_t tag, uint32_t nwg,
                                                  uint32_t wg, uint32_t nslices,
                                                  uint64_t* __restrict__ phase = nullptr) {
  constexpr uint32_t NT = S::NT;
  constexpr int kBatch = S::kBatch;
  __shared__ uint64_t s_big[S::kBig][3];  // {src_off, payload_off, length} of the larger payloads
  __shared__ uint32_t s_last;
  __shared__ uint32_t s_bkey[S::kBig];
  __shared__ uint32_t s_nbig;
  __shared__ uint32_t s_bad;
  __shared__ __attribute__((aligned(16))) uint32_t s_in[4 * S::kStage + 4];  // the staged input (+ a dword of slack)
  const uint64_t t0 = done ? gpu_ticks() : 0;
  const uint32_t c = threadIdx.x;
  if (c == 0) {
    s_nbig = 0;
    s_bad = 0;
  }
  gevws_conn_in ci{0, 0}, cprev{0, 0};
  if (c < n) {  // (in flight with the staging loads)
    ci = conns[c];
    if (c > 0) cprev = conns[c - 1];
  }
  if (n) {  // bytes [0, 16 x nst) of the input: every read below is inside [0, in_bytes + 48)
    const uint32_t nst = (uint32_t)((in_bytes + GEVWS_IN_PAD) / 16);
    u32x4* st = reinterpret_cast<u32x4*>(s_in);
    if (nwg > 1) {
      // A live pass's input sits in mapped host memory, which one workgroup
      // reads at ~2.5 GB/s (a 20 KB pass: ~8 us of staging).  So every
      // workgroup copies its slice of the input into stage_buf as tagged
      // granules (hand-offs, above: 4 a 16-byte chunk), and the last one to
      // finish (stage_done) stages the whole input from there into its LDS
      // and runs the decode; the others end here.
      const uint32_t per = (nst + nslices - 1) / nslices;
      const uint32_t k0 = wg < nslices ? wg * per : nst, k1 = k0 + per < nst ? k0 + per : nst;
      for (uint32_t kb = k0; kb < k1; kb += kBatch * NT) {
        u32x4 x[kBatch];
#pragma unroll
        for (int j = 0; j < kBatch; ++j) {
          const uint32_t k = kb + (uint32_t)j * NT + c;
          if (k < k1) x[j] = ld16u(in + 16ull * k);
        }
#pragma unroll
        for (int j = 0; j < kBatch; ++j) {
          const uint32_t k = kb + (uint32_t)j * NT + c;
          if (k < k1)
#pragma unroll
            for (int i = 0; i < 4; ++i) put_granule(stage_buf + 4ull * k + i, x[j][i], tag);
        }
      }
      __builtin_amdgcn_s_waitcnt(0);  // this workgroup's stores are done before it counts itself
      __syncthreads();
      if (c == 0)
        s_last = __hip_atomic_fetch_add(stage_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nwg - 1 ? 1u : 0u;
      __syncthreads();
      if (!s_last) return false;
      if (c == 0) __hip_atomic_store(stage_done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the next launch's
      uint32_t bad = 0;
      for (uint32_t kb = 0; kb < nst; kb += kBatch * NT) {
        uint64_t g[kBatch][4];
#pragma unroll
        for (int j = 0; j < kBatch; ++j) {
          const uint32_t k = kb + (uint32_t)j * NT + c;
          if (k < nst)
#pragma unroll
            for (int i = 0; i < 4; ++i) g[j][i] = load_granule(stage_buf + 4ull * k + i);
        }
#pragma unroll
        for (int j = 0; j < kBatch; ++j) {
          const uint32_t k = kb + (uint32_t)j * NT + c;
          if (k < nst) {
            const uint64_t* q = stage_buf + 4ull * k;
            st[k] = u32x4{take_granule(q, g[j][0], tag, bad), take_granule(q + 1, g[j][1], tag, bad),
                          take_granule(q + 2, g[j][2], tag, bad), take_granule(q + 3, g[j][3], tag, bad)};
          }
        }
      }
      if (bad) s_bad = 1;
    } else for (uint32_t k0 = 0; k0 < nst; k0 += kBatch * NT) {
      u32x4 x[kBatch];
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        const uint32_t k = k0 + (uint32_t)j * NT + c;
        if (k < nst) x[j] = ld16u(in + 16ull * k);
      }
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        const uint32_t k = k0 + (uint32_t)j * NT + c;
        if (k < nst) st[k] = x[j];
      }
    }
  }
  __syncthreads();
  if (phase && c == 0) phase[0] = gpu_ticks();  // (measurement: the input is in LDS)
  if (s_bad) {  // a staged granule never carried this launch's tag (workgroup-uniform)
    if (c == 0) {
      gevws_summary sm;
      memset(&sm, 0, sizeof(sm));
      sm.status = GEVWS_ERR_DEVICE;
      *sum = sm;
    }
    signal_done(done, seq, ticks, t0, 0);
    return true;
  }
  uint64_t nf = 0, pb = 0, pl = 0, err = 0, same = 0, lastf = ~0ull, pos = 0;
  int32_t st = GEVWS_OK;
  if (c < n) {
    if (c > 0 && (ci.off < cprev.off || ci.off - cprev.off < cprev.len))
      err = 1ull << 32;  // out of order (out_of_order): informational, as k_walk_count
    if (ci.off > in_bytes || ci.len > in_bytes - ci.off) {
      ci.off = 0;
      ci.len = 0;
      st = GEVWS_ERR_INVALID;
      err += 1;
    }
    for (;;) {  // read.go:19-84 + the protocol.go:47 gate, frame after frame
      uint64_t lo, hi;
      lds_window(s_in, (uint32_t)(ci.off + pos), lo, hi);
      DevHdr h;
      const int r = parse_header(lo, hi, ci.len - pos, h);
      if (r == GEVWS_ERR_LEN_MSB) {
        st = GEVWS_ERR_LEN_MSB;
        err += 1;
      }
      if (r != GEVWS_OK || ci.len - pos - h.hlen < h.length) break;
      ++nf;
      pb += round16(h.length);
      pl += h.length;
      const uint64_t f = h.hlen + h.length;
      same += f == lastf;
      lastf = f;
      pos += f;
    }
  }
  // The five sums fit 32 bits here (input <= 128 KiB, <= 1 024 lanes): the
  // DPP scan (block_excl_scan32) instead of the 64-bit shuffle scan, 2.5 us
  // of a 100-connection pass (tools/live_pass_probe.py, GEVWS_PHASE_TICKS).
  // Field 3 carries the errors (<= 2 a lane) in its low 16 bits and the
  // out-of-order lanes in its high 16.
  const uint32_t v[kDecFields] = {(uint32_t)nf, (uint32_t)pb, (uint32_t)pl,
                                  (uint32_t)(err & 0xffffu) | ((uint32_t)(err >> 32) << 16), (uint32_t)same};
  uint32_t ex[kDecFields], tot[kDecFields];
  if (phase && c == 0) phase[1] = gpu_ticks();  // (measurement: this lane's chain parsed)
  block_excl_scan32<NT, kDecFields>(v, ex, tot);
  if (phase && c == 0) phase[2] = gpu_ticks();  // (measurement: the workgroup's scan done)
  const bool ok = tot[0] <= max_frames && tot[1] <= payload_cap;
  if (c == 0) {
    gevws_summary sm;
    memset(&sm, 0, sizeof(sm));
    sm.frames = tot[0];
    sm.payload_bytes = tot[1];
    sm.payload_len = tot[2];
    sm.errors = tot[3] & 0xffffu;
    sm.flags = (tot[3] >> 16) ? GEVWS_SUMMARY_UNORDERED : 0u;
    sm.run_frames = tot[4];
    sm.status = ok ? GEVWS_OK : GEVWS_ERR_CAPACITY;
    *sum = sm;
  }
  if (!ok) {  // capacity error: nothing written (uniform)
    signal_done(done, seq, ticks, t0, 0);
    return true;
  }
  if (c < n) {
    gevws_conn_out o;
    o.first_frame = ex[0];
    o.consumed = pos;
    o.payload_base = ex[1];
    o.nframes = (uint32_t)nf;
    o.status = st;
    cout[c] = o;
    // records + the lane's own payloads
    uint64_t q = 0, poff = ex[1];
    for (uint64_t k = 0; k < nf; ++k) {
      uint64_t lo, hi;
      lds_window(s_in, (uint32_t)(ci.off + q), lo, hi);
      DevHdr h;
      parse_header(lo, hi, ci.len - q, h);  // succeeded in the walk above
      const uint64_t src = ci.off + q + h.hlen;
      const uint32_t flags = (h.b0 >> 7) | (((h.b0 & 0x70) >> 4) << 8) | ((h.b0 & 0x0f) << 16) | ((h.masked & 1) << 24);
      u32x4* rp = reinterpret_cast<u32x4*>(frames + ex[0] + k);
      rp[0] = u32x4{flags, h.mask, (uint32_t)h.length, (uint32_t)(h.length >> 32)};
      rp[1] = u32x4{(uint32_t)poff, (uint32_t)(poff >> 32), (uint32_t)src, (uint32_t)(src >> 32)};
      if (h.length <= kSmallLaneBytes) {
        constexpr int NCH = kSmallLaneBytes / 16;
        const uint32_t nch = (uint32_t)((h.length + 15) >> 4);
        u32x4 x[NCH];
#pragma unroll
        for (int j = 0; j < NCH; ++j)
          if ((uint32_t)j < nch) x[j] = lds16(s_in, (uint32_t)(src + 16ull * j));
#pragma unroll
        for (int j = 0; j < NCH; ++j)
          if ((uint32_t)j < nch) {
            u32x4 y = x[j] ^ h.mask;
            const int64_t rem = (int64_t)h.length - 16 * j;
            if (rem < 16) y = keep_bytes(y, rem);
            *reinterpret_cast<u32x4*>(payload + poff + 16ull * j) = y;
          }
      } else {
        const uint32_t b = atomicAdd(&s_nbig, 1u);
        s_big[b][0] = src;
        s_big[b][1] = poff;
        s_big[b][2] = h.length;
        s_bkey[b] = h.mask;
      }
      poff += round16(h.length);
      q += h.hlen + h.length;
    }
  }
  __syncthreads();
  const uint32_t nbig = s_nbig;
  for (uint32_t b = 0; b < nbig; ++b) {  // the larger payloads, by the whole workgroup
    const uint64_t src = s_big[b][0], poff = s_big[b][1], L = s_big[b][2];
    const uint32_t key = s_bkey[b];
    for (uint64_t j = c; 16 * j < L; j += NT) {
      u32x4 y = lds16(s_in, (uint32_t)(src + 16 * j)) ^ key;
      const int64_t rem = (int64_t)L - (int64_t)(16 * j);
      if (rem < 16) y = keep_bytes(y, rem);
      *reinterpret_cast<u32x4*>(payload + poff + 16 * j) = y;
    }
  }
  if (phase && c == 0) phase[3] = gpu_ticks();  // (measurement: every output store issued)
  signal_done(done, seq, ticks, t0, 0);
  return true;
}

// The launched live pass's input slices (launch_decode_small), at most g.
__host__ __device__ inline uint32_t small_slices(uint64_t in_bytes, uint32_t n, uint32_t g) {
  const uint64_t w = ((in_bytes + GEVWS_IN_PAD) / 16 + kSmallSliceChunks - 1) / kSmallSliceChunks;
  return n == 0 ? 1u : w < g ? (uint32_t)w : g;
}


// A live pass's staging granules (4 per 16-byte chunk of the wide shape's input), zeroed once.
inline bool ensure_small_stage(gevws_ctx* ctx, hipStream_t st) {
  if (ctx->d_small_stage) return true;
  const size_t sbytes = 4ull * sizeof(uint64_t) * SmallWide::kStage;
  if (hipMalloc(reinterpret_cast<void**>(&ctx->d_small_stage), sbytes) != hipSuccess ||
      hipMemsetAsync(ctx->d_small_stage, 0, sbytes, st) != hipSuccess) {
    if (ctx->d_small_stage) (void)hipFree(ctx->d_small_stage);
    ctx->d_small_stage = nullptr;
    return false;
  }
  return true;
}

}  // namespace
