// gevws_encode.hip -- the two next rows of SURVEY.md §8f on the device:
// outbound encode, ws.WriteHeader (write.go:48-84) + ws.FrameToBytes
// (frame.go:274-278) for a batch of reply frames written back to back as
// handlerProtocol's send buffer (connection.go:213); and control-frame
// dispatch, HandlerWrap.OnMessage (wrap.go:38-90) + util.HandleClose /
// HandlePing / HandlePong / CheckCloseFrameData (util.go:27-85).
#include "gevws_internal.hpp"

namespace {

// ------------------------------------------------------------------ outbound encode (§8f row 1)
// ws.WriteHeader (write.go:48-84) + ws.FrameToBytes (frame.go:274-278) for a
// batch of frames: wire[f] = WriteHeader(hdr_f) || payload_f, frames back to
// back (as handlerProtocol appends Packet output to its tmpBuffer,
// connection.go:213).  Go's byte arithmetic is kept: Rsv << 4 truncated to a
// byte, OpCode OR-ed as a whole byte, byte(Length) for any Length <= 125.

__device__ __forceinline__ uint32_t enc_header(const gevws_header& h, uint64_t& lo, uint64_t& hi) {
  const uint32_t b0 = ((h.fin ? 0x80u : 0u) | ((uint32_t)h.rsv << 4) | h.opcode) & 0xffu;
  const int64_t L = h.length;
  uint32_t b1, n;
  lo = 0;
  hi = 0;
  if (L <= 125) {
    b1 = (uint32_t)L & 0xffu;
    n = 2;
  } else if (L <= 0xFFFF) {
    b1 = 126;
    lo = ((uint64_t)((L >> 8) & 0xff) << 16) | ((uint64_t)(L & 0xff) << 24);
    n = 4;
  } else {
    b1 = 127;
    const uint64_t be = __builtin_bswap64((uint64_t)L);  // bytes 2..9, big-endian
    lo = be << 16;
    hi = be >> 48;
    n = 10;
  }
  if (h.masked) {
    b1 |= 0x80;
    uint32_t k;
    memcpy(&k, h.mask, 4);
    if (n == 2) lo |= (uint64_t)k << 16;
    else if (n == 4) lo |= (uint64_t)k << 32;
    else hi |= (uint64_t)k << 16;
    n += 4;
  }
  lo |= (uint64_t)b0 | ((uint64_t)b1 << 8);
  return n;
}

__device__ __forceinline__ uint32_t enc_hlen(const gevws_header& h) {
  const int64_t L = h.length;
  return (L <= 125 ? 2u : (L <= 0xFFFF ? 4u : 10u)) + (h.masked ? 4u : 0u);
}

// A workgroup sizes kEncSlabs consecutive slabs of kWalkBlock frames (one
// frame per lane per slab, coalesced), so the batch has one block partial per
// 4 096 frames and the single-workgroup scan of partials stays short (C4:
// 10.7 K partials instead of 171 K).
constexpr int kEncSlabs = 16;
// Tile-map entries a lane writes itself in k_enc_emit (unrolled, predicated);
// a frame with more has the rest written by its whole wave.  16 as a plain
// loop: C5 emit 79 -> 16 us but C4 138 -> 466 us
// (profiles/r03/r03_encode_emit_lane16_*), so 4.
constexpr int kEncLaneTiles = 4;
// k_encode6's run mode 2: one run counter per XCD, 64 bytes apart (zeroed by k_enc_emit)
constexpr uint32_t kEnc6Counters = 8;
// The frame count of a chained pass (decode -> dispatch -> encode with no host
// round trip): the producing step's summary gates the consumer -- its frames,
// or none when it failed (a capacity error leaves stale records behind).
__device__ __forceinline__ uint64_t gated_count(uint64_t n, const gevws_summary* __restrict__ gate) {
  if (!gate) return n;
  const gevws_summary g = *gate;
  return g.status != GEVWS_OK ? 0 : (g.frames < n ? g.frames : n);
}

// Also writes each frame's wire size (h + L) into out_off[f], which k_enc_emit
// turns into the offset in place: the emit pass reads 8 bytes per frame
// instead of the 32-byte record again (C4: 0.35 instead of 1.4 GB).
__global__ __launch_bounds__(kWalkBlock) void k_enc_size(const gevws_out_frame* __restrict__ fr, uint64_t n,
                                                         uint64_t* __restrict__ blk, uint64_t* __restrict__ out_off,
                                                         const gevws_summary* __restrict__ gate = nullptr) {
  n = gated_count(n, gate);
  const uint64_t f0 = (uint64_t)blockIdx.x * kWalkBlock * kEncSlabs + threadIdx.x;
  uint64_t one = 0, wire = 0, pl = 0;
#pragma unroll 4
  for (int j = 0; j < kEncSlabs; ++j) {
    const uint64_t f = f0 + (uint64_t)j * kWalkBlock;
    if (f < n) {
      const gevws_out_frame o = fr[f];
      const uint64_t w = enc_hlen(o.hdr) + o.payload_len;
      one += 1;
      pl += o.payload_len;
      wire += w;
      out_off[f] = w;
    }
  }
  __shared__ uint64_t s_part[3][kWalkBlock / 64];
  const uint64_t vals[3] = {one, wire, pl};
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const uint64_t sm = wave_sum(vals[k]);
    if (lane == 0) s_part[k][w] = sm;
  }
  __syncthreads();
  if (threadIdx.x < kBlkFields) {
    uint64_t sm = 0;
    if (threadIdx.x < 3)
      for (int j = 0; j < kWalkBlock / 64; ++j) sm += s_part[threadIdx.x][j];
    blk[(uint64_t)blockIdx.x * kBlkFields + threadIdx.x] = sm;
  }
}

__global__ __launch_bounds__(kWalkBlock) void k_enc_emit(uint64_t n,
                                                         const uint64_t* __restrict__ blk,
                                                         const gevws_summary* __restrict__ sum,
                                                         uint64_t* __restrict__ out_off,
                                                         uint32_t* __restrict__ tile_first,
                                                         const gevws_summary* __restrict__ gate = nullptr,
                                                         uint32_t* __restrict__ work = nullptr) {
  if (work && blockIdx.x == 0 && threadIdx.x < kEnc6Counters) work[threadIdx.x * 16] = 0;  // k_encode6's run counters
  if (sum->status != GEVWS_OK) return;
  n = gated_count(n, gate);
  const uint64_t f0 = (uint64_t)blockIdx.x * kWalkBlock * kEncSlabs + threadIdx.x;
  const uint64_t carry = blk[(uint64_t)blockIdx.x * kBlkFields + 1];
  // every slab's wire sizes (k_enc_size left them in out_off) loaded at once,
  // then ONE workgroup scan over all slabs: a wave scan per slab, and the 64
  // (slab, wave) totals scanned by one wave in frame order -- two barriers per
  // workgroup instead of two per slab
  constexpr int NW = kWalkBlock / 64;
  static_assert(kEncSlabs * NW == 64, "one lane per (slab, wave) total");
  __shared__ uint64_t s_base[kEncSlabs * NW];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t ws[kEncSlabs], inc[kEncSlabs];
#pragma unroll
  for (int j = 0; j < kEncSlabs; ++j) {
    const uint64_t f = f0 + (uint64_t)j * kWalkBlock;
    ws[j] = f < n ? out_off[f] : 0;
  }
#pragma unroll
  for (int j = 0; j < kEncSlabs; ++j) {
    inc[j] = wave_incl_scan(ws[j]);
    if (lane == 63) s_base[j * NW + wv] = inc[j];
  }
  __syncthreads();
  if (wv == 0) {
    const uint64_t x = s_base[lane];
    s_base[lane] = wave_incl_scan(x) - x;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kEncSlabs; ++j) {  // (fully unrolled: ws / inc stay in registers)
    const uint64_t f = f0 + (uint64_t)j * kWalkBlock;
    if (f - threadIdx.x >= n) break;  // workgroup-uniform: slab past the batch
    // tile map: tiles whose first byte lies in the frame's wire bytes [o, o + v).
    // A lane writes up to kEncLaneTiles entries itself; the rest of a big
    // frame's range (a 1 MiB frame has 256) is written by its whole wave, 64
    // entries a store.
    const uint64_t end = carry + s_base[j * NW + wv] + inc[j];
    const uint64_t o = end - ws[j];
    uint64_t t = (o + kTile - 1) / kTile;
    const uint64_t te = f < n ? (end + kTile - 1) / kTile : t;
    if (f < n) out_off[f] = o;
#pragma unroll
    for (int k = 0; k < kEncLaneTiles; ++k, ++t)
      if (t < te) tile_first[t] = (uint32_t)f;
    for (uint64_t rest = __ballot(t < te); rest; rest &= rest - 1) {  // (whole wave active here)
      const int src = __builtin_ctzll(rest);
      const uint64_t bt = __shfl((unsigned long long)t, src), be = __shfl((unsigned long long)te, src);
      const uint32_t bf = (uint32_t)__shfl((unsigned long long)f, src);
      for (uint64_t x = bt + (uint64_t)lane; x < be; x += 64) tile_first[x] = bf;
    }
  }
}

// One output byte at absolute position `a` of frame f (global-memory form, used
// by the fallback path).
__device__ __forceinline__ uint8_t enc_byte_global(const gevws_out_frame* __restrict__ fr,
                                                   const uint64_t* __restrict__ out_off,
                                                   const uint8_t* __restrict__ payload, uint64_t f, uint64_t a) {
  const gevws_out_frame o = fr[f];
  uint64_t lo, hi;
  const uint32_t hl = enc_header(o.hdr, lo, hi);
  const uint64_t r = a - out_off[f];
  if (r < hl) return (uint8_t)(r < 8 ? (lo >> (8 * r)) : (hi >> (8 * (r - 8))));
  return payload[o.payload_off + (r - hl)];
}

constexpr int kEncWinFrames = 1024;
// bytes [k0, k1) of a 16-byte lane (0 <= k0 < k1 <= 16)
__device__ __forceinline__ u128 byte_mask(int k0, int k1) {
  const u128 hi = (k1 >= 16) ? ~(u128)0 : (((u128)1 << (8 * k1)) - 1);
  const u128 lo = ((u128)1 << (8 * k0)) - 1;
  return hi & ~lo;
}

// The LDS table of the replies k_handle_small assembles (one workgroup).
struct EncWin {
  const int32_t* start;  // wire start relative to the window, clamped >= -64
  const int32_t* pend;   // payload end relative to the window, clamped
  const uint8_t* hlen;
  const uint64_t* delta;  // payload_off - out_off - hlen (mod 2^64)
  const uint64_t* h0;     // serialised header bytes 0-7 / 8-15
  const uint64_t* h1;
};

// Assemble the 16 output bytes at window-relative position `rel` (absolute `a`)
// from the frames overlapping it (at most 8: every frame is >= 2 wire bytes),
// starting at frame lo: header bytes from the frame's serialised header,
// payload bytes from ONE unaligned 16-byte load per frame.  The first two
// frames' loads are issued together (most boundary chunks hold the end of one
// payload and the header + start of the next: C2 -2.6 %, C5 -1.6 % against one
// at a time, profiles/r01/r01_encode_ab_asm2_*.json); further frames (frames of a
// few bytes) continue one by one.
__device__ __forceinline__ void enc_assemble_from(u128& acc, int32_t rel, uint64_t a, int kmax, uint32_t j, uint32_t F,
                                                  const EncWin& W, const uint8_t* __restrict__ payload) {
  for (; j < F && W.start[j] < rel + kmax; ++j) {
    const int32_t hs = W.start[j];
    const int32_t ps = hs + (int32_t)W.hlen[j];
    const int32_t pe = W.pend[j];
    // header bytes [max(hs, rel), min(ps, rel + kmax))
    const int32_t h0 = hs > rel ? hs : rel;
    const int32_t h1 = ps < rel + kmax ? ps : rel + kmax;
    if (h0 < h1) {
      const u128 H = (u128)W.h0[j] | ((u128)W.h1[j] << 64);
      acc |= ((H >> (8 * (h0 - hs))) << (8 * (h0 - rel))) & byte_mask(h0 - rel, h1 - rel);
    }
    // payload bytes [max(ps, rel), min(pe, rel + kmax))
    const int32_t p0 = ps > rel ? ps : rel;
    const int32_t p1 = pe < rel + kmax ? pe : rel + kmax;
    if (p0 < p1) {
      const int k0 = p0 - rel;
      const u128 v = u128_of(ld16u(payload + (a + (uint64_t)k0 + W.delta[j])));
      acc |= (v << (8 * k0)) & byte_mask(k0, p1 - rel);
    }
  }
}

// enc_assemble in two halves, so a caller can have several chunks' payload
// loads in flight before it combines any (k_handle_small: over PCIe each
// round of loads is a round trip): enc_prep computes the first two frames'
// ranges and issues their loads, enc_finish combines them (and walks the rare
// further frames of a few bytes one by one).
struct EncPrep {
  int kmax;
  int32_t hs[2], h0[2], h1[2], p0[2], p1[2];
  u32x4 pv[2];
  u64x2 hv[2];
};

__device__ __forceinline__ void enc_prep(EncPrep& P, int32_t rel, uint64_t a, uint64_t total, uint32_t lo, uint32_t F,
                                         const EncWin& W, const uint8_t* __restrict__ payload) {
  P.kmax = (a + 16 <= total) ? 16 : (int)(total - a);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const uint32_t j = lo + k;
    const bool in = j < F && W.start[j < F ? j : lo] < rel + P.kmax;
    const uint32_t jj = in ? j : lo;
    P.hs[k] = W.start[jj];
    const int32_t ps = P.hs[k] + (int32_t)W.hlen[jj];
    const int32_t pe = W.pend[jj];
    P.h0[k] = P.hs[k] > rel ? P.hs[k] : rel;
    P.h1[k] = in ? (ps < rel + P.kmax ? ps : rel + P.kmax) : P.h0[k];
    P.p0[k] = ps > rel ? ps : rel;
    P.p1[k] = in ? (pe < rel + P.kmax ? pe : rel + P.kmax) : P.p0[k];
    P.pv[k] = u32x4{0, 0, 0, 0};
    P.hv[k] = u64x2{0, 0};
    if (P.p0[k] < P.p1[k]) P.pv[k] = ld16u(payload + (a + (uint64_t)(P.p0[k] - rel) + W.delta[jj]));
    if (P.h0[k] < P.h1[k]) P.hv[k] = u64x2{W.h0[jj], W.h1[jj]};
  }
}

__device__ __forceinline__ u32x4 enc_finish(const EncPrep& P, int32_t rel, uint64_t a, uint32_t lo, uint32_t F,
                                            const EncWin& W, const uint8_t* __restrict__ payload) {
  u128 acc = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    if (P.h0[k] < P.h1[k]) {
      const u128 H = (u128)P.hv[k][0] | ((u128)P.hv[k][1] << 64);
      acc |= ((H >> (8 * (P.h0[k] - P.hs[k]))) << (8 * (P.h0[k] - rel))) & byte_mask(P.h0[k] - rel, P.h1[k] - rel);
    }
    if (P.p0[k] < P.p1[k]) {
      const int k0 = P.p0[k] - rel;
      acc |= (u128_of(P.pv[k]) << (8 * k0)) & byte_mask(k0, P.p1[k] - rel);
    }
  }
  if (lo + 2 < F && W.start[lo + 2] < rel + P.kmax)  // more frames in these 16 bytes
    enc_assemble_from(acc, rel, a, P.kmax, lo + 2, F, W, payload);
  return u32x4_of(acc);
}

// The encode's byte stream, one wave per step (k_encode6; k_enc_size /
// k_enc_emit placed every frame's wire bytes and the output-tile -> frame
// map).  Every wave walks its own runs of tiles, ST = U / 4 tiles a step, with
// no workgroup barrier.
//  * A step inside one payload is streamed (a misaligned source as the
//    unmask's streaming path: wave-contiguous 1 KiB spans, aligned
//    non-temporal loads, DPP rotate + v_alignbyte; an aligned one with plain
//    loads), aligned non-temporal stores.
//  * Otherwise the step's frames (at most 16 U, one or two per lane) go into
//    the wave's LDS table, each frame that is the last to start in its chunk
//    marks that chunk in a one-byte-per-chunk map (its end, the next frame's
//    start, lies in a later chunk: one writer per slot), and one per-wave
//    prefix max turns the marks into every chunk's frame -- no search.  A
//    chunk inside one payload is loaded (unaligned) and stored.  A 64-byte
//    group holding any other chunk is queued whole in the wave's LDS (slots
//    from a ballot, no atomics) and assembled after the interior loads are in
//    flight, one chunk per lane: the frame holding the byte before the chunk
//    and the next one, both payload loads issued together.  Queuing the whole
//    group makes one store write its 64 bytes: otherwise every frame boundary
//    left its line to HBM as two partial writes (C4: 46 M 32-byte write
//    requests per launch; the encode 10.70 -> 9.11 ms, profiles/r02/r02_encode_ab_g64_*.json;
//    queuing only the boundary chunks with plain stores for the shared lines
//    measured slower again, profiles/r04/r04_encode6_dev.jsonl).
// It replaced round 3's workgroup-window kernels k_encode (4-tile windows, a
// binary search per chunk) and k_encode5 (8-tile windows with a chunk map):
// C4 -9 %, C2 -7 %, C1-shaped -19 %, C5 -7 %, C3 equal (profiles/r04/r04_encode6_ab.jsonl).
// LDS written by some lanes of a wave and read by others: the hardware keeps a
// wave's LDS operations in order, the fence keeps the compiler from moving them.
__device__ __forceinline__ void wave_lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// How waves share the tiles (`mode`, -1 = chosen on the device):
//  0  one contiguous run per wave -- batches of big frames (mean >= kBigFrameBytes,
//     the streaming path: long runs keep DRAM pages open);
//  1  each wave takes every nwaves-th run of K tiles (K <= kEnc6Run, at least
//     8 runs a wave): a run's cost follows the local frame density, and runs
//     spread over the whole batch even it out -- small batches (fewer than
//     kEnc6CounterMinTiles tiles a wave);
//  2  runs of kEnc6CounterRun tiles from a work counter, one counter per XCD
//     over its eighth of the tiles (one lane's vector atomic per run; k_enc_emit
//     zeroes them) -- every other batch.  One counter for the whole grid
//     saturated at runs of 4 tiles (C4 14.3 ms); eight keep C4 at 8.2 ms
//     against 9.0 with runs of 64 (profiles/r04/r04_encode6_counter_ab.jsonl).
constexpr uint64_t kEnc6Run = 64;
constexpr uint64_t kEnc6CounterRun = 4;
constexpr uint64_t kEnc6CounterMinTiles = 16;  // per wave, for mode 2
template <int U>
__global__ __launch_bounds__(kUnmaskBlock) __attribute__((amdgpu_waves_per_eu(U == 4 ? 8 : 4))) void k_encode6(
    const gevws_out_frame* __restrict__ fr, const uint8_t* __restrict__ payload, const uint64_t* __restrict__ out_off,
    const uint32_t* __restrict__ tile_first, const gevws_summary* __restrict__ sum, uint8_t* __restrict__ out,
    uint32_t big_grid, uint32_t* __restrict__ work, int mode) {
  static_assert(U == 4 || U == 8, "one or two tiles a step");
  constexpr int NW = kUnmaskBlock / 64, ST = U / 4, TF = 16 * U, MW = U / 4;
  // frame i of the step: wire start (step-relative, >= -64) * 16 | header
  // length, payload end (step-relative, clamped), payload_off - wire start -
  // header length (lo / hi)
  __shared__ u32x4 s_ta[NW][TF];
  __shared__ u64x2 s_tb[NW][TF];            // header bytes 0-7, bytes 8-13
  __shared__ uint32_t s_map[NW][64 * MW];  // chunk -> frame, one byte per chunk (lane l: chunks U l ..)
  __shared__ uint16_t s_q[NW][64 * U];     // queued chunks (0xffff: a group's slot past the run)
  if (sum->status != GEVWS_OK) return;
  const uint64_t total = sum->payload_bytes;  // wire bytes
  const uint64_t nframes = sum->frames;
  const uint64_t ntiles = (total + kTile - 1) / kTile;
  if (ntiles == 0) return;
  const uint32_t groups = active_groups(total, nframes, big_grid);
  if (blockIdx.x >= groups) return;
  const uint32_t w = uniform32(threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)groups * NW;
  const uint64_t per = (ntiles + nwaves - 1) / nwaves;
  const uint64_t gw = (uint64_t)blockIdx.x * NW + w;
  if (mode < 0)
    mode = total / nframes >= kBigFrameBytes ? 0 : (ntiles >= kEnc6CounterMinTiles * nwaves ? 2 : 1);
  uint64_t t = mode ? 0 : gw * per;
  uint64_t tend = mode ? 0 : (t + per < ntiles ? t + per : ntiles);
  // modes 1 / 2: run length K (a multiple of the step) and the wave's next run
  uint64_t K = ntiles / (nwaves * 8);
  K = K > kEnc6Run ? kEnc6Run : K;
  K = K < (uint64_t)ST ? (uint64_t)ST : K - K % ST;
  if (mode == 2 && groups < kEnc6Counters) mode = 1;  // (every counter needs its workgroups)
  if (mode == 2) K = kEnc6CounterRun;
  // mode 2: the workgroups of each XCD (blockIdx.x mod 8, the dispatch's
  // round robin) share one counter over their eighth of the tiles
  const uint32_t xc = blockIdx.x % kEnc6Counters;
  const uint64_t segn = ((ntiles + kEnc6Counters - 1) / kEnc6Counters + K - 1) / K * K;
  const uint64_t seg0 = xc * segn < ntiles ? xc * segn : ntiles;
  const uint64_t seg1 = seg0 + segn < ntiles ? seg0 + segn : ntiles;
  uint64_t run = gw;
  uint8_t* const mb = reinterpret_cast<uint8_t*>(s_map[w]);
  uint64_t c_f = ~0ull, c_ps = 0, c_pe = 0, c_delta = 0;  // cached frame: payload [c_ps, c_pe) in wire coordinates
  for (;;) {
    if (t >= tend) {
      if (mode == 0) break;
      if (mode == 2) {
        uint32_t g = 0;
        if ((fresh_tid() & 63) == 0) g = atomicAdd(work + xc * 16, 1u);
        t = seg0 + (uint64_t)uniform32((uint32_t)__shfl((int)g, 0, 64)) * K;
        if (t >= seg1) break;
        tend = t + K < seg1 ? t + K : seg1;
        continue;
      }
      t = run * K;
      if (t >= ntiles) break;
      tend = t + K < ntiles ? t + K : ntiles;
      run += nwaves;
      continue;
    }
    const uint64_t B = t * kTile;
    const uint64_t nt = tend - t < (uint64_t)ST ? tend - t : (uint64_t)ST;  // tiles this step
    const uint64_t send = B + nt * kTile;
    const uint64_t lim = send < total ? send : total;  // the step writes [B, lim)
    uint64_t fa = c_f, fb = c_f;
    if (!(B >= c_ps && send <= c_pe)) {
      // the step's first and last frames; a step with one frame may lie in its payload
      fa = uniform32(tile_first[t]);
      fb = t + nt < ntiles ? (uint64_t)uniform32(tile_first[t + nt]) : nframes - 1;
      if (fa == fb && fa != c_f) {
        c_f = fa;
        const uint64_t* rec = reinterpret_cast<const uint64_t*>(fr + fa);
        const uint64_t w0 = uniform64(rec[0]), len = uniform64(rec[1]);
        const uint64_t po = uniform64(rec[2]), pl = uniform64(rec[3]);
        gevws_header h;
        memcpy(&h, &w0, 8);
        h.length = (int64_t)len;
        c_ps = uniform64(out_off[fa]) + enc_hlen(h);
        c_pe = c_ps + pl;
        c_delta = po - c_ps;
      }
    }
    if (B >= c_ps && send <= c_pe) {  // inside one payload: stream the step
      const uint8_t* s0 = payload + (B + c_delta);
      const uint32_t mis = (uint32_t)(reinterpret_cast<uint64_t>(s0) & 15);  // wave-uniform
      const uint32_t lane = fresh_tid() & 63;
      const int nu = (int)nt * 4;
      u32x4 v[U];  // (zeroed: else carried round the loop, 121 VGPRs instead of 89)
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = u32x4{0, 0, 0, 0};
      if (mis != 0) {
        const uint8_t* a = s0 + lane * 16 - mis;
        uint8_t* d = out + B + lane * 16;
        const bool last = lane == 63;
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (u < nu) v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a + u * 1024));
        u32x4 e = u32x4{0, 0, 0, 0};
        if (last) e = *reinterpret_cast<const u32x4*>(a + (nu - 1) * 1024 + 16);
        u32x4 r = rot_next_lane(v[0]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (u < nu) {
            const u32x4 rn = u + 1 < nu ? rot_next_lane(v[u + 1 < U ? u + 1 : u]) : e;
            st16_nt(d + u * 1024, funnel16(v[u], last ? rn : r, mis));
            r = rn;
          }
        }
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (u < nu) v[u] = ld16u(s0 + u * 1024 + lane * 16);
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (u < nu) st16_nt(out + B + u * 1024 + lane * 16, v[u]);
      }
      t += nt;
      continue;
    }
    const uint64_t n = fb - fa + 1;
    if (n > (uint64_t)TF) {
      // frames of a few bytes: per-lane global lookup and byte assembly (as k_encode)
      const uint32_t lane = fresh_tid() & 63;
#pragma unroll 1
      for (int u = 0; u < U; ++u) {
        const uint64_t p = B + (uint64_t)u * 1024 + lane * 16;
        if (p < lim) {
          uint64_t lo = fa, hi = fb;
          while (lo < hi) {
            const uint64_t mid = (lo + hi + 1) >> 1;
            if (out_off[mid] <= p) lo = mid; else hi = mid - 1;
          }
          uint32_t wd[4] = {0, 0, 0, 0};
          uint64_t j = lo;
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            while (j + 1 < nframes && out_off[j + 1] <= p + k) ++j;
            const uint32_t byte = (p + k < total) ? enc_byte_global(fr, out_off, payload, j, p + k) : 0u;
            wd[k >> 2] |= byte << (8 * (k & 3));
          }
          *reinterpret_cast<u32x4*>(out + p) = u32x4{wd[0], wd[1], wd[2], wd[3]};
        }
      }
      t += nt;
      continue;
    }
    // the step's frame table and chunk marks
    {
      const uint32_t lane = fresh_tid() & 63;
#pragma unroll
      for (int k = 0; k < MW; ++k) s_map[w][lane * MW + k] = 0;
      wave_lds_order();
      // frame i's wire offset from the step's first one: out_off[fa] (one
      // scalar load) + fa's wire size + the sizes of frames 1 .. i-1 (a wave
      // scan; each of frames 1 .. n-2 starts and ends inside the step's
      // U KiB window, so their sum is below U KiB and fits 32 bits; frame 0
      // and frame n - 1 may be any size and are added in 64 bits) -- no
      // per-frame out_off reads (C4: 0.35 GB a launch)
      static_assert((uint64_t)U * 1024 < (1ull << 32), "the interior frames' 32-bit wire-size scan");
      const uint64_t o_fa = uniform64(out_off[fa]);
      uint64_t w_fa = 0;
      uint32_t carry = 0;
#pragma unroll
      for (int k = 0; k < TF / 64; ++k) {
        if ((uint64_t)(64 * k) >= n) break;  // (wave-uniform)
        const uint32_t i = lane + 64 * k;
        const bool have = i < n;
        const uint64_t f = fa + (have ? i : 0);
        const u64x2* r = reinterpret_cast<const u64x2*>(fr + f);
        const u64x2 h2 = r[0], p2 = r[1];
        gevws_header h;
        memcpy(&h, &h2, 16);
        uint64_t hlo, hhi;
        const uint32_t hl = enc_header(h, hlo, hhi);
        const uint64_t wsz = hl + p2[1];
        if (k == 0)
          w_fa = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)wsz, 0) |
                 ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(wsz >> 32), 0) << 32);
        const uint32_t w32 = (have && i >= 1 && (uint64_t)i + 1 < n) ? (uint32_t)wsz : 0u;
        const uint32_t inc = wave_incl_scan32(w32);
        const uint32_t ex = carry + inc - w32;
        carry += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        if (have) {
          const uint64_t oo = i == 0 ? o_fa : o_fa + w_fa + ex;
          const int64_t st = (int64_t)(oo - B);
          const int64_t end = st + hl + (int64_t)p2[1];  // the next frame's start
          const int32_t stc = st < -64 ? -64 : (int32_t)st;
          const uint64_t d = p2[0] - oo - hl;
          s_ta[w][i] = u32x4{(uint32_t)(stc * 16) | hl, end > 0x7fffffffll ? 0x7fffffffu : (uint32_t)end,
                             (uint32_t)d, (uint32_t)(d >> 32)};
          s_tb[w][i] = u64x2{hlo, hhi};
          // the last frame to start in its chunk marks it (the batch's last frame always)
          if (st >= 0 && st < (int64_t)(U * 1024)) {
            const int64_t sc = st >> 4;
            if (end >= (sc + 1) * 16 || f == nframes - 1) mb[sc] = (uint8_t)i;
          }
        }
      }
      wave_lds_order();
      // prefix max over the chunks (lane l holds chunks U l .. U l + U - 1)
      uint32_t b[U];
#pragma unroll
      for (int k = 0; k < MW; ++k) {
        const uint32_t m = s_map[w][lane * MW + k];
#pragma unroll
        for (int j = 0; j < 4; ++j) b[4 * k + j] = (m >> (8 * j)) & 0xffu;
      }
#pragma unroll
      for (int j = 1; j < U; ++j) b[j] = b[j] > b[j - 1] ? b[j] : b[j - 1];
      uint32_t inc = b[U - 1];
#pragma unroll
      for (int dd = 1; dd < 64; dd <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)inc, dd, 64);
        if (lane >= (uint32_t)dd) inc = inc > y ? inc : y;
      }
      uint32_t exc = (uint32_t)__shfl_up((int)inc, 1, 64);
      if (lane == 0) exc = 0;
#pragma unroll
      for (int k = 0; k < MW; ++k) {
        uint32_t m = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) m |= (b[4 * k + j] > exc ? b[4 * k + j] : exc) << (8 * j);
        s_map[w][lane * MW + k] = m;
      }
      wave_lds_order();
    }
    // classify the lane's chunks (chunk u * 64 + lane, byte u * 1 KiB + 16 lane),
    // queue the 64-byte groups holding a chunk that is not inside one payload
    // (whole, in order), and load the rest
    uint32_t interior = 0, nb = 0;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t lane = fresh_tid() & 63;
      const uint32_t c = (uint32_t)u * 64 + lane;
      const int32_t x = (int32_t)(c * 16);
      const bool valid = B + (uint64_t)x < lim;
      const u32x4 ta = s_ta[w][mb[c]];
      const int32_t ps = ((int32_t)ta[0] >> 4) + (int32_t)(ta[0] & 15u);
      const bool in = valid && ps <= x && x + 16 <= (int32_t)ta[1];
      const uint64_t bal = __ballot(valid && !in);
      const bool defer = ((bal >> (lane & ~3u)) & 0xFull) != 0;  // (group-uniform)
      const uint64_t dbal = __ballot(defer);
      if (defer) {
        const uint32_t slot =
            nb + __builtin_amdgcn_mbcnt_hi((uint32_t)(dbal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)dbal, 0u));
        s_q[w][slot] = valid ? (uint16_t)c : (uint16_t)0xffffu;
      }
      nb += (uint32_t)__builtin_popcountll(dbal);
      const bool ld = in && !defer;
      interior |= (ld ? 1u : 0u) << u;
      // every lane loads; a chunk not stored here from payload[0]
      v[u] = ld16u(payload + (ld ? B + (uint64_t)x + ((uint64_t)ta[2] | ((uint64_t)ta[3] << 32)) : 0ull));
    }
    wave_lds_order();
    // a queued chunk: header and payload bytes of the frames overlapping it.
    // Payload bytes come from the 16 bytes at the chunk's position in the
    // frame's payload coordinates (no shift), unless those would start before
    // the buffer.
    auto paddr = [&](const u32x4& ta, int32_t x, int32_t kend) -> uint64_t {
      const int32_t hs = (int32_t)ta[0] >> 4, ps = hs + (int32_t)(ta[0] & 15u), pe = (int32_t)ta[1];
      const int32_t p0 = ps > x ? ps : x, p1 = pe < kend ? pe : kend;
      if (hs >= kend || p0 >= p1) return 0;  // (payload[0], always readable, unused)
      const uint64_t d = (uint64_t)ta[2] | ((uint64_t)ta[3] << 32);
      const uint64_t off = B + (uint64_t)x + d;
      return (int64_t)off >= 0 ? off : B + (uint64_t)p0 + d;
    };
    auto piece = [&](u128& acc, uint32_t j, const u32x4& ta, const u32x4& pv4, int32_t x, int32_t kend) {
      const int32_t hs = (int32_t)ta[0] >> 4;
      if (hs >= kend) return;
      const int32_t ps = hs + (int32_t)(ta[0] & 15u), pe = (int32_t)ta[1];
      const int32_t h0 = hs > x ? hs : x, h1 = ps < kend ? ps : kend;
      if (h0 < h1) {
        const u64x2 tb = s_tb[w][j];
        const u128 H = (u128)tb[0] | ((u128)tb[1] << 64);
        acc |= ((H >> (8 * (h0 - hs))) << (8 * (h0 - x))) & byte_mask(h0 - x, h1 - x);
      }
      const int32_t p0 = ps > x ? ps : x, p1 = pe < kend ? pe : kend;
      if (p0 < p1) {
        const uint64_t d = (uint64_t)ta[2] | ((uint64_t)ta[3] << 32);
        const bool at_x = (int64_t)(B + (uint64_t)x + d) >= 0;
        const u128 pv = u128_of(pv4);
        acc |= (at_x ? pv : (pv << (8 * (p0 - x)))) & byte_mask(p0 - x, p1 - x);
      }
    };
    auto assemble = [&](uint32_t c) -> u32x4 {
      const int32_t x = (int32_t)(c * 16);
      const uint64_t a = B + (uint64_t)x;
      const int32_t kend = x + ((a + 16 <= total) ? 16 : (int32_t)(total - a));
      // the frame holding the byte before the chunk (the step's first frame
      // for chunk 0) and the next one: both payload loads issued together
      const uint32_t j0 = c ? (uint32_t)mb[c - 1] : 0u;
      const uint32_t j1 = j0 + 1 < (uint32_t)n ? j0 + 1 : j0;
      const u32x4 t0 = s_ta[w][j0], t1 = s_ta[w][j1];
      const uint64_t a0 = paddr(t0, x, kend);
      const uint64_t a1 = j1 != j0 ? paddr(t1, x, kend) : 0ull;
      const u32x4 v0 = ld16u(payload + a0), v1 = ld16u(payload + a1);
      u128 acc = 0;
      piece(acc, j0, t0, v0, x, kend);
      if (j1 != j0) piece(acc, j1, t1, v1, x, kend);
      for (uint32_t j = j0 + 2; j < (uint32_t)n; ++j) {  // frames of a few bytes
        const u32x4 ta = s_ta[w][j];
        if (((int32_t)ta[0] >> 4) >= kend) break;
        piece(acc, j, ta, ld16u(payload + paddr(ta, x, kend)), x, kend);
      }
      return u32x4_of(acc);
    };
    const uint32_t i0 = fresh_tid() & 63;
    u32x4 x0 = u32x4{0, 0, 0, 0};
    uint32_t q0 = 0xffffu;
    if (i0 < nb) {
      q0 = s_q[w][i0];
      if (q0 != 0xffffu) x0 = assemble(q0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (interior & (1u << u)) st16_nt(out + B + (uint64_t)u * 1024 + (fresh_tid() & 63) * 16, v[u]);
    if (q0 != 0xffffu) st16_nt(out + B + (uint64_t)q0 * 16, x0);
    for (uint32_t i = i0 + 64; i < nb; i += 64) {
      const uint32_t q = s_q[w][i];
      if (q != 0xffffu) st16_nt(out + B + (uint64_t)q * 16, assemble(q));
    }
    wave_lds_order();  // this step's readers are done with the table, the map and the queue
    t += nt;
  }
}

// ------------------------------------------------------------------ control-frame dispatch (§8f row 2)
// HandlerWrap.OnMessage (plugins/websocket/wrap.go:38-90) for decoded frames:
// close -> util.HandleClose (util.go:27-46) + ShutdownWrite; ping -> pong with
// the same payload (util.go:49-51); pong -> ping (util.go:54-56, kept as the
// reference has it); other control opcodes -> nothing; data frames -> the echo
// policy standing in for the user's WSHandler (empty replies send nothing,
// wrap.go:72).  Replies are gevws_out_frame records for gevws_encode_batch.

constexpr uint32_t kAuxSlot = 128;  // one close body (<= 125 bytes) per slot

__device__ __constant__ char kErrNotInUse[] = "status code is not in use";
__device__ __constant__ char kErrAppLevel[] = "status code is only application level";
__device__ __constant__ char kErrNoMeaning[] = "status code has no meaning yet";
__device__ __constant__ char kErrUnknown[] = "status code is not defined in spec";
__device__ __constant__ char kErrUtf8[] = "invalid utf8 sequence in close reason";

// unicode/utf8.ValidString: strict UTF-8.
__device__ bool utf8_valid(const uint8_t* p, uint64_t n) {
  uint64_t i = 0;
  while (i < n) {
    const uint32_t c = p[i];
    if (c < 0x80) { ++i; continue; }
    uint32_t need, lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) need = 1;
    else if (c == 0xE0) { need = 2; lo = 0xA0; }
    else if ((c >= 0xE1 && c <= 0xEC) || c == 0xEE || c == 0xEF) need = 2;
    else if (c == 0xED) { need = 2; hi = 0x9F; }
    else if (c == 0xF0) { need = 3; lo = 0x90; }
    else if (c >= 0xF1 && c <= 0xF3) need = 3;
    else if (c == 0xF4) { need = 3; hi = 0x8F; }
    else return false;
    if (i + need >= n) return false;  // truncated sequence
    const uint32_t c1 = p[i + 1];
    if (c1 < lo || c1 > hi) return false;
    for (uint32_t k = 2; k <= need; ++k)
      if ((p[i + k] & 0xC0) != 0x80) return false;
    i += need + 1;
  }
  return true;
}

// 0: no reply, 1: reply with the frame's own payload, 2: close reply (aux body), 3: bare close header
__device__ __forceinline__ int disp_kind(const gevws_header& h, int policy, uint32_t& op_out) {
  const uint32_t op = h.opcode;
  if (op & 8) {
    if (op == 0x8) return h.length == 0 ? 3 : 2;
    if (op == 0x9) { op_out = 0xA; return 1; }
    if (op == 0xA) { op_out = 0x9; return 1; }
    return 0;
  }
  if (policy == GEVWS_HANDLER_NONE || h.length <= 0) return 0;
  op_out = policy == GEVWS_HANDLER_ECHO_BINARY ? 0x2u : 0x1u;
  return 1;
}

__global__ __launch_bounds__(kWalkBlock) void k_disp_count(const gevws_frame* __restrict__ fr, uint64_t n, int policy,
                                                           uint64_t* __restrict__ blk,
                                                           const gevws_summary* __restrict__ gate = nullptr) {
  n = gated_count(n, gate);
  const uint64_t f0 = (uint64_t)blockIdx.x * kWalkBlock * kEncSlabs + threadIdx.x;  // as k_enc_size
  uint64_t rep = 0, aux = 0, shut = 0;
#pragma unroll 4
  for (int j = 0; j < kEncSlabs; ++j) {
    const uint64_t f = f0 + (uint64_t)j * kWalkBlock;
    if (f < n) {
      uint32_t op;
      const int k = disp_kind(fr[f].hdr, policy, op);
      rep += k != 0;
      aux += k == 2;
      shut += k >= 2;
    }
  }
  __shared__ uint64_t s_part[3][kWalkBlock / 64];
  const uint64_t vals[3] = {rep, aux, shut};
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const uint64_t sm = wave_sum(vals[k]);
    if (lane == 0) s_part[k][w] = sm;
  }
  __syncthreads();
  if (threadIdx.x < kBlkFields) {
    uint64_t sm = 0;
    const int fld = threadIdx.x == 3 ? 2 : (threadIdx.x == 2 ? -1 : threadIdx.x);
    if (fld >= 0)
      for (int j = 0; j < kWalkBlock / 64; ++j) sm += s_part[fld][j];
    blk[(uint64_t)blockIdx.x * kBlkFields + threadIdx.x] = sm;  // [replies, aux slots, 0, shutdowns]
  }
}

__device__ void put_close_body(uint8_t* dst, uint32_t code, const uint8_t* reason, uint64_t rlen, uint32_t& n) {
  // ws.NewCloseFrameBody (frame.go:251-259): BE16 code + reason cropped to 123 bytes
  const uint64_t crop = rlen < 123 ? rlen : 123;
  dst[0] = (uint8_t)(code >> 8);
  dst[1] = (uint8_t)code;
  for (uint64_t i = 0; i < crop; ++i) dst[2 + i] = reason[i];
  n = (uint32_t)(2 + crop);
}

__device__ void put_close_error(uint8_t* dst, const char* msg, uint32_t& n) {
  uint64_t len = 0;
  while (msg[len]) ++len;
  put_close_body(dst, 1002, reinterpret_cast<const uint8_t*>(msg), len, n);  // StatusProtocolError
}

// One reply record (and for a close its aux-slot body) for decoded frame f.
__device__ __forceinline__ void disp_reply(const gevws_frame& in, int kind, uint32_t op, uint64_t f, uint64_t r,
                                        uint64_t slot, const uint8_t* __restrict__ payload, uint64_t aux_off,
                                        gevws_out_frame* __restrict__ rep, int64_t* __restrict__ reply_of,
                                        uint8_t* __restrict__ aux_base) {
  reply_of[f] = (int64_t)r;
  gevws_out_frame o;
  memset(&o, 0, sizeof(o));
  o.hdr.fin = 1;
  if (kind == 1) {
    o.hdr.opcode = (uint8_t)op;
    o.hdr.length = in.hdr.length;
    o.payload_off = in.payload_off;
    o.payload_len = (uint64_t)in.hdr.length;
  } else if (kind == 3) {
    o.hdr.opcode = 0x8;  // WriteHeader(&Header{Fin: true, OpCode: OpClose}), util.go:28-33
  } else {
    uint8_t* body = aux_base + slot * kAuxSlot;
    const uint8_t* p = payload + in.payload_off;
    const uint64_t L = (uint64_t)in.hdr.length;
    uint32_t code = 0;
    const uint8_t* reason = p;
    uint64_t rlen = 0;
    if (L >= 2) {  // ParseCloseFrameData, read.go:89-102
      code = ((uint32_t)p[0] << 8) | p[1];
      reason = p + 2;
      rlen = L - 2;
    }
    uint32_t nb;
    const bool defined = code == 1000 || code == 1001 || code == 1002 || code == 1003 || code == 1007 ||
                         code == 1008 || code == 1009 || code == 1010 || code == 1011 || code == 1005 ||
                         code == 1006 || code == 1015;
    if (code <= 999) put_close_error(body, kErrNotInUse, nb);
    else if (code == 1005 || code == 1006 || code == 1015) put_close_error(body, kErrAppLevel, nb);
    else if (code == 1004) put_close_error(body, kErrNoMeaning, nb);
    else if (code >= 1000 && code <= 2999 && !defined) put_close_error(body, kErrUnknown, nb);
    else if (!utf8_valid(reason, rlen)) put_close_error(body, kErrUtf8, nb);
    else put_close_body(body, code, reason, rlen, nb);
    o.hdr.opcode = 0x8;
    o.hdr.length = nb;
    o.payload_off = aux_off + slot * kAuxSlot;
    o.payload_len = nb;
  }
  rep[r] = o;
}

__global__ __launch_bounds__(kWalkBlock) void k_disp_emit(const gevws_frame* __restrict__ fr, uint64_t n, int policy,
                                                          const uint8_t* __restrict__ payload, uint64_t aux_off,
                                                          const uint64_t* __restrict__ blk,
                                                          const gevws_summary* __restrict__ sum,
                                                          gevws_out_frame* __restrict__ rep,
                                                          int64_t* __restrict__ reply_of,
                                                          uint8_t* __restrict__ aux_base,
                                                          const gevws_summary* __restrict__ gate = nullptr) {
  if (sum->status != GEVWS_OK) return;
  n = gated_count(n, gate);
  const uint64_t f0 = (uint64_t)blockIdx.x * kWalkBlock * kEncSlabs + threadIdx.x;  // as k_enc_emit
  uint64_t c_rep = blk[(uint64_t)blockIdx.x * kBlkFields + 0], c_aux = blk[(uint64_t)blockIdx.x * kBlkFields + 1];
  for (int j = 0; j < kEncSlabs; ++j) {
    const uint64_t f = f0 + (uint64_t)j * kWalkBlock;
    if (f - threadIdx.x >= n) break;  // workgroup-uniform: slab past the batch
    uint32_t op = 0;
    int kind = 0;
    gevws_frame in;
    if (f < n) {
      in = fr[f];
      kind = disp_kind(in.hdr, policy, op);
    }
    uint64_t v[2] = {(uint64_t)(kind != 0), (uint64_t)(kind == 2)};
    uint64_t ex[2], tot[2];
    block_excl_scan<kWalkBlock, 2>(v, ex, tot);
    if (f < n) {
      if (kind == 0)
        reply_of[f] = -1;
      else
        disp_reply(in, kind, op, f, c_rep + ex[0], c_aux + ex[1], payload, aux_off, rep, reply_of, aux_base);
    }
    c_rep += tot[0];
    c_aux += tot[1];
  }
}


// A live pass's handler step in ONE launch (gevws_handle_decoded_async on a
// pass of at most kHandleSmallFrames decoded frames): k_disp_count /
// k_disp_emit's dispatch and the encode's size / scan / FrameToBytes for the
// replies, in one workgroup -- each step's counts by block scans, the replies'
// wire image assembled 16 bytes per lane from an LDS table of every reply
// (enc_prep / enc_finish: serialised headers from the table, payloads by
// unaligned loads).  Outputs and summaries are exactly the two-step chain's (seven
// launches, ~5 us of GPU time each whatever their size).
constexpr uint64_t kHandleSmallFrames = kEncWinFrames;
__global__ __launch_bounds__(kWalkBlock) void k_handle_small(const gevws_frame* __restrict__ fr, uint64_t max_frames,
                                                            const gevws_summary* __restrict__ dec, int policy,
                                                            uint8_t* __restrict__ payload, uint64_t aux_off,
                                                            uint64_t aux_cap, gevws_out_frame* __restrict__ rep,
                                                            int64_t* __restrict__ reply_of,
                                                            gevws_summary* __restrict__ dsum, uint8_t* __restrict__ out,
                                                            uint64_t out_cap, uint64_t* __restrict__ out_off,
                                                            gevws_summary* __restrict__ esum,
                                                            uint32_t* __restrict__ done = nullptr,
                                                            uint32_t seq = 0, uint64_t* __restrict__ ticks = nullptr) {
  constexpr int WF = (int)kHandleSmallFrames;
  const uint64_t t0 = done ? gpu_ticks() : 0;
  __shared__ int32_t s_start[WF];
  __shared__ int32_t s_pend[WF];
  __shared__ uint8_t s_hlen[WF];
  __shared__ uint64_t s_delta[WF];
  __shared__ uint64_t s_h0[WF], s_h1[WF];
  __shared__ uint32_t s_status;
  const uint32_t tid = threadIdx.x;
  // the decode's summary and the first kWalkBlock records in flight together
  // (mapped host memory in a live pass: one round trip instead of three)
  gevws_frame in0;
  if (tid < max_frames) in0 = fr[tid];  // (inside the records' capacity; used below only for f < n)
  const uint64_t n = gated_count(max_frames, dec);
  // 1. dispatch counts (k_disp_count + k_scan_blocks)
  uint64_t rep_n = 0, aux_n = 0, shut_n = 0;
  for (uint64_t f0 = 0; f0 < n; f0 += kWalkBlock) {  // workgroup-uniform
    const uint64_t f = f0 + tid;
    uint32_t op = 0;
    const int k = f < n ? disp_kind((f0 == 0 ? in0 : fr[f]).hdr, policy, op) : 0;
    const uint64_t v[3] = {(uint64_t)(k != 0), (uint64_t)(k == 2), (uint64_t)(k >= 2)};
    uint64_t ex[3], tot[3];
    block_excl_scan<kWalkBlock, 3>(v, ex, tot);
    rep_n += tot[0];
    aux_n += tot[1];
    shut_n += tot[2];
  }
  const bool disp_ok = rep_n <= n && aux_n <= aux_cap / kAuxSlot;
  if (tid == 0) {
    gevws_summary sm;
    memset(&sm, 0, sizeof(sm));
    sm.frames = rep_n;
    sm.payload_bytes = aux_n;
    sm.errors = shut_n;
    sm.status = disp_ok ? GEVWS_OK : GEVWS_ERR_CAPACITY;
    *dsum = sm;
  }
  // 2. replies (k_disp_emit)
  if (disp_ok) {
    uint64_t c_rep = 0, c_aux = 0;
    for (uint64_t f0 = 0; f0 < n; f0 += kWalkBlock) {
      const uint64_t f = f0 + tid;
      uint32_t op = 0;
      int kind = 0;
      gevws_frame in;
      if (f < n) {
        in = f0 == 0 ? in0 : fr[f];
        kind = disp_kind(in.hdr, policy, op);
      }
      const uint64_t v[2] = {(uint64_t)(kind != 0), (uint64_t)(kind == 2)};
      uint64_t ex[2], tot[2];
      block_excl_scan<kWalkBlock, 2>(v, ex, tot);
      if (f < n) {
        if (kind == 0) reply_of[f] = -1;
        else disp_reply(in, kind, op, f, c_rep + ex[0], c_aux + ex[1], payload, aux_off, rep, reply_of,
                        payload + aux_off);
      }
      c_rep += tot[0];
      c_aux += tot[1];
    }
  }
  __threadfence_block();  // the reply records before other lanes read them
  __syncthreads();
  // 3. encode sizes, wire offsets and the summary (k_enc_size + scan + k_enc_emit)
  const uint64_t nr = disp_ok ? (rep_n < n ? rep_n : n) : 0;
  uint64_t wire = 0, pl = 0;
  for (uint64_t r0 = 0; r0 < nr; r0 += kWalkBlock) {
    const uint64_t r = r0 + tid;
    uint64_t w = 0, L = 0;
    gevws_out_frame o;
    if (r < nr) {
      o = rep[r];
      w = enc_hlen(o.hdr) + o.payload_len;
      L = o.payload_len;
    }
    const uint64_t v[2] = {w, L};
    uint64_t ex[2], tot[2];
    block_excl_scan<kWalkBlock, 2>(v, ex, tot);
    if (r < nr) {
      const uint64_t oo = wire + ex[0];
      out_off[r] = oo;
      uint64_t lo, hi;
      const uint32_t hl = enc_header(o.hdr, lo, hi);
      s_start[r] = (int32_t)oo;
      s_pend[r] = (int32_t)(oo + hl + o.payload_len);
      s_hlen[r] = (uint8_t)hl;
      s_delta[r] = o.payload_off - oo - hl;
      s_h0[r] = lo;
      s_h1[r] = hi;
    }
    wire += tot[0];
    pl += tot[1];
  }
  if (tid == 0) {
    gevws_summary sm;
    memset(&sm, 0, sizeof(sm));
    sm.frames = nr;
    sm.payload_bytes = wire;
    sm.payload_len = pl;
    sm.status = wire > out_cap ? GEVWS_ERR_CAPACITY : GEVWS_OK;
    s_status = (uint32_t)sm.status;
    *esum = sm;
  }
  __syncthreads();
  if (s_status != (uint32_t)GEVWS_OK || wire == 0) {  // (workgroup-uniform)
    signal_done(done, seq, ticks, t0, 1);
    return;
  }
  // 4. the wire image, 16 bytes per lane (the last chunk's tail zeroed inside
  // the GEVWS_OUT_PAD slack)
  // (kHandleBatch chunks a lane with their payload loads in flight together:
  // the payloads sit in mapped host memory, a round trip per round of loads)
  constexpr int kHandleBatch = 4;
  const EncWin W{s_start, s_pend, s_hlen, s_delta, s_h0, s_h1};
  for (uint64_t a0 = (uint64_t)tid * 16; a0 < wire; a0 += (uint64_t)kWalkBlock * 16 * kHandleBatch) {
    EncPrep P[kHandleBatch];
    uint32_t lo[kHandleBatch];
#pragma unroll
    for (int j = 0; j < kHandleBatch; ++j) {
      const uint64_t a = a0 + (uint64_t)j * kWalkBlock * 16;
      lo[j] = 0;
      if (a < wire) {
        const int32_t rel = (int32_t)a;
        uint32_t hi = (uint32_t)nr - 1;  // the last reply starting at or before a
        while (lo[j] < hi) {
          const uint32_t mid = (lo[j] + hi + 1) >> 1;
          if (s_start[mid] <= rel) lo[j] = mid; else hi = mid - 1;
        }
        enc_prep(P[j], rel, a, wire, lo[j], (uint32_t)nr, W, payload);
      }
    }
#pragma unroll
    for (int j = 0; j < kHandleBatch; ++j) {
      const uint64_t a = a0 + (uint64_t)j * kWalkBlock * 16;
      if (a < wire) {
        const u32x4 x = enc_finish(P[j], (int32_t)a, a, lo[j], (uint32_t)nr, W, payload);
        __builtin_memcpy(out + a, &x, 16);
      }
    }
  }
  signal_done(done, seq, ticks, t0, 1);
}

// GEVWS_TUNE_ENCODE_VARIANT: 0 = two tiles a wave step when the caller's
// capacity per frame exceeds kEnc6MinMeanBytes, else one (C1-shaped 128-byte
// frames 0.097 vs 0.104 ms, C4 8.83 vs 8.97, C2 0.431 vs 0.454), the run mode
// chosen on the device; 1 / 2 = one / two tiles a step; 3 / 4 / 5 = two tiles
// a step in run mode 0 / 1 / 2 (measurement).
constexpr int kNumEncodeVariants = 7;
constexpr uint64_t kEnc6MinMeanBytes = 256;

}  // namespace

namespace gevws_impl {

int encode_variant_count() { return kNumEncodeVariants; }

}  // namespace gevws_impl

using namespace gevws_impl;

extern "C" {

static int encode_impl(gevws_ctx* ctx, void* stream, const gevws_out_frame* d_frames, uint64_t n,
                       const gevws_summary* gate, const uint8_t* d_payload, uint8_t* d_out, uint64_t out_cap,
                       uint64_t* d_out_off, gevws_summary* d_summary) {
  if (!ctx || !d_summary || (n && (!d_frames || !d_out || !d_out_off))) return GEVWS_ERR_INVALID;
  if (n > 0xFFFFFFFFull) return GEVWS_ERR_INVALID;
  DeviceGuard g(ctx->device);
  hipStream_t st = pick_stream(ctx, stream);
  const uint64_t nblk64 = (n + (uint64_t)kWalkBlock * kEncSlabs - 1) / ((uint64_t)kWalkBlock * kEncSlabs);
  const uint32_t nblk = (uint32_t)nblk64;
  const uint64_t ntiles_cap = (out_cap + kTile - 1) / kTile + 1;
  const size_t blk_bytes = ((size_t)nblk * kBlkFields * sizeof(uint64_t) + 255) & ~size_t(255);
  int r = order_after_last(ctx, st);
  if (r != GEVWS_OK) return r;
  const size_t tile_bytes = (ntiles_cap * sizeof(uint32_t) + 255) & ~size_t(255);
  r = ensure_scratch(ctx, blk_bytes + tile_bytes + kEnc6Counters * 64);
  if (r != GEVWS_OK) return r;
  uint64_t* blk = reinterpret_cast<uint64_t*>(ctx->scratch);
  uint32_t* tile_first = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(ctx->scratch) + blk_bytes);
  uint32_t* work = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(ctx->scratch) + blk_bytes + tile_bytes);
  if (nblk) k_enc_size<<<nblk, kWalkBlock, 0, st>>>(d_frames, n, blk, d_out_off, gate);
  k_scan_blocks<false><<<1, kScanBlock, 0, st>>>(blk, nblk, n, out_cap, d_summary);
  if (nblk) k_enc_emit<<<nblk, kWalkBlock, 0, st>>>(n, blk, d_summary, d_out_off, tile_first, gate, work);
  // k_encode6's step: two tiles a wave for frames of more than
  // kEnc6MinMeanBytes (by the caller's capacity), at 4 workgroups per CU (121
  // VGPRs), else one tile at 8 (64 VGPRs)
  const int v = ctx->encode_variant;
  const bool u8 = v == 2 || (v >= 3 && v < 6) || (v == 0 && n && out_cap / n > kEnc6MinMeanBytes);
  const uint64_t per_cu = u8 ? 4 : 8;
  const uint64_t wtiles = u8 ? 8 : 4;  // tiles per workgroup step
  uint64_t grid = (out_cap / kTile + wtiles - 1) / wtiles;
  // (GEVWS_TUNE_UNMASK_GRID, when set, caps the encode's grid too: measurement)
  const uint64_t gcap = ctx->unmask_grid ? (uint64_t)ctx->unmask_grid : per_cu * (uint64_t)ctx->num_cus;
  if (grid > gcap) grid = gcap;
  if (grid < 1) grid = 1;
  // batches of big frames (mean >= kBigFrameBytes) keep 4 workgroups per CU
  // (the rest return at once)
  const uint32_t big = grid > 4ull * ctx->num_cus ? 4u * (uint32_t)ctx->num_cus : 0u;
  const int mode = v == 6 ? 1 : v >= 3 ? v - 3 : -1;  // 6: MEASUREMENT
  (u8 ? k_encode6<8> : k_encode6<4>)<<<(uint32_t)grid, kUnmaskBlock, 0, st>>>(
      d_frames, d_payload, d_out_off, tile_first, d_summary, d_out, big, work, mode);
  GEVWS_HIP(hipGetLastError());
  return mark_last(ctx, st);
}

int gevws_encode_batch_async(gevws_ctx* ctx, void* stream, const gevws_out_frame* d_frames, uint64_t n,
                             const uint8_t* d_payload, uint8_t* d_out, uint64_t out_cap, uint64_t* d_out_off,
                             gevws_summary* d_summary) {
  return encode_impl(ctx, stream, d_frames, n, nullptr, d_payload, d_out, out_cap, d_out_off, d_summary);
}

int gevws_encode_replies_async(gevws_ctx* ctx, void* stream, const gevws_out_frame* d_replies,
                               uint64_t max_replies, const gevws_summary* d_dispatched, const uint8_t* d_payload,
                               uint8_t* d_out, uint64_t out_cap, uint64_t* d_out_off, gevws_summary* d_summary) {
  if (!d_dispatched) return GEVWS_ERR_INVALID;
  return encode_impl(ctx, stream, d_replies, max_replies, d_dispatched, d_payload, d_out, out_cap, d_out_off,
                     d_summary);
}

static int dispatch_impl(gevws_ctx* ctx, void* stream, const gevws_frame* d_frames, uint64_t n,
                         const gevws_summary* gate, int policy, uint8_t* d_payload, uint64_t aux_off,
                         uint64_t aux_cap, gevws_out_frame* d_replies, int64_t* d_reply_of,
                         gevws_summary* d_summary) {
  if (!ctx || !d_summary || (n && (!d_frames || !d_payload || !d_replies || !d_reply_of))) return GEVWS_ERR_INVALID;
  if (policy < GEVWS_HANDLER_NONE || policy > GEVWS_HANDLER_ECHO_TEXT) return GEVWS_ERR_INVALID;
  DeviceGuard g(ctx->device);
  hipStream_t st = pick_stream(ctx, stream);
  const uint64_t nblk64 = (n + (uint64_t)kWalkBlock * kEncSlabs - 1) / ((uint64_t)kWalkBlock * kEncSlabs);
  if (nblk64 > 0xFFFFFFFFull) return GEVWS_ERR_INVALID;
  const uint32_t nblk = (uint32_t)nblk64;
  const size_t blk_bytes = ((size_t)nblk * kBlkFields * sizeof(uint64_t) + 255) & ~size_t(255);
  int r = order_after_last(ctx, st);
  if (r != GEVWS_OK) return r;
  r = ensure_scratch(ctx, blk_bytes);
  if (r != GEVWS_OK) return r;
  uint64_t* blk = reinterpret_cast<uint64_t*>(ctx->scratch);
  if (nblk) k_disp_count<<<nblk, kWalkBlock, 0, st>>>(d_frames, n, policy, blk, gate);
  k_scan_blocks<false><<<1, kScanBlock, 0, st>>>(blk, nblk, n, aux_cap / kAuxSlot, d_summary);
  if (nblk)
    k_disp_emit<<<nblk, kWalkBlock, 0, st>>>(d_frames, n, policy, d_payload, aux_off, blk, d_summary, d_replies,
                                              d_reply_of, d_payload + aux_off, gate);
  GEVWS_HIP(hipGetLastError());
  return mark_last(ctx, st);
}

int gevws_dispatch_async(gevws_ctx* ctx, void* stream, const gevws_frame* d_frames, uint64_t n, int policy,
                         uint8_t* d_payload, uint64_t aux_off, uint64_t aux_cap, gevws_out_frame* d_replies,
                         int64_t* d_reply_of, gevws_summary* d_summary) {
  return dispatch_impl(ctx, stream, d_frames, n, nullptr, policy, d_payload, aux_off, aux_cap, d_replies,
                       d_reply_of, d_summary);
}

int gevws_dispatch_decoded_async(gevws_ctx* ctx, void* stream, const gevws_frame* d_frames, uint64_t max_frames,
                                 const gevws_summary* d_decoded, int policy, uint8_t* d_payload, uint64_t aux_off,
                                 uint64_t aux_cap, gevws_out_frame* d_replies, int64_t* d_reply_of,
                                 gevws_summary* d_summary) {
  if (!d_decoded) return GEVWS_ERR_INVALID;
  return dispatch_impl(ctx, stream, d_frames, max_frames, d_decoded, policy, d_payload, aux_off, aux_cap, d_replies,
                       d_reply_of, d_summary);
}

int gevws_handle_decoded_async(gevws_ctx* ctx, void* stream, const gevws_frame* d_frames, uint64_t max_frames,
                               const gevws_summary* d_decoded, int policy, uint8_t* d_payload, uint64_t aux_off,
                               uint64_t aux_cap, gevws_out_frame* d_replies, int64_t* d_reply_of,
                               gevws_summary* d_disp_summary, uint8_t* d_out, uint64_t out_cap, uint64_t* d_out_off,
                               gevws_summary* d_enc_summary) {
  if (!ctx || !d_decoded || !d_disp_summary || !d_enc_summary) return GEVWS_ERR_INVALID;
  if (max_frames > kHandleSmallFrames || out_cap > 0x7fffffffull) {  // the two-step chain
    int r = gevws_dispatch_decoded_async(ctx, stream, d_frames, max_frames, d_decoded, policy, d_payload, aux_off,
                                         aux_cap, d_replies, d_reply_of, d_disp_summary);
    if (r != GEVWS_OK) return r;
    return gevws_encode_replies_async(ctx, stream, d_replies, max_frames, d_disp_summary, d_payload, d_out, out_cap,
                                      d_out_off, d_enc_summary);
  }
  if (max_frames && (!d_frames || !d_payload || !d_replies || !d_reply_of || !d_out || !d_out_off))
    return GEVWS_ERR_INVALID;
  if (policy < GEVWS_HANDLER_NONE || policy > GEVWS_HANDLER_ECHO_TEXT) return GEVWS_ERR_INVALID;
  DeviceGuard g(ctx->device);
  hipStream_t st = pick_stream(ctx, stream);
  int r = order_after_last(ctx, st);
  if (r != GEVWS_OK) return r;
  const uint32_t seq = ctx->done_flag ? ++ctx->done_seq : 0u;
  k_handle_small<<<1, kWalkBlock, 0, st>>>(d_frames, max_frames, d_decoded, policy, d_payload, aux_off, aux_cap,
                                           d_replies, d_reply_of, d_disp_summary, d_out, out_cap, d_out_off,
                                           d_enc_summary, ctx->done_flag, seq, ctx->done_flag ? ctx->ticks : nullptr);
  GEVWS_HIP(hipGetLastError());
  r = mark_last(ctx, st);  // (recorded now: see mark_last_lazy)
  if (ctx->done_flag) ctx->last_signal = seq;
  return r;
}

}  // extern "C"
