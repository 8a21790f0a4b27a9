// gevws_unmask.hip -- the payload unmask / compaction (SURVEY.md §8a rows
// a1, a3): ws.Cipher (cipher.go:14-53) of every frame's payload into its
// 16-aligned slot of the payload arena -- the zeroed make + Read + Cipher of
// protocol.go:50-55, the key phase restarting at 0 per frame (protocol.go:54);
// HBM-bound at h + 2L bytes per frame.  Also ws.Cipher on a device buffer
// (gevws_cipher_async) and the streaming-copy ceiling bench.py measures.
#include "gevws_internal.hpp"

namespace {

// Largest frame index f in [tile_first[t], tile_first[t+1]] with payload_off <= p.
__device__ __forceinline__ uint64_t find_frame(const gevws_frame* __restrict__ frames,
                                               const uint32_t* __restrict__ tile_first, uint64_t t,
                                               uint64_t ntiles, uint64_t nframes, uint64_t p) {
  uint64_t lo = tile_first[t];
  uint64_t hi = (t + 1 < ntiles) ? (uint64_t)tile_first[t + 1] : nframes - 1;
  while (lo < hi) {
    const uint64_t mid = (lo + hi + 1) >> 1;
    if (frames[mid].payload_off <= p) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// One 16-byte chunk of a frame the per-lane fallback path takes (windows of
// more than kWinFrames frames: runs of empty frames), found by a search in
// the tile map's frame range.
__device__ __forceinline__ void unmask_chunk_lookup(const uint8_t* __restrict__ in,
                                                    const gevws_frame* __restrict__ frames,
                                                    const uint32_t* __restrict__ tile_first, uint64_t t,
                                                    uint64_t ntiles, uint64_t nframes, uint64_t p,
                                                    uint8_t* __restrict__ out) {
  const gevws_frame* fr = frames + find_frame(frames, tile_first, t, ntiles, nframes, p);
  const uint64_t rel = p - fr->payload_off;
  uint32_t k;
  memcpy(&k, fr->hdr.mask, 4);
  u32x4 x = ld16u(in + fr->src_off + rel) ^ (fr->hdr.masked ? k : 0u);
  const int64_t r = fr->hdr.length - (int64_t)rel;
  if (r < 16) x = keep_bytes(x, r);
  st16_nt(out + p, x);
}

// Measurement helper (not on the reference path): the unmask kernel's
// streaming loop with the frame lookup and the XOR taken out -- each workgroup
// owns a contiguous run of 4 KiB tiles, U 16-byte loads per lane, aligned
// non-temporal stores.  bench.py times it over the same bytes as the
// achievable-bandwidth ceiling beside the 8 TB/s spec peak.  NTL: loads
// non-temporal like the unmask's streaming loads (else plain); WSPAN: the
// unmask's streaming layout -- in steps of U tiles of which wave w copies the
// contiguous U KiB at w * U KiB (16 aligned bytes per lane per KiB).
template <bool NT>
__device__ __forceinline__ u32x4 copy_ld(const uint8_t* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));  // unaligned nt load
  else return ld16u(p);
}

template <bool PS>
__device__ __forceinline__ void copy_st(uint8_t* p, u32x4 x) {
  if constexpr (PS) *reinterpret_cast<u32x4*>(p) = x;  // (p may be misaligned: gfx950 unaligned access mode)
  else st16_nt(p, x);
}

template <int U, bool NTL, bool WSPAN, bool PS = false>
__global__ __launch_bounds__(kUnmaskBlock) void k_copy_stream(const uint8_t* __restrict__ src,
                                                              uint8_t* __restrict__ dst, uint64_t n) {
  const uint64_t ntiles = n / kTile;
  const uint32_t lane_off = threadIdx.x * 16;
  const uint64_t per = (ntiles + gridDim.x - 1) / gridDim.x;
  uint64_t t = (uint64_t)blockIdx.x * per;
  const uint64_t tend = t + per < ntiles ? t + per : ntiles;
  const uint64_t wrel = WSPAN ? (uint64_t)(threadIdx.x >> 6) * U * 1024 + (threadIdx.x & 63) * 16 : lane_off;
  constexpr uint64_t kStride = WSPAN ? 1024 : kTile;  // between a lane's U chunks of a step
  for (; t + U <= tend; t += U) {
    const uint64_t base = t * kTile + wrel;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = copy_ld<NTL>(src + base + u * kStride);
#pragma unroll
    for (int u = 0; u < U; ++u) copy_st<PS>(dst + base + u * kStride, v[u]);
  }
  for (; t < tend; ++t) {
    const uint64_t base = t * kTile + lane_off;
    copy_st<PS>(dst + base, copy_ld<NTL>(src + base));
  }
  // bytes past the last whole tile: 16 per lane, workgroup 0
  const uint64_t tail = ntiles * kTile;
  if (blockIdx.x == 0)
    for (uint64_t p = tail + lane_off; p < n; p += kTile) copy_st<PS>(dst + p, copy_ld<NTL>(src + p));
}

// The unmask = ws.Cipher (cipher.go:14-53) of every frame's payload into its
// 16-aligned slot of the payload arena (protocol.go:50-55: the zeroed make +
// Read + Cipher; pad bytes zero).  Each workgroup owns a contiguous run of 4
// KiB output tiles.  While one frame covers the next U tiles the loop streams
// (stream_step); otherwise it takes a window of tiles whose frames' records it
// loads into LDS, and each lane looks up the frame of each of its chunks.
constexpr int kWinFrames = 1024;  // frames a window's LDS table holds (more: the per-lane fallback)

// One streaming step: U whole tiles [base, base + U*kTile) of the output
// arena inside one frame (payload offset f_po, source f_src, length f_len,
// key f_key).  A misaligned source is read with aligned non-temporal loads
// over wave-contiguous U KiB spans and realigned in registers (DPP lane rotate
// + v_alignbyte): wave w covers U KiB-chunks [base + w*U KiB, +U KiB) of the
// step, lane 63's successor chunk at step u is lane 0's chunk at u+1, so only
// u = U-1 needs one extra load, by lane 63.  An aligned source: plain loads.
// Stores: aligned, non-temporal.
template <int U>
__device__ __forceinline__ void stream_step(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                            uint64_t base, uint64_t f_po, uint64_t f_src, int64_t f_len,
                                            uint32_t f_key) {
  const uint32_t lane_off = threadIdx.x * 16;
  const uint64_t rel0 = base - f_po + lane_off;
  const uint8_t* src = in + f_src + rel0;
  uint8_t* dst = out + base + lane_off;
  u32x4 v[U];
  const uint32_t mis = (uint32_t)(reinterpret_cast<uint64_t>(src) & 15);  // uniform: lanes 16 B apart
  if (mis != 0) {
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t wrel = (uint64_t)wave * U * 1024 + lane * 16;  // this lane's offset in the step
    const uint8_t* a = in + f_src + (base - f_po) + wrel - mis;
    uint8_t* d = out + base + wrel;
    const bool last = lane == 63;
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a + u * 1024));
    u32x4 e = u32x4{0, 0, 0, 0};
    if (last) e = *reinterpret_cast<const u32x4*>(a + (U - 1) * 1024 + 16);
    u32x4 r = rot_next_lane(v[0]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const u32x4 rn = u + 1 < U ? rot_next_lane(v[u + 1 < U ? u + 1 : u]) : e;
      const u32x4 nx = last ? rn : r;
      u32x4 x = funnel16(v[u], nx, mis) ^ f_key;
      const int64_t rem = f_len - (int64_t)(base - f_po + wrel + u * 1024);
      if (rem < 16) x = keep_bytes(x, rem);
      st16_nt(d + u * 1024, x);
      r = rn;
    }
    return;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = ld16u(src + u * kTile);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    u32x4 x = v[u] ^ f_key;
    const int64_t rem = f_len - (int64_t)(rel0 + u * kTile);
    if (rem < 16) x = keep_bytes(x, rem);
    st16_nt(dst + u * kTile, x);
  }
}

// The LDS frame table of a v3 window (kWinFrames entries each).
struct WinLds {
  uint32_t* start;   // frame start relative to the window (clamped at 0)
  int32_t* lend;     // payload end relative to the window (clamped)
  uint64_t* delta;   // src_off - payload_off (mod 2^64)
  uint32_t* key;
};

// v3: 16-tile streaming steps; a window is 4 tiles: the records of every frame
// overlapping it (index range from the tile map) go into LDS with one
// coalesced pass and each lane binary-searches LDS for the frame of each of
// its 4 chunks, whose loads are unaligned non-temporal 16-byte loads.  The
// scheme of batches of equal-size frames (C1, C2, C3, C5: -5 % on C1-shaped
// and -2.4 % on C2 batches against v4's 8-tile windows, equal on C3;
// profiles/r02/r02_ab2.log).
template <int U>
__device__ __forceinline__ void unmask_v3_body(const uint8_t* __restrict__ in, const gevws_frame* __restrict__ frames,
                                               const uint32_t* __restrict__ tile_first,
                                               const gevws_summary* __restrict__ sum, uint8_t* __restrict__ out,
                                               uint32_t big_grid, const WinLds& L, uint32_t* __restrict__ runs = nullptr,
                                               uint32_t* __restrict__ s_run = nullptr) {
  constexpr int WT = kWinTiles;
  uint32_t* const s_start = L.start;
  int32_t* const s_lend = L.lend;
  uint64_t* const s_delta = L.delta;
  uint32_t* const s_key = L.key;
  if (sum->status != GEVWS_OK) return;
  const uint64_t total = sum->payload_bytes;
  const uint64_t nframes = sum->frames;
  const uint64_t ntiles = (total + kTile - 1) / kTile;
  const uint32_t groups = active_groups(total, nframes, big_grid);
  if (blockIdx.x >= groups) return;
  const uint64_t per = (ntiles + groups - 1) / groups;
  // counter runs as the v5 path's, for batches of frames below kBigFrameBytes
  // with at least kUnmaskRunMinTiles tiles a workgroup: C2 -4 %, C5 equal;
  // big frames want long runs (C3 +15 %) and small batches few (C1-shaped +13
  // %, profiles/r04/r04_unmask_counter_ab.jsonl)
  const bool dyn = runs != nullptr && groups >= kUnmaskRunCounters && nframes && total / nframes < kBigFrameBytes &&
                   ntiles >= kUnmaskRunMinTiles * groups;
  uint64_t t = dyn ? 0 : (uint64_t)blockIdx.x * per;
  uint64_t tend = dyn ? 0 : (t + per < ntiles ? t + per : ntiles);
  const uint32_t xc = blockIdx.x % kUnmaskRunCounters;
  const uint64_t segn = ((ntiles + kUnmaskRunCounters - 1) / kUnmaskRunCounters + kUnmaskRun - 1) / kUnmaskRun * kUnmaskRun;
  const uint64_t seg0 = xc * segn < ntiles ? xc * segn : ntiles;
  const uint64_t seg1 = seg0 + segn < ntiles ? seg0 + segn : ntiles;
  const uint32_t lane_off = threadIdx.x * 16;
  uint64_t f_po = 0, f_end = 0, f_src = 0;
  int64_t f_len = 0;
  uint32_t f_key = 0;
  for (;;) {
  if (dyn) {
    __syncthreads();
    if (threadIdx.x == 0) *s_run = atomicAdd(runs + xc * 16, 1u);
    __syncthreads();
    t = seg0 + (uint64_t)*s_run * kUnmaskRun;
    if (t >= seg1) break;
    tend = t + kUnmaskRun < seg1 ? t + kUnmaskRun : seg1;
  }
  while (t < tend) {
    const uint64_t base = t * kTile;
    if (base >= f_end) {  // workgroup-uniform: refresh the cached frame (scalar loads)
      const uint64_t* rec = reinterpret_cast<const uint64_t*>(frames + tile_first[t]);
      const uint64_t w0 = rec[0];
      f_len = (int64_t)rec[1];
      f_po = rec[2];
      f_src = rec[3];
      f_end = f_po + round16((uint64_t)f_len);
      f_key = ((w0 >> 24) & 0xff) ? (uint32_t)(w0 >> 32) : 0u;
    }
    if (t + U <= tend && base + U * kTile <= f_end) {
      stream_step<U>(in, out, base, f_po, f_src, f_len, f_key);
      t += U;
      continue;
    }
    // ---- window path
    const uint64_t wt = (tend - t) < (uint64_t)WT ? (tend - t) : (uint64_t)WT;
    const uint64_t wend_t = t + wt;
    const uint64_t wbase = base;
    const uint64_t f_lo = tile_first[t];
    const uint64_t f_hi = wend_t < ntiles ? (uint64_t)tile_first[wend_t] : nframes - 1;
    const uint64_t F = f_hi - f_lo + 1;
    if (F <= (uint64_t)kWinFrames) {
      __syncthreads();  // previous window's readers are done with the LDS table
      for (uint64_t i = threadIdx.x; i < F; i += kUnmaskBlock) {
        const uint64_t* rec = reinterpret_cast<const uint64_t*>(frames + f_lo + i);
        const uint64_t w0 = rec[0];
        const uint64_t Ln = rec[1];
        const uint64_t po = rec[2];
        const uint64_t so = rec[3];
        s_start[i] = po > wbase ? (uint32_t)(po - wbase) : 0u;
        const uint64_t lend = po + Ln;  // end of payload bytes
        s_lend[i] = lend <= wbase ? 0 : (lend - wbase > 0x7fffffffull ? 0x7fffffff : (int32_t)(lend - wbase));
        s_delta[i] = so - po;
        s_key[i] = ((w0 >> 24) & 0xff) ? (uint32_t)(w0 >> 32) : 0u;
      }
      __syncthreads();
      u32x4 v[WT];
      uint32_t key[WT];
      int32_t rem[WT];
#pragma unroll
      for (int u = 0; u < WT; ++u) {
        const uint32_t rel = (uint32_t)(u * kTile) + lane_off;
        const uint64_t p = wbase + rel;
        rem[u] = 0;
        key[u] = 0;
        v[u] = u32x4{0, 0, 0, 0};
        if ((uint64_t)u < wt && p < total) {
          uint32_t lo = 0, hi = (uint32_t)F - 1;
          while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (s_start[mid] <= rel) lo = mid; else hi = mid - 1;
          }
          rem[u] = s_lend[lo] - (int32_t)rel;
          key[u] = s_key[lo];
          v[u] = ld16u_stream<true>(in + (p + s_delta[lo]));
        }
      }
#pragma unroll
      for (int u = 0; u < WT; ++u) {
        if (rem[u] > 0) {
          u32x4 x = v[u] ^ key[u];
          if (rem[u] < 16) x = keep_bytes(x, rem[u]);
          st16_nt(out + wbase + (uint32_t)(u * kTile) + lane_off, x);
        }
      }
      t = wend_t;
      continue;
    }
    // ---- too many frames in the window (runs of empty frames): per-lane lookup, one tile
    const uint64_t p = base + lane_off;
    if (p < total) unmask_chunk_lookup(in, frames, tile_first, t, ntiles, nframes, p, out);
    t += 1;
  }
  if (!dyn) break;
  }
}

// v5: the window path for batches of mixed sizes (C4), software-pipelined and
// with its two latency chains out of the critical path.  8-tile windows; the
// NEXT step is decided while the current window's payload loads are in flight
// (its tile-map entries -- first frame a, last frame b and the frame at tile
// +U, which equals a iff one frame covers the next U tiles -- and, for a
// window, its first 256 records into registers, one per lane).  Profiled
// (round 3, cycle counters; profiles/r03/r03_unmask_profile*.jsonl) an 8-tile
// window of round 2's v4 spent a quarter of its ~37 K cycles in the per-chunk
// searches and a third in the next-step decision.  v5:
//  * chunk -> frame by a map instead of a search: every non-empty frame marks
//    its first 16-byte chunk in the window (payloads are 16-aligned and
//    contiguous, so each chunk belongs to exactly one frame: the last one
//    starting at or before it), and a workgroup prefix-max over the 2 048
//    chunk slots turns the marks into the owner of every chunk; a lane then
//    reads its 8 owners and their attributes in two LDS round trips, all
//    chunks at once.  The map is double-buffered: window k clears the buffer
//    window k+1 fills.
//  * the tile map through an LDS cache of kTmapN entries (refilled by the
//    whole workgroup every ~60 windows): a decision is LDS reads, not global.
// C4 7.75 -> 7.40 ms against v4 (profiles/r03/r03_unmask_v5*_ab.jsonl).
// amdgpu_waves_per_eu(4): four workgroups per CU (128 VGPRs); 5 or 6 measured
// slower (r03_unmask_occ_ab.jsonl).  Every lane id is re-derived where it is
// used (fresh_tid): held across the loop, the fill's per-lane LDS / record
// addresses were spilled, and each spill reload -- a scratch load queued
// behind the window's global loads, vmcnt being in order -- serialised them
// (C4: 2 GB of the 22.9 GB read per launch in round 1).
constexpr int kWin5Frames = 1024;
constexpr uint32_t kWinChunks = 8 * (uint32_t)kTile / 16;  // 2 048 chunks in an 8-tile window
constexpr uint32_t kQuarter = kWinChunks / (kUnmaskBlock / 64);  // chunks per wave
constexpr uint32_t kTmapN = 512;

struct WinRec {
  u64x2 lo;  // header word (fin, rsv, opcode, masked, mask[4]), length
  u64x2 hi;  // payload_off, src_off
};

__device__ __forceinline__ WinRec load_rec(const gevws_frame* __restrict__ frames, uint64_t f) {
  const u64x2* r = reinterpret_cast<const u64x2*>(frames + f);
  return WinRec{r[0], r[1]};
}

struct WinLds5 {
  int32_t* lend;    // [kWin5Frames] payload end relative to the window (clamped)
  uint64_t* delta;  // [kWin5Frames] src_off - payload_off
  uint32_t* key;    // [kWin5Frames]
  uint16_t* own;    // [2][kWinChunks] window chunk -> frame index + 1 (marks, then their prefix max)
  uint32_t* wtot;   // [2][kUnmaskBlock / 64] per map: frame index + 1 covering each wave quarter's first chunk
  uint32_t* tmap;   // [kTmapN + 1] tile_first[tm0 ...], then the run index of a grab
};

template <int U>
__device__ __forceinline__ void unmask_v5_body(const uint8_t* __restrict__ in, const gevws_frame* __restrict__ frames,
                                               const uint32_t* __restrict__ tile_first,
                                               const gevws_summary* __restrict__ sum, uint8_t* __restrict__ out,
                                               uint32_t big_grid, const WinLds5& L, bool wide = false,
                                               uint32_t* __restrict__ runs = nullptr) {
  constexpr int WT = 8;
  static_assert(WT * kTile / 16 == kWinChunks && kWinChunks == 8 * kUnmaskBlock, "8 chunks per thread");
  if (sum->status != GEVWS_OK) return;
  const uint64_t total = sum->payload_bytes;
  const uint64_t nframes = sum->frames;
  const uint64_t ntiles = (total + kTile - 1) / kTile;
  const uint32_t groups = active_groups(total, nframes, big_grid, wide);
  if (blockIdx.x >= groups) return;
  const uint64_t per = (ntiles + groups - 1) / groups;
  // counter runs (kUnmaskRun tiles of this XCD's eighth) when every counter
  // has workgroups, else one contiguous run per workgroup
  const bool dyn = runs != nullptr && groups >= kUnmaskRunCounters;
  uint64_t t = dyn ? 0 : (uint64_t)blockIdx.x * per;
  uint64_t tend = dyn ? 0 : (t + per < ntiles ? t + per : ntiles);
  const uint32_t xc = blockIdx.x % kUnmaskRunCounters;
  const uint64_t segn = ((ntiles + kUnmaskRunCounters - 1) / kUnmaskRunCounters + kUnmaskRun - 1) / kUnmaskRun * kUnmaskRun;
  const uint64_t seg0 = xc * segn < ntiles ? xc * segn : ntiles;
  const uint64_t seg1 = seg0 + segn < ntiles ? seg0 + segn : ntiles;
  {  // both chunk maps (and their wave seeds) start empty
    const uint32_t tid = fresh_tid();
    reinterpret_cast<u32x4*>(L.own)[tid] = u32x4{0, 0, 0, 0};
    reinterpret_cast<u32x4*>(L.own + kWinChunks)[tid] = u32x4{0, 0, 0, 0};
    if (tid < 2 * (kUnmaskBlock / 64)) L.wtot[tid] = 0;
  }
  __syncthreads();
  uint64_t f_po = 0, f_end = 0, f_src = 0;  // the cached (streaming) frame
  int64_t f_len = 0;
  uint32_t f_key = 0;
  uint64_t pf_t = ~0ull, pf_a = 0, pf_b = 0;  // decision for tile pf_t, made during the previous window
  bool pf_stream = false;
  WinRec r0 = {};  // record pf_a + tid when !pf_stream
  uint32_t buf = 0;          // chunk map of this window
  uint64_t tm0 = ~0ull;      // first tile of the cached tile map
  auto cache_frame = [&](uint64_t f) {  // wave-uniform: SGPRs
    const uint64_t* rec = reinterpret_cast<const uint64_t*>(frames + f);
    const uint64_t w0 = uniform64(rec[0]);
    f_len = (int64_t)uniform64(rec[1]);
    f_po = uniform64(rec[2]);
    f_src = uniform64(rec[3]);
    f_end = f_po + round16((uint64_t)f_len);
    f_key = ((w0 >> 24) & 0xff) ? (uint32_t)(w0 >> 32) : 0u;
  };
  // tile_first[x] for x < ntiles from the LDS cache, which holds [x, x + 16]
  // after the call (a refill is a workgroup step: callers are uniform)
  auto tmap_at = [&](uint64_t x) -> uint64_t {
    if (tm0 == ~0ull || x < tm0 || x + 16 >= tm0 + kTmapN) {
      __syncthreads();  // every wave done with the old entries
      tm0 = x;
      for (uint32_t i = fresh_tid(); i < kTmapN; i += kUnmaskBlock) {
        const uint64_t y = x + i;
        L.tmap[i] = y < ntiles ? tile_first[y] : 0u;
      }
      __syncthreads();
    }
    return uniform32(L.tmap[x - tm0]);
  };
  // step decision for tile x: a = first frame; stream iff one frame covers
  // [x, x+U) -- the tile map puts frame a at tile x+U-1 too, and its record
  // (then cached for the streaming step) ends at or past tile x+U; otherwise
  // b = last frame of the window [x, x+WT)
  auto decide = [&](uint64_t x, uint64_t& a, uint64_t& b, bool& stream) {
    a = tmap_at(x);
    stream = false;
    if (x + U <= tend && tmap_at(x + U - 1) == a) {
      cache_frame(a);
      stream = x * kTile >= f_po && (x + U) * kTile <= f_end;
    }
    const uint64_t wt = (tend - x) < (uint64_t)WT ? (tend - x) : (uint64_t)WT;
    b = x + wt < ntiles ? tmap_at(x + wt) : nframes - 1;
  };
  for (;;) {
  if (dyn) {  // the next run: thread 0's vector atomic, through LDS
    __syncthreads();
    if (threadIdx.x == 0) L.tmap[kTmapN] = atomicAdd(runs + xc * 16, 1u);
    __syncthreads();
    t = seg0 + (uint64_t)L.tmap[kTmapN] * kUnmaskRun;
    if (t >= seg1) break;
    tend = t + kUnmaskRun < seg1 ? t + kUnmaskRun : seg1;
    pf_t = ~0ull;
    r0 = WinRec{};
  }
  while (t < tend) {
    const uint64_t base = t * kTile;
    if (t + U <= tend && base >= f_po && base + U * kTile <= f_end) {  // still inside the cached frame
      stream_step<U>(in, out, base, f_po, f_src, f_len, f_key);
      t += U;
      pf_t = ~0ull;
      r0 = WinRec{};  // (redefined: dead across the step)
      continue;
    }
    uint64_t a, b;
    bool stream, have = false;
    if (pf_t == t) {
      a = pf_a;
      b = pf_b;
      stream = pf_stream;
      have = !pf_stream;
    } else {
      decide(t, a, b, stream);
    }
    if (stream) {  // decide() cached frame a, which covers [t, t+U)
      stream_step<U>(in, out, base, f_po, f_src, f_len, f_key);
      t += U;
      pf_t = ~0ull;
      r0 = WinRec{};
      continue;
    }
    const uint64_t wt = (tend - t) < (uint64_t)WT ? (tend - t) : (uint64_t)WT;
    const uint64_t wend_t = t + wt;
    const uint64_t wbase = base;
    const uint64_t F = b - a + 1;
    if (F > (uint64_t)kWin5Frames) {  // runs of empty frames: per-lane lookup, one tile
      const uint64_t p = base + fresh_tid() * 16;
      if (p < total) unmask_chunk_lookup(in, frames, tile_first, t, ntiles, nframes, p, out);
      t += 1;
      pf_t = ~0ull;
      r0 = WinRec{};
      continue;
    }
    uint16_t* const own = L.own + buf * kWinChunks;
    uint32_t* const carry = L.wtot + buf * (kUnmaskBlock / 64);
    __syncthreads();  // previous window's readers are done with the frame table
    auto fill = [&](uint64_t i, const WinRec& q) {
      const uint64_t Ln = q.lo[1], po = q.hi[0], so = q.hi[1];
      const uint64_t lend = po + Ln;
      L.lend[i] = lend <= wbase ? 0 : (lend - wbase > 0x7fffffffull ? 0x7fffffff : (int32_t)(lend - wbase));
      L.delta[i] = so - po;
      L.key[i] = ((q.lo[0] >> 24) & 0xff) ? (uint32_t)(q.lo[0] >> 32) : 0u;
      if (Ln) {  // the frame's first chunk in the window (frame a's is chunk 0)
        const uint64_t sc = po > wbase ? (po - wbase) >> 4 : 0;
        if (sc < kWinChunks) own[sc] = (uint16_t)(i + 1);
        // the frame covering the first chunk of wave w's quarter (w > 0)
        // seeds that wave's scan: no cross-wave step
        const uint64_t ec = (po + round16(Ln) - wbase) >> 4;  // one past its last chunk
#pragma unroll
        for (uint32_t w = 1; w < kUnmaskBlock / 64; ++w)
          if (sc < w * kQuarter && w * kQuarter < ec) carry[w] = (uint32_t)(i + 1);
      }
    };
    const uint32_t tid = fresh_tid();
    if (tid < F) fill(tid, have ? r0 : load_rec(frames, a + tid));
    for (uint64_t i = tid + kUnmaskBlock; i < F; i += kUnmaskBlock) fill(i, load_rec(frames, a + i));
    __syncthreads();
    // prefix max over the chunk marks, per wave over its own quarter of the
    // window (wave w: chunks [512 w, 512 (w + 1)), lane l the 8 from 512 w + 8 l),
    // seeded with the frame covering the quarter's first chunk; the wave then
    // reads only its quarter's owners, so no barrier follows
    {
      const uint32_t j = fresh_tid(), lane = j & 63, w = j >> 6;
      u32x4 m = reinterpret_cast<const u32x4*>(own)[j];
      uint32_t run[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        run[2 * k] = m[k] & 0xffffu;
        run[2 * k + 1] = m[k] >> 16;
      }
#pragma unroll
      for (int k = 1; k < 8; ++k) run[k] = run[k] > run[k - 1] ? run[k] : run[k - 1];
      uint32_t inc = run[7];
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)inc, d, 64);
        if (lane >= (uint32_t)d) inc = inc > y ? inc : y;
      }
      uint32_t exc = (uint32_t)__shfl_up((int)inc, 1, 64);
      const uint32_t seed = w ? carry[w] : 0u;
      if (lane == 0) exc = 0;
      exc = exc > seed ? exc : seed;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t lo16 = run[2 * k] > exc ? run[2 * k] : exc;
        const uint32_t hi16 = run[2 * k + 1] > exc ? run[2 * k + 1] : exc;
        m[k] = lo16 | (hi16 << 16);
      }
      reinterpret_cast<u32x4*>(own)[j] = m;
      // the next window's map and seeds start empty (their last readers
      // finished before this window's first barrier)
      reinterpret_cast<u32x4*>(L.own + (buf ^ 1) * kWinChunks)[j] = u32x4{0, 0, 0, 0};
      if (lane == 0) L.wtot[(buf ^ 1) * (kUnmaskBlock / 64) + w] = 0;
    }
    u32x4 v[WT];
    uint32_t key[WT];
    int32_t rem[WT];
    uint32_t lov[WT];
    // wave w, step u: the 64 contiguous chunks 512 w + 64 u + lane (1 KiB)
#pragma unroll
    for (int u = 0; u < WT; ++u) {
      const uint32_t tq = fresh_tid();
      const uint32_t c = (tq >> 6) * kQuarter + (uint32_t)u * 64 + (tq & 63);
      const uint32_t o = own[c];
      lov[u] = o ? o - 1 : 0;
    }
    const uint32_t tl = fresh_tid();
    const uint32_t loff = (tl >> 6) * kQuarter * 16 + (tl & 63) * 16;
#pragma unroll
    for (int u = 0; u < WT; ++u) {
      const uint32_t rel = (uint32_t)u * 1024 + loff;
      const uint64_t p = wbase + rel;
      rem[u] = 0;
      key[u] = 0;
      v[u] = u32x4{0, 0, 0, 0};
      if ((uint64_t)rel < wt * kTile && p < total) {
        const uint32_t lo = lov[u];
        rem[u] = L.lend[lo] - (int32_t)rel;
        key[u] = L.key[lo];
        v[u] = ld16u_stream<true>(in + (p + L.delta[lo]));
      }
    }
    // decide the next step (and fetch the next window's records) while this
    // window's payload loads are in flight
    __asm__ volatile("" ::: "memory");
    pf_t = ~0ull;
    if (wend_t < tend) {
      decide(wend_t, pf_a, pf_b, pf_stream);
      pf_t = wend_t;
      if (!pf_stream) {
        const uint64_t nF = pf_b - pf_a + 1;
        const uint32_t tid2 = fresh_tid();
        if (tid2 < nF) r0 = load_rec(frames, pf_a + tid2);
      }
    }
    const uint32_t ts = fresh_tid();
    const uint32_t soff = (ts >> 6) * kQuarter * 16 + (ts & 63) * 16;
#pragma unroll
    for (int u = 0; u < WT; ++u) {
      if (rem[u] > 0) {
        u32x4 x = v[u] ^ key[u];
        if (rem[u] < 16) x = keep_bytes(x, rem[u]);
        st16_nt(out + wbase + (uint32_t)u * 1024 + soff, x);
      }
    }
    buf ^= 1;
    t = wend_t;
  }
  if (!dyn) break;
  }
}

// The default unmask: the batch's own statistics pick the window scheme --
// batches of equal-size frames (at least half of the frames the size of the
// one before them on the connection: C1, C2, C3, C5) take v3's 4-tile windows,
// mixed ones (C4) v5's pipelined 8-tile windows, with the whole (wide) grid
// for a batch of fewer than kWideGridTiles tiles.  One kernel, one LDS
// budget, the choice is a uniform branch on the summary the walk wrote.
__global__ __launch_bounds__(kUnmaskBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_unmask_auto5(
    const uint8_t* __restrict__ in, const gevws_frame* __restrict__ frames, const uint32_t* __restrict__ tile_first,
    const gevws_summary* __restrict__ sum, uint8_t* __restrict__ out, uint32_t big_grid, uint32_t* __restrict__ runs) {
  static_assert(kWinFrames == kWin5Frames, "one frame table for both bodies");
  __shared__ uint32_t s_start[kWinFrames];
  __shared__ int32_t s_lend[kWinFrames];
  __shared__ uint64_t s_delta[kWinFrames];
  __shared__ uint32_t s_key[kWinFrames];
  __shared__ __attribute__((aligned(16))) uint16_t s_own[2 * kWinChunks];
  __shared__ uint32_t s_wtot[2 * (kUnmaskBlock / 64)];
  __shared__ uint32_t s_tmap[kTmapN + 1];
  if (2 * sum->run_frames >= sum->frames)
    unmask_v3_body<16>(in, frames, tile_first, sum, out, big_grid, WinLds{s_start, s_lend, s_delta, s_key}, runs,
                       s_tmap + kTmapN);
  else
    unmask_v5_body<16>(in, frames, tile_first, sum, out, big_grid,
                       WinLds5{s_lend, s_delta, s_key, s_own, s_wtot, s_tmap},
                       sum->payload_bytes / kTile < kWideGridTiles, runs);
}

// v5 for every batch (GEVWS_TUNE_UNMASK_VARIANT 1): the mixed-size path on any
// batch, so the parity tests run it over equal-size frames too.
__global__ __launch_bounds__(kUnmaskBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_unmask_v5(
    const uint8_t* __restrict__ in, const gevws_frame* __restrict__ frames, const uint32_t* __restrict__ tile_first,
    const gevws_summary* __restrict__ sum, uint8_t* __restrict__ out, uint32_t big_grid, uint32_t* __restrict__ runs) {
  __shared__ int32_t s_lend[kWin5Frames];
  __shared__ uint64_t s_delta[kWin5Frames];
  __shared__ uint32_t s_key[kWin5Frames];
  __shared__ __attribute__((aligned(16))) uint16_t s_own[2 * kWinChunks];
  __shared__ uint32_t s_wtot[2 * (kUnmaskBlock / 64)];
  __shared__ uint32_t s_tmap[kTmapN + 1];
  unmask_v5_body<16>(in, frames, tile_first, sum, out, big_grid,
                     WinLds5{s_lend, s_delta, s_key, s_own, s_wtot, s_tmap},
                     sum->payload_bytes / kTile < kWideGridTiles, runs);
}

// ------------------------------------------------------------------ ws.Cipher on a device buffer
// p[i] ^= mask[(offset + i) & 3] for i in [0, n): 16-byte aligned chunks of the
// address space; interior chunks use one rotated 32-bit key, edge chunks go
// byte by byte.
__global__ __launch_bounds__(256) void k_cipher(uint8_t* __restrict__ p, uint64_t n, uint32_t key,
                                                uint64_t offset, uint64_t nchunks) {
  const uint64_t a0 = reinterpret_cast<uint64_t>(p) & ~uint64_t(15);
  const uint64_t pe = reinterpret_cast<uint64_t>(p) + n;
  const uint32_t s = (uint32_t)((offset - reinterpret_cast<uint64_t>(p)) & 3);
  const uint32_t krot = s ? ((key >> (8 * s)) | (key << (32 - 8 * s))) : key;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nchunks;
       k += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t a = a0 + 16 * k;
    if (a >= reinterpret_cast<uint64_t>(p) && a + 16 <= pe) {
      u32x4* q = reinterpret_cast<u32x4*>(a);
      *q = *q ^ krot;
    } else {
      for (uint32_t b = 0; b < 16; ++b) {
        const uint64_t x = a + b;
        if (x >= reinterpret_cast<uint64_t>(p) && x < pe) {
          const uint32_t idx = (uint32_t)((offset + (x - reinterpret_cast<uint64_t>(p))) & 3);
          *reinterpret_cast<uint8_t*>(x) ^= (uint8_t)(key >> (8 * idx));
        }
      }
    }
  }
}

using UnmaskFn = void (*)(const uint8_t*, const gevws_frame*, const uint32_t*, const gevws_summary*, uint8_t*,
                         uint32_t, uint32_t*);
struct UnmaskVariant {
  UnmaskFn fn;
  int unroll;
  const char* name;
  bool wide = false;  // may launch the wide grid (k_unmask_auto)
  bool runs = true;   // the v5 path's counter runs (else one contiguous run per workgroup)
};
// Variant 0 is the default (gevws_ctx_set_tuning(ctx, GEVWS_TUNE_UNMASK_VARIANT, i)).
// The measurement variants of rounds 1-3 (v3 / v4 window shapes, interleaved
// searches, phase-profiled builds, other occupancies) are gone from the
// library; their measurements stay in profiles/ and DESIGN.md §5.
const UnmaskVariant kUnmaskVariants[] = {
    {k_unmask_auto5, 16,
     "auto: v3 4-tile windows for batches of equal-size frames, v5 (pipelined 8-tile windows with a chunk -> frame "
     "map and the tile map cached in LDS) otherwise; non-temporal streaming and window loads; a wide grid for a "
     "smaller batch of mixed sizes after one on this context", true},
    {k_unmask_v5, 16, "v5 for every batch (the default's mixed-batch path alone)", true},
    {k_unmask_auto5, 16, "the default with one contiguous run per workgroup on the v5 path (rounds 1-3; measurement)",
     true, false},
};
constexpr int kNumUnmaskVariants = sizeof(kUnmaskVariants) / sizeof(kUnmaskVariants[0]);

}  // namespace

namespace gevws_impl {

int unmask_variant_count() { return kNumUnmaskVariants; }
const char* unmask_variant_name(int i) { return i >= 0 && i < kNumUnmaskVariants ? kUnmaskVariants[i].name : nullptr; }

int launch_unmask(gevws_ctx* ctx, hipStream_t st, uint64_t payload_cap, const uint8_t* d_in,
                  const gevws_frame* d_frames, const uint32_t* tile_first, const gevws_summary* d_summary,
                  uint8_t* d_payload) {
  const UnmaskVariant& v = kUnmaskVariants[ctx->unmask_variant];
  const uint64_t ntiles = (payload_cap + kTile - 1) / kTile;
  const uint32_t ucus = (uint32_t)ctx->num_cus;
  const uint64_t norm = 4 * (uint64_t)ucus;
  // the wide grid (kWideGridPerCU per CU) when the previous decode on this
  // context was a batch of mixed sizes (run frames < half) below
  // kWideGridTiles; the kernel still uses `norm` workgroups unless this
  // batch is one too
  const bool wide = v.wide && !ctx->unmask_grid && ctx->stats_known && ctx->prev_mixed &&
                    ntiles < kWideGridTiles && norm <= 0xffffu;
  uint64_t grid = ctx->unmask_grid ? (uint64_t)ctx->unmask_grid : wide ? kWideGridPerCU * (uint64_t)ucus : norm;
  const uint64_t useful = (ntiles + v.unroll - 1) / v.unroll;
  if (grid > useful) grid = useful;
  if (grid < 1) grid = 1;
  ctx->last_unmask_grid = (uint32_t)grid;
  v.fn<<<(uint32_t)grid, kUnmaskBlock, 0, st>>>(d_in, d_frames, tile_first, d_summary, d_payload,
                                                ctx->unmask_grid ? 0u : ucus | (wide ? (uint32_t)norm << 16 : 0u),
                                                v.runs ? ctx->unmask_runs : nullptr);
  return GEVWS_OK;
}

}  // namespace gevws_impl

using namespace gevws_impl;

extern "C" {

int gevws_copy_async(gevws_ctx* ctx, void* stream, uint8_t* d_dst, const uint8_t* d_src, uint64_t n,
                     uint32_t grid) {
  if (!ctx || (n && (!d_dst || !d_src))) return GEVWS_ERR_INVALID;
  if (grid & 0x80000000u) return GEVWS_ERR_INVALID;  // no such flag (ABI 2: unknown bits are rejected)
  // bit 30: plain loads (else non-temporal); bit 29: the unmask's
  // wave-contiguous spans (else tile-strided lanes); bit 28: plain stores to
  // a destination of any alignment (else non-temporal, 16-aligned)
  // bit 27: non-temporal stores to a destination of any alignment
  const bool plain = grid & 0x40000000u, wspan = grid & 0x20000000u, pstore = grid & 0x10000000u,
             anyal = pstore || (grid & 0x08000000u);
  if ((n & 15) || (!anyal && (reinterpret_cast<uint64_t>(d_dst) & 15))) return GEVWS_ERR_INVALID;
  if (n == 0) return GEVWS_OK;
  DeviceGuard g(ctx->device);
  hipStream_t st = pick_stream(ctx, stream);
  grid &= 0x07ffffffu;
  if (grid == 0) grid = (uint32_t)ctx->num_cus;
  auto k = pstore ? (plain ? k_copy_stream<16, false, false, true> : k_copy_stream<16, true, false, true>)
           : wspan ? (plain ? k_copy_stream<16, false, true> : k_copy_stream<16, true, true>)
                   : (plain ? k_copy_stream<16, false, false> : k_copy_stream<16, true, false>);
  k<<<grid, kUnmaskBlock, 0, st>>>(d_src, d_dst, n);
  GEVWS_HIP(hipGetLastError());
  return GEVWS_OK;
}

int gevws_cipher_async(gevws_ctx* ctx, void* stream, uint8_t* d_p, uint64_t n, const uint8_t mask[4],
                       uint64_t offset) {
  if (!ctx || !mask || (n && !d_p)) return GEVWS_ERR_INVALID;
  if (n == 0) return GEVWS_OK;
  DeviceGuard g(ctx->device);
  hipStream_t st = pick_stream(ctx, stream);
  uint32_t key;
  memcpy(&key, mask, 4);
  const uint64_t a0 = reinterpret_cast<uint64_t>(d_p) & ~uint64_t(15);
  const uint64_t nchunks = (reinterpret_cast<uint64_t>(d_p) + n - a0 + 15) / 16;
  uint64_t grid = (nchunks + 255) / 256;
  if (grid > 4096) grid = 4096;
  k_cipher<<<(uint32_t)grid, 256, 0, st>>>(d_p, n, key, offset, nchunks);
  GEVWS_HIP(hipGetLastError());
  return GEVWS_OK;
}

}  // extern "C"
