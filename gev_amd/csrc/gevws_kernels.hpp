// gevws_kernels.hpp -- device-side building blocks shared by the kernel files
// of libgevws.so (gfx950 / MI355X): common types and constants, the header
// parse of ws.VirtualReadHeader (read.go:19-84), wave / block scans, the
// scan of block partials, and the byte-stream helpers the unmask and the
// encode share.  Every file includes it inside its own anonymous namespace
// copy; nothing here has external linkage.
//
//   gevws_walk.hip    header walk (count / split / bases / record pass) and
//                     the one-launch small-batch decode (read.go + protocol.go:47)
//   gevws_unmask.hip  payload unmask / compaction (cipher.go:14-53, protocol.go:50-55),
//                     ws.Cipher on a device buffer, the copy ceiling
//   gevws_encode.hip  outbound encode (write.go:48-84, frame.go:274-278) and
//                     control-frame dispatch (wrap.go:38-90, util.go:27-85)
//   gevws_device.hip  the context and the C ABI of include/gevws.h, synth / verify
//
// No MFMA anywhere: this is a byte stream, not a contraction.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>

#include "gevws.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

namespace {

constexpr int kWalkBlock = 256;
// The counting walk and the per-connection bases run one wave per workgroup
// over `cpb` <= 64 connections each: small batches spread their few chains
// over every CU (one chain's dependent loads share a CU's memory pipeline with
// fewer others), big ones keep 64 per workgroup.
constexpr int kCountBlock = 64;
constexpr int kScanBlock = 1024;
constexpr int kUnmaskBlock = 256;
constexpr uint64_t kTile = GEVWS_TILE;
static_assert(kTile == kUnmaskBlock * 16, "one tile = one 16-byte chunk per lane");
constexpr int kBlkFields = 4;  // frames, padded payload bytes, payload length, errors
// decode partials: the four above + frames of a connection's equal-size runs
// (the size of the frame before them on the connection) -> summary.run_frames
constexpr int kDecFields = 5;
// up to this many walk blocks the last one to finish scans the partials
// (no separate k_scan_blocks launch); more take the scan kernel: every block
// counts itself with an atomic on one address, and 1 024 of them serialise
// for longer than the launch they save (C1-shaped batch: walk + scan 46 ->
// 54 us fused; 256 blocks -- C2, C3, C5, an 8-way C4 share -- save 4-8 us)
constexpr uint32_t kFusedScanMaxBlocks = 256;
// their partials as tagged granules (gevws_walk.hip, hand-offs): two per field
constexpr size_t kWalkPartBytes = (size_t)kFusedScanMaxBlocks * kDecFields * 2 * sizeof(uint64_t);

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ u32x4 ld16u(const uint8_t* p) {
  u32x4 v;
  __builtin_memcpy(&v, p, 16);  // gfx950 unaligned global_load_dwordx4
  return v;
}

__device__ __forceinline__ uint64_t round16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

__device__ __forceinline__ u32x4 keep_bytes(u32x4 x, int64_t rem) {
  // zero bytes at positions >= rem (rem in 1..15): Go's make() zero-fill of the pad
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t valid = rem - 4 * j;
    const uint32_t m = valid >= 4 ? 0xffffffffu : (valid <= 0 ? 0u : ((1u << (8 * valid)) - 1u));
    x[j] &= m;
  }
  return x;
}

// 32-bit field starting at byte `off` (0..12) of the 16-byte window lo|hi.
__device__ __forceinline__ uint32_t window32(uint64_t lo, uint64_t hi, uint32_t off) {
  const uint32_t sh = off * 8;
  uint64_t x = (sh == 0) ? lo : (sh < 64 ? ((lo >> sh) | (hi << (64 - sh))) : (hi >> (sh - 64)));
  return (uint32_t)x;
}

static_assert(sizeof(gevws_frame) == 32 && offsetof(gevws_frame, payload_off) == 16 &&
                  offsetof(gevws_frame, src_off) == 24, "emit_record writes gevws_frame as two 16-byte halves");

struct DevHdr {
  uint32_t b0;
  uint32_t masked;
  uint32_t mask;  // little-endian key bytes
  uint32_t hlen;
  uint64_t length;
};

// ws.VirtualReadHeader (read.go:19-84) on the 16 bytes at the cursor.
// avail < 6 -> NEED_MORE (read.go:20-23); FIN/RSV/opcode (read.go:29-31);
// MASK + len7 (read.go:33-49); BE16/BE64 extended length (read.go:60-77) with
// the MSB check (read.go:71-73); key = last 4 header bytes (read.go:78-81).
// avail < header length (Appendix A U1, ringbuffer-dependent in the reference)
// -> NEED_MORE.
__device__ __forceinline__ int parse_header(uint64_t lo, uint64_t hi, uint64_t avail, DevHdr& h) {
  if (avail < 6) return GEVWS_NEED_MORE;
  const uint32_t b0 = (uint32_t)(lo & 0xff);
  const uint32_t b1 = (uint32_t)((lo >> 8) & 0xff);
  const uint32_t masked = b1 >> 7;
  const uint32_t len7 = b1 & 0x7f;
  const uint32_t ext = len7 < 126 ? 0u : (len7 == 126 ? 2u : 8u);
  const uint32_t hlen = 2 + ext + 4 * masked;
  if (avail < hlen) return GEVWS_NEED_MORE;
  uint64_t L;
  if (len7 < 126) {
    L = len7;
  } else if (len7 == 126) {
    L = (((lo >> 16) & 0xff) << 8) | ((lo >> 24) & 0xff);
  } else {
    L = __builtin_bswap64((lo >> 16) | (hi << 48));  // header bytes 2..9, big-endian
    if (L >> 63) return GEVWS_ERR_LEN_MSB;
  }
  h.b0 = b0;
  h.masked = masked;
  h.mask = masked ? window32(lo, hi, 2 + ext) : 0u;
  h.hlen = hlen;
  h.length = L;
  return GEVWS_OK;
}

template <bool NT = false>
__device__ __forceinline__ void load_window(const uint8_t* p, uint64_t& lo, uint64_t& hi) {
  u32x4 v;
  if constexpr (NT) v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));  // unaligned nt load
  else v = ld16u(p);
  lo = (uint64_t)v[0] | ((uint64_t)v[1] << 32);
  hi = (uint64_t)v[2] | ((uint64_t)v[3] << 32);
}

typedef unsigned __int128 u128;

__device__ __forceinline__ u128 u128_of(u32x4 v) {
  return (u128)v[0] | ((u128)v[1] << 32) | ((u128)v[2] << 64) | ((u128)v[3] << 96);
}
__device__ __forceinline__ u32x4 u32x4_of(u128 x) {
  return u32x4{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)(x >> 64), (uint32_t)(x >> 96)};
}

// Wave-level (64 lanes) inclusive scan of a u64.
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}

// Block exclusive scan of NV u64 values per thread (blockDim.x = BS; every
// lane of the workgroup calls it).  Returns exclusive prefixes in ex[],
// block totals in tot[].  DPP wave scans (wave_incl_scan64_dpp, below) and
// one LDS exchange of the wave totals: the shuffle form's ds_bpermute round
// trips cost the one-launch decode 2.5 us of a 100-connection pass
// (profiles/r06/README.md, r06z / r06aa).
template <int BS, int NV>
__device__ __forceinline__ void block_excl_scan(const uint64_t (&v)[NV], uint64_t (&ex)[NV],
                                                uint64_t (&tot)[NV]);

// Wave64 inclusive scans by DPP (no LDS round trips; every lane active):
// row_shr 1 / 2 / 4 / 8 scan each row of 16 lanes (lanes shifted in from
// outside the row read 0: bound_ctrl), then row_bcast:15 adds row 0's total
// into row 1 and row 2's into row 3, and row_bcast:31 adds lane 31's running
// total into rows 2 and 3 (the masked-off rows keep `old` = 0).  The shuffle
// forms above cost a ds_bpermute (an LDS round trip) per step and 32-bit half.
template <int CTRL, int ROWS, bool BOUND>
__device__ __forceinline__ uint32_t dpp32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xf, BOUND);
}
template <int CTRL, int ROWS, bool BOUND>
__device__ __forceinline__ uint64_t dpp64(uint64_t x) {
  return (uint64_t)dpp32<CTRL, ROWS, BOUND>((uint32_t)x) | ((uint64_t)dpp32<CTRL, ROWS, BOUND>((uint32_t)(x >> 32)) << 32);
}
__device__ __forceinline__ uint32_t wave_incl_scan32_dpp(uint32_t x) {
  x += dpp32<0x111, 0xf, true>(x);   // row_shr:1
  x += dpp32<0x112, 0xf, true>(x);   // row_shr:2
  x += dpp32<0x114, 0xf, true>(x);   // row_shr:4
  x += dpp32<0x118, 0xf, true>(x);   // row_shr:8
  x += dpp32<0x142, 0xa, false>(x);  // row_bcast:15 -> rows 1, 3
  x += dpp32<0x143, 0xc, false>(x);  // row_bcast:31 -> rows 2, 3
  return x;
}
__device__ __forceinline__ uint64_t wave_incl_scan64_dpp(uint64_t x) {
  x += dpp64<0x111, 0xf, true>(x);
  x += dpp64<0x112, 0xf, true>(x);
  x += dpp64<0x114, 0xf, true>(x);
  x += dpp64<0x118, 0xf, true>(x);
  x += dpp64<0x142, 0xa, false>(x);
  x += dpp64<0x143, 0xc, false>(x);
  return x;
}

template <int BS, int NV>
__device__ __forceinline__ void block_excl_scan(const uint64_t (&v)[NV], uint64_t (&ex)[NV],
                                                uint64_t (&tot)[NV]) {
  constexpr int NW = BS / 64;
  __shared__ uint64_t s_w[NV][NW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t inc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    inc[k] = wave_incl_scan64_dpp(v[k]);
    if (lane == 63) s_w[k][w] = inc[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    uint64_t before = 0, all = 0;
#pragma unroll
    for (int j = 0; j < NW; ++j) {  // (broadcast LDS reads: every lane the same word)
      const uint64_t t = s_w[k][j];
      before += j < w ? t : 0u;
      all += t;
    }
    ex[k] = before + inc[k] - v[k];
    tot[k] = all;
  }
  __syncthreads();
}

// Block exclusive scan of NV u32 values per thread (blockDim.x = BS) on DPP
// wave scans: one LDS exchange of the wave totals.  For sums known to fit
// 32 bits (the one-launch decode's, whose input is at most 128 KiB).
template <int BS, int NV>
__device__ __forceinline__ void block_excl_scan32(const uint32_t (&v)[NV], uint32_t (&ex)[NV], uint32_t (&tot)[NV]) {
  constexpr int NW = BS / 64;
  __shared__ uint32_t s_w[NV][NW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    inc[k] = wave_incl_scan32_dpp(v[k]);
    if (lane == 63) s_w[k][w] = inc[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int j = 0; j < NW; ++j) {  // (broadcast LDS reads: every lane the same word)
      const uint32_t t = s_w[k][j];
      before += j < w ? t : 0u;
      all += t;
    }
    ex[k] = before + inc[k] - v[k];
    tot[k] = all;
  }
  __syncthreads();
}

// threadIdx.x as a fresh value the compiler cannot hoist or keep live across
// a loop: addresses derived from it are recomputed where they are used
// instead of being held in (and spilled from) registers.
__device__ __forceinline__ uint32_t fresh_tid() {
  uint32_t t = threadIdx.x;
  __asm__ volatile("" : "+v"(t));
  return t;
}

// A value every lane of the wave loaded from the same address, kept in SGPRs
// (the compiler cannot always prove such loads uniform once the loop stores).
__device__ __forceinline__ uint32_t uniform32(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
  return (uint64_t)uniform32((uint32_t)x) | ((uint64_t)uniform32((uint32_t)(x >> 32)) << 32);
}

// ------------------------------------------------------------------ 2. scan of block partials
// SPLIT (decode): field 3 holds errors in its low 32 bits and the count of
// out-of-order connections in its high 32 (k_walk_count) -> summary.errors and
// GEVWS_SUMMARY_UNORDERED.
// BS: the workgroup (the decode's scan runs 256 threads: a workgroup of 4
// waves finds room on a CU beside another batch's unmask, 16 waves do not).
template <bool SPLIT, int NF = kBlkFields, int BS = kScanBlock>
__global__ __launch_bounds__(BS) void k_scan_blocks(uint64_t* __restrict__ blk, uint32_t nblk,
                                                    uint64_t max_frames, uint64_t payload_cap,
                                                    gevws_summary* __restrict__ sum) {
  // kScanPer consecutive partials per thread: a batch of per-frame blocks
  // (encode / dispatch of 43.8 M frames: 171 K partials) takes a few rounds of
  // the workgroup instead of one round per 1 024 partials
  constexpr int kScanPer = 8;
  uint64_t carry[NF] = {};
  for (uint64_t base = 0; base < nblk; base += (uint64_t)BS * kScanPer) {
    const uint64_t i0 = base + (uint64_t)threadIdx.x * kScanPer;
    uint64_t loc[NF] = {}, ex[NF], tot[NF];
#pragma unroll
    for (int r = 0; r < kScanPer; ++r)
#pragma unroll
      for (int k = 0; k < NF; ++k) loc[k] += (i0 + r < nblk) ? blk[(i0 + r) * NF + k] : 0;
    block_excl_scan<BS, NF>(loc, ex, tot);
    // fields 0/1 become exclusive bases (frames, arena bytes)
    uint64_t b0 = carry[0] + ex[0], b1 = carry[1] + ex[1];
#pragma unroll
    for (int r = 0; r < kScanPer; ++r) {
      if (i0 + r < nblk) {  // re-read (cached) rather than held across the scan: register budget
        uint64_t* p = blk + (i0 + r) * NF;
        const uint64_t f0 = p[0], f1 = p[1];
        p[0] = b0;
        p[1] = b1;
        b0 += f0;
        b1 += f1;
      }
    }
#pragma unroll
    for (int k = 0; k < NF; ++k) carry[k] += tot[k];
  }
  if (threadIdx.x == 0) {
    gevws_summary s;
    memset(&s, 0, sizeof(s));
    s.frames = carry[0];
    s.payload_bytes = carry[1];
    s.payload_len = carry[2];
    s.errors = SPLIT ? (carry[3] & 0xffffffffull) : carry[3];
    s.flags = (SPLIT && (carry[3] >> 32)) ? GEVWS_SUMMARY_UNORDERED : 0u;
    if constexpr (NF > 4) s.run_frames = carry[4];
    s.status = (carry[0] > max_frames || carry[1] > payload_cap) ? GEVWS_ERR_CAPACITY : GEVWS_OK;
    *sum = s;
  }
}

// ------------------------------------------------------------------ one-launch passes
// The small-batch decode (k_decode_small, gevws_walk.hip) and the one-launch
// handler step (k_handle_small, gevws_encode.hip) run in ONE workgroup.  The
// decode has two shapes: 256 lanes and 64 KiB of input staged in LDS (a loop's
// usual pass), and 1 024 lanes and 128 KiB (146 KB of the 160 KiB LDS: passes
// of up to 1 024 connections, e.g. the 4 000-connection live shape's ~500).
constexpr uint32_t kSmallConns = 256;
constexpr uint64_t kSmallBytes = 64 * 1024;
constexpr uint32_t kOneLaunchConns = GEVWS_ONE_LAUNCH_MAX_CONNS;
constexpr uint64_t kOneLaunchBytes = GEVWS_ONE_LAUNCH_MAX_BYTES;
static_assert(kOneLaunchConns == 1024 && kOneLaunchBytes == 128 * 1024, "k_decode_small's wide shape");
// A live pass's last kernel announces its end in mapped host memory: every
// thread's writes (records, payload, summaries) are fenced at system scope,
// then one lane stores `seq` with a system-scope release (a vector store), so
// a host that sees the flag sees the results -- it spins on host memory
// instead of waiting in hipStreamSynchronize (gevws_ctx_set_completion_flag).
// Before the flag, with `ticks` set (gevws_ctx_set_timeline_ticks), thread 0
// also stores the kernel's start tick t0 and its end tick (s_memrealtime, the
// GPU's constant-rate wall clock) at ticks[2 slot], ticks[2 slot + 1] (slot 0:
// the decode, 1: the handler step): the host's per-pass timeline
// (gevws_protocol_get_timeline).  Callers reach it with the whole workgroup
// (it holds a barrier).
__device__ __forceinline__ uint64_t gpu_ticks() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ void signal_done(uint32_t* done, uint32_t seq, uint64_t* ticks = nullptr, uint64_t t0 = 0,
                                            int slot = 0) {
  if (!done) return;
  if (ticks && threadIdx.x == 0) {
    ticks[2 * slot] = t0;
    ticks[2 * slot + 1] = gpu_ticks();
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------------ split walk bounds (host defaults too)
constexpr uint64_t kSplitMinBytes = 16384;        // a connection's segments are at least this long
constexpr uint32_t kSplitMaxLanes = 32;
constexpr uint64_t kSplitLanesPerCU = 512;        // auto: split while the walk has fewer lanes per CU

// ------------------------------------------------------------------ unmask / encode byte streams
// Streams of big frames run fastest with one workgroup per CU (fewer
// concurrent streams: better DRAM row locality); small frames need more
// workgroups to hide the window path's latency (profiles/r01/r01_grid_*.json).  The
// batch's mean frame size is only known on the device, so kernels are launched
// with 4 workgroups per CU and, for big frames, all but the first `big_grid`
// return at once.  big_grid = 0 disables the adaptation (explicit grid).
constexpr uint64_t kBigFrameBytes = 48 * 1024;
// k_unmask_auto5's wide grid (kWideGridPerCU workgroups per CU instead of 4),
// launched when the context's previous decode was a batch of mixed frame
// sizes below kWideGridTiles output tiles: there the contiguous runs of 4
// workgroups per CU finish unevenly (the window path's cost follows the local
// frame density) and more, shorter runs balance -- C4's 8-way share (590 K
// tiles) 1.15 -> 0.99 ms, its 4-way share (1.2 M) 2.15 -> 2.09; the 2-way
// share (2.4 M), the full C4 (4.7 M tiles), C2, C3, C5 are best at 4 per CU
// (profiles/r02/r02_grid_sweep.jsonl)
constexpr uint32_t kWideGridPerCU = 32;
constexpr uint64_t kWideGridTiles = 2ull << 20;
// The unmask v5 path's runs: the workgroups of each XCD (blockIdx.x mod 8, the
// dispatch's round robin) take runs of kUnmaskRun tiles of their eighth of the
// output from one counter (k_walk_bases zeroes them) instead of one contiguous
// run each -- a run's cost follows the local frame density, and short runs
// even it out (C4 7.44 -> 6.90 ms, its 2-way share 4.28 -> 3.72, 4-way 2.05
// -> 1.86; runs of 32 / 64 tiles in between; profiles/r04/r04_unmask_counter_ab.jsonl).
// One counter per XCD: one for the whole grid saturates (k_encode6 measured it).
constexpr uint32_t kUnmaskRunCounters = 8;
constexpr uint64_t kUnmaskRun = 16;
constexpr uint64_t kUnmaskRunMinTiles = 64;  // the v3 path's counter runs: tiles a workgroup at least

// Workgroups that take a run of the output: big_grid (low 16 bits: one per CU)
// for batches of big frames, else the whole grid -- or, when the host
// launched a wide grid (high 16 bits: the usual grid), the usual grid unless
// the caller asks for the wide one.
__device__ __forceinline__ uint32_t active_groups(uint64_t total, uint64_t nframes, uint32_t big_grid,
                                                  bool wide = false) {
  const uint32_t ncu = big_grid & 0xffffu, norm = big_grid >> 16;
  if (ncu == 0 || gridDim.x <= ncu || nframes == 0) return gridDim.x;
  if (total / nframes >= kBigFrameBytes) return ncu;
  return (norm == 0 || wide || gridDim.x <= norm) ? gridDim.x : norm;
}

template <bool NT>
__device__ __forceinline__ u32x4 ld16u_stream(const uint8_t* p) {
  if constexpr (NT) {
    // unaligned 16-byte nontemporal load (gfx950 unaligned access mode)
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  } else {
    return ld16u(p);
  }
}

__device__ __forceinline__ void st16_nt(uint8_t* p, u32x4 x) {
  __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p));
}

constexpr int kWinTiles = 4;  // a window of the unmask's v3 path and of the encode (tiles)

// Value of `x` in lane+1, lane 63 gets lane 0's (DPP wave_rol:1).
__device__ __forceinline__ u32x4 rot_next_lane(u32x4 x) {
  return u32x4{(uint32_t)__builtin_amdgcn_update_dpp(0, (int)x[0], 0x134, 0xf, 0xf, false),
               (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x[1], 0x134, 0xf, 0xf, false),
               (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x[2], 0x134, 0xf, 0xf, false),
               (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x[3], 0x134, 0xf, 0xf, false)};
}

// Bytes [m, m+16) of the 32-byte concatenation a|b (m in 1..15, wave-uniform).
__device__ __forceinline__ u32x4 funnel16(u32x4 a, u32x4 b, uint32_t m) {
  const uint32_t r = m & 3;
  u32x4 o;
  switch (m >> 2) {
    case 0:
      o = u32x4{__builtin_amdgcn_alignbyte(a[1], a[0], r), __builtin_amdgcn_alignbyte(a[2], a[1], r),
                __builtin_amdgcn_alignbyte(a[3], a[2], r), __builtin_amdgcn_alignbyte(b[0], a[3], r)};
      break;
    case 1:
      o = u32x4{__builtin_amdgcn_alignbyte(a[2], a[1], r), __builtin_amdgcn_alignbyte(a[3], a[2], r),
                __builtin_amdgcn_alignbyte(b[0], a[3], r), __builtin_amdgcn_alignbyte(b[1], b[0], r)};
      break;
    case 2:
      o = u32x4{__builtin_amdgcn_alignbyte(a[3], a[2], r), __builtin_amdgcn_alignbyte(b[0], a[3], r),
                __builtin_amdgcn_alignbyte(b[1], b[0], r), __builtin_amdgcn_alignbyte(b[2], b[1], r)};
      break;
    default:
      o = u32x4{__builtin_amdgcn_alignbyte(b[0], a[3], r), __builtin_amdgcn_alignbyte(b[1], b[0], r),
                __builtin_amdgcn_alignbyte(b[2], b[1], r), __builtin_amdgcn_alignbyte(b[3], b[2], r)};
      break;
  }
  return o;
}

}  // namespace
