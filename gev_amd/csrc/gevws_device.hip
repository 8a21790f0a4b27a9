// gevws_device.hip -- gfx950 (MI355X / CDNA4) kernels and the device half of
// the C ABI declared in include/gevws.h.
//
// Hot path: for a batch of connections, the
// repeated websocket.(*Protocol).UnPacket loop of Connection.handlerProtocol
// (connection.go:208-218 -> plugins/websocket/protocol.go:38-62) is done as
// four stages (five launches) on one stream:
//
//   1. k_walk_count  one lane per connection walks its header chain
//                    (ws.VirtualReadHeader, read.go:19-84, plus the
//                    completeness gate, protocol.go:47), counts frames,
//                    payload bytes and consumed bytes and records a 16-byte
//                    entry per frame; one wave per workgroup, block sums.
//   2. k_scan_blocks one workgroup scans the block partials -> batch totals,
//                    capacity check.
//   3. k_walk_bases  per-connection bases (block-level scan), then
//      k_walk_emit   one wave per connection turns its entries into 32-byte
//                    records (wave scan of the padded lengths -> payload
//                    offsets) and the output-tile -> frame map.
//   4. k_unmask_v4   the byte stream (ws.Cipher, cipher.go:14-53; the key phase
//                    restarts at 0 per frame, protocol.go:54): contiguous runs
//                    of 4 KiB output tiles per workgroup, streamed with aligned
//                    loads while one frame covers 16 tiles, else an LDS window
//                    of frame records searched per 16-byte chunk.  HBM-bound:
//                    h + 2L bytes per frame.
//
// No MFMA: this is a byte stream, not a contraction.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "gevws.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

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

__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}

// Block exclusive scan of NV u64 values per thread (blockDim.x = BS).
// Returns exclusive prefixes in ex[], block totals in tot[].
template <int BS, int NV>
__device__ __forceinline__ void block_excl_scan(const uint64_t (&v)[NV], uint64_t (&ex)[NV],
                                                uint64_t (&tot)[NV]) {
  constexpr int NW = BS / 64;
  __shared__ uint64_t s_w[NV][NW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t inc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    inc[k] = wave_incl_scan(v[k]);
    if (lane == 63) s_w[k][w] = inc[k];
  }
  __syncthreads();
  // lane j reads wave j's total: one LDS load per field instead of NW
  // (unrolled over NV x NW it took 160 VGPRs at NV = 5 and spilled)
  static_assert(NW <= 64, "one lane per wave total");
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const uint64_t sj = lane < NW ? s_w[k][lane] : 0;
    ex[k] = wave_sum(lane < w ? sj : 0) + inc[k] - v[k];
    tot[k] = wave_sum(sj);
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

// The decode's partials scan by ONE wave (the walk's last block, see
// walk_block_done): per round each lane takes 8 consecutive block partials,
// fields 0/1 become exclusive bases (frames, arena bytes) for k_walk_bases,
// every field is totalled into the summary, with the capacity check.
__device__ void scan_partials_wave(uint64_t* __restrict__ blk, uint32_t nblk, uint64_t max_frames,
                                   uint64_t payload_cap, gevws_summary* __restrict__ sum) {
  constexpr int P = 8;
  const int lane = threadIdx.x & 63;
  uint64_t carry[kDecFields] = {0, 0, 0, 0, 0};
  for (uint64_t base = 0; base < nblk; base += 64 * P) {  // wave-uniform
    const uint64_t i0 = base + (uint64_t)lane * P;
    uint64_t loc[kDecFields] = {0, 0, 0, 0, 0};
    uint64_t loc0[P], loc1[P];  // this lane's partials of fields 0 / 1, for the bases
#pragma unroll
    for (int r = 0; r < P; ++r) {
      loc0[r] = (i0 + r < nblk) ? __hip_atomic_load(blk + (i0 + r) * kDecFields, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT) : 0;
      loc1[r] = (i0 + r < nblk) ? __hip_atomic_load(blk + (i0 + r) * kDecFields + 1, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT) : 0;
    }
#pragma unroll
    for (int r = 0; r < P; ++r)
#pragma unroll
      for (int k = 0; k < kDecFields; ++k)
        loc[k] += (i0 + r < nblk) ? __hip_atomic_load(blk + (i0 + r) * kDecFields + k, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT)
                                  : 0;
    const uint64_t inc0 = wave_incl_scan(loc[0]), inc1 = wave_incl_scan(loc[1]);
    uint64_t b0 = carry[0] + inc0 - loc[0], b1 = carry[1] + inc1 - loc[1];
#pragma unroll
    for (int r = 0; r < P; ++r) {
      if (i0 + r < nblk) {
        uint64_t* q = blk + (i0 + r) * kDecFields;
        const uint64_t f0 = loc0[r], f1 = loc1[r];
        q[0] = b0;
        q[1] = b1;
        b0 += f0;
        b1 += f1;
      }
    }
#pragma unroll
    for (int k = 0; k < kDecFields; ++k) carry[k] += wave_sum(loc[k]);
  }
  if (lane == 0) {
    gevws_summary sm;
    memset(&sm, 0, sizeof(sm));
    sm.frames = carry[0];
    sm.payload_bytes = carry[1];
    sm.payload_len = carry[2];
    sm.errors = carry[3] & 0xffffffffull;
    sm.flags = (carry[3] >> 32) ? GEVWS_SUMMARY_UNORDERED : 0u;
    sm.run_frames = carry[4];
    sm.status = (carry[0] > max_frames || carry[1] > payload_cap) ? GEVWS_ERR_CAPACITY : GEVWS_OK;
    *sum = sm;
  }
}

// The last of the walk's workgroups to finish (a device-scope counter) scans
// the partials, so the decode needs no k_scan_blocks launch.  L2 is per XCD
// and not coherent, and a release fence would write back the whole L2 (the
// walk's entry stores: measured 2x slower), so only the partials travel
// coherently: they are stored and loaded as agent-scope atomics (write-through
// / L2-bypassing), each writer waits for its stores before its workgroup counts
// itself, and the last workgroup resets the counter for the context's next call.
__device__ __forceinline__ void put_partial(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void walk_block_done(uint32_t* __restrict__ done, uint32_t nblk, uint64_t* __restrict__ blk,
                                                uint64_t max_frames, uint64_t payload_cap,
                                                gevws_summary* __restrict__ sum, bool wrote) {
  __shared__ uint32_t s_last;
  if (wrote) __builtin_amdgcn_s_waitcnt(0);  // the partials' write-through stores are done
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblk - 1 ? 1u : 0u;
  __syncthreads();
  if (s_last) {
    if (threadIdx.x < 64) scan_partials_wave(blk, nblk, max_frames, payload_cap, sum);
    if (threadIdx.x == 0) __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ------------------------------------------------------------------ 1. walk (count)
// Frame entries recorded by the counting walk so the emit pass need not
// re-fetch every header line from HBM: 8 bytes per frame in a per-connection
// slot run whose base derives from the stream's arena offset (no scan needed):
// base_c = S (off_c / SG + c), capacity S (len_c / SG + 1) with S = kSlotAlign
// = 32, the granularity G the smallest power of two >= 64 B that keeps the
// table within kEntryBudget; runs start on 256-byte boundaries, so the walk can
// store its entries as whole groups (the LDS-ring writer: 256 bytes of 32).
// The runs are
// disjoint when the whole table is in increasing input order with no overlap
// (for c < d: base_c + cap_c <= S ((off_c + len_c) / SG + 1 + c) <= base_d);
// a neighbour check per connection cannot establish that (an
// unsorted table can pass every local check and still collide), so every
// workgroup reports whether any of its connections starts before the previous
// one ends, k_scan_blocks ORs that into summary.flags, and on an unordered
// table the emit pass ignores the entries and re-walks every chain.  Entries
// are written either way: base + cap <= n_entries holds for any table, so the
// stores stay inside the table.  A connection whose frames outnumber its slots
// (mean frame < G bytes) or whose stream is >= 4 GiB is re-walked too.
constexpr uint64_t kWriterChainsPerCU = 128;  // k_walk_count ST 2 (the writer wave) from n_conns >= this x CUs
constexpr uint32_t kEntryGranMinShift = 6;        // 64-byte granularity when the table fits
constexpr uint64_t kEntryBudget = 1ull << 29;     // entries (8 GiB of scratch) at most
// slot runs start on 32-entry (256-byte) boundaries: the writer wave of the
// LDS-ring walk stores whole 256-byte groups (k_walk_count ST 2)
constexpr uint32_t kSlotShift = 5;
constexpr uint64_t kSlotAlign = 1ull << kSlotShift;
// 8-byte entry: the key, and b0 | masked << 8 | length form << 9 | payload
// length << 11.  The header's position is not stored: a row's frames are
// contiguous from its start, so the record pass recomputes each position as
// the prefix sum of the frame sizes before it (hlen + L).  A payload length
// >= kLenEsc is stored as kLenEsc and re-read from the header by the record
// pass, where the prefix sum gives its position (rare: frames of 2 MiB and
// more, whose unmask dwarfs one header load).  Round 2's 16-byte entry
// (position, key, length, meta) cost the walk 0.71 GB of C4's writes and the
// record pass as many reads (profiles/r03/r03_pmc_split.json).
constexpr uint32_t kLenEsc = (1u << 21) - 1;
struct WalkEntry {
  uint32_t mask;
  uint32_t w;
};
static_assert(sizeof(WalkEntry) == 8, "one dwordx2 per entry");
// meta: b0 | masked << 8 | hlen << 16 (walk_parse / walk_chain)
__device__ __forceinline__ WalkEntry make_entry(uint32_t key, uint64_t L, uint32_t meta) {
  const uint32_t hlen = meta >> 16, masked = (meta >> 8) & 1u;
  const uint32_t ext = hlen - 2 - 4 * masked;  // 0, 2 or 8 length bytes
  const uint32_t form = ext == 0 ? 0u : (ext == 2 ? 1u : 2u);
  const uint32_t l21 = L < kLenEsc ? (uint32_t)L : kLenEsc;
  return WalkEntry{key, (meta & 0x1ffu) | (form << 9) | (l21 << 11)};
}
__device__ __forceinline__ uint32_t entry_hlen(const WalkEntry& e) {
  const uint32_t form = (e.w >> 9) & 3u;
  return 2 + (form == 2 ? 8u : 2u * form) + 4 * ((e.w >> 8) & 1u);
}
__device__ __forceinline__ uint32_t entry_len21(const WalkEntry& e) { return e.w >> 11; }

__device__ __forceinline__ bool entry_slots_of(const gevws_conn_in& ci, uint32_t c, uint64_t n_entries,
                                              uint32_t gshift, uint64_t& base, uint64_t& cap) {
  if (n_entries == 0 || ci.len >= (1ull << 32)) return false;
  base = kSlotAlign * ((ci.off >> (gshift + kSlotShift)) + (uint64_t)c);
  cap = kSlotAlign * ((ci.len >> (gshift + kSlotShift)) + 1);
  return base + cap <= n_entries;
}

// Connection c breaks the increasing, non-overlapping order the slot runs rely
// on (its stream starts before the previous one ends).
__device__ __forceinline__ bool out_of_order(const gevws_conn_in* __restrict__ conns, uint32_t c,
                                             const gevws_conn_in& ci) {
  if (c == 0) return false;
  const gevws_conn_in p = conns[c - 1];
  return ci.off < p.off || ci.off - p.off < p.len;
}

// The counting walk's header parse (read.go:19-84 + the protocol.go:47 gate)
// on the 16-byte window at a frame start with `avail` bytes buffered from it:
// OK, NEED_MORE (fewer than 6 / header / payload bytes) or ERR_LEN_MSB.
__device__ __forceinline__ int walk_parse(uint64_t lo, uint64_t hi, uint64_t avail, uint32_t& meta, uint32_t& hlen,
                                          uint64_t& L, uint32_t& key) {
  const uint32_t b1 = (uint32_t)(lo >> 8) & 0xffu;
  const uint32_t masked = b1 >> 7, len7 = b1 & 0x7fu;
  const bool e16 = len7 == 126, e64 = len7 == 127;
  hlen = 2 + (e64 ? 8u : (e16 ? 2u : 0u)) + 4 * masked;
  const uint64_t L64 = __builtin_bswap64((lo >> 16) | (hi << 48));
  const uint64_t L16 = (((lo >> 16) & 0xff) << 8) | ((lo >> 24) & 0xff);
  L = e64 ? L64 : (e16 ? L16 : (uint64_t)len7);
  key = (e64 ? (uint32_t)(hi >> 16) : (e16 ? (uint32_t)(lo >> 32) : (uint32_t)(lo >> 16))) & (0u - masked);
  meta = ((uint32_t)lo & 0xffu) | (masked << 8) | (hlen << 16);
  const bool have_hdr = avail >= 6 && avail >= hlen;
  if (have_hdr && e64 && (L64 >> 63)) return GEVWS_ERR_LEN_MSB;
  return (have_hdr && avail - hlen >= L) ? GEVWS_OK : GEVWS_NEED_MORE;
}

// D > 0: uniform-stream speculation.  After three consecutive frames of equal
// size F the lane requests the windows at pos, pos + F, ..., pos + (D-1)F
// (within the stream) at once and parses them in order while the frames keep
// size F, so a run of equal-size frames costs one memory latency per D frames
// instead of one per frame.  The first frame of another size ends the batch
// (the windows after it are dropped) and the walk goes on from the true
// position, so the result never depends on the guess.  Requiring three equal
// frames keeps the batch path (and the wave divergence it costs) out of
// mixed-size traffic.  Interleaved A/B against D = 0
// (profiles/r01/r01_ab_walk2_*.json): the walk of fixed-size traffic takes 23-28 %
// less time (C2, C3), mixed traffic 0-5 % more (C4, C5: a longer loop body on
// a latency-bound chain), so the host runs D = 0 after a mixed batch.
// The chain walk of one stream (k_walk_count's loop; also each segment of
// k_walk_split): entries into [ebase, ebase + ecap) while rec, per-frame
// counts into R (R.err / R.st carry in the caller's values).
struct WalkRes {
  uint64_t pos, nf, pb, pl, same, lastf, firstf, err;
  int32_t st;
  bool rec;
};
__device__ __forceinline__ WalkRes walk_res_fresh(uint64_t err = 0, int32_t st = GEVWS_OK) {
  WalkRes R;
  R.pos = R.nf = R.pb = R.pl = R.same = R.firstf = 0;
  R.lastf = ~0ull;
  R.err = err;
  R.st = st;
  R.rec = false;
  return R;
}

// ST: where entries go.  0 = global memory, one 8-byte store per frame from the
// walking lane (batches of few chains: latency-bound, the stores overlap the
// next header load); 2 = this lane's LDS ring (WalkRing), drained to global
// memory by the workgroup's writer wave (k_walk_count ST 2): the walker then
// issues no global stores at all, so waiting for its header load (vmcnt counts
// loads and stores in order) never waits for an entry store.  Batches of many
// chains, whose walk is bound by line traffic: single entry stores scattered
// among the random header reads cost far more than their bytes (C4: 1.60 ms
// against 1.00 without entries, 1.26 through the writer;
// profiles/r03/r03_walk_writer_grp_ab.jsonl, r03_compact_entries_ab.jsonl).
constexpr uint32_t kRingDone = 0x80000000u;   // head flag: the chain is finished
constexpr uint32_t kWriterGroup = 32;         // entries per writer store group (256 bytes)
constexpr uint32_t kRing = 2 * kWriterGroup;  // entries per lane's LDS ring
struct WalkRing {
  WalkEntry* e;    // kRing entries (LDS)
  uint32_t* head;  // entries published (whole groups of 4; | kRingDone with the count at the end)
  uint32_t* tail;  // entries the writer has taken
};
__device__ __forceinline__ uint32_t lds_ld(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int D, int ST = 0>
__device__ __forceinline__ void walk_chain(const uint8_t* __restrict__ s, const uint64_t len, bool rec,
                                           const uint64_t ebase, const uint64_t ecap,
                                           WalkEntry* __restrict__ entries, WalkEntry* __restrict__ sink,
                                           WalkRes& R, WalkRing ring = WalkRing{nullptr, nullptr, nullptr}) {
    static_assert(ST == 0 || ST == 2, "entries from the lane or through the writer wave");
    uint64_t nf = R.nf, pb = R.pb, pl = R.pl, same = R.same, lastf = R.lastf, firstf = R.firstf, err = R.err;
    int32_t st = R.st;
    uint64_t pos = R.pos;
    // software-pipelined: the next header's 16 bytes are requested before this
    // frame's entry is stored, so waiting for that load (vmcnt counts loads and
    // stores in issue order) never waits for the store's completion.  Reading
    // 16 bytes at any pos <= len stays inside the GEVWS_IN_PAD slack.
    // Every path into the loop head has exactly [header load, entry store]
    // outstanding (lanes not recording store to their own sink slot past the
    // table), so the compiler waits vmcnt(1), not vmcnt(0).
    uint64_t lo, hi;
    load_window(s + pos, lo, hi);
    if constexpr (ST == 0) *sink = WalkEntry{0, 0};
    uint64_t prev_fsz = 0;  // speculation (D > 0): size of the last frame and the run of equal sizes
    uint32_t run = 0;
    auto put_entry = [&](uint32_t key, uint64_t L, uint32_t meta) {
      rec = rec && nf < ecap;
      const WalkEntry e = make_entry(key, L, meta);
      if constexpr (ST == 2) {
        // room for this group in the ring? (the writer is normally far ahead:
        // it copies a group in a few hundred cycles, a step takes ~1 us)
        if ((nf & 3) == 0)
          while ((uint32_t)nf + 4 - lds_ld(ring.tail) > kRing) __builtin_amdgcn_s_sleep(1);
        ring.e[nf & (kRing - 1)] = e;
        __asm__ volatile("" ::: "memory");  // the entry before the head that publishes it (DS ops run in order)
        if ((nf & 3) == 3) lds_st(ring.head, (uint32_t)nf + 1);
      } else {
        *(rec ? entries + ebase + nf : sink) = e;
      }
      ++nf;
      pb += round16(L);
      pl += L;
      const uint64_t f = (uint64_t)(meta >> 16) + L;  // frame size (hlen + L)
      same += f == lastf;
      firstf = lastf == ~0ull ? f : firstf;
      lastf = f;
    };
    // One chain step on the window (clo, chi) at pos; the next header's window
    // is loaded into (nlo, nhi).  false: the chain ends here.
    auto step = [&](const uint64_t clo, const uint64_t chi, uint64_t& nlo, uint64_t& nhi) -> bool {
      // The chain is latency-bound (one load per frame, few lanes per SIMD):
      // only the next frame's position is computed before its header load is
      // issued -- at min(next, len), always inside the stream + GEVWS_IN_PAD
      // -- and the checks run while that load is in flight.
      const uint32_t b1 = (uint32_t)(clo >> 8) & 0xffu;
      const uint32_t masked = b1 >> 7, len7 = b1 & 0x7fu;
      const bool e16 = len7 == 126, e64 = len7 == 127;
      const uint32_t hlen = 2 + (e64 ? 8u : (e16 ? 2u : 0u)) + 4 * masked;
      const uint64_t L64 = __builtin_bswap64((clo >> 16) | (chi << 48));
      const uint64_t L16 = (((clo >> 16) & 0xff) << 8) | ((clo >> 24) & 0xff);
      const uint64_t L = e64 ? L64 : (e16 ? L16 : (uint64_t)len7);
      const uint64_t fsz = hlen + L;
      const uint64_t next = pos + fsz;
      load_window(s + (next <= len ? next : len), nlo, nhi);  // (a wrapped next is <= len or clamped)
      const uint64_t avail = len - pos;
      const bool have_hdr = avail >= 6 && avail >= hlen;   // read.go:20-23, U1
      const bool msb = e64 && (L64 >> 63);                  // read.go:71-73
      if (!have_hdr || msb || avail - hlen < L) {           // protocol.go:47 gate
        if (have_hdr && msb) { st = GEVWS_ERR_LEN_MSB; err += 1; }
        return false;
      }
      const uint32_t key = (e64 ? (uint32_t)(chi >> 16) : (e16 ? (uint32_t)(clo >> 32) : (uint32_t)(clo >> 16))) &
                           (0u - masked);
      const uint32_t meta = ((uint32_t)clo & 0xffu) | (masked << 8) | (hlen << 16);
      put_entry(key, L, meta);
      pos = next;
      if constexpr (D > 0) {
        run = fsz == prev_fsz ? run + 1 : 1;
        prev_fsz = fsz;
        if (run >= 3) {
          // third equal frame in a row: take the following frames in batches
          // of D windows at stride fsz while their size stays fsz; (nlo, nhi),
          // in flight, is the window at pos
          bool fail = false;
          for (;;) {
            // unconditional loads (addresses clamped to the stream end: 16
            // bytes at any q <= len stay inside GEVWS_IN_PAD); the first qn
            // windows are real
            uint64_t qlo[D], qhi[D];
            uint32_t qn = 1;  // windows at positions <= len (pos itself is)
#pragma unroll
            for (int j = 1; j < D; ++j) {
              const uint64_t q = pos + (uint64_t)j * fsz;
              const bool in = q <= len;
              qn += in ? 1u : 0u;
              load_window(s + (in ? q : len), qlo[j], qhi[j]);
            }
            qlo[0] = nlo;
            qhi[0] = nhi;
            bool stop = false;
#pragma unroll
            for (int j = 0; j < D; ++j) {
              if (!stop && (uint32_t)j < qn) {
                uint32_t m2, h2, k2;
                uint64_t L2;
                const int r = walk_parse(qlo[j], qhi[j], len - pos, m2, h2, L2, k2);
                if (r != GEVWS_OK) {
                  if (r == GEVWS_ERR_LEN_MSB) { st = GEVWS_ERR_LEN_MSB; err += 1; }
                  fail = stop = true;
                } else {
                  put_entry(k2, L2, m2);
                  pos += h2 + L2;
                  if (h2 + L2 != fsz) {
                    stop = true;
                    run = 1;
                    prev_fsz = h2 + L2;
                  }
                }
              }
            }
            if (fail) break;
            load_window(s + pos, nlo, nhi);  // the next batch's first window, or the chain's next header
            if (stop || qn < (uint32_t)D || pos + fsz > len) break;
          }
          if (fail) return false;
          if constexpr (ST == 0) *sink = WalkEntry{0, 0};  // same [load, store] in flight as the plain path
        }
      }
      return true;
    };
    // two window buffers in turn: the window a step loads is the next step's
    // current one in the same registers.  (With one buffer the compiler copies
    // the loaded window into the loop-carried registers at the back edge -- a
    // copy that waits for the load and, vmcnt being in order, for every entry
    // store after it: each step then paid the load AND the stores' latency
    // instead of overlapping them with the checks; C4 walk 1.61 -> 1.59 ms,
    // profiles/r03/r03_walk_unr_ab.jsonl.)
    uint64_t lo2 = 0, hi2 = 0;
    for (;;) {
      if (!step(lo, hi, lo2, hi2)) break;
      if (!step(lo2, hi2, lo, hi)) break;
    }
    R.pos = pos;
    R.nf = nf;
    R.pb = pb;
    R.pl = pl;
    R.same = same;
    R.lastf = lastf;
    R.firstf = firstf;
    R.err = err;
    R.st = st;
    R.rec = rec;
    if constexpr (ST == 2) {  // the rest of the entries, and the end of the chain
      __asm__ volatile("" ::: "memory");
      lds_st(ring.head, (uint32_t)nf | kRingDone);
    }
}

// The writer wave of k_walk_count ST 2: lane j copies walker lane j's ring to
// its entry slots (ebase ~0: none) in groups of kWriterGroup entries (256
// bytes, aligned: slot runs start on kSlotAlign entries) as they are
// published, the last partial group when the chain is done; every slot below
// ecap only.  Whole groups: a 64-byte group is half an L2 line, and scattered
// half-line writes among the walk's random line reads cost far more than their
// bytes (256-byte groups 1.262 ms on C4, 128-byte 1.284, 64-byte 1.345;
// profiles/r03/r03_compact_entries_ab.jsonl).
__device__ __forceinline__ void walk_ring_writer(WalkEntry* __restrict__ entries, WalkRing ring, uint64_t ebase,
                                                 uint64_t ecap) {
  static_assert(kWriterGroup <= kSlotAlign, "groups aligned by the slot runs");
  uint32_t t = 0;
  bool fin = false;
  for (;;) {
    if (!fin) {
      const uint32_t hv = lds_ld(ring.head);
      __asm__ volatile("" ::: "memory");  // the entries after the head that published them
      const uint32_t h = hv & ~kRingDone;
      while (h - t >= kWriterGroup) {
        WalkEntry g[kWriterGroup];
#pragma unroll
        for (uint32_t k = 0; k < kWriterGroup; ++k) g[k] = ring.e[(t + k) & (kRing - 1)];
        if (ebase != ~0ull && t + kWriterGroup <= ecap) {
          u32x4* d = reinterpret_cast<u32x4*>(entries + ebase + t);  // 256-byte aligned
#pragma unroll
          for (uint32_t k = 0; k < kWriterGroup / 2; ++k)
            d[k] = u32x4{g[2 * k].mask, g[2 * k].w, g[2 * k + 1].mask, g[2 * k + 1].w};
        }
        t += kWriterGroup;
        __asm__ volatile("" ::: "memory");
        lds_st(ring.tail, t);
      }
      if (hv & kRingDone) {
        for (; t < h; ++t)
          if (ebase != ~0ull && t < ecap) entries[ebase + t] = ring.e[t & (kRing - 1)];
        fin = true;
      }
    }
    if (__all(fin)) break;
    __builtin_amdgcn_s_sleep(2);
  }
}

// 1. The counting walk: one lane per connection (wave 0), and with ST 2 a
// second wave that writes the walkers' entries.
template <int D, int ST>
__global__ __launch_bounds__(ST == 2 ? 2 * kCountBlock : kCountBlock) void k_walk_count(
    const uint8_t* __restrict__ in, const gevws_conn_in* __restrict__ conns, uint32_t n,
    gevws_conn_out* __restrict__ cout, uint64_t* __restrict__ blk, WalkEntry* __restrict__ entries, uint64_t n_entries,
    uint32_t gshift, uint32_t cpb, uint64_t in_bytes, uint32_t* __restrict__ done, uint64_t max_frames,
    uint64_t payload_cap, gevws_summary* __restrict__ sum) {
  __shared__ WalkEntry s_ring[ST == 2 ? kCountBlock * kRing : 1];
  __shared__ uint32_t s_head[ST == 2 ? kCountBlock : 1], s_tail[ST == 2 ? kCountBlock : 1];
  __shared__ uint64_t s_ebase[ST == 2 ? kCountBlock : 1], s_ecap[ST == 2 ? kCountBlock : 1];
  const uint32_t lane = threadIdx.x & 63;
  const bool walker = ST != 2 || threadIdx.x < 64;
  const uint32_t c = blockIdx.x * cpb + lane;
  const bool active = walker && lane < cpb && c < n;
  uint64_t nf = 0, pb = 0, pl = 0, err = 0, same = 0;
  gevws_conn_in ci = {0, 0};
  int32_t st = GEVWS_OK;
  uint64_t ebase = 0, ecap = 0;
  bool rec0 = false;
  if (active) {
    ci = conns[c];
    // the order flag rides in the high half of the error count (k_scan_blocks SPLIT)
    if (out_of_order(conns, c, ci)) err = 1ull << 32;
    if (ci.off > in_bytes || ci.len > in_bytes - ci.off) {
      // a stream outside the input arena: nothing is read, the connection
      // reports GEVWS_ERR_INVALID (and counts as an error), the rest decode
      ci.off = 0;
      ci.len = 0;
      st = GEVWS_ERR_INVALID;
      err += 1;
    }
    rec0 = entry_slots_of(ci, c, n_entries, gshift, ebase, ecap);
  }
  const WalkRing ring = {s_ring + lane * kRing, s_head + lane, s_tail + lane};
  if constexpr (ST == 2) {
    if (walker) {
      s_head[lane] = active ? 0u : kRingDone;
      s_tail[lane] = 0;
      s_ebase[lane] = rec0 ? ebase : ~0ull;
      s_ecap[lane] = ecap;
    }
    __syncthreads();
    if (!walker) walk_ring_writer(entries, ring, s_ebase[lane], s_ecap[lane]);
  }
  if (active) {
    WalkRes R = walk_res_fresh(err, st);
    walk_chain<D, ST>(in + ci.off, ci.len, rec0, ebase, ecap, entries, entries + n_entries + c, R, ring);
    nf = R.nf;
    pb = R.pb;
    pl = R.pl;
    err = R.err;
    same = R.same;
    gevws_conn_out o;
    o.first_frame = R.rec ? 1 : 0;  // scratch flag for k_walk_emit: entries recorded
    o.consumed = R.pos;
    o.payload_base = pb;  // per-connection arena bytes; k_walk_emit turns it into a base
    o.nframes = (uint32_t)nf;
    o.status = R.st;
    cout[c] = o;
  }
  // block partial sums (one wave)
  const uint64_t vals[kDecFields] = {nf, pb, pl, err, same};
#pragma unroll
  for (int k = 0; k < kDecFields; ++k) {
    const uint64_t s = wave_sum(vals[k]);
    if (threadIdx.x == 0) {
      if (done) put_partial(blk + (uint64_t)blockIdx.x * kDecFields + k, s);
      else blk[(uint64_t)blockIdx.x * kDecFields + k] = s;
    }
  }
  if (done) walk_block_done(done, gridDim.x, blk, max_frames, payload_cap, sum, threadIdx.x == 0);
}

// ------------------------------------------------------------------ 1a''. walk (count), split
// A chain costs one memory round trip per frame, so a batch of few, long
// chains (an 8-way C4 share: 8 192 connections, 1 100+ frames on the longest)
// walks for (longest chain) x (latency) with most of the chip idle.
// k_walk_split gives each connection KS lanes.  Lane i > 0 guesses a frame
// start near i/KS of the stream: it searches up to kSyncWindows windows of
// kSyncWin bytes spread over the first half of its segment for a
// position whose header and the kSyncDepth - 1 headers its chain reaches are
// all plausible (sync_frame: RSV clear, a defined opcode, control frames final
// and short, the mask bit of the connection's first frame, minimal length
// encodings, frames inside the stream), and guesses the chain's last header
// (sync_search).  WebSocket headers are not
// self-synchronising, so a guess is only a guess: each lane walks its segment
// [its guess, the next lane's guess) with k_walk_count's rules, and the
// connection's result is accepted only when every segment but the last ends
// exactly on its end (consumed == segment length, status OK) -- segment 0
// starts at a true frame start, so by induction every accepted guess is one,
// and the segments' frames, in order, are exactly the serial chain's.  If any
// segment misses, lane 0 re-walks the whole connection serially (a guess can
// cost time, never a different result).  The segments become the rows of a
// virtual connection table (segs / sout / srec) that the record pass walks
// like connections, with each segment's frame / payload offsets relative to
// its connection (k_walk_emit adds the connection's bases); per-connection
// results, block partials and summary are exactly k_walk_count's (the
// equal-size run count is stitched across segment boundaries).
constexpr uint32_t kSyncWin = 256;                // bytes searched after a split point
constexpr uint32_t kSyncRow = kSyncWin / 4 + 5;   // dwords per lane's LDS row (window + 16 B; odd stride)
constexpr int kSyncDepth = 5;                     // consecutive plausible headers confirm a guess
constexpr uint64_t kSplitMinBytes = 16384;        // a connection's segments are at least this long
constexpr uint32_t kSplitMaxLanes = 32;
constexpr uint32_t kSplitAutoMaxLanes = 16;  // the auto choice's largest split
constexpr uint64_t kSplitLanesPerCU = 512;        // auto: split while the walk has fewer lanes per CU
// auto: split only after a decode on this context whose connections averaged
// this many frames of at most this many payload bytes (the long chains of
// small frames splitting shortens; a batch of big frames -- C2, C3, C5 --
// pays the guesses for nothing)
constexpr uint64_t kSplitMinFramesPerConn = 256;
constexpr uint64_t kSplitMaxConnsPerCU = 32;  // more chains keep the walk busy unsplit (C4 1/4 share: +5 %)
constexpr uint64_t kSplitMaxFrameBytes = 4096;

__device__ __forceinline__ bool sync_plausible1(uint32_t b0, uint32_t b1, uint32_t m0) {
  const uint32_t op = b0 & 0x0fu;
  const bool data = op <= 2, ctrl = op >= 8 && op <= 10;
  return (b0 & 0x70u) == 0 && (b1 >> 7) == m0 && (data || (ctrl && (b0 & 0x80u) && (b1 & 0x7fu) <= 125));
}

// The frame size of a plausible header in the 16 bytes lo|hi with rem stream
// bytes from it, else 0.
__device__ __forceinline__ uint64_t sync_frame(uint64_t lo, uint64_t hi, uint64_t rem, uint32_t m0) {
  const uint32_t b0 = (uint32_t)lo & 0xffu, b1 = (uint32_t)(lo >> 8) & 0xffu;
  if (!sync_plausible1(b0, b1, m0)) return 0;
  const uint32_t len7 = b1 & 0x7fu;
  const uint32_t hlen = 2 + (len7 == 127 ? 8u : (len7 == 126 ? 2u : 0u)) + 4 * (b1 >> 7);
  uint64_t L = len7;
  if (len7 == 126) {
    L = (((lo >> 16) & 0xff) << 8) | ((lo >> 24) & 0xff);
    if (L < 126) return 0;
  } else if (len7 == 127) {
    L = __builtin_bswap64((lo >> 16) | (hi << 48));
    if ((L >> 63) || L < 65536) return 0;
  }
  if (rem < hlen || rem - hlen < L) return 0;
  return hlen + L;
}

// The guess is the LAST header of a confirmed chain of kSyncDepth, not its
// first: chains converge (a false start inside a payload often hops onto a
// true header and from there follows the true chain), so a chain's far end is
// a frame start far more often than its first header -- for the last header
// to be a false start the chain must have stayed inside payload bytes for
// every hop.  (16-byte loads at q < len stay inside the stream + GEVWS_IN_PAD.)
// 16 bytes at byte x of an LDS row
__device__ __forceinline__ void row_window(const uint32_t* __restrict__ row, uint32_t x, uint64_t& lo, uint64_t& hi) {
  const uint32_t k = x >> 2, e = x & 3;
  const uint32_t w0 = row[k], w1 = row[k + 1], w2 = row[k + 2], w3 = row[k + 3], w4 = row[k + 4];
  lo = (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, e) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, e) << 32);
  hi = (uint64_t)__builtin_amdgcn_alignbyte(w3, w2, e) | ((uint64_t)__builtin_amdgcn_alignbyte(w4, w3, e) << 32);
}

// Level-1 candidates among the 4 byte positions of dword w (wn: the next
// dword): bit e set when byte e could open a frame -- RSV clear, opcode & 7
// <= 2 (0-2, 8-10), the next byte's mask bit == m0 (mpat: m0 in every byte's
// bit 7).  SWAR, so a window's 256 positions cost 64 such steps on every lane
// alike instead of a divergent test per position.
__device__ __forceinline__ uint32_t sync_l1_mask4(uint32_t w, uint32_t wn, uint32_t mpat) {
  const uint32_t w1 = __builtin_amdgcn_alignbyte(wn, w, 1);  // byte p + 1 of every position p
  const uint32_t bad = (w & 0x74747474u) | (w & (w >> 1) & 0x01010101u) | ((w1 ^ mpat) & 0x80808080u);
  const uint32_t z = ~(((bad & 0x7f7f7f7fu) + 0x7f7f7f7fu) | bad | 0x7f7f7f7fu);  // 0x80 where bad's byte is 0
  return ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
}

// A confirmed frame start reached from one of kSyncWindows windows of
// kSyncWin bytes at t, t + step, ..., below qmax (every window inside the
// stream).  Per window: (1) the window into this lane's LDS row and a bitmask
// of its level-1 candidates (sync_l1_mask4); (2) the lane's candidates in
// order -- a loop over set bits, so the wave iterates as often as its busiest
// lane has candidates, not once per position -- until the first whose chain
// stays plausible for every hop inside the window; (3) all lanes at once
// continue that candidate's chain with global loads to kSyncDepth headers.
constexpr int kSyncWindows = 4;
// headers a candidate's chain must show inside the window before its global
// confirmation (a lone plausible header is common in payload bytes, and
// confirming it costs the whole wave memory round trips; 2 finds fewer guesses)
constexpr int kSyncMinInWindow = 1;
__device__ __forceinline__ bool sync_search(const uint8_t* __restrict__ s, uint64_t len, uint64_t t, uint64_t step,
                                            uint64_t qmax, uint32_t m0, uint32_t* __restrict__ row, uint64_t& b) {
  const uint32_t mpat = m0 ? 0x80808080u : 0u;
  for (int win = 0; win < kSyncWindows; ++win, t += step) {
    if (t + kSyncWin + 16 > len || t >= qmax) return false;
    uint32_t wv[kSyncRow - 1];
#pragma unroll
    for (uint32_t j = 0; j < (kSyncWin + 16) / 16; ++j) {
      const u32x4 v = ld16u(s + t + 16 * j);
#pragma unroll
      for (int e = 0; e < 4; ++e) wv[4 * j + e] = v[e];
    }
#pragma unroll
    for (uint32_t k = 0; k < kSyncRow - 1; ++k) row[k] = wv[k];
    row[kSyncRow - 1] = 0;
    uint64_t cm[kSyncWin / 64];
#pragma unroll
    for (uint32_t j = 0; j < kSyncWin / 64; ++j) {
      uint64_t m = 0;
#pragma unroll
      for (uint32_t k = 0; k < 16; ++k) m |= (uint64_t)sync_l1_mask4(wv[16 * j + k], wv[16 * j + k + 1], mpat) << (4 * k);
      cm[j] = m;
    }
    // (2) the first candidate whose in-window hops are all plausible
    bool have = false;
    uint64_t q = 0, lb = 0;
    int h = 0;
#pragma unroll
    for (uint32_t j = 0; j < kSyncWin / 64; ++j) {
      uint64_t m = have ? 0 : cm[j];
      while (m) {
        uint32_t x = 64 * j + (uint32_t)__builtin_ctzll(m);
        m &= m - 1;
        uint64_t lo, hi;
        row_window(row, x, lo, hi);
        uint64_t f = sync_frame(lo, hi, len - (t + x), m0);
        if (f == 0) continue;
        int hh = 1;
        uint32_t last = x;
        while (hh < kSyncDepth && x + f < kSyncWin) {
          x += (uint32_t)f;
          row_window(row, x, lo, hi);
          f = sync_frame(lo, hi, len - (t + x), m0);
          if (f == 0) break;
          last = x;
          ++hh;
        }
        if (f == 0 || (hh < kSyncMinInWindow && t + x + f < len)) continue;
        have = true;
        q = t + x + f;
        lb = t + last;
        h = hh;
        m = 0;
      }
    }
    if (!have) continue;
    // (3) the rest of its chain from memory
    bool ok = true;
    while (h < kSyncDepth) {
      if (q >= qmax || q >= len) {
        ok = false;
        break;
      }
      uint64_t lo, hi;
      load_window(s + q, lo, hi);
      const uint64_t g = sync_frame(lo, hi, len - q, m0);
      if (g == 0) {
        ok = false;
        break;
      }
      lb = q;
      q += g;
      ++h;
    }
    if (ok && lb < qmax) {
      b = lb;
      return true;
    }
  }
  return false;
}

template <int KS, int D>
__global__ __launch_bounds__(kCountBlock) void k_walk_split(const uint8_t* __restrict__ in,
                                                            const gevws_conn_in* __restrict__ conns, uint32_t n,
                                                            gevws_conn_out* __restrict__ cout,
                                                            uint64_t* __restrict__ blk,
                                                            WalkEntry* __restrict__ entries, uint64_t n_entries,
                                                            uint32_t gshift, uint32_t cpb, uint64_t in_bytes,
                                                            uint32_t* __restrict__ done, uint64_t max_frames,
                                                            uint64_t payload_cap, gevws_summary* __restrict__ sum,
                                                            gevws_conn_in* __restrict__ segs,
                                                            gevws_conn_out* __restrict__ sout,
                                                            uint8_t* __restrict__ srec,
                                                            uint64_t min_seg = kSplitMinBytes) {
  static_assert(KS >= 2 && KS <= (int)kSplitMaxLanes && (KS & (KS - 1)) == 0, "KS: a power of two");
  __shared__ uint32_t s_row[kCountBlock * kSyncRow];
  const uint32_t lane = threadIdx.x & 63, i = lane % KS;
  const uint32_t c = blockIdx.x * cpb + threadIdx.x / KS;
  const bool active = threadIdx.x / KS < cpb && c < n;
  const uint64_t v = (uint64_t)c * KS + i;
  gevws_conn_in ci = {0, 0};
  bool oob = false;
  if (active) {
    ci = conns[c];
    oob = ci.off > in_bytes || ci.len > in_bytes - ci.off;
    if (oob) ci = gevws_conn_in{0, 0};  // nothing of it is read (k_walk_count's rule)
  }
  const uint8_t* s = in + ci.off;
  // 1. guesses: lane 0 starts at 0; lane i at the first confirmed frame start
  // after i/kc of the stream (kc: segments of >= kSplitMinBytes)
  bool found = active && i == 0;
  uint64_t b = 0;
  if (active && i > 0) {
    const uint64_t kc = ci.len / min_seg < KS ? ci.len / min_seg : KS;
    if (i < kc) {
      // windows spread over the first half of the segment; guesses below
      // 3/4 of it, so they stay in increasing lane order
      const uint64_t seg = ci.len / kc, t = ci.len * i / kc;
      const uint64_t step = seg / (2 * kSyncWindows) > kSyncWin ? seg / (2 * kSyncWindows) : kSyncWin;
      const uint32_t m0 = (uint32_t)s[1] >> 7;  // the first frame's mask bit (len >= 2 x kSplitMinBytes)
      found = sync_search(s, ci.len, t, step, t + seg * 3 / 4, m0, s_row + (threadIdx.x) * kSyncRow, b);
    }
  }
  // 2. a segment ends at the next lane's guess (or the stream's end);
  // lanes without a guess hold an empty segment there
  const uint64_t mine = found ? b : ~0ull;
  uint64_t end = ci.len;
#pragma unroll
  for (int j = KS - 1; j >= 1; --j) {
    const uint64_t y = __shfl(mine, (int)((lane + j) & 63), 64);
    if ((int)i + j < KS && y != ~0ull) end = y;
  }
  const uint64_t sb = found ? b : end;
  const uint64_t slen = found ? end - b : 0;
  gevws_conn_in sg = {ci.off + sb, slen};
  // 3. walk the segment (entries in its own slot run)
  uint64_t ebase = 0, ecap = 0;
  const bool rec0 = active && entry_slots_of(sg, (uint32_t)v, n_entries, gshift, ebase, ecap);
  WalkRes R = walk_res_fresh();
  if (active) walk_chain<D>(in + sg.off, sg.len, rec0, ebase, ecap, entries, entries + n_entries + v, R);
  // 4. stitch the group's KS lanes (every lane takes part in the shuffles)
  const bool last = found && end == ci.len;
  const bool ok = !found || last || (R.st == GEVWS_OK && R.pos == slen);
  uint64_t prevlast = ~0ull;
  bool got = false;
#pragma unroll
  for (int d = 1; d < KS; ++d) {
    const uint64_t ynf = __shfl_up(R.nf, d, 64), ylast = __shfl_up(R.lastf, d, 64);
    if (!got && (int)i >= d && ynf > 0) {
      prevlast = ylast;
      got = true;
    }
  }
  const uint64_t same = R.same + ((R.nf > 0 && got && R.firstf == prevlast) ? 1 : 0);
  uint64_t inf = R.nf, ipb = R.pb;  // inclusive prefixes within the group
#pragma unroll
  for (int d = 1; d < KS; d <<= 1) {
    const uint64_t a = __shfl_up(inf, d, 64), q = __shfl_up(ipb, d, 64);
    if ((int)i >= d) {
      inf += a;
      ipb += q;
    }
  }
  uint64_t t_nf = R.nf, t_pb = R.pb, t_pl = R.pl, t_same = same;
  uint64_t t_cons = last ? sb + R.pos : 0;
  int32_t t_st = last ? R.st : 0;
  int t_ok = ok ? 1 : 0;
#pragma unroll
  for (int d = KS / 2; d >= 1; d >>= 1) {
    t_nf += __shfl_xor(t_nf, d, 64);
    t_pb += __shfl_xor(t_pb, d, 64);
    t_pl += __shfl_xor(t_pl, d, 64);
    t_same += __shfl_xor(t_same, d, 64);
    t_cons += __shfl_xor(t_cons, d, 64);
    t_st += __shfl_xor(t_st, d, 64);
    t_ok &= __shfl_xor(t_ok, d, 64);
  }
  const bool valid = t_ok != 0 && !oob;
  uint64_t nf = 0, pb = 0, pl = 0, err = 0, rs = 0;
  if (active) {
    if (valid) {
      segs[v] = sg;
      gevws_conn_out so;
      so.first_frame = inf - R.nf;  // relative to the connection's first frame
      so.consumed = R.pos;
      so.payload_base = ipb - R.pb;  // relative to the connection's payload base
      so.nframes = (uint32_t)R.nf;
      so.status = R.st;
      sout[v] = so;
      srec[v] = R.rec ? 1 : 0;
    }
    if (i == 0) {
      gevws_conn_out o;
      o.first_frame = 0;
      if (oob) {
        o.consumed = 0;
        o.payload_base = 0;
        o.nframes = 0;
        o.status = GEVWS_ERR_INVALID;
      } else if (valid) {
        nf = t_nf;
        pb = t_pb;
        pl = t_pl;
        rs = t_same;
        o.consumed = t_cons;
        o.payload_base = pb;
        o.nframes = (uint32_t)nf;
        o.status = t_st;
      } else {
        // a guess missed: the whole chain, serially (no entries: the record
        // pass re-walks it as one segment)
        WalkRes S = walk_res_fresh();
        walk_chain<0>(s, ci.len, false, 0, 0, entries, entries + n_entries + v, S);
        nf = S.nf;
        pb = S.pb;
        pl = S.pl;
        rs = S.same;
        o.consumed = S.pos;
        o.payload_base = pb;
        o.nframes = (uint32_t)nf;
        o.status = S.st;
      }
      err = (o.status < 0 ? 1ull : 0ull) + (out_of_order(conns, c, conns[c]) ? (1ull << 32) : 0ull);
      cout[c] = o;
    }
    if (!valid) {  // one segment: the whole connection, re-walked by the record pass
      segs[v] = i == 0 ? ci : gevws_conn_in{ci.off + ci.len, 0};
      gevws_conn_out so;
      so.first_frame = 0;
      so.consumed = 0;
      so.payload_base = 0;
      so.nframes = (uint32_t)(i == 0 ? nf : 0);
      so.status = GEVWS_OK;
      sout[v] = so;
      srec[v] = 0;
    }
  }
  // block partials (one wave), as k_walk_count
  const uint64_t vals[kDecFields] = {nf, pb, pl, err, rs};
#pragma unroll
  for (int k = 0; k < kDecFields; ++k) {
    const uint64_t x = wave_sum(vals[k]);
    if (threadIdx.x == 0) {
      if (done) put_partial(blk + (uint64_t)blockIdx.x * kDecFields + k, x);
      else blk[(uint64_t)blockIdx.x * kDecFields + k] = x;
    }
  }
  if (done) walk_block_done(done, gridDim.x, blk, max_frames, payload_cap, sum, threadIdx.x == 0);
}

// ------------------------------------------------------------------ 2. scan of block partials
// SPLIT (decode): field 3 holds errors in its low 32 bits and the count of
// out-of-order connections in its high 32 (k_walk_count) -> summary.errors and
// GEVWS_SUMMARY_UNORDERED.
template <bool SPLIT, int NF = kBlkFields>
__global__ __launch_bounds__(kScanBlock) void k_scan_blocks(uint64_t* __restrict__ blk, uint32_t nblk,
                                                            uint64_t max_frames, uint64_t payload_cap,
                                                            gevws_summary* __restrict__ sum) {
  // kScanPer consecutive partials per thread: a batch of per-frame blocks
  // (encode / dispatch of 43.8 M frames: 171 K partials) takes a few rounds of
  // the workgroup instead of one round per 1 024 partials
  constexpr int kScanPer = 8;
  uint64_t carry[NF] = {};
  for (uint64_t base = 0; base < nblk; base += (uint64_t)kScanBlock * kScanPer) {
    const uint64_t i0 = base + (uint64_t)threadIdx.x * kScanPer;
    uint64_t loc[NF] = {}, ex[NF], tot[NF];
#pragma unroll
    for (int r = 0; r < kScanPer; ++r)
#pragma unroll
      for (int k = 0; k < NF; ++k) loc[k] += (i0 + r < nblk) ? blk[(i0 + r) * NF + k] : 0;
    block_excl_scan<kScanBlock, NF>(loc, ex, tot);
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

// ------------------------------------------------------------------ 3. walk (emit)
// 3a. per-connection bases: block-level exclusive scan of (frames, arena bytes)
// on top of the scanned block partials.
__global__ __launch_bounds__(kCountBlock) void k_walk_bases(uint32_t n, gevws_conn_out* __restrict__ cout,
                                                            const uint64_t* __restrict__ blk,
                                                            const gevws_summary* __restrict__ sum,
                                                            uint8_t* __restrict__ rec_flags, uint32_t cpb,
                                                            uint64_t* __restrict__ stats = nullptr) {
  if (stats && blockIdx.x == 0 && threadIdx.x == 0) {  // the context's history (split walk, D, wide grid)
    stats[0] = sum->frames;
    stats[1] = sum->payload_len;
    stats[2] = sum->run_frames;
  }
  if (sum->status != GEVWS_OK) return;  // capacity error: nothing written
  const uint32_t c = blockIdx.x * cpb + threadIdx.x;
  const bool active = threadIdx.x < cpb && c < n;
  uint64_t v[2] = {0, 0};
  gevws_conn_out o;
  if (active) {
    o = cout[c];
    v[0] = o.nframes;
    v[1] = o.payload_base;  // this connection's arena bytes (k_walk_count)
  }
  uint64_t ex[2], tot[2];
  block_excl_scan<kCountBlock, 2>(v, ex, tot);
  if (!active) return;
  rec_flags[c] = o.first_frame != 0 ? 1 : 0;  // k_walk_count's "entries recorded" flag
  o.first_frame = blk[(uint64_t)blockIdx.x * kDecFields + 0] + ex[0];
  o.payload_base = blk[(uint64_t)blockIdx.x * kDecFields + 1] + ex[1];
  cout[c] = o;
}

__device__ __forceinline__ void emit_record(gevws_frame* __restrict__ frames, uint32_t* __restrict__ tile_first,
                                            uint64_t f, uint64_t poff, uint64_t src_off, const DevHdr& h) {
  // the 32-byte record as two 16-byte stores: {fin, rsv, opcode, masked,
  // mask[4], length} and {payload_off, src_off} (gevws_frame's layout)
  // (C4's emit 0.64 -> 0.55 ms against the field-by-field struct store, which
  // compiled to three stores of 8 + 16 + 8 bytes; profiles/r01/r01_ab_emit_store_*.json)
  const uint32_t flags = (h.b0 >> 7) | (((h.b0 & 0x70) >> 4) << 8) | ((h.b0 & 0x0f) << 16) | ((h.masked & 1) << 24);
  u32x4* r = reinterpret_cast<u32x4*>(frames + f);
  const u32x4 r0 = u32x4{flags, h.mask, (uint32_t)h.length, (uint32_t)(h.length >> 32)};
  const u32x4 r1 = u32x4{(uint32_t)poff, (uint32_t)(poff >> 32), (uint32_t)src_off, (uint32_t)(src_off >> 32)};
  r[0] = r0;  // (plain stores: the unmask reads the records from L2 right after;
  r[1] = r1;  // non-temporal ones made C4's record pass 0.494 -> 0.551 ms, r02_emit_nt_ab.jsonl)
  const uint64_t padded = round16(h.length);
  // output tiles whose first byte lies in [poff, poff + padded)
  for (uint64_t t = (poff + kTile - 1) / kTile; t * kTile < poff + padded; ++t) tile_first[t] = (uint32_t)f;
}

// 3b. records + tile map from the walk's entries.  A wave takes G
// consecutive connections at a time, their metadata in one coalesced load
// (lane j = connection j).  Phase 1: when their recorded frames number at most
// 64 R, the group's frames are enumerated across connection boundaries --
// lane l of round r takes the group's frame r*64 + l, finds its connection by
// a binary search over the lanes' frame prefix sums (__shfl), and the payload
// offsets come from a segmented wave scan plus a per-connection carry kept in
// lane j -- so connections of a few frames (C1: 16 frames of 136 B) fill whole
// waves instead of 16 lanes of one, and all R rounds' entries are requested at
// once (C4 0.53 -> 0.49 ms against one wave per connection,
// profiles/r02/r02_emit_ab.jsonl).  Phase 2: longer connections one wave each, 64
// entries per round, U rounds' entries requested at once (a connection of N
// frames costs ceil(N / 64U) entry-load latencies), wave prefix sum of the
// padded lengths -> payload offsets, 64 contiguous 32-byte records per store.
// Connections without recorded entries are re-walked afterwards, one lane per
// connection.

// Segmented inclusive wave scan: a segment starts at every lane with head set
// (and at lane 0).  Every lane must take part.
__device__ __forceinline__ uint64_t wave_seg_scan(uint64_t v, bool head) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t vu = __shfl_up(v, d, 64);
    const bool hu = __shfl_up((int)head, d, 64) != 0;
    if (lane >= d && !head) {
      v += vu;
      head = hu;
    }
  }
  return v;
}

// One round of entries (lane = frame): each frame's payload length L and the
// segmented inclusive prefix `ip` of the frame sizes (hlen + L), so a frame
// starts at (its row's position carry) + ip - (hlen + L).  Escaped lengths
// (>= kLenEsc) are re-read from the header, lowest lane first: every frame
// before it in its row is then resolved, so its position is exact.  `head`:
// the lane starts a row in this round; pbase / coff: the position carry and
// input offset of the lane's row (every lane must take part: shuffles).
__device__ __forceinline__ void entry_round(const uint8_t* __restrict__ in, const WalkEntry& q, bool valid, bool head,
                                            uint64_t pbase, uint64_t coff, uint64_t& L, uint64_t& ip) {
  L = valid ? entry_len21(q) : 0;
  bool esc = valid && L == kLenEsc;
  uint64_t fsz = (valid && !esc) ? entry_hlen(q) + L : 0;
  ip = wave_seg_scan(fsz, head);
  for (;;) {
    const uint64_t m = __ballot(esc);
    if (m == 0) break;  // wave-uniform
    if ((threadIdx.x & 63) == (uint32_t)__builtin_ctzll(m)) {
      uint64_t lo, hi;
      load_window(in + coff + pbase + ip, lo, hi);  // (fsz == 0: ip is the frame's start)
      DevHdr h;
      parse_header(lo, hi, ~0ull, h);  // parsed by the walk: complete
      L = h.length;
      fsz = h.hlen + L;
      esc = false;
    }
    ip = wave_seg_scan(fsz, head);
  }
}

constexpr int kEmitGroup = 16;
constexpr uint64_t kEmitSplitPerCU = 32;  // record-pass workgroups per CU over k_walk_split's rows
// (Measured and not kept: phase 2 software-pipelined, the next batch's entry
// loads issued before this batch's rounds -- C4 0.448 -> 0.477 ms, 8-way share
// 0.094 -> 0.108: the record pass is not bound by its entry loads' latency.)
__global__ __launch_bounds__(kWalkBlock) void k_walk_emit(const uint8_t* __restrict__ in,
                                                          const gevws_conn_in* __restrict__ conns, uint32_t n,
                                                          const gevws_conn_out* __restrict__ cout,
                                                          const gevws_summary* __restrict__ sum,
                                                          gevws_frame* __restrict__ frames,
                                                          uint32_t* __restrict__ tile_first,
                                                          const WalkEntry* __restrict__ entries, uint64_t n_entries,
                                                          uint32_t gshift, const uint8_t* __restrict__ rec_flags,
                                                          const gevws_conn_out* __restrict__ pout = nullptr,
                                                          uint32_t ks = 0) {
  constexpr int U = 4, G = kEmitGroup;
  if (sum->status != GEVWS_OK) return;
  // k_walk_split's segments: frame / payload offsets relative to connection c / ks
  auto out_of = [&](uint64_t c) {
    gevws_conn_out o = cout[c];
    if (ks) {
      const gevws_conn_out p = pout[c / ks];
      o.first_frame += p.first_frame;
      o.payload_base += p.payload_base;
    }
    return o;
  };
  const bool unordered = (sum->flags & GEVWS_SUMMARY_UNORDERED) != 0;  // entry runs may collide: unused
  const int lane = threadIdx.x & 63;
  const uint64_t nwaves = (uint64_t)gridDim.x * (kWalkBlock / 64);
  // the record of entry q: payload length L, frame f, payload offset poff,
  // header at input offset hpos
  auto record = [&](const WalkEntry& q, uint64_t L, uint64_t f, uint64_t poff, uint64_t hpos) {
    DevHdr h;
    h.b0 = q.w & 0xff;
    h.masked = (q.w >> 8) & 1;
    h.hlen = entry_hlen(q);
    h.mask = q.mask;
    h.length = L;
    emit_record(frames, tile_first, f, poff, hpos + h.hlen, h);
  };
  // the per-connection rounds (64 entries per round, U rounds per load)
  auto one_conn = [&](uint64_t cnt, uint64_t first_frame, uint64_t payload_base, uint64_t coff, uint64_t ebase) {
    const WalkEntry* ce = entries + ebase;
    uint64_t carry = payload_base, pcarry = 0;
    auto round = [&](const WalkEntry& q, uint64_t r0) {
      const uint64_t k = r0 + lane;
      const bool valid = k < cnt;
      uint64_t L, ip;
      entry_round(in, q, valid, lane == 0, pcarry, coff, L, ip);
      const uint64_t fsz = valid ? entry_hlen(q) + L : 0;
      const uint64_t padded = valid ? round16(L) : 0;
      const uint64_t incl = wave_incl_scan(padded);
      if (valid) record(q, L, first_frame + k, carry + incl - padded, coff + pcarry + ip - fsz);
      carry += __shfl(incl, 63, 64);
      pcarry += __shfl(ip, 63, 64);
    };
    if (cnt <= 64) {  // wave-uniform
      for (uint64_t k0 = 0; k0 < cnt; k0 += 64) {
        WalkEntry q = {0, 0};
        if (k0 + lane < cnt) q = ce[k0 + lane];
        round(q, k0);
      }
    } else {
      for (uint64_t k0 = 0; k0 < cnt; k0 += 64 * U) {
        WalkEntry q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          // unconditional (clamped to the last entry): a branch around the
          // load would make the compiler wait for it inside the branch
          const uint64_t k = k0 + (uint64_t)u * 64 + lane;
          q[u] = ce[k < cnt ? k : cnt - 1];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (k0 + (uint64_t)u * 64 >= cnt) break;  // wave-uniform
          round(q[u], k0 + (uint64_t)u * 64);
        }
      }
    }
  };
  {
    // phase 1: groups of G connections, their short connections (<= kShort
    // frames, so a group has at most 64 R) enumerated across boundaries
    constexpr int R = 4;
    constexpr uint64_t kShort = 64ull * R / G;
    const uint64_t ngroups = ((uint64_t)n + G - 1) / G;
    for (uint64_t g = (uint64_t)blockIdx.x * (kWalkBlock / 64) + (threadIdx.x >> 6); g < ngroups; g += nwaves) {
      const uint64_t c = g * G + lane;
      uint64_t nf = 0, ff = 0, pbase = 0, coff = 0, ebase = 0;
      if (lane < G && c < n) {
        const gevws_conn_out o = out_of(c);
        const gevws_conn_in ci = conns[c];
        uint64_t ecap = 0;
        const bool rec = rec_flags[c] && !unordered && entry_slots_of(ci, (uint32_t)c, n_entries, gshift, ebase, ecap);
        nf = (rec && o.nframes <= kShort) ? o.nframes : 0;  // long: phase 2; unrecorded: re-walked below
        ff = o.first_frame;
        pbase = o.payload_base;
        coff = ci.off;
      }
      const uint64_t inc = wave_incl_scan(nf);
      const uint64_t T = uniform64(__shfl(inc, 63, 64));  // <= 64 R
      if (T == 0) continue;
      const uint64_t tstart = inc - nf;  // lane j: group index of its connection's first frame
      WalkEntry q[R];
      uint32_t jr[R];
      uint64_t kr[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint64_t t = (uint64_t)r * 64 + lane;
        static_assert((G & (G - 1)) == 0, "G: a power of two");
        uint32_t lo = 0, hi = G - 1;  // smallest j with inc_j > t
#pragma unroll
        for (int it = 0; (1 << it) < G; ++it) {  // fixed trip count: the __shfl sees every lane
          const uint32_t mid = (lo + hi) >> 1;
          if (__shfl(inc, (int)mid, 64) > t) hi = mid; else lo = mid + 1;
        }
        jr[r] = lo;
        kr[r] = t - __shfl(tstart, (int)lo, 64);
        const uint64_t eb = __shfl(ebase, (int)lo, 64);  // (outside the t < T branch: see below)
        q[r] = WalkEntry{0, 0};
        if (t < T) q[r] = entries[eb + kr[r]];
      }
      // lane j: its connection's padded bytes and stream bytes already placed
      uint64_t carry = 0, pcarry = 0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if ((uint64_t)r * 64 >= T) break;  // wave-uniform
        const uint64_t t = (uint64_t)r * 64 + lane;
        const bool valid = t < T;
        const uint32_t j = jr[r];
        // a segment starts at a connection's first frame and at lane 0
        const bool head = kr[r] == 0 || lane == 0;
        // every __shfl runs with the whole wave active: a ds_bpermute reads
        // nothing from a lane masked off by a branch (here: lane j of a
        // connection whose frames are all taken, in a round's short tail)
        const uint64_t cj = __shfl(carry, (int)j, 64), pcj = __shfl(pcarry, (int)j, 64);
        const uint64_t fj = __shfl(ff, (int)j, 64), pj = __shfl(pbase, (int)j, 64), oj = __shfl(coff, (int)j, 64);
        uint64_t L, ip;
        entry_round(in, q[r], valid, head, pcj, oj, L, ip);
        const uint64_t fsz = valid ? entry_hlen(q[r]) + L : 0;
        const uint64_t padded = valid ? round16(L) : 0;
        const uint64_t v = wave_seg_scan(padded, head);
        if (valid) record(q[r], L, fj + kr[r], pj + cj + v - padded, oj + pcj + ip - fsz);
        // lane j adds its connection's bytes in this round (from the lane of its last frame here)
        const uint64_t r0 = (uint64_t)r * 64, r1 = r0 + 64;
        const uint64_t a = tstart > r0 ? tstart : r0, b = inc < r1 ? inc : r1;
        const int src = (int)((b > a ? b - 1 : r0) - r0);
        const uint64_t got = __shfl(v, src, 64), gotp = __shfl(ip, src, 64);
        if (lane < G && b > a) {
          carry += got;
          pcarry += gotp;
        }
      }
    }
    // phase 2: connections of more than kShort frames, one wave per
    // connection, GL consecutive connections per wave (their metadata in one
    // load) when the batch has more connections than the grid has waves
    // (half the grid's waves busy: C4's 65 536 connections 0.43 ms in groups of
    // 16 vs 0.53 ms in groups of 8 over every wave -- fewer record streams
    // interleave in DRAM; profiles/r02/r02_emit_ab.jsonl)
    const uint64_t per = (2 * (uint64_t)n + nwaves - 1) / nwaves;
    const uint64_t GL = per < 1 ? 1 : (per > 16 ? 16 : per);
    const uint64_t nl = ((uint64_t)n + GL - 1) / GL;
    for (uint64_t g = (uint64_t)blockIdx.x * (kWalkBlock / 64) + (threadIdx.x >> 6); g < nl; g += nwaves) {
      const uint64_t c = g * GL + lane;
      uint64_t nf = 0, ff = 0, pbase = 0, coff = 0, ebase = 0;
      if (lane < GL && c < n) {
        const gevws_conn_out o = out_of(c);
        const gevws_conn_in ci = conns[c];
        uint64_t ecap = 0;
        const bool rec = rec_flags[c] && !unordered && entry_slots_of(ci, (uint32_t)c, n_entries, gshift, ebase, ecap);
        nf = (rec && o.nframes > kShort) ? o.nframes : 0;
        ff = o.first_frame;
        pbase = o.payload_base;
        coff = ci.off;
      }
      // the group's connections with long chains (a ballot: groups of only
      // short or empty connections -- all of C1's -- cost one instruction;
      // C1's record pass 0.030 -> 0.025 ms, profiles/r03/r03_emit_pf_ab.jsonl)
      for (uint64_t m = __ballot(lane < GL && nf > 0); m; m &= m - 1) {  // wave-uniform
        const int j = __builtin_ctzll(m);
        const uint64_t cnt = uniform64(__shfl(nf, j, 64));
        const uint64_t fj = uniform64(__shfl(ff, j, 64)), pj = uniform64(__shfl(pbase, j, 64));
        const uint64_t oj = uniform64(__shfl(coff, j, 64)), ej = uniform64(__shfl(ebase, j, 64));
        one_conn(cnt, fj, pj, oj, ej);
      }
    }
  }
  // connections without recorded entries: one lane per connection re-walks
  const uint64_t nthreads = (uint64_t)gridDim.x * kWalkBlock;
  for (uint64_t c = (uint64_t)blockIdx.x * kWalkBlock + threadIdx.x; c < n; c += nthreads) {
    if (rec_flags[c] && !unordered) continue;
    const gevws_conn_out o = out_of(c);
    const gevws_conn_in ci = conns[c];
    const uint8_t* s = in + ci.off;
    uint64_t pos = 0, poff = o.payload_base;
    for (uint64_t k = 0; k < o.nframes; ++k) {
      uint64_t lo, hi;
      load_window(s + pos, lo, hi);
      DevHdr h;
      parse_header(lo, hi, ci.len - pos, h);  // succeeded in k_walk_count
      emit_record(frames, tile_first, o.first_frame + k, poff, ci.off + pos + h.hlen, h);
      poff += round16(h.length);
      pos += h.hlen + h.length;
    }
  }
}

// ------------------------------------------------------------------ 3c. small batches, one launch
// A live server's pass is small (C1: ~100 connections x 136 B per loop
// iteration) and pays per launch, not per byte: four kernels cost ~5 us each
// of GPU time whatever their size (profiles/r02/r02_loopback_*), plus their host
// launch costs.  Batches of at most kSmallConns connections and
// GEVWS_TUNE_SMALL_BATCH bytes (default kSmallBytes) run the whole decode in
// ONE workgroup: each lane walks its connection (k_walk_count's rules), a
// block scan gives the bases and the summary, each lane re-walks its chain
// writing the records and unmasking payloads of up to kSmallLaneBytes itself
// (all its chunk loads at once), and the workgroup unmasks the larger ones
// together.  Output identical to the multi-kernel decode.
// A live pass's last kernel announces its end in mapped host memory: every
// thread's writes (records, payload, summaries) are fenced at system scope,
// then one lane stores `seq` with a system-scope release (a vector store), so
// a host that sees the flag sees the results -- it spins on host memory
// instead of waiting in hipStreamSynchronize (gevws_ctx_set_completion_flag).
// Callers reach it with the whole workgroup (it holds a barrier).
__device__ __forceinline__ void signal_done(uint32_t* done, uint32_t seq) {
  if (!done) return;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr uint32_t kSmallConns = 256;
constexpr uint64_t kSmallBytes = 64 * 1024;
constexpr uint32_t kSmallLaneBytes = 256;
constexpr uint32_t kSmallBig = kSmallBytes / kSmallLaneBytes;  // larger payloads fit in the input at most this often

__global__ __launch_bounds__(kSmallConns) void k_decode_small(const uint8_t* __restrict__ in, uint64_t in_bytes,
                                                              const gevws_conn_in* __restrict__ conns, uint32_t n,
                                                              gevws_frame* __restrict__ frames, uint64_t max_frames,
                                                              uint8_t* __restrict__ payload, uint64_t payload_cap,
                                                              gevws_conn_out* __restrict__ cout,
                                                              gevws_summary* __restrict__ sum,
                                                              uint32_t* __restrict__ done = nullptr,
                                                              uint32_t seq = 0) {
  __shared__ uint64_t s_big[kSmallBig][3];  // {src_off, payload_off, length} of the larger payloads
  __shared__ uint32_t s_bkey[kSmallBig];
  __shared__ uint32_t s_nbig;
  const uint32_t c = threadIdx.x;
  if (c == 0) s_nbig = 0;
  gevws_conn_in ci{0, 0};
  uint64_t nf = 0, pb = 0, pl = 0, err = 0, same = 0, lastf = ~0ull, pos = 0;
  int32_t st = GEVWS_OK;
  if (c < n) {
    ci = conns[c];
    if (out_of_order(conns, c, ci)) err = 1ull << 32;  // informational, as k_walk_count
    if (ci.off > in_bytes || ci.len > in_bytes - ci.off) {
      ci.off = 0;
      ci.len = 0;
      st = GEVWS_ERR_INVALID;
      err += 1;
    }
    const uint8_t* s = in + ci.off;
    for (;;) {  // read.go:19-84 + the protocol.go:47 gate, frame after frame
      uint64_t lo, hi;
      load_window(s + pos, lo, hi);
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
  const uint64_t v[kDecFields] = {nf, pb, pl, err, same};
  uint64_t ex[kDecFields], tot[kDecFields];
  block_excl_scan<kSmallConns, kDecFields>(v, ex, tot);
  const bool ok = tot[0] <= max_frames && tot[1] <= payload_cap;
  if (c == 0) {
    gevws_summary sm;
    memset(&sm, 0, sizeof(sm));
    sm.frames = tot[0];
    sm.payload_bytes = tot[1];
    sm.payload_len = tot[2];
    sm.errors = tot[3] & 0xffffffffull;
    sm.flags = (tot[3] >> 32) ? GEVWS_SUMMARY_UNORDERED : 0u;
    sm.run_frames = tot[4];
    sm.status = ok ? GEVWS_OK : GEVWS_ERR_CAPACITY;
    *sum = sm;
  }
  if (!ok) {  // capacity error: nothing written (uniform)
    signal_done(done, seq);
    return;
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
    const uint8_t* s = in + ci.off;
    uint64_t q = 0, poff = ex[1];
    for (uint64_t k = 0; k < nf; ++k) {
      uint64_t lo, hi;
      load_window(s + q, lo, hi);
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
          if ((uint32_t)j < nch) x[j] = ld16u(in + src + 16ull * j);
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
    for (uint64_t j = c; 16 * j < L; j += kSmallConns) {
      u32x4 y = ld16u(in + src + 16 * j) ^ key;
      const int64_t rem = (int64_t)L - (int64_t)(16 * j);
      if (rem < 16) y = keep_bytes(y, rem);
      *reinterpret_cast<u32x4*>(payload + poff + 16 * j) = y;
    }
  }
  signal_done(done, seq);
}

// ------------------------------------------------------------------ 4. unmask / compact
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

template <int U, bool NTL, bool WSPAN>
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
    for (int u = 0; u < U; ++u) st16_nt(dst + base + u * kStride, v[u]);
  }
  for (; t < tend; ++t) {
    const uint64_t base = t * kTile + lane_off;
    st16_nt(dst + base, copy_ld<NTL>(src + base));
  }
  // bytes past the last whole tile: 16 per lane, workgroup 0
  const uint64_t tail = ntiles * kTile;
  if (blockIdx.x == 0)
    for (uint64_t p = tail + lane_off; p < n; p += kTile) st16_nt(dst + p, copy_ld<NTL>(src + p));
}

// The unmask = ws.Cipher (cipher.go:14-53) of every frame's payload into its
// 16-aligned slot of the payload arena (protocol.go:50-55: the zeroed make +
// Read + Cipher; pad bytes zero).  Each workgroup owns a contiguous run of 4
// KiB output tiles.  While one frame covers the next U tiles the loop streams
// (stream_step); otherwise it takes a window of tiles whose frames' records it
// loads into LDS, and each lane looks up the frame of each of its chunks.
constexpr int kWinTiles = 4;      // v3 window (tiles)
constexpr int kWinFrames = 1024;  // frames a window's LDS table holds (more: the per-lane fallback)

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
                                               uint32_t big_grid, const WinLds& L) {
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
  uint64_t t = (uint64_t)blockIdx.x * per;
  const uint64_t tend = t + per < ntiles ? t + per : ntiles;
  const uint32_t lane_off = threadIdx.x * 16;
  uint64_t f_po = 0, f_end = 0, f_src = 0;
  int64_t f_len = 0;
  uint32_t f_key = 0;
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
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

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
  uint32_t* tmap;   // [kTmapN] tile_first[tm0 ...]
};

template <int U>
__device__ __forceinline__ void unmask_v5_body(const uint8_t* __restrict__ in, const gevws_frame* __restrict__ frames,
                                               const uint32_t* __restrict__ tile_first,
                                               const gevws_summary* __restrict__ sum, uint8_t* __restrict__ out,
                                               uint32_t big_grid, const WinLds5& L, bool wide = false) {
  constexpr int WT = 8;
  static_assert(WT * kTile / 16 == kWinChunks && kWinChunks == 8 * kUnmaskBlock, "8 chunks per thread");
  if (sum->status != GEVWS_OK) return;
  const uint64_t total = sum->payload_bytes;
  const uint64_t nframes = sum->frames;
  const uint64_t ntiles = (total + kTile - 1) / kTile;
  const uint32_t groups = active_groups(total, nframes, big_grid, wide);
  if (blockIdx.x >= groups) return;
  const uint64_t per = (ntiles + groups - 1) / groups;
  uint64_t t = (uint64_t)blockIdx.x * per;
  const uint64_t tend = t + per < ntiles ? t + per : ntiles;
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
}

// The default unmask: the batch's own statistics pick the window scheme --
// batches of equal-size frames (at least half of the frames the size of the
// one before them on the connection: C1, C2, C3, C5) take v3's 4-tile windows,
// mixed ones (C4) v5's pipelined 8-tile windows, with the whole (wide) grid
// for a batch of fewer than kWideGridTiles tiles.  One kernel, one LDS
// budget, the choice is a uniform branch on the summary the walk wrote.
__global__ __launch_bounds__(kUnmaskBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_unmask_auto5(
    const uint8_t* __restrict__ in, const gevws_frame* __restrict__ frames, const uint32_t* __restrict__ tile_first,
    const gevws_summary* __restrict__ sum, uint8_t* __restrict__ out, uint32_t big_grid) {
  static_assert(kWinFrames == kWin5Frames, "one frame table for both bodies");
  __shared__ uint32_t s_start[kWinFrames];
  __shared__ int32_t s_lend[kWinFrames];
  __shared__ uint64_t s_delta[kWinFrames];
  __shared__ uint32_t s_key[kWinFrames];
  __shared__ __attribute__((aligned(16))) uint16_t s_own[2 * kWinChunks];
  __shared__ uint32_t s_wtot[2 * (kUnmaskBlock / 64)];
  __shared__ uint32_t s_tmap[kTmapN];
  if (2 * sum->run_frames >= sum->frames)
    unmask_v3_body<16>(in, frames, tile_first, sum, out, big_grid, WinLds{s_start, s_lend, s_delta, s_key});
  else
    unmask_v5_body<16>(in, frames, tile_first, sum, out, big_grid,
                       WinLds5{s_lend, s_delta, s_key, s_own, s_wtot, s_tmap},
                       sum->payload_bytes / kTile < kWideGridTiles);
}

// v5 for every batch (GEVWS_TUNE_UNMASK_VARIANT 1): the mixed-size path on any
// batch, so the parity tests run it over equal-size frames too.
__global__ __launch_bounds__(kUnmaskBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_unmask_v5(
    const uint8_t* __restrict__ in, const gevws_frame* __restrict__ frames, const uint32_t* __restrict__ tile_first,
    const gevws_summary* __restrict__ sum, uint8_t* __restrict__ out, uint32_t big_grid) {
  __shared__ int32_t s_lend[kWin5Frames];
  __shared__ uint64_t s_delta[kWin5Frames];
  __shared__ uint32_t s_key[kWin5Frames];
  __shared__ __attribute__((aligned(16))) uint16_t s_own[2 * kWinChunks];
  __shared__ uint32_t s_wtot[2 * (kUnmaskBlock / 64)];
  __shared__ uint32_t s_tmap[kTmapN];
  unmask_v5_body<16>(in, frames, tile_first, sum, out, big_grid,
                     WinLds5{s_lend, s_delta, s_key, s_own, s_wtot, s_tmap},
                     sum->payload_bytes / kTile < kWideGridTiles);
}

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
                                                         const gevws_summary* __restrict__ gate = nullptr) {
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

// The LDS frame table of an encode window.  LH: the serialised headers are
// not kept in LDS (h0 / h1 unused) but rebuilt from the frame's record (an L2
// hit: the window just loaded it), which frees 16 KiB of LDS per workgroup for
// occupancy -- k_encode; the one-workgroup k_handle_small keeps them in LDS.
struct EncWin {
  const int32_t* start;  // wire start relative to the window, clamped >= -64
  const int32_t* pend;   // payload end relative to the window, clamped
  const uint8_t* hlen;
  const uint64_t* delta;  // payload_off - out_off - hlen (mod 2^64)
  const uint64_t* h0;     // !LH: serialised header bytes 0-7 / 8-15
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
template <bool LH>
__device__ __forceinline__ void enc_assemble_from(u128& acc, int32_t rel, uint64_t a, int kmax, uint32_t j, uint32_t F,
                                                  const EncWin& W, const uint8_t* __restrict__ payload,
                                                  const gevws_out_frame* __restrict__ fr, uint64_t f_lo) {
  for (; j < F && W.start[j] < rel + kmax; ++j) {
    const int32_t hs = W.start[j];
    const int32_t ps = hs + (int32_t)W.hlen[j];
    const int32_t pe = W.pend[j];
    // header bytes [max(hs, rel), min(ps, rel + kmax))
    const int32_t h0 = hs > rel ? hs : rel;
    const int32_t h1 = ps < rel + kmax ? ps : rel + kmax;
    if (h0 < h1) {
      u128 H;
      if constexpr (LH) {
        uint64_t hl, hh;
        enc_header(fr[f_lo + j].hdr, hl, hh);
        H = (u128)hl | ((u128)hh << 64);
      } else {
        H = (u128)W.h0[j] | ((u128)W.h1[j] << 64);
      }
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

template <bool LH>
__device__ __forceinline__ u32x4 enc_assemble(int32_t rel, uint64_t a, uint64_t total, uint32_t lo, uint32_t F,
                                              const EncWin& W, const uint8_t* __restrict__ payload,
                                              const gevws_out_frame* __restrict__ fr, uint64_t f_lo) {
  const int kmax = (a + 16 <= total) ? 16 : (int)(total - a);
  int32_t hs[2], h0[2], h1[2], p0[2], p1[2];
  u32x4 pv[2];
  u64x2 hv[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const uint32_t j = lo + k;
    const bool in = j < F && W.start[j < F ? j : lo] < rel + kmax;
    const uint32_t jj = in ? j : lo;
    hs[k] = W.start[jj];
    const int32_t ps = hs[k] + (int32_t)W.hlen[jj];
    const int32_t pe = W.pend[jj];
    h0[k] = hs[k] > rel ? hs[k] : rel;
    h1[k] = in ? (ps < rel + kmax ? ps : rel + kmax) : h0[k];
    p0[k] = ps > rel ? ps : rel;
    p1[k] = in ? (pe < rel + kmax ? pe : rel + kmax) : p0[k];
    pv[k] = u32x4{0, 0, 0, 0};
    hv[k] = u64x2{0, 0};
    if (p0[k] < p1[k]) pv[k] = ld16u(payload + (a + (uint64_t)(p0[k] - rel) + W.delta[jj]));
    if (h0[k] < h1[k]) {
      if constexpr (LH) hv[k] = *reinterpret_cast<const u64x2*>(fr + f_lo + jj);  // the header half of the record
      else hv[k] = u64x2{W.h0[jj], W.h1[jj]};
    }
  }
  u128 acc = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    if (h0[k] < h1[k]) {
      u128 H;
      if constexpr (LH) {
        gevws_header hd;
        memcpy(&hd, &hv[k], 16);
        uint64_t hl, hh;
        enc_header(hd, hl, hh);
        H = (u128)hl | ((u128)hh << 64);
      } else {
        H = (u128)hv[k][0] | ((u128)hv[k][1] << 64);
      }
      acc |= ((H >> (8 * (h0[k] - hs[k]))) << (8 * (h0[k] - rel))) & byte_mask(h0[k] - rel, h1[k] - rel);
    }
    if (p0[k] < p1[k]) {
      const int k0 = p0[k] - rel;
      acc |= (u128_of(pv[k]) << (8 * k0)) & byte_mask(k0, p1[k] - rel);
    }
  }
  if (lo + 2 < F && W.start[lo + 2] < rel + kmax)  // more frames in these 16 bytes
    enc_assemble_from<LH>(acc, rel, a, kmax, lo + 2, F, W, payload, fr, f_lo);
  return u32x4_of(acc);
}

// The encode's byte stream (k_enc_size / k_enc_emit placed every frame's wire
// bytes and the output-tile -> frame map).  Each workgroup owns a contiguous
// run of output tiles.
//  * Inside one payload for the next U tiles: stream (a misaligned source as
//    the unmask's streaming path: wave-contiguous U KiB spans, aligned
//    non-temporal loads, DPP rotate + v_alignbyte; an aligned one with plain
//    loads), aligned non-temporal stores.
//  * Otherwise a window of kWinTiles tiles: its frames' wire starts, payload
//    ends, header lengths and payload offsets in LDS; each lane finds the
//    frame of each of its chunks by binary search; a chunk inside one payload
//    is loaded (unaligned) and stored; a chunk that straddles a frame boundary
//    (header bytes or two frames' pieces) is queued in LDS and assembled
//    afterwards by the whole workgroup, one chunk per lane, instead of by the
//    one or two lanes of each wave that meet them while the other lanes wait.
//    A 64-byte group of chunks holding a boundary is queued whole (its
//    interior chunks with it, four consecutive slots), so one store writes the
//    group's 64 bytes: otherwise every frame boundary left its line to HBM as
//    two partial writes (C4: 46 M 32-byte write requests per launch, 0 with
//    it; the whole C4 encode 10.70 -> 9.11 ms, profiles/r02/r02_encode_ab_g64_*.json).
//    All the window's payload loads are issued before its stores, and the
//    interior chunks are stored only after the queue barrier and the lane's
//    first queued chunk has been assembled, so the interior loads and the first
//    assembly's loads are in flight together (C4 9.39 -> 9.17 ms,
//    profiles/r03/r03_encode_eo_ab.jsonl).
// The window path is latency-bound: the kernel is held to 72 VGPRs for 7
// workgroups per CU (amdgpu_waves_per_eu(7): C2 -4 %, C4 -2 % against 6 per
// CU; 8 per CU at 64 VGPRs was slower on C5, profiles/r01/r01_encode_ab_occ_*.json).
// Measured and not kept: 8-tile windows (C4 9.71 -> 12.23 ms), a chunk ->
// frame map instead of the search (C4 9.35 -> 9.57 ms), non-temporal window
// loads (C4 +8.8 %) -- DESIGN.md §5.
__global__ __launch_bounds__(kUnmaskBlock) __attribute__((amdgpu_waves_per_eu(7))) void k_encode(
    const gevws_out_frame* __restrict__ fr, const uint8_t* __restrict__ payload, const uint64_t* __restrict__ out_off,
    const uint32_t* __restrict__ tile_first, const gevws_summary* __restrict__ sum, uint8_t* __restrict__ out,
    uint32_t big_grid) {
  constexpr int U = 4, WT = kWinTiles, WF = kEncWinFrames;
  __shared__ int32_t s_start[WF];
  __shared__ int32_t s_pend[WF];
  __shared__ uint8_t s_hlen[WF];
  __shared__ uint32_t s_bnd[WT * kUnmaskBlock];  // queued chunk: rel / 16 | frame << 16 (~0: a group's filler)
  __shared__ uint32_t s_nb;
  __shared__ uint64_t s_delta[WF];
  const EncWin W{s_start, s_pend, s_hlen, s_delta, nullptr, nullptr};
  if (sum->status != GEVWS_OK) return;
  const uint64_t total = sum->payload_bytes;  // wire bytes
  const uint64_t nframes = sum->frames;
  const uint64_t ntiles = (total + kTile - 1) / kTile;
  const uint32_t groups = active_groups(total, nframes, big_grid);
  if (blockIdx.x >= groups) return;
  const uint64_t per = (ntiles + groups - 1) / groups;
  uint64_t t = (uint64_t)blockIdx.x * per;
  const uint64_t tend = t + per < ntiles ? t + per : ntiles;
  uint64_t c_ps = 0, c_pe = 0, c_delta = 0;  // cached frame: payload [c_ps, c_pe) in wire coordinates
  while (t < tend) {
    const uint32_t lane_off = fresh_tid() * 16;  // recomputed per step: held, it was spilled
    const uint64_t base = t * kTile;
    if (base >= c_pe) {  // workgroup-uniform refresh (scalar loads)
      const uint64_t f = tile_first[t];
      const gevws_out_frame o = fr[f];
      c_ps = out_off[f] + enc_hlen(o.hdr);
      c_pe = c_ps + o.payload_len;
      c_delta = o.payload_off - c_ps;
    }
    if (t + U <= tend && base >= c_ps && base + U * kTile <= c_pe) {  // inside one payload: stream
      u32x4 v[U];
      const uint8_t* s0 = payload + (base + c_delta);
      const uint32_t mis = (uint32_t)(reinterpret_cast<uint64_t>(s0) & 15);  // wave-uniform
      if (mis != 0) {
        const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
        const uint64_t wrel = (uint64_t)wave * U * 1024 + lane * 16;
        const uint8_t* a = s0 + wrel - mis;
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
          st16_nt(d + u * 1024, funnel16(v[u], last ? rn : r, mis));
          r = rn;
        }
        t += U;
        continue;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = ld16u(payload + (base + u * kTile + lane_off + c_delta));
#pragma unroll
      for (int u = 0; u < U; ++u) st16_nt(out + base + u * kTile + lane_off, v[u]);
      t += U;
      continue;
    }
    const uint64_t wt = (tend - t) < (uint64_t)WT ? (tend - t) : (uint64_t)WT;
    const uint64_t wbase = base;
    const uint64_t f_lo = tile_first[t];
    const uint64_t f_hi = (t + wt) < ntiles ? (uint64_t)tile_first[t + wt] : nframes - 1;
    const uint64_t F = f_hi - f_lo + 1;
    if (F <= (uint64_t)WF) {
      __syncthreads();
      for (uint64_t i = fresh_tid(); i < F; i += kUnmaskBlock) {
        const gevws_out_frame o = fr[f_lo + i];
        const uint32_t hl = enc_hlen(o.hdr);
        const uint64_t oo = out_off[f_lo + i];
        const int64_t st = (int64_t)(oo - wbase);
        s_start[i] = st < -64 ? -64 : (int32_t)st;
        const int64_t pe = st + hl + (int64_t)o.payload_len;
        s_pend[i] = pe > 0x7fffffffll ? 0x7fffffff : (int32_t)pe;
        s_hlen[i] = hl;
        s_delta[i] = o.payload_off - oo - hl;
      }
      if (threadIdx.x == 0) s_nb = 0;
      __syncthreads();
      // every chunk's frame and kind first (interior of one payload, or a
      // boundary to queue); a load inside the interior/boundary branch made
      // the compiler wait for it at the branch's join
      u32x4 v[WT];
      uint32_t interior = 0, queued = 0;
      uint32_t qlo[WT];
#pragma unroll
      for (int u = 0; u < WT; ++u) {
        const int32_t rel = u * (int32_t)kTile + (int32_t)lane_off;
        const uint64_t a = wbase + (uint64_t)rel;
        const bool valid = (uint64_t)u < wt && a < total;
        uint32_t lo = 0, hi = valid ? (uint32_t)F - 1 : 0u;
        while (lo < hi) {
          const uint32_t mid = (lo + hi + 1) >> 1;
          if (s_start[mid] <= rel) lo = mid; else hi = mid - 1;
        }
        const bool in = valid && rel >= s_start[lo] + (int32_t)s_hlen[lo] && rel + 16 <= s_pend[lo];
        qlo[u] = lo;
        interior |= (in ? 1u : 0u) << u;
        queued |= (valid && !in ? 1u : 0u) << u;
      }
      // 64-byte groups holding a queued chunk go to the queue whole
      const uint32_t lane = threadIdx.x & 63, g0 = lane & ~3u;
#pragma unroll
      for (int u = 0; u < WT; ++u) {
        const uint64_t bal = __ballot((queued >> u) & 1u);  // whole wave active
        const bool defer = ((bal >> g0) & 0xFull) != 0;     // (group-uniform)
        uint32_t slot = 0;
        if (defer && (lane & 3u) == 0) slot = atomicAdd(&s_nb, 4u);
        slot = __shfl(slot, (int)g0);
        if (defer) {
          const bool valid = (interior | queued) & (1u << u);
          s_bnd[slot + (lane & 3u)] =
              valid ? ((uint32_t)(u * (int32_t)kTile + (int32_t)lane_off) >> 4) | (qlo[u] << 16) : 0xffffffffu;
          interior &= ~(1u << u);
        }
      }
      // the interior loads (the queue pass loads its chunks itself; every lane
      // loads, a non-interior chunk from payload[0], always readable, unused)
#pragma unroll
      for (int u = 0; u < WT; ++u) {
        const bool in = (interior >> u) & 1u;
        const uint64_t a = wbase + (uint64_t)(u * (int32_t)kTile + (int32_t)lane_off);
        v[u] = ld16u(payload + (in ? a + s_delta[qlo[u]] : 0ull));
      }
      __syncthreads();  // the queue is complete
      const uint32_t nb = s_nb;
      const uint32_t i0 = fresh_tid();
      u32x4 x0 = u32x4{0, 0, 0, 0};
      uint32_t q0 = 0xffffffffu;
      if (i0 < nb) {
        q0 = s_bnd[i0];
        if (q0 != 0xffffffffu) {
          const int32_t rel = (int32_t)((q0 & 0xffffu) << 4);
          x0 = enc_assemble<true>(rel, wbase + (uint64_t)rel, total, q0 >> 16, (uint32_t)F, W, payload, fr, f_lo);
        }
      }
#pragma unroll
      for (int u = 0; u < WT; ++u)
        if (interior & (1u << u)) st16_nt(out + wbase + u * kTile + fresh_tid() * 16, v[u]);
      if (q0 != 0xffffffffu) st16_nt(out + wbase + (uint64_t)((q0 & 0xffffu) << 4), x0);
      for (uint32_t i = i0 + kUnmaskBlock; i < nb; i += kUnmaskBlock) {
        const uint32_t q = s_bnd[i];
        if (q == 0xffffffffu) continue;  // a group's slot past the batch's end
        const int32_t rel = (int32_t)((q & 0xffffu) << 4);
        const uint64_t a = wbase + (uint64_t)rel;
        st16_nt(out + a, enc_assemble<true>(rel, a, total, q >> 16, (uint32_t)F, W, payload, fr, f_lo));
      }
      t += wt;
      continue;
    }
    // more than kEncWinFrames frames in the window (frames of a few bytes):
    // one tile, per-lane global lookup and byte assembly
    {
      const uint64_t a = t * kTile + lane_off;
      if (a < total) {
        uint64_t lo = tile_first[t];
        uint64_t hi = (t + 1 < ntiles) ? (uint64_t)tile_first[t + 1] : nframes - 1;
        while (lo < hi) {
          const uint64_t mid = (lo + hi + 1) >> 1;
          if (out_off[mid] <= a) lo = mid; else hi = mid - 1;
        }
        uint32_t w[4] = {0, 0, 0, 0};
        uint64_t j = lo;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          while (j + 1 < nframes && out_off[j + 1] <= a + k) ++j;
          const uint32_t byte = (a + k < total) ? enc_byte_global(fr, out_off, payload, j, a + k) : 0u;
          w[k >> 2] |= byte << (8 * (k & 3));
        }
        *reinterpret_cast<u32x4*>(out + a) = u32x4{w[0], w[1], w[2], w[3]};
      }
      t += 1;
    }
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
// (enc_assemble: headers rebuilt from the records, payloads by unaligned
// loads).  Outputs and summaries are exactly the two-step chain's (seven
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
                                                            uint32_t seq = 0) {
  constexpr int WF = (int)kHandleSmallFrames;
  __shared__ int32_t s_start[WF];
  __shared__ int32_t s_pend[WF];
  __shared__ uint8_t s_hlen[WF];
  __shared__ uint64_t s_delta[WF];
  __shared__ uint64_t s_h0[WF], s_h1[WF];
  __shared__ uint32_t s_status;
  const uint32_t tid = threadIdx.x;
  const uint64_t n = gated_count(max_frames, dec);
  // 1. dispatch counts (k_disp_count + k_scan_blocks)
  uint64_t rep_n = 0, aux_n = 0, shut_n = 0;
  for (uint64_t f0 = 0; f0 < n; f0 += kWalkBlock) {  // workgroup-uniform
    const uint64_t f = f0 + tid;
    uint32_t op = 0;
    const int k = f < n ? disp_kind(fr[f].hdr, policy, op) : 0;
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
        in = fr[f];
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
    signal_done(done, seq);
    return;
  }
  // 4. the wire image, 16 bytes per lane (the last chunk's tail zeroed inside
  // the GEVWS_OUT_PAD slack)
  for (uint64_t a = (uint64_t)tid * 16; a < wire; a += (uint64_t)kWalkBlock * 16) {
    const int32_t rel = (int32_t)a;
    uint32_t lo = 0, hi = (uint32_t)nr - 1;  // the last reply starting at or before a
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (s_start[mid] <= rel) lo = mid; else hi = mid - 1;
    }
    const u32x4 x = enc_assemble<false>(rel, a, wire, lo, (uint32_t)nr, EncWin{s_start, s_pend, s_hlen, s_delta, s_h0, s_h1},
                                        payload, nullptr, 0);
    __builtin_memcpy(out + a, &x, 16);
  }
  signal_done(done, seq);
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

// ------------------------------------------------------------------ synthetic frames
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ u32x4 plain16(uint64_t seed, uint64_t g, uint64_t i) {
  const uint64_t b = seed ^ (g * 0x9E3779B97F4A7C15ull);
  const uint64_t w0 = splitmix64(b + (i >> 3));
  const uint64_t w1 = splitmix64(b + (i >> 3) + 1);
  return u32x4{(uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)};
}

__device__ __forceinline__ uint32_t synth_hlen(const gevws_synth_desc& d) {
  return 2 + (d.len_form == 7 ? 0 : (d.len_form == 16 ? 2 : 8)) + (d.masked ? 4 : 0);
}

__global__ __launch_bounds__(256) void k_synth(uint8_t* __restrict__ in,
                                               const gevws_synth_desc* __restrict__ desc,
                                               uint64_t n_frames, uint64_t seed) {
  for (uint64_t g = blockIdx.x; g < n_frames; g += gridDim.x) {
    const gevws_synth_desc d = desc[g];
    const uint32_t hlen = synth_hlen(d);
    uint8_t* h = in + d.hdr_off;
    if (threadIdx.x == 0) {
      h[0] = d.b0;
      const uint8_t mbit = d.masked ? 0x80 : 0;
      uint32_t e = 2;
      if (d.len_form == 7) {
        h[1] = mbit | (uint8_t)d.length;
      } else if (d.len_form == 16) {
        h[1] = mbit | 126;
        h[2] = (uint8_t)(d.length >> 8);
        h[3] = (uint8_t)d.length;
        e = 4;
      } else {
        h[1] = mbit | 127;
        for (int k = 0; k < 8; ++k) h[2 + k] = (uint8_t)(d.length >> (56 - 8 * k));
        e = 10;
      }
      if (d.masked)
        for (int k = 0; k < 4; ++k) h[e + k] = (uint8_t)(d.mask >> (8 * k));
    }
    uint8_t* pl = h + hlen;
    const uint32_t key = d.masked ? d.mask : 0u;
    for (uint64_t i = (uint64_t)threadIdx.x * 16; i < d.length; i += 256 * 16) {
      const u32x4 x = plain16(seed, g, i) ^ key;
      if (i + 16 <= d.length) {
        __builtin_memcpy(pl + i, &x, 16);
      } else {
        for (uint32_t b = 0; b < d.length - i; ++b) pl[i + b] = (uint8_t)(x[b >> 2] >> (8 * (b & 3)));
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_synth_verify(const gevws_synth_desc* __restrict__ desc,
                                                      uint64_t n_frames, uint64_t seed,
                                                      const gevws_frame* __restrict__ frames,
                                                      const uint8_t* __restrict__ payload,
                                                      uint64_t payload_cap,
                                                      unsigned long long* __restrict__ mismatch) {
  uint64_t bad = 0;
  for (uint64_t g = blockIdx.x; g < n_frames; g += gridDim.x) {
    const gevws_synth_desc d = desc[g];
    const gevws_frame fr = frames[g];
    if (fr.payload_off > payload_cap || round16(d.length) > payload_cap - fr.payload_off) {
      bad += threadIdx.x == 0 ? d.length + 1 : 0;  // record out of range: never dereferenced
      continue;
    }
    if (threadIdx.x == 0) {
      uint32_t k;
      memcpy(&k, fr.hdr.mask, 4);
      bad += fr.hdr.fin != (d.b0 >> 7);
      bad += fr.hdr.rsv != ((d.b0 & 0x70) >> 4);
      bad += fr.hdr.opcode != (d.b0 & 0x0f);
      bad += fr.hdr.masked != d.masked;
      bad += k != (d.masked ? d.mask : 0u);
      bad += (uint64_t)fr.hdr.length != d.length;
      bad += fr.src_off != d.hdr_off + synth_hlen(d);
      bad += (fr.payload_off & 15) != 0;
    }
    const uint64_t padded = round16(d.length);
    for (uint64_t i = (uint64_t)threadIdx.x * 16; i < padded; i += 256 * 16) {
      u32x4 want = plain16(seed, g, i);
      if (d.length - i < 16) want = keep_bytes(want, (int64_t)(d.length - i));
      const u32x4 got = *reinterpret_cast<const u32x4*>(payload + fr.payload_off + i);
      const u32x4 x = got ^ want;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        for (int b = 0; b < 4; ++b) bad += ((x[j] >> (8 * b)) & 0xff) != 0;
    }
  }
  const uint64_t w = wave_sum(bad);
  if ((threadIdx.x & 63) == 0 && w) atomicAdd(mismatch, (unsigned long long)w);
}

}  // namespace

// ====================================================================== C ABI
struct gevws_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  bool timing = false;
  struct EventSet {
    hipEvent_t e[5];
  };
  std::vector<EventSet> evs;  // one set per timed call since the last gevws_ctx_timing
  size_t evs_used = 0;
  gevws_summary* d_sum = nullptr;  // summary slot of the synchronous entry point
  int unmask_variant = 0;  // GEVWS_TUNE_UNMASK_VARIANT (kUnmaskVariants)
  int unmask_grid = 0;     // 0 = auto
  int encode_variant = 0;  // GEVWS_TUNE_ENCODE_VARIANT (kNumEncodeVariants)
  uint64_t small_bytes = kSmallBytes;  // one-launch decode (k_decode_small) up to this many input bytes
  uint32_t* done_flag = nullptr;  // mapped host word the one-launch kernels signal (gevws_ctx_set_completion_flag)
  uint32_t done_seq = 0;
  int64_t last_signal = -1;  // the value the last call's last kernel stores there, -1: none
  // the context's history: the last multi-kernel decode's frame / payload /
  // equal-size-run totals (written by k_walk_bases into mapped host memory)
  // and its connection count, read once that decode has finished; it picks
  // the split walk, the walk's speculation and the unmask's wide grid
  uint64_t* h_stats = nullptr;
  uint64_t* d_stats = nullptr;
  bool stats_pending = false, stats_known = false;
  uint64_t stats_conns = 0, prev_frames_per_conn = 0, prev_frame_bytes = 0;
  bool prev_mixed = false;
  uint32_t last_unmask_grid = 0;  // workgroups of the last decode's unmask launch
  uint32_t last_ks = 1;    // lanes per connection of the last multi-kernel decode's walk
  uint32_t split_lanes = 0;  // lanes per connection (k_walk_split); 0 = auto, 1 = off
  uint64_t split_min_bytes = kSplitMinBytes;        // split walk: bytes per segment at least
  uint64_t split_lanes_per_cu = kSplitLanesPerCU;   // split walk auto: lanes per CU at most
  int walk_variant = 0;    // 0 = speculation (D = 8) unless the history is mixed, 1 = plain chain walk
                           // (D = 0), 2 = no entry table (the record pass re-walks every chain), 3 =
                           // the writer wave whatever the batch size
  // Scratch is per context: calls on a different stream than the previous one
  // first wait for it (one in-flight batch per context; use one context per
  // stream for concurrency).
  hipEvent_t last_done = nullptr;
  hipStream_t last_stream = nullptr;
  bool has_last = false;
  int num_cus = 256;
  uint32_t* d_done = nullptr;  // the decode walk's finished-workgroup counter (zero between calls)
  // split-stream decode (gevws_ctx_set_unmask_stream): the unmask on its own
  // stream after the record pass (front_done), its grid for unmask_cus CUs
  hipStream_t unmask_stream = nullptr;
  int unmask_cus = 0;
  hipEvent_t front_done = nullptr;
};

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

#define GEVWS_HIP(call)                                                                \
  do {                                                                                  \
    hipError_t e_ = (call);                                                             \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "[gevws] %s failed: %s\n", #call, hipGetErrorString(e_));          \
      return GEVWS_ERR_DEVICE;                                                          \
    }                                                                                   \
  } while (0)

// NULL = the HIP default (null) stream, as in every HIP/CUDA API; callers
// that want the context's own stream pass gevws_ctx_stream(ctx).
hipStream_t pick_stream(gevws_ctx* ctx, void* stream) {
  (void)ctx;
  return reinterpret_cast<hipStream_t>(stream);
}

// Orders this call after the context's previous one when the stream changes.
int order_after_last(gevws_ctx* ctx, hipStream_t st) {
  if (ctx->has_last && ctx->last_stream != st) GEVWS_HIP(hipStreamWaitEvent(st, ctx->last_done, 0));
  return GEVWS_OK;
}

int mark_last(gevws_ctx* ctx, hipStream_t st) {
  ctx->last_signal = -1;  // (the one-launch paths set it after this)
  GEVWS_HIP(hipEventRecord(ctx->last_done, st));
  ctx->last_stream = st;
  ctx->has_last = true;
  return GEVWS_OK;
}

int ensure_scratch(gevws_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->scratch_bytes) return GEVWS_OK;
  if (ctx->scratch) {
    GEVWS_HIP(hipDeviceSynchronize());
    GEVWS_HIP(hipFree(ctx->scratch));
    ctx->scratch = nullptr;
    ctx->scratch_bytes = 0;
  }
  size_t want = bytes + bytes / 4 + 4096;
  GEVWS_HIP(hipMalloc(&ctx->scratch, want));
  ctx->scratch_bytes = want;
  return GEVWS_OK;
}

using UnmaskFn = void (*)(const uint8_t*, const gevws_frame*, const uint32_t*, const gevws_summary*, uint8_t*,
                         uint32_t);
struct UnmaskVariant {
  UnmaskFn fn;
  int unroll;
  const char* name;
  bool wide = false;  // may launch the wide grid (k_unmask_auto)
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
};
constexpr int kNumUnmaskVariants = sizeof(kUnmaskVariants) / sizeof(kUnmaskVariants[0]);

// GEVWS_TUNE_WALK_VARIANT values (0 = the default choice per batch).
const char* const kWalkVariants[] = {
    "default: one lane per connection with uniform-stream speculation (D = 8; plain D = 0 after a batch of mixed "
    "sizes on this context); from 128 connections per CU the entries go through an LDS ring to a writer wave "
    "(256-byte groups); the split walk for few long chains of small frames",
    "one lane per connection, plain chain walk (D = 0)",
    "no entry table (the record pass re-walks every chain)",
    "entries through the writer wave whatever the batch size (the default's path for >= 128 connections per CU)",
};
constexpr int kNumWalkVariants = sizeof(kWalkVariants) / sizeof(kWalkVariants[0]);
constexpr int kNumEncodeVariants = 1;  // GEVWS_TUNE_ENCODE_VARIANT: 0 = k_encode

}  // namespace

static int launch_unmask(gevws_ctx* ctx, hipStream_t st, uint64_t payload_cap, const uint8_t* d_in,
                  const gevws_frame* d_frames, const uint32_t* tile_first, const gevws_summary* d_summary,
                  uint8_t* d_payload);

extern "C" {

int gevws_abi_version(void) { return GEVWS_ABI_VERSION; }

const char* gevws_status_string(int s) {
  switch (s) {
    case GEVWS_OK: return "ok";
    case GEVWS_NEED_MORE: return "header error: not enough";  // ws.ErrHeaderNotReady text
    case GEVWS_ERR_LEN_MSB: return "header error: the most significant bit must be 0";
    case GEVWS_ERR_CAPACITY: return "output capacity exceeded";
    case GEVWS_ERR_INVALID: return "invalid argument";
    case GEVWS_ERR_DEVICE: return "HIP device error";
    case GEVWS_HANDSHAKE: return "handshake response";
    case GEVWS_ERR_NOT_UPGRADED: return "connection not upgraded and the protocol has no upgrader";
    case GEVWS_ERR_HANDSHAKE: return "websocket upgrade failed";
    default: return "unknown status";
  }
}

int gevws_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

gevws_ctx* gevws_ctx_create(int device) {
  int n = gevws_device_count();
  if (device < 0 || device >= n) {
    fprintf(stderr, "[gevws] gevws_ctx_create: device %d not available (%d visible)\n", device, n);
    return nullptr;
  }
  DeviceGuard g(device);
  gevws_ctx* ctx = new gevws_ctx();
  ctx->device = device;
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return nullptr;
  }
  if (hipEventCreateWithFlags(&ctx->last_done, hipEventDisableTiming) != hipSuccess) {
    gevws_ctx_destroy(ctx);
    return nullptr;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    ctx->num_cus = prop.multiProcessorCount;
  if (hipMalloc(reinterpret_cast<void**>(&ctx->d_sum), sizeof(gevws_summary)) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&ctx->d_done), 256) != hipSuccess ||
      hipMemset(ctx->d_done, 0, 256) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&ctx->h_stats), 64, hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->d_stats), ctx->h_stats, 0) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    gevws_ctx_destroy(ctx);
    return nullptr;
  }
  return ctx;
}

void gevws_ctx_destroy(gevws_ctx* ctx) {
  if (!ctx) return;
  DeviceGuard g(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->d_sum) (void)hipFree(ctx->d_sum);
  if (ctx->d_done) (void)hipFree(ctx->d_done);
  if (ctx->h_stats) (void)hipHostFree(ctx->h_stats);
  if (ctx->last_done) (void)hipEventDestroy(ctx->last_done);
  if (ctx->front_done) (void)hipEventDestroy(ctx->front_done);
  for (auto& set : ctx->evs)
    for (auto& e : set.e) (void)hipEventDestroy(e);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

int gevws_ctx_device(const gevws_ctx* ctx) { return ctx ? ctx->device : -1; }

void* gevws_ctx_stream(const gevws_ctx* ctx) { return ctx ? reinterpret_cast<void*>(ctx->stream) : nullptr; }

// (also used by the multi-GPU count reduce, gevws_comm.cpp)
int gevws_ctx_order_after_last(gevws_ctx* ctx, void* stream) {
  if (!ctx) return GEVWS_ERR_INVALID;
  DeviceGuard g(ctx->device);
  return order_after_last(ctx, reinterpret_cast<hipStream_t>(stream));
}

int gevws_stream_cu_count(int device, void* stream) {
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n <= 0) return 0;
  if (!stream) return n;
  std::vector<uint32_t> m((size_t)(n + 31) / 32, 0u);
  if (hipExtStreamGetCUMask(reinterpret_cast<hipStream_t>(stream), (uint32_t)m.size(), m.data()) != hipSuccess)
    return n;
  int c = 0;
  for (int i = 0; i < n; ++i) c += (m[(size_t)i / 32] >> (i % 32)) & 1u;
  return c > 0 ? c : n;
}

int gevws_stream_create_cu_mask(int device, const uint32_t* cu_mask, uint32_t n_words, void** stream) {
  if (!cu_mask || !n_words || !stream || device < 0 || device >= gevws_device_count()) return GEVWS_ERR_INVALID;
  *stream = nullptr;
  uint32_t any = 0;
  for (uint32_t i = 0; i < n_words; ++i) any |= cu_mask[i];
  if (!any) return GEVWS_ERR_INVALID;
  DeviceGuard g(device);
  hipStream_t s = nullptr;
  GEVWS_HIP(hipExtStreamCreateWithCUMask(&s, n_words, cu_mask));
  *stream = reinterpret_cast<void*>(s);
  return GEVWS_OK;
}

int gevws_stream_destroy(void* stream) {
  if (!stream) return GEVWS_OK;
  return hipStreamDestroy(reinterpret_cast<hipStream_t>(stream)) == hipSuccess ? GEVWS_OK : GEVWS_ERR_DEVICE;
}

int gevws_ctx_set_unmask_stream(gevws_ctx* ctx, void* unmask_stream) {
  if (!ctx) return GEVWS_ERR_INVALID;
  DeviceGuard g(ctx->device);
  ctx->unmask_stream = reinterpret_cast<hipStream_t>(unmask_stream);
  ctx->unmask_cus = unmask_stream ? gevws_stream_cu_count(ctx->device, unmask_stream) : 0;
  if (ctx->unmask_cus <= 0 || ctx->unmask_cus > ctx->num_cus) ctx->unmask_cus = ctx->num_cus;
  if (unmask_stream && !ctx->front_done &&
      hipEventCreateWithFlags(&ctx->front_done, hipEventDisableTiming) != hipSuccess) {
    ctx->unmask_stream = nullptr;
    return GEVWS_ERR_DEVICE;
  }
  return GEVWS_OK;
}

int gevws_ctx_set_tuning(gevws_ctx* ctx, int key, int64_t value) {
  if (!ctx) return GEVWS_ERR_INVALID;
  switch (key) {
    case GEVWS_TUNE_UNMASK_VARIANT:
      if (value < 0 || value >= kNumUnmaskVariants) return GEVWS_ERR_INVALID;
      ctx->unmask_variant = (int)value;
      return GEVWS_OK;
    case GEVWS_TUNE_UNMASK_GRID:
      if (value < 0 || value > (1 << 20)) return GEVWS_ERR_INVALID;
      ctx->unmask_grid = (int)value;
      return GEVWS_OK;
    case GEVWS_TUNE_ENCODE_VARIANT:
      if (value < 0 || value >= kNumEncodeVariants) return GEVWS_ERR_INVALID;
      ctx->encode_variant = (int)value;
      return GEVWS_OK;
    case GEVWS_TUNE_SMALL_BATCH:
      if (value < 0 || (uint64_t)value > kSmallBytes) return GEVWS_ERR_INVALID;
      ctx->small_bytes = (uint64_t)value;
      return GEVWS_OK;
    case GEVWS_TUNE_SPLIT_LANES:
      if (value < 0 || value > kSplitMaxLanes || (value > 1 && (value & (value - 1)))) return GEVWS_ERR_INVALID;
      ctx->split_lanes = (uint32_t)value;
      return GEVWS_OK;
    case GEVWS_TUNE_WALK_VARIANT:
      if (value < 0 || value >= kNumWalkVariants) return GEVWS_ERR_INVALID;
      ctx->walk_variant = (int)value;
      return GEVWS_OK;
    case GEVWS_TUNE_SPLIT_MIN_BYTES:
      if (value < 1024 || value > (1ll << 30)) return GEVWS_ERR_INVALID;
      ctx->split_min_bytes = (uint64_t)value;
      return GEVWS_OK;
    case GEVWS_TUNE_SPLIT_LANES_PER_CU:
      if (value < 64 || value > 4096) return GEVWS_ERR_INVALID;
      ctx->split_lanes_per_cu = (uint64_t)value;
      return GEVWS_OK;
    default:
      return GEVWS_ERR_INVALID;
  }
}

const char* gevws_tuning_name(int key, int64_t value) {
  if (key == GEVWS_TUNE_UNMASK_VARIANT && value >= 0 && value < kNumUnmaskVariants)
    return kUnmaskVariants[value].name;
  if (key == GEVWS_TUNE_WALK_VARIANT && value >= 0 && value < kNumWalkVariants) return kWalkVariants[value];
  return nullptr;
}

int gevws_ctx_last_split_lanes(const gevws_ctx* ctx) { return ctx ? (int)ctx->last_ks : -1; }

int gevws_ctx_set_completion_flag(gevws_ctx* ctx, uint32_t* d_flag) {
  if (!ctx) return GEVWS_ERR_INVALID;
  ctx->done_flag = d_flag;
  ctx->last_signal = -1;
  return GEVWS_OK;
}

int64_t gevws_ctx_completion_seq(const gevws_ctx* ctx) { return ctx ? ctx->last_signal : -1; }

int gevws_ctx_last_unmask_grid(const gevws_ctx* ctx) { return ctx ? (int)ctx->last_unmask_grid : -1; }

int gevws_ctx_set_timing(gevws_ctx* ctx, int enable) {
  if (!ctx) return GEVWS_ERR_INVALID;
  ctx->timing = enable != 0;
  return GEVWS_OK;
}

int gevws_ctx_timing(gevws_ctx* ctx, float ms_sum[4], uint32_t* calls) {
  if (!ctx || !ms_sum || !calls) return GEVWS_ERR_INVALID;
  DeviceGuard g(ctx->device);
  float acc[4] = {0, 0, 0, 0};
  for (size_t k = 0; k < ctx->evs_used; ++k) {
    auto& set = ctx->evs[k];
    GEVWS_HIP(hipEventSynchronize(set.e[4]));
    for (int i = 0; i < 4; ++i) {
      float t = 0;
      GEVWS_HIP(hipEventElapsedTime(&t, set.e[i], set.e[i + 1]));
      acc[i] += t;
    }
  }
  for (int i = 0; i < 4; ++i) ms_sum[i] = acc[i];
  *calls = (uint32_t)ctx->evs_used;
  ctx->evs_used = 0;
  return GEVWS_OK;
}

int gevws_decode_batch_async(gevws_ctx* ctx, void* stream, const uint8_t* d_in, uint64_t in_bytes,
                             const gevws_conn_in* d_conns, uint32_t n_conns, gevws_frame* d_frames,
                             uint64_t max_frames, uint8_t* d_payload, uint64_t payload_cap,
                             gevws_conn_out* d_conn_out, gevws_summary* d_summary) {
  if (!ctx || !d_summary) return GEVWS_ERR_INVALID;
  if (n_conns && (!d_in || !d_conns || !d_conn_out)) return GEVWS_ERR_INVALID;
  if (max_frames > 0xFFFFFFFFull) return GEVWS_ERR_INVALID;  // tile map holds 32-bit frame ids
  DeviceGuard g(ctx->device);
  hipStream_t st = pick_stream(ctx, stream);
  // a small batch with the default kernels: the whole decode in one launch
  // (per-phase timing and the variant knobs keep the multi-kernel path)
  if (n_conns <= kSmallConns && in_bytes <= ctx->small_bytes && !ctx->timing && ctx->walk_variant == 0 &&
      ctx->unmask_variant == 0 && ctx->unmask_grid == 0) {
    int r = order_after_last(ctx, st);
    if (r != GEVWS_OK) return r;
    const uint32_t seq = ctx->done_flag ? ++ctx->done_seq : 0u;
    k_decode_small<<<1, kSmallConns, 0, st>>>(d_in, in_bytes, d_conns, n_conns, d_frames, max_frames, d_payload,
                                               payload_cap, d_conn_out, d_summary, ctx->done_flag, seq);
    GEVWS_HIP(hipGetLastError());
    r = mark_last(ctx, st);
    if (ctx->done_flag) ctx->last_signal = seq;
    return r;
  }
  const uint32_t ncu = (uint32_t)ctx->num_cus;
  // connections per counting workgroup: 64, or fewer so a small batch covers every CU
  const uint32_t cpb = n_conns >= (uint32_t)kCountBlock * ncu ? (uint32_t)kCountBlock
                                                             : (n_conns + ncu - 1) / ncu > 0 ? (n_conns + ncu - 1) / ncu : 1;
  // the context's history, once its last multi-kernel decode has finished
  if (ctx->stats_pending && hipEventQuery(ctx->last_done) == hipSuccess) {
    ctx->stats_pending = false;
    ctx->stats_known = true;
    const uint64_t fr = ctx->h_stats[0], pl = ctx->h_stats[1];
    ctx->prev_frames_per_conn = ctx->stats_conns ? fr / ctx->stats_conns : 0;
    ctx->prev_frame_bytes = fr ? pl / fr : 0;
    ctx->prev_mixed = 2 * ctx->h_stats[2] < fr;  // k_unmask_auto5's v5 choice
  }
  // split walk (k_walk_split): ks lanes per connection when the batch has too
  // few connections to keep kSplitLanesPerCU lanes per CU walking, and they
  // are long chains of small frames (the previous decode's)
  const int wv = ctx->walk_variant;
  uint32_t ks = 1;
  if (wv == 0 && n_conns) {
    if (ctx->split_lanes >= 2) {
      ks = ctx->split_lanes;
    } else if (ctx->split_lanes == 0 && in_bytes / n_conns >= 2 * kSplitMinBytes && ctx->stats_known &&
               ctx->prev_frames_per_conn >= kSplitMinFramesPerConn && ctx->prev_frame_bytes <= kSplitMaxFrameBytes) {
      if ((uint64_t)n_conns <= kSplitMaxConnsPerCU * ncu)
        while (ks < kSplitAutoMaxLanes && (uint64_t)n_conns * ks * 2 <= ctx->split_lanes_per_cu * ncu) ks *= 2;
    }
  }
  if ((uint64_t)n_conns * ks > 0xFFFFFFFFull) ks = 1;
  ctx->last_ks = ks;
  const uint32_t cpb_w = ks > 1 ? (kCountBlock / ks < cpb ? kCountBlock / ks : cpb) : cpb;
  const uint32_t nblk = (n_conns + cpb_w - 1) / cpb_w;
  const uint64_t n_v = (uint64_t)n_conns * ks;  // rows of the record pass's connection table
  const uint64_t ntiles_cap = (payload_cap + kTile - 1) / kTile + 1;
  const size_t blk_bytes = ((size_t)nblk * kDecFields * sizeof(uint64_t) + 255) & ~size_t(255);
  const size_t tile_bytes = (ntiles_cap * sizeof(uint32_t) + 255) & ~size_t(255);
  uint32_t gshift = kEntryGranMinShift;
  while ((in_bytes >> gshift) > kEntryBudget) ++gshift;
  const uint64_t n_entries = kSlotAlign * ((in_bytes >> (gshift + kSlotShift)) + n_v + 1);
  const size_t flag_bytes = ((size_t)n_conns + 255) & ~size_t(255);
  const size_t seg_bytes = ks > 1 ? ((n_v * (sizeof(gevws_conn_in) + sizeof(gevws_conn_out) + 1) + 1023) & ~size_t(255)) : 0;
  // + one sink slot per walk lane after the table (k_walk_count / k_walk_split)
  int r = order_after_last(ctx, st);
  if (r != GEVWS_OK) return r;
  r = ensure_scratch(ctx, blk_bytes + tile_bytes + flag_bytes + seg_bytes + (n_entries + n_v) * sizeof(WalkEntry));
  if (r != GEVWS_OK) return r;
  char* sp = reinterpret_cast<char*>(ctx->scratch);
  uint64_t* blk = reinterpret_cast<uint64_t*>(sp);
  uint32_t* tile_first = reinterpret_cast<uint32_t*>(sp + blk_bytes);
  uint8_t* rec_flags = reinterpret_cast<uint8_t*>(sp + blk_bytes + tile_bytes);
  char* segp = sp + blk_bytes + tile_bytes + flag_bytes;
  gevws_conn_in* segs = reinterpret_cast<gevws_conn_in*>(segp);
  gevws_conn_out* sout = reinterpret_cast<gevws_conn_out*>(segp + n_v * sizeof(gevws_conn_in));
  uint8_t* srec = reinterpret_cast<uint8_t*>(segp + n_v * (sizeof(gevws_conn_in) + sizeof(gevws_conn_out)));
  WalkEntry* entries = reinterpret_cast<WalkEntry*>(segp + seg_bytes);
  const bool timed = ctx->timing;
  hipEvent_t* ev = nullptr;
  if (timed) {
    if (ctx->evs_used == ctx->evs.size()) {
      gevws_ctx::EventSet set;
      for (auto& e : set.e) GEVWS_HIP(hipEventCreate(&e));
      ctx->evs.push_back(set);
    }
    ev = ctx->evs[ctx->evs_used++].e;
    GEVWS_HIP(hipEventRecord(ev[0], st));
  }
  // walk variant 2: no entry table -- the counting walk stores nothing per
  // frame and the record pass re-walks every chain
  const uint64_t ne = wv == 2 ? 0 : n_entries;
  // The walk's last workgroup scans the partials itself (walk_block_done) and
  // saves the k_scan_blocks launch (with release / acquire fences instead of
  // coherent partials it was slower: C1-shaped walk 0.034 -> 0.074 ms,
  // profiles/r02/r02_steps_fused.jsonl).
  const bool fused = nblk > 0 && nblk <= kFusedScanMaxBlocks;
  uint32_t* done = fused ? ctx->d_done : nullptr;
  // the walk's uniform-stream speculation (D = 8) pays on long runs of equal
  // frames (C2, C3: -23..-28 %) and costs 2-7 % elsewhere (C1, C4,
  // profiles/r02/r02_walk_store_count_ab.jsonl); after a decode on this context
  // whose frames were mostly NOT the size of their predecessor the plain
  // chain walk (D = 0) runs instead
  const bool plain = wv == 1 || (wv != 1 && ctx->stats_known && ctx->prev_mixed);
  if (nblk && ks > 1) {
#define GEVWS_SPLIT(K)                                                                                            \
  (plain ? k_walk_split<K, 0> : k_walk_split<K, 8>)<<<nblk, kCountBlock, 0, st>>>(                                \
      d_in, d_conns, n_conns, d_conn_out, blk, entries, ne, gshift, cpb_w, in_bytes, done, max_frames, payload_cap, \
      d_summary, segs, sout, srec, ctx->split_min_bytes)
    if (ks == 2) GEVWS_SPLIT(2);
    else if (ks == 4) GEVWS_SPLIT(4);
    else if (ks == 8) GEVWS_SPLIT(8);
    else if (ks == 16) GEVWS_SPLIT(16);
    else GEVWS_SPLIT(32);
#undef GEVWS_SPLIT
  } else if (nblk && (wv == 3 || (uint64_t)n_conns >= kWriterChainsPerCU * (uint64_t)ncu)) {
    // many chains: the walk is bound by its line traffic -- entries through
    // each lane's LDS ring to the workgroup's writer wave (k_walk_count ST 2)
    (plain ? k_walk_count<0, 2> : k_walk_count<8, 2>)<<<nblk, 2 * kCountBlock, 0, st>>>(
        d_in, d_conns, n_conns, d_conn_out, blk, entries, ne, gshift, cpb, in_bytes, done, max_frames, payload_cap,
        d_summary);
  } else if (nblk) {
    (plain ? k_walk_count<0, 0> : k_walk_count<8, 0>)<<<nblk, kCountBlock, 0, st>>>(
        d_in, d_conns, n_conns, d_conn_out, blk, entries, ne, gshift, cpb, in_bytes, done, max_frames, payload_cap,
        d_summary);
  }
  if (timed) GEVWS_HIP(hipEventRecord(ev[1], st));
  if (!fused) k_scan_blocks<true, kDecFields><<<1, kScanBlock, 0, st>>>(blk, nblk, max_frames, payload_cap, d_summary);
  if (timed) GEVWS_HIP(hipEventRecord(ev[2], st));
  if (nblk) {
    k_walk_bases<<<nblk, kCountBlock, 0, st>>>(n_conns, d_conn_out, blk, d_summary, rec_flags, cpb_w, ctx->d_stats);
    ctx->stats_pending = true;
    ctx->stats_conns = n_conns;
    // the record pass walks the segments when the walk was split
    const gevws_conn_in* e_conns = ks > 1 ? segs : d_conns;
    const gevws_conn_out* e_out = ks > 1 ? sout : d_conn_out;
    const uint8_t* e_rec = ks > 1 ? srec : rec_flags;
    const gevws_conn_out* e_parent = ks > 1 ? d_conn_out : nullptr;
    uint64_t egrid = (n_v + kWalkBlock / 64 - 1) / (kWalkBlock / 64);
    // (split rows: each row is a chain of ~100 frames whose entries cost a
    // load round trip, so more waves share them out)
    const uint64_t ecap = (ks > 1 ? kEmitSplitPerCU : 8) * (uint64_t)ncu;
    if (egrid > ecap) egrid = ecap;
    k_walk_emit<<<(uint32_t)egrid, kWalkBlock, 0, st>>>(d_in, e_conns, (uint32_t)n_v, e_out, d_summary, d_frames,
                                                          tile_first, entries, ne, gshift, e_rec, e_parent,
                                                          ks > 1 ? ks : 0);
  }
  // split streams: the unmask waits for the front (walk, scan, record pass)
  // on its own stream; the next batch's front can then run beside it
  hipStream_t ust = st;
  if (ctx->unmask_stream && ctx->unmask_stream != st) {
    ust = ctx->unmask_stream;
    GEVWS_HIP(hipEventRecord(ctx->front_done, st));
    GEVWS_HIP(hipStreamWaitEvent(ust, ctx->front_done, 0));
  }
  if (timed) GEVWS_HIP(hipEventRecord(ev[3], ust));  // (split: once the unmask stream may start it)
  r = launch_unmask(ctx, ust, payload_cap, d_in, d_frames, tile_first, d_summary, d_payload);
  if (r != GEVWS_OK) return r;
  if (timed) GEVWS_HIP(hipEventRecord(ev[4], ust));
  GEVWS_HIP(hipGetLastError());
  return mark_last(ctx, ust);
}

int gevws_decode_batch(gevws_ctx* ctx, void* stream, const uint8_t* d_in, uint64_t in_bytes,
                       const gevws_conn_in* d_conns, uint32_t n_conns, gevws_frame* d_frames,
                       uint64_t max_frames, uint8_t* d_payload, uint64_t payload_cap,
                       gevws_conn_out* d_conn_out, gevws_summary* h_summary) {
  if (!ctx || !h_summary) return GEVWS_ERR_INVALID;
  DeviceGuard g(ctx->device);
  hipStream_t st = pick_stream(ctx, stream);
  gevws_summary* d_sum = ctx->d_sum;
  int r = gevws_decode_batch_async(ctx, stream, d_in, in_bytes, d_conns, n_conns, d_frames, max_frames,
                                   d_payload, payload_cap, d_conn_out, d_sum);
  if (r == GEVWS_OK) {
    GEVWS_HIP(hipMemcpyAsync(h_summary, d_sum, sizeof(gevws_summary), hipMemcpyDeviceToHost, st));
    GEVWS_HIP(hipStreamSynchronize(st));
    r = h_summary->status;
  }
  return r;
}

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
  r = ensure_scratch(ctx, blk_bytes + ntiles_cap * sizeof(uint32_t));
  if (r != GEVWS_OK) return r;
  uint64_t* blk = reinterpret_cast<uint64_t*>(ctx->scratch);
  uint32_t* tile_first = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(ctx->scratch) + blk_bytes);
  if (nblk) k_enc_size<<<nblk, kWalkBlock, 0, st>>>(d_frames, n, blk, d_out_off, gate);
  k_scan_blocks<false><<<1, kScanBlock, 0, st>>>(blk, nblk, n, out_cap, d_summary);
  if (nblk) k_enc_emit<<<nblk, kWalkBlock, 0, st>>>(n, blk, d_summary, d_out_off, tile_first, gate);
  const uint64_t per_cu = 7;  // the window path's occupancy (k_encode)
  uint64_t grid = (out_cap / kTile + kWinTiles - 1) / kWinTiles;
  // (GEVWS_TUNE_UNMASK_GRID, when set, caps the encode's grid too: measurement)
  const uint64_t gcap = ctx->unmask_grid ? (uint64_t)ctx->unmask_grid : per_cu * (uint64_t)ctx->num_cus;
  if (grid > gcap) grid = gcap;
  if (grid < 1) grid = 1;
  // every frame boundary takes the window path, which needs several
  // workgroups per CU to hide its latency (C3: 22.6 ms at 4/CU vs 36 ms at
  // 1/CU); it runs 7 per CU (C2 -18 %, C4 -4 % against 4,
  // profiles/r01/r01_encode_ab_lds_*.json, r01_encode_ab_occ_*.json), and
  // batches of big frames (mean >= kBigFrameBytes) keep 4 per CU (the rest
  // return at once)
  const uint32_t big = grid > 4ull * ctx->num_cus ? 4u * (uint32_t)ctx->num_cus : 0u;
  k_encode<<<(uint32_t)grid, kUnmaskBlock, 0, st>>>(d_frames, d_payload, d_out_off, tile_first, d_summary, d_out,
                                                     big);
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
                                           d_enc_summary, ctx->done_flag, seq);
  GEVWS_HIP(hipGetLastError());
  r = mark_last(ctx, st);
  if (ctx->done_flag) ctx->last_signal = seq;
  return r;
}

int gevws_copy_async(gevws_ctx* ctx, void* stream, uint8_t* d_dst, const uint8_t* d_src, uint64_t n,
                     uint32_t grid) {
  if (!ctx || (n && (!d_dst || !d_src))) return GEVWS_ERR_INVALID;
  if ((n & 15) || (reinterpret_cast<uint64_t>(d_dst) & 15)) return GEVWS_ERR_INVALID;
  if (n == 0) return GEVWS_OK;
  DeviceGuard g(ctx->device);
  hipStream_t st = pick_stream(ctx, stream);
  // bit 30: plain loads (else non-temporal); bit 29: the unmask's
  // wave-contiguous spans (else tile-strided lanes)
  const bool plain = grid & 0x40000000u, wspan = grid & 0x20000000u;
  grid &= 0x1fffffffu;
  if (grid == 0) grid = (uint32_t)ctx->num_cus;
  auto k = wspan ? (plain ? k_copy_stream<16, false, true> : k_copy_stream<16, true, true>)
                 : (plain ? k_copy_stream<16, false, false> : k_copy_stream<16, true, false>);
  k<<<grid, kUnmaskBlock, 0, st>>>(d_src, d_dst, n);
  GEVWS_HIP(hipGetLastError());
  return GEVWS_OK;
}

int gevws_pinned_alloc(uint64_t bytes, void** host_ptr, void** dev_ptr) {
  if (!host_ptr || !dev_ptr || bytes == 0) return GEVWS_ERR_INVALID;
  *host_ptr = nullptr;
  *dev_ptr = nullptr;
  void* h = nullptr;
  if (hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess || !h)
    return GEVWS_ERR_DEVICE;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d) {
    (void)hipHostFree(h);
    return GEVWS_ERR_DEVICE;
  }
  *host_ptr = h;
  *dev_ptr = d;
  return GEVWS_OK;
}

int gevws_pinned_free(void* host_ptr) {
  if (!host_ptr) return GEVWS_OK;
  return hipHostFree(host_ptr) == hipSuccess ? GEVWS_OK : GEVWS_ERR_DEVICE;
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

int gevws_synth_async(gevws_ctx* ctx, void* stream, uint8_t* d_in, const gevws_synth_desc* d_desc,
                      uint64_t n_frames, uint64_t seed) {
  if (!ctx || (n_frames && (!d_in || !d_desc))) return GEVWS_ERR_INVALID;
  if (n_frames == 0) return GEVWS_OK;
  DeviceGuard g(ctx->device);
  hipStream_t st = pick_stream(ctx, stream);
  uint64_t grid = n_frames < (1u << 20) ? n_frames : (1u << 20);
  k_synth<<<(uint32_t)grid, 256, 0, st>>>(d_in, d_desc, n_frames, seed);
  GEVWS_HIP(hipGetLastError());
  return GEVWS_OK;
}

int gevws_synth_verify_async(gevws_ctx* ctx, void* stream, const gevws_synth_desc* d_desc,
                             uint64_t n_frames, uint64_t seed, const gevws_frame* d_frames,
                             const uint8_t* d_payload, uint64_t payload_cap, uint64_t* d_mismatch) {
  if (!ctx || !d_mismatch || (n_frames && (!d_desc || !d_frames || !d_payload))) return GEVWS_ERR_INVALID;
  if (n_frames == 0) return GEVWS_OK;
  DeviceGuard g(ctx->device);
  hipStream_t st = pick_stream(ctx, stream);
  uint64_t grid = n_frames < (1u << 16) ? n_frames : (1u << 16);
  k_synth_verify<<<(uint32_t)grid, 256, 0, st>>>(d_desc, n_frames, seed, d_frames, d_payload, payload_cap,
                                                  reinterpret_cast<unsigned long long*>(d_mismatch));
  GEVWS_HIP(hipGetLastError());
  return GEVWS_OK;
}

}  // extern "C"

static int launch_unmask(gevws_ctx* ctx, hipStream_t st, uint64_t payload_cap, const uint8_t* d_in,
                  const gevws_frame* d_frames, const uint32_t* tile_first, const gevws_summary* d_summary,
                  uint8_t* d_payload) {
  const UnmaskVariant& v = kUnmaskVariants[ctx->unmask_variant];
  const uint64_t ntiles = (payload_cap + kTile - 1) / kTile;
  // CUs the unmask's stream may use (all of the device's, or its CU mask's)
  const uint32_t ucus = (uint32_t)(st == ctx->unmask_stream && ctx->unmask_cus > 0 ? ctx->unmask_cus : ctx->num_cus);
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
                                                ctx->unmask_grid ? 0u : ucus | (wide ? (uint32_t)norm << 16 : 0u));
  return GEVWS_OK;
}
