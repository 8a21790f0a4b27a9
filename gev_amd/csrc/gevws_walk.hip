// gevws_walk.hip -- the decode up to the unmask:
// for every connection of a batch, the repeated websocket.(*Protocol).UnPacket
// loop of Connection.handlerProtocol (connection.go:208-218 ->
// plugins/websocket/protocol.go:38-62) up to the payload copy:
//
//   k_walk_count   one lane per connection walks its header chain
//                  (ws.VirtualReadHeader, read.go:19-84, plus the completeness
//                  gate, protocol.go:47), counts frames, payload bytes and
//                  consumed bytes and records an 8-byte entry per frame; the
//                  last workgroup scans the block partials (small batches)
//   k_walk_split   the same for few long chains: KS lanes per connection
//   k_scan_blocks  the partials scan for big batches -> batch totals, capacity
//   k_walk_bases   per-connection bases (block-level scan)
//   k_walk_emit    the 32-byte records (= ws.Header + offsets) and the
//                  output-tile -> frame map the unmask reads
//   k_decode_small a batch of <= 1 024 connections and 128 KiB: the whole
//                  decode, unmask included, in one workgroup
#include <chrono>

#include "gevws_internal.hpp"
#include "gevws_small.hpp"

namespace {

// A walk block's partial of field k as two granules (low, high 32 bits).
__device__ __forceinline__ void put_partial(uint64_t* part, uint32_t b, int k, uint64_t v, uint32_t tag) {
  uint64_t* p = part + 2 * ((uint64_t)b * kDecFields + k);
  put_granule(p, (uint32_t)v, tag);
  put_granule(p + 1, (uint32_t)(v >> 32), tag);
}

// The decode's partials scan by ONE wave (the walk's last block, see
// walk_block_done): per round each lane takes P consecutive block partials
// (tagged granules, all loads in flight before any is checked), fields 0/1
// become exclusive bases (frames, arena bytes) for k_walk_bases in blk,
// every field is totalled into the summary, with the capacity check.
__device__ void scan_partials_wave(const uint64_t* __restrict__ part, uint32_t tag, uint64_t* __restrict__ blk,
                                   uint32_t nblk, uint64_t max_frames, uint64_t payload_cap,
                                   gevws_summary* __restrict__ sum) {
  constexpr int P = 4;  // 64 x 4 = kFusedScanMaxBlocks: one round
  const int lane = threadIdx.x & 63;
  uint64_t carry[kDecFields] = {0, 0, 0, 0, 0};
  uint32_t bad = 0;
  for (uint64_t base = 0; base < nblk; base += 64 * P) {  // wave-uniform
    const uint64_t i0 = base + (uint64_t)lane * P;
    uint64_t g[P][kDecFields][2];
#pragma unroll
    for (int r = 0; r < P; ++r)
#pragma unroll
      for (int k = 0; k < kDecFields; ++k)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          g[r][k][h] = (i0 + r < nblk) ? load_granule(part + 2 * ((i0 + r) * kDecFields + k) + h) : 0;
    uint64_t loc[kDecFields] = {0, 0, 0, 0, 0};
    uint64_t loc0[P], loc1[P];  // this lane's partials of fields 0 / 1, for the bases
#pragma unroll
    for (int r = 0; r < P; ++r)
#pragma unroll
      for (int k = 0; k < kDecFields; ++k) {
        uint64_t v = 0;
        if (i0 + r < nblk) {
          const uint64_t* q = part + 2 * ((i0 + r) * kDecFields + k);
          v = (uint64_t)take_granule(q, g[r][k][0], tag, bad) | ((uint64_t)take_granule(q + 1, g[r][k][1], tag, bad) << 32);
        }
        loc[k] += v;
        if (k == 0) loc0[r] = v;
        if (k == 1) loc1[r] = v;
      }
    const uint64_t inc0 = wave_incl_scan(loc[0]), inc1 = wave_incl_scan(loc[1]);
    uint64_t b0 = carry[0] + inc0 - loc[0], b1 = carry[1] + inc1 - loc[1];
#pragma unroll
    for (int r = 0; r < P; ++r) {
      if (i0 + r < nblk) {
        uint64_t* q = blk + (i0 + r) * kDecFields;
        q[0] = b0;
        q[1] = b1;
        b0 += loc0[r];
        b1 += loc1[r];
      }
    }
#pragma unroll
    for (int k = 0; k < kDecFields; ++k) carry[k] += wave_sum(loc[k]);
  }
  bad = (uint32_t)wave_sum(bad);
  if (lane == 0) {
    gevws_summary sm;
    memset(&sm, 0, sizeof(sm));
    sm.frames = carry[0];
    sm.payload_bytes = carry[1];
    sm.payload_len = carry[2];
    sm.errors = carry[3] & 0xffffffffull;
    sm.flags = (carry[3] >> 32) ? GEVWS_SUMMARY_UNORDERED : 0u;
    sm.run_frames = carry[4];
    sm.status = bad ? GEVWS_ERR_DEVICE
                    : (carry[0] > max_frames || carry[1] > payload_cap) ? GEVWS_ERR_CAPACITY : GEVWS_OK;
    *sum = sm;
  }
}

// The last of the walk's workgroups to finish (a device-scope counter) scans
// the partials, so a decode of <= kFusedScanMaxBlocks blocks needs no
// k_scan_blocks launch.  The partials travel as tagged granules (hand-offs,
// above); each writer waits for its stores before its workgroup counts itself
// (not needed for correctness: it makes the first load of each granule the
// one that carries the tag), and the last workgroup resets the counter for the
// context's next call (ordered after this launch by the kernel boundary).
__device__ __forceinline__ void walk_block_done(uint32_t* __restrict__ done, uint32_t nblk, const uint64_t* __restrict__ part,
                                                uint32_t tag, uint64_t* __restrict__ blk, uint64_t max_frames,
                                                uint64_t payload_cap, gevws_summary* __restrict__ sum, bool wrote) {
  __shared__ uint32_t s_last;
  if (wrote) __builtin_amdgcn_s_waitcnt(0);  // the partials' write-through stores are done
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblk - 1 ? 1u : 0u;
  __syncthreads();
  if (s_last) {
    if (threadIdx.x < 64) scan_partials_wave(part, tag, blk, nblk, max_frames, payload_cap, sum);
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

template <int D, int ST = 0, uint32_t RING = kRing>
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
          while ((uint32_t)nf + 4 - lds_ld(ring.tail) > RING) __builtin_amdgcn_s_sleep(1);
        ring.e[nf & (RING - 1)] = e;
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
template <uint32_t GROUP = kWriterGroup, uint32_t RING = kRing>
__device__ __forceinline__ void walk_ring_writer(WalkEntry* __restrict__ entries, WalkRing ring, uint64_t ebase,
                                                 uint64_t ecap) {
  static_assert(GROUP <= kSlotAlign && kSlotAlign % GROUP == 0 && RING % GROUP == 0 && GROUP % 4 == 0,
                "groups aligned by the slot runs, whole groups in the ring");
  uint32_t t = 0;
  bool fin = false;
  for (;;) {
    if (!fin) {
      const uint32_t hv = lds_ld(ring.head);
      __asm__ volatile("" ::: "memory");  // the entries after the head that published them
      const uint32_t h = hv & ~kRingDone;
      while (h - t >= GROUP) {
        WalkEntry g[GROUP];
#pragma unroll
        for (uint32_t k = 0; k < GROUP; ++k) g[k] = ring.e[(t + k) & (RING - 1)];
        if (ebase != ~0ull && t + GROUP <= ecap) {
          u32x4* d = reinterpret_cast<u32x4*>(entries + ebase + t);  // 8 x GROUP-byte aligned
#pragma unroll
          for (uint32_t k = 0; k < GROUP / 2; ++k)
            d[k] = u32x4{g[2 * k].mask, g[2 * k].w, g[2 * k + 1].mask, g[2 * k + 1].w};
        }
        t += GROUP;
        __asm__ volatile("" ::: "memory");
        lds_st(ring.tail, t);
      }
      if (hv & kRingDone) {
        for (; t < h; ++t)
          if (ebase != ~0ull && t < ecap) entries[ebase + t] = ring.e[t & (RING - 1)];
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
    uint32_t gshift, uint32_t cpb, uint64_t in_bytes, uint32_t* __restrict__ done, uint64_t* __restrict__ part,
    uint32_t tag, uint64_t max_frames, uint64_t payload_cap, gevws_summary* __restrict__ sum) {
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
      if (done) put_partial(part, blockIdx.x, k, s, tag);
      else blk[(uint64_t)blockIdx.x * kDecFields + k] = s;
    }
  }
  if (done) walk_block_done(done, gridDim.x, part, tag, blk, max_frames, payload_cap, sum, threadIdx.x == 0);
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
constexpr uint32_t kSplitAutoMaxLanes = 16;  // the auto choice's largest split
// auto: split only after a decode on this context whose connections averaged
// this many frames of at most this many payload bytes (the long chains of
// small frames splitting shortens; a batch of big frames -- C2, C3, C5 --
// pays the guesses for nothing)
constexpr uint64_t kSplitMinFramesPerConn = 256;
// more chains keep the walk busy unsplit: with the writer wave the 4-way C4
// share (64 per CU) walks faster split 8 ways (2.698 -> 2.645 ms a step), the
// 2-way (128 per CU) and the full batch slower at any split
// (profiles/r06/r06i_split_rule.jsonl; round 2-5, without the writer, the
// 4-way share lost 5 % split)
constexpr uint64_t kSplitMaxConnsPerCU = 64;
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

// ST 2: the walkers' entries go through each lane's LDS ring to a second
// (writer) wave, as k_walk_count's ST 2 -- a walking lane then issues no
// global stores, so its header loads never wait behind entry stores.  The
// ring (kSplitRing entries a lane, stored in kSplitGroup-entry groups) shares
// its LDS with the guess rows, which are done with before the first entry:
// 19 KB a workgroup, 8 workgroups of two waves per CU.
constexpr uint32_t kSplitRing = 32;
constexpr uint32_t kSplitGroup = 16;
constexpr uint32_t kSplitLdsWords = (kCountBlock * kSyncRow > 2 * kCountBlock * kSplitRing)
                                        ? kCountBlock * kSyncRow
                                        : 2 * kCountBlock * kSplitRing;  // dwords: guess rows | rings

template <int KS, int D, int ST>
__global__ __launch_bounds__(ST == 2 ? 2 * kCountBlock : kCountBlock) void k_walk_split(const uint8_t* __restrict__ in,
                                                            const gevws_conn_in* __restrict__ conns, uint32_t n,
                                                            gevws_conn_out* __restrict__ cout,
                                                            uint64_t* __restrict__ blk,
                                                            WalkEntry* __restrict__ entries, uint64_t n_entries,
                                                            uint32_t gshift, uint32_t cpb, uint64_t in_bytes,
                                                            uint32_t* __restrict__ done,
                                                            uint64_t* __restrict__ part, uint32_t tag,
                                                            uint64_t max_frames,
                                                            uint64_t payload_cap, gevws_summary* __restrict__ sum,
                                                            gevws_conn_in* __restrict__ segs,
                                                            gevws_conn_out* __restrict__ sout,
                                                            uint8_t* __restrict__ srec,
                                                            uint64_t min_seg = kSplitMinBytes,
                                                            uint32_t* __restrict__ fallbacks = nullptr) {
  static_assert(KS >= 2 && KS <= (int)kSplitMaxLanes && (KS & (KS - 1)) == 0, "KS: a power of two");
  static_assert(ST == 0 || ST == 2, "entries from the lanes or through the writer wave");
  __shared__ __attribute__((aligned(16))) uint32_t s_lds[ST == 2 ? kSplitLdsWords : kCountBlock * kSyncRow];
  __shared__ uint32_t s_head[ST == 2 ? kCountBlock : 1], s_tail[ST == 2 ? kCountBlock : 1];
  __shared__ uint64_t s_ebase[ST == 2 ? kCountBlock : 1], s_ecap[ST == 2 ? kCountBlock : 1];
  uint32_t* const s_row = s_lds;  // the guess rows (step 1), then the rings (step 3)
  const bool walker = ST != 2 || threadIdx.x < 64;
  const uint32_t lane = threadIdx.x & 63, i = lane % KS;
  const uint32_t c = blockIdx.x * cpb + lane / KS;
  const bool active = walker && lane / KS < cpb && c < n;
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
      found = sync_search(s, ci.len, t, step, t + seg * 3 / 4, m0, s_row + lane * kSyncRow, b);
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
  if constexpr (ST == 2) {
    const WalkRing ring = {reinterpret_cast<WalkEntry*>(s_lds) + lane * kSplitRing, s_head + lane, s_tail + lane};
    if (walker) {
      s_head[lane] = active ? 0u : kRingDone;
      s_tail[lane] = 0;
      s_ebase[lane] = rec0 ? ebase : ~0ull;
      s_ecap[lane] = ecap;
    }
    __syncthreads();  // every guess row read: the rings may take the LDS
    if (!walker) walk_ring_writer<kSplitGroup, kSplitRing>(entries, ring, s_ebase[lane], s_ecap[lane]);
    else if (active)
      walk_chain<D, 2, kSplitRing>(in + sg.off, sg.len, rec0, ebase, ecap, entries, entries + n_entries + v, R, ring);
  } else if (active) {
    walk_chain<D>(in + sg.off, sg.len, rec0, ebase, ecap, entries, entries + n_entries + v, R);
  }
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
        if (fallbacks) atomicAdd(fallbacks, 1u);  // (gevws_ctx_last_split_fallbacks)
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
      if (done) put_partial(part, blockIdx.x, k, x, tag);
      else blk[(uint64_t)blockIdx.x * kDecFields + k] = x;
    }
  }
  if (done) walk_block_done(done, gridDim.x, part, tag, blk, max_frames, payload_cap, sum, threadIdx.x == 0);
}

// ------------------------------------------------------------------ 3. walk (emit)
// 3a. per-connection bases: block-level exclusive scan of (frames, arena bytes)
// on top of the scanned block partials.
__global__ __launch_bounds__(kCountBlock) void k_walk_bases(uint32_t n, gevws_conn_out* __restrict__ cout,
                                                            const uint64_t* __restrict__ blk,
                                                            const gevws_summary* __restrict__ sum,
                                                            uint8_t* __restrict__ rec_flags, uint32_t cpb,
                                                            uint64_t* __restrict__ stats = nullptr,
                                                            uint32_t* __restrict__ runs = nullptr) {
  // the unmask's per-XCD run counters start at zero (before the capacity check:
  // the unmask reads them whatever the status)
  if (runs && blockIdx.x == 0 && threadIdx.x < kUnmaskRunCounters) runs[threadIdx.x * 16] = 0;
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
  // The wave's plain inclusive scan (DPP) minus its value just before this
  // lane's segment, whose first lane is the highest head at or below it (the
  // wave's lane 0 if none): one ballot and one shuffle instead of a shuffled
  // value and head flag at each of six steps.
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t incl = wave_incl_scan64_dpp(v);
  const uint64_t heads = __ballot(head);
  const uint64_t upto = lane == 63 ? heads : heads & ((2ull << lane) - 1);
  const int h = upto ? 63 - __builtin_clzll(upto) : 0;
  const uint64_t before = __shfl(incl, h > 0 ? h - 1 : 0, 64);
  return h > 0 ? incl - before : incl;
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

template <class S>
__global__ __launch_bounds__(S::NT) void k_decode_small(const uint8_t* __restrict__ in, uint64_t in_bytes,
                                                        const gevws_conn_in* __restrict__ conns, uint32_t n,
                                                        gevws_frame* __restrict__ frames, uint64_t max_frames,
                                                        uint8_t* __restrict__ payload, uint64_t payload_cap,
                                                        gevws_conn_out* __restrict__ cout,
                                                        gevws_summary* __restrict__ sum,
                                                        uint32_t* __restrict__ done = nullptr,
                                                        uint32_t seq = 0, uint64_t* __restrict__ ticks = nullptr,
                                                        uint64_t* __restrict__ stage_buf = nullptr,
                                                        uint32_t* __restrict__ stage_done = nullptr,
                                                        uint32_t tag = 0, uint64_t* __restrict__ phase = nullptr) {
  (void)decode_small_body<S>(in, in_bytes, conns, n, frames, max_frames, payload, payload_cap, cout, sum, done, seq,
                             ticks, stage_buf, stage_done, tag, gridDim.x, blockIdx.x, gridDim.x, phase);
}

// The same with its arguments in one by-value struct: the form a dispatch
// written straight into the context's own AQL queue takes (gevws_direct.cpp).
template <class S>
__global__ __launch_bounds__(S::NT) void k_decode_small_direct(DirectDecodeArgs a) {
  (void)decode_small_body<S>(a.in, a.in_bytes, a.conns, a.n, a.frames, a.max_frames, a.payload, a.payload_cap,
                             a.cout, a.sum, a.done, a.seq, a.ticks, a.stage_buf, a.stage_done, a.tag, a.nwg,
                             blockIdx.x, a.nwg, a.phase);
}

// ------------------------------------------------------------------ 3d. the resident decode service
// A live pass's launch call costs its loop ~5 us of host time whatever the
// pass (the HIP runtime's).  With the service on (gevws_ctx_set_service), a
// context keeps one instance of this kernel resident on its stream --
// kSmallStageWGs workgroups, as many as a launched live pass stages its input
// with -- and the host posts passes to it instead of launching them: the
// pass's arguments into the mailbox in mapped host memory, then a 64-bit word
// {generation, pass number}.
//
// Lane 0 of workgroup 0 polls the mailbox and broadcasts each pass it takes
// to the other workgroups as tagged granules in device memory (ctl: the
// command, the arguments' halves), tag t0 + k for the instance's k-th pass
// (the host reserves the instance's tags [t0, t0 + kServiceMaxPasses)).  A
// pass then runs as the launched one does (decode_small_body, narrow shape):
// the first `slices` workgroups each stage a slice and count themselves in,
// the last one decodes and signals the completion word (a pass of one slice:
// workgroup 0 alone, from the input); the rest skip it.
//
// Every wave reaches an exit.  With no pass of its own pending, workgroup 0
// ends the instance when the mailbox's live generation is no longer its own
// (the host bumps it before any other work on the context's stream, before a
// new instance, and to stop) or at its deadline (life_ticks of the GPU's
// constant-rate clock after its start; the host posts only within half of
// it): it waits for its last pass's done granule -- every workgroup has taken
// that pass -- and then stores the exit granule (tag t0), which the others
// poll beside the command; they also end at twice the deadline on their own.
// A posted pass is tagged with its instance's generation and the host posts
// the next only once the last has signalled, so none is lost (the one posted
// before a stop still runs, the work behind it waits on the stream) and none
// runs twice.
constexpr uint32_t kServiceMaxPasses = 1u << 16;
// ctl: the command {the pass's slices}, its number, the arguments' halves, exit, done
constexpr uint32_t kSvcCmd = 0, kSvcSeq = 1, kSvcArgs = 2, kSvcExit = kSvcArgs + 2 * kServiceArgs,
                   kSvcDone = kSvcExit + 1, kSvcCtlGranules = kSvcDone + 1;

template <class S>
__global__ __launch_bounds__(S::NT) void k_decode_service(ServiceBox* __restrict__ box, uint32_t gen, uint32_t req0,
                                                          uint64_t life_ticks, uint32_t* __restrict__ done,
                                                          uint64_t* __restrict__ ticks, uint64_t* __restrict__ ctl,
                                                          uint64_t* __restrict__ stage_buf,
                                                          uint32_t* __restrict__ stage_done, uint32_t t0) {
  __shared__ uint32_t s_k, s_slices, s_req;
  __shared__ uint64_t s_a[kServiceArgs];
  const uint64_t t_start = gpu_ticks();
  const uint32_t wg = blockIdx.x, G = gridDim.x;
  uint32_t last = req0;  // (lane 0 of workgroup 0) the last pass taken
  uint32_t k = 0;        // (lane 0) the instance's last pass number seen
  for (;;) {
    if (threadIdx.x == 0) {
      uint32_t slices = 0, req = 0;  // 0: end
      if (wg == 0) {
        while (k + 1 < kServiceMaxPasses) {
          const uint64_t w = __hip_atomic_load(&box->req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
          if ((uint32_t)(w >> 32) == gen && (uint32_t)w != last) {  // a pass of this instance's
            last = req = (uint32_t)w;
            break;
          }
          if (__hip_atomic_load(&box->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != gen ||
              gpu_ticks() - t_start >= life_ticks)
            break;
          __builtin_amdgcn_s_sleep(2);
        }
        if (req) {
          const uint32_t tag = t0 + ++k;
          for (int i = 0; i < kServiceArgs; ++i)
            s_a[i] = __hip_atomic_load(&box->args[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(&box->ack, req, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);  // (the box is free)
          slices = small_slices(s_a[1], (uint32_t)s_a[3], G);
          if (slices > 1) {  // (the workgroups past its slices take a pass as a number only)
            for (int i = 0; i < kServiceArgs; ++i) {
              put_granule(ctl + kSvcArgs + 2 * i, (uint32_t)s_a[i], tag);
              put_granule(ctl + kSvcArgs + 2 * i + 1, (uint32_t)(s_a[i] >> 32), tag);
            }
            put_granule(ctl + kSvcSeq, req, tag);
          }
          put_granule(ctl + kSvcCmd, slices, tag);
        } else {
          // pass k is done, so every workgroup has taken it
          if (k)
            for (uint64_t t1 = gpu_ticks(); (uint32_t)(load_granule(ctl + kSvcDone) >> 32) != t0 + k &&
                                            gpu_ticks() - t1 < life_ticks;)
              __builtin_amdgcn_s_sleep(2);
          put_granule(ctl + kSvcExit, 0u, t0);
        }
      } else {
        for (;;) {
          const uint64_t g = load_granule(ctl + kSvcCmd);
          const uint32_t d = (uint32_t)(g >> 32) - t0;
          if (d > k && d < kServiceMaxPasses) {  // a pass not seen yet (skipped unless it has a slice for us)
            k = d;
            if ((uint32_t)g > wg) {
              slices = (uint32_t)g;
              break;
            }
            continue;
          }
          if ((uint32_t)(load_granule(ctl + kSvcExit) >> 32) == t0 || gpu_ticks() - t_start >= 2 * life_ticks) break;
          __builtin_amdgcn_s_sleep(2);
        }
        // a pass with a slice for us: its arguments stay until every workgroup with one has taken it
        uint32_t bad = 0;
        const uint32_t tag = t0 + k;
        for (int i = 0; slices && i < kServiceArgs; ++i) {
          const uint64_t* p = ctl + kSvcArgs + 2 * i;
          const uint32_t lo = take_granule(p, load_granule(p), tag, bad);
          const uint32_t hi = take_granule(p + 1, load_granule(p + 1), tag, bad);
          s_a[i] = (uint64_t)lo | ((uint64_t)hi << 32);
        }
        if (slices) req = take_granule(ctl + kSvcSeq, load_granule(ctl + kSvcSeq), tag, bad);
        if (bad) slices = 0;  // (never seen: the pass then waits for the host's fallback)
      }
      s_k = k;
      s_slices = slices;
      s_req = req;
    }
    __syncthreads();
    const uint32_t slices = s_slices;
    if (!slices) return;
    // The pass's input was written after this kernel started (a launched
    // kernel's start would have dropped stale lines): without a launch, each
    // wave drops them itself -- the host's release of the pass (its req store)
    // reaches this workgroup through the granules, so acquire at system scope.
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    const uint32_t tag = t0 + s_k;
    const bool decoded = decode_small_body<S>(
        reinterpret_cast<const uint8_t*>(s_a[0]), s_a[1], reinterpret_cast<const gevws_conn_in*>(s_a[2]),
        (uint32_t)s_a[3], reinterpret_cast<gevws_frame*>(s_a[4]), s_a[5], reinterpret_cast<uint8_t*>(s_a[6]), s_a[7],
        reinterpret_cast<gevws_conn_out*>(s_a[8]), reinterpret_cast<gevws_summary*>(s_a[9]), done, s_req, ticks,
        stage_buf, stage_done, tag, slices, wg, slices);
    if (decoded && threadIdx.x == 0) put_granule(ctl + kSvcDone, 0u, tag);
    __syncthreads();  // (s_a and the body's LDS reused by the next pass)
  }
}

// GEVWS_TUNE_WALK_VARIANT values (0 = the default choice per batch).
const char* const kWalkVariants[] = {
    "default: one lane per connection with uniform-stream speculation (D = 8; plain D = 0 after a batch of mixed "
    "sizes on this context); from 128 connections per CU the entries go through an LDS ring to a writer wave "
    "(256-byte groups); the split walk for few long chains of small frames",
    "one lane per connection, plain chain walk (D = 0)",
    "no entry table (the record pass re-walks every chain)",
    "entries through the writer wave whatever the batch size (the default's path for >= 128 connections per CU)",
    "the default, with the split walk's entries stored by the walking lanes (no writer wave; measurement)",
};
constexpr int kNumWalkVariants = sizeof(kWalkVariants) / sizeof(kWalkVariants[0]);

}  // namespace

namespace gevws_impl {

int walk_variant_count() { return kNumWalkVariants; }
const void* direct_kernel_stub(int wide) {
  return wide ? reinterpret_cast<const void*>(&k_decode_small_direct<SmallWide>)
              : reinterpret_cast<const void*>(&k_decode_small_direct<SmallNarrow>);
}
uint32_t split_fallback_counter() { return kSplitFallbackCounter; }
const char* walk_variant_name(int i) { return i >= 0 && i < kNumWalkVariants ? kWalkVariants[i] : nullptr; }

// GEVWS_PHASE_TICKS=1 (measurement, tools/live_pass_probe.py): a one-launch
// decode also stamps, into the timeline ticks' words 2-5 (past the 4 the ABI
// documents: the caller's buffer must hold 6), when its input was in LDS,
// lane 0's chain parsed, the workgroup's scan done, its last store issued.
static uint64_t* phase_ticks(const gevws_ctx* ctx) {
  static const bool on = [] {
    const char* e = getenv("GEVWS_PHASE_TICKS");
    return e && e[0] == '1';
  }();
  return on && ctx->done_flag && ctx->ticks ? ctx->ticks + 2 : nullptr;
}

template <class S>
static int launch_decode_small(gevws_ctx* ctx, hipStream_t st, const uint8_t* d_in, uint64_t in_bytes,
                               const gevws_conn_in* d_conns, uint32_t n_conns, gevws_frame* d_frames,
                               uint64_t max_frames, uint8_t* d_payload, uint64_t payload_cap,
                               gevws_conn_out* d_conn_out, gevws_summary* d_summary) {
  const uint32_t seq = ctx->done_flag ? ++ctx->done_seq : 0u;
  // a pass that signals a mapped flag is a live pass over mapped host memory:
  // its input is read by kSmallStageWGs-wide slices (k_decode_small)
  uint32_t nwg = 1;
  if (ctx->done_flag && n_conns) {
    nwg = small_slices(in_bytes, n_conns, kSmallStageWGs);
    if (nwg > 1 && !ensure_small_stage(ctx, st)) nwg = 1;
  }
  const uint32_t tag = nwg > 1 ? next_hand_tag(ctx) : 0u;
  k_decode_small<S><<<nwg, S::NT, 0, st>>>(d_in, in_bytes, d_conns, n_conns, d_frames, max_frames, d_payload,
                                           payload_cap, d_conn_out, d_summary, ctx->done_flag, seq,
                                           ctx->done_flag ? ctx->ticks : nullptr, ctx->d_small_stage,
                                           ctx->d_done + kSmallStageCounter, tag, phase_ticks(ctx));
  GEVWS_HIP(hipGetLastError());
  const int r = ctx->prev_small_decode ? mark_last_lazy(ctx, st) : mark_last(ctx, st);
  ctx->prev_small_decode = true;
  if (ctx->done_flag) ctx->last_signal = seq;
  return r;
}

// The service's instance lives kServiceLifeMs of the GPU's clock from its
// start; the host posts to it only within kServiceUseMs of its launch, then
// replaces it (the old one returns at the generation bump, the new one starts
// behind it on the stream), so a posted pass always finds its instance.
constexpr uint64_t kServiceLifeMs = 200;
constexpr int64_t kServiceUseMs = 100;

static int64_t host_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// A narrow-shape live pass posted to the context's resident service (an
// instance launched first when none is live, or the live one is too old or
// signals elsewhere), or false: launch it as usual.  The mailbox is never
// overwritten before the instance has taken the last pass posted (ack), and
// the live instance gets the next pass only once the last has signalled (its
// workgroups are free); otherwise the pass is launched, behind the instance.
bool service_post(gevws_ctx* ctx, hipStream_t st, const uint8_t* d_in, uint64_t in_bytes,
                  const gevws_conn_in* d_conns, uint32_t n_conns, gevws_frame* d_frames, uint64_t max_frames,
                  uint8_t* d_payload, uint64_t payload_cap, gevws_conn_out* d_conn_out, gevws_summary* d_summary) {
  if (!ctx->svc_enabled || !ctx->svc_box || !ctx->done_flag || st != ctx->stream || n_conns > kSmallConns ||
      in_bytes > kSmallBytes)
    return false;
  if (__atomic_load_n(&ctx->svc_box->ack, __ATOMIC_ACQUIRE) != ctx->svc_last) return false;
  const int64_t now = host_ns();
  if (ctx->svc_live) {
    if (now - ctx->svc_t_launch_ns > kServiceUseMs * 1000000 || ctx->svc_flag != ctx->done_flag ||
        ctx->svc_ticks != ctx->ticks || ctx->svc_passes + 2 >= kServiceMaxPasses)
      service_stop(ctx);  // (replaced below, behind it on the stream)
    else if ((int32_t)(__atomic_load_n(ctx->svc_flag_host, __ATOMIC_ACQUIRE) - ctx->svc_last) < 0)
      return false;  // the last pass still runs
  }
  if (!ctx->svc_live) {
    if (ctx->last_direct) {  // (passes on the context's own queue finish first)
      if (direct_drain(ctx) != GEVWS_OK) return false;
      ctx->last_direct = false;
    }
    hipPointerAttribute_t pa;
    if (hipPointerGetAttributes(&pa, ctx->done_flag) != hipSuccess || !pa.hostPointer) return false;
    if (!ensure_small_stage(ctx, st)) return false;
    if (!ctx->d_svc_ctl) {
      const size_t cb = kSvcCtlGranules * sizeof(uint64_t);
      if (hipMalloc(reinterpret_cast<void**>(&ctx->d_svc_ctl), cb) != hipSuccess) {
        ctx->d_svc_ctl = nullptr;
        return false;
      }
      if (hipMemsetAsync(ctx->d_svc_ctl, 0, cb, st) != hipSuccess) return false;
    }
    if (ctx->has_last && ctx->last_stream != st &&
        (last_event(ctx) != GEVWS_OK || hipStreamWaitEvent(st, ctx->last_done, 0) != hipSuccess))
      return false;
    const uint32_t gen = ++ctx->svc_gen;
    const uint32_t t0 = reserve_hand_tags(ctx, kServiceMaxPasses);
    __atomic_store_n(&ctx->svc_box->gen, gen, __ATOMIC_RELEASE);
    k_decode_service<SmallNarrow><<<kSmallStageWGs, SmallNarrow::NT, 0, st>>>(
        ctx->svc_box_dev, gen, ctx->svc_last, kServiceLifeMs * ctx->wall_khz, ctx->done_flag, ctx->ticks,
        ctx->d_svc_ctl, ctx->d_small_stage, ctx->d_done + kSmallStageCounter, t0);
    if (hipGetLastError() != hipSuccess || mark_last_lazy(ctx, st) != GEVWS_OK) {
      __atomic_store_n(&ctx->svc_box->gen, ++ctx->svc_gen, __ATOMIC_RELEASE);
      return false;
    }
    ctx->svc_live = true;
    ctx->svc_t_launch_ns = now;
    ctx->svc_flag = ctx->done_flag;
    ctx->svc_flag_host = static_cast<const uint32_t*>(pa.hostPointer);
    ctx->svc_ticks = ctx->ticks;
    ctx->svc_t0 = t0;
    ctx->svc_passes = 0;
    ++ctx->svc_launches;
  }
  uint32_t seq = ++ctx->done_seq;
  if (seq == 0) seq = ++ctx->done_seq;  // (0: no pass, to the kernel)
  const uint64_t a[kServiceArgs] = {reinterpret_cast<uint64_t>(d_in),      in_bytes,
                                    reinterpret_cast<uint64_t>(d_conns),   n_conns,
                                    reinterpret_cast<uint64_t>(d_frames),  max_frames,
                                    reinterpret_cast<uint64_t>(d_payload), payload_cap,
                                    reinterpret_cast<uint64_t>(d_conn_out), reinterpret_cast<uint64_t>(d_summary)};
  for (int k = 0; k < kServiceArgs; ++k) __atomic_store_n(&ctx->svc_box->args[k], a[k], __ATOMIC_RELAXED);
  __atomic_store_n(&ctx->svc_box->req, ((uint64_t)ctx->svc_gen << 32) | seq, __ATOMIC_RELEASE);  // after the args
  ctx->svc_last = seq;
  ctx->last_signal = seq;
  ++ctx->svc_passes;
  ++ctx->svc_posts;
  return true;
}

int decode_small(gevws_ctx* ctx, hipStream_t st, const uint8_t* d_in, uint64_t in_bytes,
                 const gevws_conn_in* d_conns, uint32_t n_conns, gevws_frame* d_frames, uint64_t max_frames,
                 uint8_t* d_payload, uint64_t payload_cap, gevws_conn_out* d_conn_out, gevws_summary* d_summary) {
  if (n_conns > kOneLaunchConns || in_bytes > kOneLaunchBytes) return GEVWS_ERR_INVALID;
  const int r = order_after_last(ctx, st);
  if (r != GEVWS_OK) return r;
  // the narrow shape whenever the pass fits it: a quarter of the lanes to
  // launch and synchronise, and a CU keeps room for other work
  if (n_conns <= kSmallConns && in_bytes <= kSmallBytes)
    return launch_decode_small<SmallNarrow>(ctx, st, d_in, in_bytes, d_conns, n_conns, d_frames, max_frames,
                                            d_payload, payload_cap, d_conn_out, d_summary);
  return launch_decode_small<SmallWide>(ctx, st, d_in, in_bytes, d_conns, n_conns, d_frames, max_frames, d_payload,
                                        payload_cap, d_conn_out, d_summary);
}

// A live pass written into the context's own AQL queue (gevws_direct.cpp),
// or false: launch it as usual.  Same kernel body, shape and staging as the
// launched one-launch decode.
bool direct_post(gevws_ctx* ctx, const uint8_t* d_in, uint64_t in_bytes, const gevws_conn_in* d_conns,
                 uint32_t n_conns, gevws_frame* d_frames, uint64_t max_frames, uint8_t* d_payload,
                 uint64_t payload_cap, gevws_conn_out* d_conn_out, gevws_summary* d_summary) {
  if (!ctx->direct_enabled || !ctx->done_flag || n_conns > kOneLaunchConns || in_bytes > kOneLaunchBytes)
    return false;
  service_stop(ctx);
  const int wide = n_conns <= kSmallConns && in_bytes <= kSmallBytes ? 0 : 1;
  uint32_t nwg = n_conns ? small_slices(in_bytes, n_conns, kSmallStageWGs) : 1u;
  if (nwg > 1 && !ctx->d_small_stage) {  // (allocated and zeroed on the stream, once)
    if (!ensure_small_stage(ctx, ctx->stream)) nwg = 1;
    else if (hipStreamSynchronize(ctx->stream) != hipSuccess) return false;
  }
  DirectDecodeArgs a;
  a.in = d_in;
  a.in_bytes = in_bytes;
  a.conns = d_conns;
  a.frames = d_frames;
  a.max_frames = max_frames;
  a.payload = d_payload;
  a.payload_cap = payload_cap;
  a.cout = d_conn_out;
  a.sum = d_summary;
  a.done = ctx->done_flag;
  a.ticks = ctx->ticks;
  a.stage_buf = ctx->d_small_stage;
  a.stage_done = ctx->d_done + kSmallStageCounter;
  a.n = n_conns;
  uint32_t seq = ctx->done_seq + 1;
  if (seq == 0) seq = 1;
  a.seq = seq;
  a.tag = nwg > 1 ? next_hand_tag(ctx) : 0u;
  a.nwg = nwg;
  a.phase = phase_ticks(ctx);
  if (!direct_dispatch(ctx, wide, a)) return false;
  ctx->done_seq = seq;
  ctx->last_signal = seq;
  return true;
}

int decode_front(gevws_ctx* ctx, hipStream_t st, const uint8_t* d_in, uint64_t in_bytes,
                 const gevws_conn_in* d_conns, uint32_t n_conns, gevws_frame* d_frames, uint64_t max_frames,
                 uint64_t payload_cap, gevws_conn_out* d_conn_out, gevws_summary* d_summary, hipEvent_t* ev,
                 uint32_t** tile_first_out) {
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
  if ((wv == 0 || wv == 4) && n_conns) {
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
  const size_t run_bytes = kUnmaskRunCounters * 64;  // the unmask's run counters, 64 bytes apart
  r = ensure_scratch(ctx, blk_bytes + tile_bytes + run_bytes + flag_bytes + seg_bytes +
                              (n_entries + n_v) * sizeof(WalkEntry));
  if (r != GEVWS_OK) return r;
  char* sp = reinterpret_cast<char*>(ctx->scratch);
  uint64_t* blk = reinterpret_cast<uint64_t*>(sp);
  uint32_t* tile_first = reinterpret_cast<uint32_t*>(sp + blk_bytes);
  ctx->unmask_runs = reinterpret_cast<uint32_t*>(sp + blk_bytes + tile_bytes);
  uint8_t* rec_flags = reinterpret_cast<uint8_t*>(sp + blk_bytes + tile_bytes + run_bytes);
  char* segp = sp + blk_bytes + tile_bytes + run_bytes + flag_bytes;
  gevws_conn_in* segs = reinterpret_cast<gevws_conn_in*>(segp);
  gevws_conn_out* sout = reinterpret_cast<gevws_conn_out*>(segp + n_v * sizeof(gevws_conn_in));
  uint8_t* srec = reinterpret_cast<uint8_t*>(segp + n_v * (sizeof(gevws_conn_in) + sizeof(gevws_conn_out)));
  WalkEntry* entries = reinterpret_cast<WalkEntry*>(segp + seg_bytes);
  *tile_first_out = tile_first;
  if (ev) GEVWS_HIP(hipEventRecord(ev[0], st));
  // walk variant 2: no entry table -- the counting walk stores nothing per
  // frame and the record pass re-walks every chain
  const uint64_t ne = wv == 2 ? 0 : n_entries;
  // The walk's last workgroup scans the partials itself (walk_block_done) and
  // saves the k_scan_blocks launch (with release / acquire fences instead of
  // coherent partials it was slower: C1-shaped walk 0.034 -> 0.074 ms,
  // profiles/r02/r02_steps_fused.jsonl).
  const bool fused = nblk > 0 && nblk <= kFusedScanMaxBlocks;
  constexpr int kDecScanBlock = 256;
  uint32_t* done = fused ? ctx->d_done : nullptr;
  const uint32_t tag = fused ? next_hand_tag(ctx) : 0u;
  // the walk's uniform-stream speculation (D = 8) pays on long runs of equal
  // frames (C2, C3: -23..-28 %) and costs 2-7 % elsewhere (C1, C4,
  // profiles/r02/r02_walk_store_count_ab.jsonl); after a decode on this context
  // whose frames were mostly NOT the size of their predecessor the plain
  // chain walk (D = 0) runs instead
  const bool plain = wv == 1 || (wv != 1 && ctx->stats_known && ctx->prev_mixed);
  if (nblk && ks > 1) {
    // entries through the writer wave (walk variant 4: from the walking lanes, the round-5 form)
    const bool writer = wv != 4;
    GEVWS_HIP(hipMemsetAsync(ctx->d_done + kSplitFallbackCounter, 0, sizeof(uint32_t), st));
#define GEVWS_SPLIT(K)                                                                                            \
  (writer ? (plain ? k_walk_split<K, 0, 2> : k_walk_split<K, 8, 2>)                                               \
          : (plain ? k_walk_split<K, 0, 0> : k_walk_split<K, 8, 0>))<<<nblk, writer ? 2 * kCountBlock : kCountBlock, \
                                                                      0, st>>>(                                     \
      d_in, d_conns, n_conns, d_conn_out, blk, entries, ne, gshift, cpb_w, in_bytes, done, ctx->d_walk_part, tag,     \
      max_frames, payload_cap,                                                                                      \
      d_summary, segs, sout, srec, ctx->split_min_bytes, ctx->d_done + kSplitFallbackCounter)
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
        d_in, d_conns, n_conns, d_conn_out, blk, entries, ne, gshift, cpb, in_bytes, done, ctx->d_walk_part, tag,
        max_frames, payload_cap, d_summary);
  } else if (nblk) {
    (plain ? k_walk_count<0, 0> : k_walk_count<8, 0>)<<<nblk, kCountBlock, 0, st>>>(
        d_in, d_conns, n_conns, d_conn_out, blk, entries, ne, gshift, cpb, in_bytes, done, ctx->d_walk_part, tag,
        max_frames, payload_cap, d_summary);
  }
  if (ev) GEVWS_HIP(hipEventRecord(ev[1], st));
  if (!fused) k_scan_blocks<true, kDecFields, kDecScanBlock><<<1, kDecScanBlock, 0, st>>>(blk, nblk, max_frames, payload_cap,
                                                                                         d_summary);
  if (ev) GEVWS_HIP(hipEventRecord(ev[2], st));
  if (nblk) {
    k_walk_bases<<<nblk, kCountBlock, 0, st>>>(n_conns, d_conn_out, blk, d_summary, rec_flags, cpb_w, ctx->d_stats,
                                               ctx->unmask_runs);
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
  GEVWS_HIP(hipGetLastError());
  return GEVWS_OK;
}

}  // namespace gevws_impl
