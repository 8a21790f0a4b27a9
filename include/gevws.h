/*
 * gevws.h -- C ABI of the MI355X-native WebSocket frame-decode / payload-unmask
 * engine (gev_amd/libgevws.so).
 *
 * This is the drop-in boundary for gev's websocket Protocol plugin
 * (plugins/websocket/protocol.go:27-64, installed via gev.CustomProtocol,
 * options.go:83-87).  Every entry point names the reference interface it
 * replaces.  Conventions: plain C structs, caller-owned buffers, nothing
 * retained after return, int status (>= 0 ok, < 0 error).  One gevws_ctx per
 * event loop (thread-confined: it owns device scratch); no global mutable
 * state beyond one-time HIP runtime init.  See INTEGRATION.md for the cgo
 * binding a gev maintainer would add.
 */
#ifndef GEVWS_H
#define GEVWS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif
#if defined(__GNUC__)
#pragma GCC visibility push(default)
#endif

/* 2 (round 5): the split-stream calls gevws_ctx_set_unmask_stream,
 * gevws_stream_create_cu_mask, gevws_stream_destroy and gevws_stream_cu_count
 * are gone, gevws_copy_async rejects unknown flag bits, and the round-1..3
 * measurement exports (gevws_gather_async, gevws_unmask_profile,
 * gevws_ctx_last_walk_budget, gevws_ctx_last_resumed; tuning keys 5, 6, 9-12)
 * removed in round 4 are counted here too. */
/* 3 (round 6): gevws_protocol_stats grew two fields (service_passes,
 * service_misses) -- a caller built against version 2 passes a smaller
 * struct to gevws_protocol_get_stats -- and the one-launch decode's limits
 * rose to GEVWS_ONE_LAUNCH_MAX_CONNS / _BYTES.  Added: the resident service
 * (gevws_ctx_set_service, _service_stop, _service_stats,
 * gevws_decode_batch_post, gevws_protocol_set_service), direct dispatch
 * (gevws_ctx_set_direct, _direct_dispatches, gevws_protocol_set_direct),
 * gevws_ctx_synchronize, gevws_ctx_last_split_fallbacks. */
#define GEVWS_ABI_VERSION 3

/* ---------------------------------------------------------------- status codes */
enum {
    GEVWS_OK = 0,
    GEVWS_NEED_MORE = 1,          /* (nil, nil): ws.ErrHeaderNotReady or the
                                     completeness gate failed (read.go:20-23,
                                     protocol.go:47, 59-61) */
    GEVWS_ERR_LEN_MSB = -1,       /* ws.ErrHeaderLengthMSB (read.go:12-16, 71-73);
                                     the connection stream is poisoned */
    GEVWS_ERR_CAPACITY = -2,      /* output records / payload arena too small;
                                     the summary holds the exact sizes needed */
    GEVWS_ERR_INVALID = -3,       /* bad argument */
    GEVWS_ERR_DEVICE = -4,        /* HIP runtime error */
    GEVWS_HANDSHAKE = 2,          /* (nil, out): UnPacket ran the upgrade and `out`
                                     holds the 101 response (protocol.go:29-37) */
    GEVWS_ERR_NOT_UPGRADED = -5,  /* UnPacket before the handshake on a protocol
                                     that has no upgrader (gevws_protocol_set_upgrader) */
    GEVWS_ERR_HANDSHAKE = -6      /* Upgrader.Upgrade failed (ws.go:158-343); `out`
                                     may hold the error response, which the caller
                                     sends, as protocol.go:31-34 returns (nil, out) */
};

/* Readable slack the caller must provide after the last byte of a device input
 * arena (kernels read whole 16-byte vectors). */
#define GEVWS_IN_PAD 64
/* Every payload in the output arena starts on this boundary. */
#define GEVWS_PAYLOAD_ALIGN 16
/* Output-arena tile (bytes) of the unmask kernel's work map. */
#define GEVWS_TILE 4096
/* The one-launch decode's limits (GEVWS_TUNE_SMALL_BATCH): batches of at most
 * this many connections and input bytes run as ONE kernel launch. */
#define GEVWS_ONE_LAUNCH_MAX_CONNS 1024u
#define GEVWS_ONE_LAUNCH_MAX_BYTES (128u * 1024u)

/* ws.Header, plugins/websocket/ws/frame.go:169-176.  Byte-identical to the Go
 * struct {Fin bool; Rsv byte; OpCode OpCode; Masked bool; Mask [4]byte;
 * Length int64} (offsets 0,1,2,3,4..7,8..15; 16 bytes). */
typedef struct gevws_header {
    uint8_t fin;
    uint8_t rsv;
    uint8_t opcode;
    uint8_t masked;
    uint8_t mask[4];
    int64_t length;
} gevws_header;

/* One connection's buffered bytes inside the batch input arena: the linear
 * join of its ring buffer's PeekAll() segments (connection.go:220-251). */
typedef struct gevws_conn_in {
    uint64_t off;
    uint64_t len;
} gevws_conn_in;

/* One decoded frame = one (ctx, out) pair UnPacket would have returned
 * (protocol.go:57-58).  Records are ordered by connection, then stream order.
 * The unmasked payload is payload_arena[payload_off, payload_off+hdr.length);
 * src_off is the absolute input-arena offset of the payload's first byte, so
 * the frame's header length is src_off minus the end of the previous frame. */
typedef struct gevws_frame {
    gevws_header hdr;
    uint64_t payload_off;
    uint64_t src_off;
} gevws_frame;

/* Per-connection result: what the handlerProtocol loop (connection.go:208-218)
 * would have consumed before UnPacket returned (nil, nil). */
typedef struct gevws_conn_out {
    uint64_t first_frame;   /* index of its first record */
    uint64_t consumed;      /* bytes of complete frames (sum of h + L) */
    uint64_t payload_base;  /* arena offset of its first payload */
    uint32_t nframes;
    int32_t status;         /* GEVWS_OK, GEVWS_ERR_LEN_MSB, or GEVWS_ERR_INVALID when
                               the stream [off, off + len) is not inside d_in[0, in_bytes)
                               (nothing of it is read) */
} gevws_conn_out;

/* Batch totals (written on the device). */
typedef struct gevws_summary {
    uint64_t frames;        /* decoded frames */
    uint64_t payload_bytes; /* arena bytes used (16-byte rounded lengths) */
    uint64_t payload_len;   /* sum of payload lengths */
    uint64_t errors;        /* connections with status < 0 */
    int32_t status;         /* GEVWS_OK or GEVWS_ERR_CAPACITY */
    uint32_t flags;         /* GEVWS_SUMMARY_* (decode only; informational) */
    uint64_t run_frames;    /* decode: frames the size (h + L) of the frame before them on
                               their connection -- the batch's uniformity, which picks the
                               unmask kernel's window scheme */
    uint64_t reserved[2];
} gevws_summary;

/* summary.flags: the connection table was not in increasing, non-overlapping
 * input order, so the header walk's per-connection entry runs were not used and
 * the record pass re-walked every chain (same result, slower). */
#define GEVWS_SUMMARY_UNORDERED 1u

typedef struct gevws_ctx gevws_ctx;

/* ---------------------------------------------------------------- library */
int gevws_abi_version(void);
const char *gevws_status_string(int status);
int gevws_device_count(void);

/* One context per event loop (the reference keeps one per-connection header
 * scratch, protocol.go:37; the batch engine keeps its scratch per loop).
 * Successive contexts on a device cycle their stream's priority over the
 * normal level and the levels below it (0, 1, ...): each priority level has
 * its own hardware queues, so several loops' passes run side by side, and a
 * context never outranks the application's normal-priority work.  The
 * environment variable GEVWS_STREAM_PRIORITIES=all adds the levels above
 * normal (0, -1, 1, ...); =normal keeps every context at 0. */
gevws_ctx *gevws_ctx_create(int device);
void gevws_ctx_destroy(gevws_ctx *ctx);
int gevws_ctx_device(const gevws_ctx *ctx);
/* The context's own non-blocking hipStream_t (one per event loop). */
void *gevws_ctx_stream(const gevws_ctx *ctx);
/* Makes `stream` wait for everything the context's last call enqueued (on
 * whichever stream that call was given).  The calls that use the context's
 * scratch (decode, encode, dispatch) order themselves after its previous such
 * call when the stream changes; the helpers that do not (gevws_copy_async,
 * gevws_cipher_async, gevws_synth_async, gevws_synth_verify_async) follow
 * plain HIP stream semantics, so a caller that points one at a decode's
 * outputs from another stream orders it first, with this or an event. */
int gevws_ctx_order_after_last(gevws_ctx *ctx, void *stream);
/* Tuning knobs for measurement and parity tests (defaults are the tuned
 * choice): GEVWS_TUNE_UNMASK_VARIANT the unmask kernel (0 = default: v3 4-tile
 * windows for batches of equal-size frames, v5 pipelined 8-tile windows with
 * a chunk -> frame map for mixed sizes, its workgroups taking runs of 16
 * tiles from a per-XCD counter; 1 = v5 for every batch; 2 = the default with
 * one contiguous run per workgroup on the v5 path),
 * GEVWS_TUNE_UNMASK_GRID its workgroup count (0 = auto; when set it caps the
 * encode's grid too), GEVWS_TUNE_ENCODE_VARIANT the encode's step (0 = the
 * default: two 4 KiB tiles a wave step when out_cap / n > 256 bytes, else
 * one, and the waves' runs of tiles chosen on the device; 1 / 2 = always one /
 * two tiles; 3 / 4 / 5 = two tiles with contiguous / cyclic / counter runs),
 * GEVWS_TUNE_WALK_VARIANT the header walk (0 = the
 * default choice per batch; 1 = plain chain walk without the uniform-stream
 * speculation; 2 = no per-frame entries, the record pass re-walks every
 * chain; 3 = the entries through the writer wave whatever the batch size),
 * GEVWS_TUNE_SMALL_BATCH the input size in bytes (default and maximum
 * GEVWS_ONE_LAUNCH_MAX_BYTES = 131 072; 0 = never) up to which a batch of at
 * most GEVWS_ONE_LAUNCH_MAX_CONNS = 1 024 connections is decoded by ONE kernel
 * launch -- walk, scan, records and unmask in a single workgroup with the
 * input staged in LDS -- when every other knob is at its default and
 * per-phase timing is off, GEVWS_TUNE_SPLIT_LANES the lanes per connection of the default
 * walk's split form (k_walk_split: lanes guess frame starts inside the stream
 * and walk the segments between the guesses; a connection whose guesses do
 * not all line up is re-walked serially, so the output never depends on
 * them): 0 = auto (the batch's connections x lanes up to 256 per CU, streams
 * of >= 32 KiB mean), 1 = never, 2 / 4 / 8 / 16 / 32 = always.  Keys 5, 6,
 * 9-12 (round 1-3 measurement variants) are retired and rejected. */
#define GEVWS_TUNE_UNMASK_VARIANT 1
#define GEVWS_TUNE_UNMASK_GRID 2
#define GEVWS_TUNE_ENCODE_VARIANT 3
#define GEVWS_TUNE_WALK_VARIANT 4
#define GEVWS_TUNE_SMALL_BATCH 7
#define GEVWS_TUNE_SPLIT_LANES 8
/* Split walk (GEVWS_TUNE_SPLIT_LANES): a connection is cut into segments of at
 * least this many bytes (default 16 384; 1 024 .. 2^30) ... */
#define GEVWS_TUNE_SPLIT_MIN_BYTES 13
/* ... and the auto choice doubles the lanes per connection while the walk
 * keeps at most this many lanes per CU (default 512; 64 .. 4 096). */
#define GEVWS_TUNE_SPLIT_LANES_PER_CU 14
int gevws_ctx_set_tuning(gevws_ctx *ctx, int key, int64_t value);
/* Lanes per connection the last multi-kernel decode's header walk used (1 =
 * not split; GEVWS_TUNE_SPLIT_LANES), -1 for a null context.  The auto choice
 * splits a batch of few connections once an earlier decode on this context
 * has shown long chains of small frames (>= 256 frames per connection of <= 4
 * KiB each). */
int gevws_ctx_last_split_lanes(const gevws_ctx *ctx);
/* Connections of the last multi-kernel decode's split walk whose guesses did
 * not line up, so the walk re-walked them serially (0 when it was not split;
 * -1 for a null context or a device error).  Waits for the context's last
 * call.  Measurement: each costs its whole chain's serial walk. */
int64_t gevws_ctx_last_split_fallbacks(gevws_ctx *ctx);
/* Completion signal of the one-launch kernels (a live pass's: the small-batch
 * decode and gevws_handle_decoded_async's one-workgroup form).  With d_flag
 * (the device address of a 32-bit word in mapped, coherent host memory) set,
 * each such launch numbers itself and its kernel stores that number there
 * after all its outputs are visible at system scope; a host then spins on
 * host memory instead of hipStreamSynchronize.  NULL turns it off (the
 * default).  gevws_ctx_completion_seq: the number the last call's last kernel
 * stores, or -1 when that call ended with another kernel or copy (the caller
 * synchronises the stream as usual). */
int gevws_ctx_set_completion_flag(gevws_ctx *ctx, uint32_t *d_flag);
/* The resident decode service (opt-in; a live loop's passes without the launch
 * call's ~5 us of host time).  With it on and a completion flag set,
 * gevws_decode_batch_post hands a pass of at most 256 connections and 64 KiB
 * to a kernel kept resident on the context's stream (launched by the first
 * post; 32 workgroups, as many as a launched live pass stages its input with):
 * the pass's arguments go into a mailbox in mapped host memory, the kernel
 * polls it, decodes exactly as the one-launch decode and stores the pass's
 * number in the completion word.  One pass at a time: a post before the last
 * posted pass has signalled is launched instead, behind it.  Any other call
 * that enqueues work on the context ends the instance first (the pass posted
 * before it still runs, and that work runs behind it); an instance also ends
 * 200 ms after its start (the next post replaces it after 100 ms).  While one
 * is live the context's stream does not drain: call gevws_ctx_service_stop
 * before synchronising it directly.  enable = 0 stops it and turns posting
 * off (the default).  gevws_ctx_service_stats: instances launched and passes
 * posted to them, since the context's creation. */
int gevws_ctx_set_service(gevws_ctx *ctx, int enable);
int gevws_ctx_service_stop(gevws_ctx *ctx);
int gevws_ctx_service_stats(const gevws_ctx *ctx, int64_t *launches, int64_t *posts);
/* Direct dispatch (opt-in; takes precedence over the service): with it on and
 * a completion flag set, gevws_decode_batch_post writes a pass that fits the
 * one-launch decode (<= GEVWS_ONE_LAUNCH_MAX_CONNS / _BYTES) as one AQL
 * dispatch packet into an HSA queue the context owns -- the same kernel body,
 * without the HIP runtime's launch call on the caller's path.  Work the
 * context enqueues on a stream after such passes first waits (on the host)
 * for their completion words, and a direct pass after stream work waits for
 * that work.  If the runtime's loader does not expose the kernels, the
 * context falls back to launching (gevws_ctx_direct_dispatches stays 0).
 * enable = 0 waits for the outstanding direct passes and turns it off. */
int gevws_ctx_set_direct(gevws_ctx *ctx, int enable);
int64_t gevws_ctx_direct_dispatches(const gevws_ctx *ctx);
/* Waits for everything the context has enqueued: its stream, the passes on
 * its own queue, a live service instance (stopped first). */
int gevws_ctx_synchronize(gevws_ctx *ctx);
/* With a completion flag set: d_ticks (device address of 4 u64 in mapped,
 * coherent host memory, or NULL = off) receives, before the flag, each
 * one-launch kernel's start and end tick of the GPU's constant-rate wall
 * clock (s_memrealtime; hipDeviceAttributeWallClockRate kHz): [0] / [1] the
 * small-batch decode, [2] / [3] the one-workgroup handler step. */
int gevws_ctx_set_timeline_ticks(gevws_ctx *ctx, uint64_t *d_ticks);
int64_t gevws_ctx_completion_seq(const gevws_ctx *ctx);
/* Workgroups of the last multi-kernel decode's unmask launch (-1 for a null
 * context): 4 per CU, or 32 per CU after a decode on this context of a batch
 * of mixed frame sizes below 8 GiB of output (the kernel then uses the wide
 * grid if this batch is one too). */
int gevws_ctx_last_unmask_grid(const gevws_ctx *ctx);
/* Human-readable name of a variant (GEVWS_TUNE_UNMASK_VARIANT or
 * GEVWS_TUNE_WALK_VARIANT), or NULL past the last one. */
const char *gevws_tuning_name(int key, int64_t value);
/* Per-phase HIP-event timing of the following decode calls (0 = off). */
int gevws_ctx_set_timing(gevws_ctx *ctx, int enable);
/* Waits for the timed calls since the previous query and returns the summed
 * ms per phase -- [0] header walk (count), [1] scan, [2] header walk (emit),
 * [3] unmask/compact -- and the number of calls; then resets. */
int gevws_ctx_timing(gevws_ctx *ctx, float ms_sum[4], uint32_t *calls);

/* ---------------------------------------------------------------- hot path
 * Device-resident batch decode: for every connection, repeated
 * websocket.(*Protocol).UnPacket (plugins/websocket/protocol.go:38-62 ->
 * ws.VirtualReadHeader read.go:19-84 -> completeness gate protocol.go:47 ->
 * payload copy protocol.go:50-51 -> ws.Cipher cipher.go:14-53) until it would
 * return (nil, nil), exactly as Connection.handlerProtocol drives it
 * (connection.go:208-218).  All pointers d_* are device pointers; d_in must
 * have GEVWS_IN_PAD readable bytes past in_bytes.  Enqueued on `stream`
 * (hipStream_t; NULL = the HIP default stream).  Returns GEVWS_OK when
 * enqueued; the batch's own outcome is d_summary->status. */
int gevws_decode_batch_async(gevws_ctx *ctx, void *stream, const uint8_t *d_in, uint64_t in_bytes,
                             const gevws_conn_in *d_conns, uint32_t n_conns,
                             gevws_frame *d_frames, uint64_t max_frames,
                             uint8_t *d_payload, uint64_t payload_cap,
                             gevws_conn_out *d_conn_out, gevws_summary *d_summary);
/* A live pass on the context's own stream: posted to the resident decode
 * service when it is on (gevws_ctx_set_service), a completion flag is set and
 * the pass fits its shape (<= 256 connections, <= 64 KiB), else
 * exactly gevws_decode_batch_async on the context's stream.  Either way the
 * caller waits for gevws_ctx_completion_seq in the completion word (-1: the
 * stream). */
int gevws_decode_batch_post(gevws_ctx *ctx, const uint8_t *d_in, uint64_t in_bytes,
                            const gevws_conn_in *d_conns, uint32_t n_conns, gevws_frame *d_frames,
                            uint64_t max_frames, uint8_t *d_payload, uint64_t payload_cap,
                            gevws_conn_out *d_conn_out, gevws_summary *d_summary);

/* Synchronous form: same work, waits, copies the summary to *h_summary and
 * returns its status. */
int gevws_decode_batch(gevws_ctx *ctx, void *stream, const uint8_t *d_in, uint64_t in_bytes,
                       const gevws_conn_in *d_conns, uint32_t n_conns, gevws_frame *d_frames,
                       uint64_t max_frames, uint8_t *d_payload, uint64_t payload_cap,
                       gevws_conn_out *d_conn_out, gevws_summary *h_summary);

/* ---------------------------------------------------------------- outbound encode
 * One reply frame: the header to serialise and where its payload bytes are
 * (e.g. a decoded frame's slot in a payload arena). */
typedef struct gevws_out_frame {
    gevws_header hdr;
    uint64_t payload_off;
    uint64_t payload_len;
} gevws_out_frame;

/* Extra writable bytes the caller must provide past out_cap (the encoder
 * stores whole 16-byte vectors; bytes past the wire total are zeroed). */
#define GEVWS_OUT_PAD 16

/* ws.FrameToBytes (frame.go:274-278) = ws.WriteHeader (write.go:48-84) +
 * payload, for n frames at once, written back to back into d_out (the bytes
 * handlerProtocol appends to its send buffer, connection.go:208-218).
 * d_out_off[f] receives frame f's wire offset; d_summary->payload_bytes the
 * wire total, ->payload_len the payload total, ->status GEVWS_ERR_CAPACITY if
 * the total exceeds out_cap (nothing written to d_out; d_out_off[f] then holds
 * frame f's wire size h + L).  Payload bytes are read as
 * 16-byte vectors: d_payload needs 16 readable bytes past its last payload
 * byte (a decode's payload arena has them).  Device pointers; enqueued on
 * `stream`. */
int gevws_encode_batch_async(gevws_ctx *ctx, void *stream, const gevws_out_frame *d_frames, uint64_t n,
                             const uint8_t *d_payload, uint8_t *d_out, uint64_t out_cap,
                             uint64_t *d_out_off, gevws_summary *d_summary);

/* ---------------------------------------------------------------- control-frame dispatch
 * HandlerWrap.OnMessage (plugins/websocket/wrap.go:38-90) over decoded frames:
 * close -> util.HandleClose reply (util.go:27-46; close-code checks and UTF-8
 * validation of the reason as CheckCloseFrameData, util.go:65-85) and a
 * ShutdownWrite; ping -> pong with the same payload; pong -> ping with the
 * same payload (util.go:54-56, as the reference does); other control opcodes ->
 * nothing; data frames -> `policy` standing in for the user's WSHandler. */
enum {
    GEVWS_HANDLER_NONE = 0,        /* user handler replies nothing */
    GEVWS_HANDLER_ECHO_BINARY = 1, /* benchmarks/websocket/server.go:22-29 */
    GEVWS_HANDLER_ECHO_TEXT = 2    /* example/websocket OnMessage shape */
};
/* Bytes of aux space per close reply body (bodies are <= 125 bytes). */
#define GEVWS_AUX_SLOT 128

/* d_frames/n: a decode's records; d_payload: its payload arena, whose region
 * [aux_off, aux_off + aux_cap) receives the close-reply bodies (one
 * GEVWS_AUX_SLOT each).  Writes the replies in stream order to d_replies
 * (capacity n; payload_off relative to d_payload, ready for
 * gevws_encode_batch_async with the same d_payload) and d_reply_of[f] = reply
 * index or -1.  d_summary: frames = replies, payload_bytes = aux slots used,
 * errors = close frames (ShutdownWrite calls), status GEVWS_ERR_CAPACITY if
 * the aux region is too small. */
int gevws_dispatch_async(gevws_ctx *ctx, void *stream, const gevws_frame *d_frames, uint64_t n, int policy,
                         uint8_t *d_payload, uint64_t aux_off, uint64_t aux_cap,
                         gevws_out_frame *d_replies, int64_t *d_reply_of, gevws_summary *d_summary);

/* The same two steps chained after a decode with no host round trip (a live
 * pass: decode -> HandlerWrap.OnMessage -> FrameToBytes on the device): the
 * frame / reply count is read on the device from the previous step's summary
 * (d_decoded: the decode's; d_dispatched: the dispatch's), none when that
 * step failed; max_frames / max_replies only bound the launch and the
 * buffers (d_reply_of: max_frames entries, d_replies / d_out_off:
 * max_replies). */
int gevws_dispatch_decoded_async(gevws_ctx *ctx, void *stream, const gevws_frame *d_frames, uint64_t max_frames,
                                 const gevws_summary *d_decoded, int policy, uint8_t *d_payload, uint64_t aux_off,
                                 uint64_t aux_cap, gevws_out_frame *d_replies, int64_t *d_reply_of,
                                 gevws_summary *d_summary);
int gevws_encode_replies_async(gevws_ctx *ctx, void *stream, const gevws_out_frame *d_replies,
                               uint64_t max_replies, const gevws_summary *d_dispatched, const uint8_t *d_payload,
                               uint8_t *d_out, uint64_t out_cap, uint64_t *d_out_off, gevws_summary *d_summary);
/* Both steps at once behind a decode: gevws_dispatch_decoded_async then
 * gevws_encode_replies_async (same arguments, summaries and outputs).  A pass
 * of at most 1 024 frames with out_cap < 2^31 -- a live event loop's -- runs
 * them as ONE kernel launch (one workgroup); larger ones take the two steps'
 * seven launches.  d_out needs GEVWS_OUT_PAD bytes of slack after out_cap. */
int gevws_handle_decoded_async(gevws_ctx *ctx, void *stream, const gevws_frame *d_frames, uint64_t max_frames,
                               const gevws_summary *d_decoded, int policy, uint8_t *d_payload, uint64_t aux_off,
                               uint64_t aux_cap, gevws_out_frame *d_replies, int64_t *d_reply_of,
                               gevws_summary *d_disp_summary, uint8_t *d_out, uint64_t out_cap, uint64_t *d_out_off,
                               gevws_summary *d_enc_summary);

/* Measurement helper, not on the reference path: n bytes (n % 16 == 0, d_dst
 * 16-byte aligned, d_src any alignment) copied with the unmask kernel's
 * streaming access pattern minus the XOR and frame lookup -- the achievable
 * HBM rate bench.py reports beside the spec peak.  grid 0 = one workgroup per
 * CU (the unmask kernel's grid for large frames), each a contiguous run of
 * tiles; grid | 0x40000000 uses plain loads instead of the non-temporal ones the
 * unmask kernel's streaming path uses; grid | 0x20000000 copies in the
 * unmask's wave layout (each wave a contiguous 16 KiB span per step);
 * grid | 0x10000000 stores with plain 16-byte stores and then accepts a
 * d_dst of any alignment (the access pattern of an encode that scatters
 * aligned payload chunks to their wire positions); grid | 0x08000000 the
 * same with non-temporal stores. */
int gevws_copy_async(gevws_ctx *ctx, void *stream, uint8_t *d_dst, const uint8_t *d_src, uint64_t n,
                     uint32_t grid);

/* Host-ingress helper, not on the reference path: `bytes` of page-locked host
 * memory mapped into the device address space (hipHostMallocMapped).
 * *host_ptr is the CPU address, *dev_ptr the address kernels use; passing
 * *dev_ptr as gevws_decode_batch_async's d_payload makes the unmask kernel
 * write the decoded payload straight into host memory over PCIe (no D2H copy
 * of the arena).  GEVWS_ERR_DEVICE when the runtime refuses. */
int gevws_pinned_alloc(uint64_t bytes, void **host_ptr, void **dev_ptr);
int gevws_pinned_free(void *host_ptr);

/* Measurement helper, not on the reference path: `bytes` of device memory on
 * `device`, zeroed, of one of three kinds -- GEVWS_MEM_DEFAULT (hipMalloc:
 * coarse-grained, cached in L2), GEVWS_MEM_FINE (fine-grained) or
 * GEVWS_MEM_UNCACHED (hipDeviceMallocUncached: accesses bypass L2, so a
 * 16-byte header read need not fetch a whole 128-byte line).  An input arena
 * placed in it is decoded like any other.  Free with gevws_device_free. */
#define GEVWS_MEM_DEFAULT 0
#define GEVWS_MEM_FINE 1
#define GEVWS_MEM_UNCACHED 2
int gevws_device_alloc(int device, uint64_t bytes, int kind, void **ptr);
int gevws_device_free(int device, void *ptr);

/* ws.Cipher(payload, mask, offset), plugins/websocket/ws/cipher.go:14-53, on a
 * device buffer in place: p[i] ^= mask[(offset+i) % 4]. */
int gevws_cipher_async(gevws_ctx *ctx, void *stream, uint8_t *d_p, uint64_t n,
                       const uint8_t mask[4], uint64_t offset);

/* ---------------------------------------------------------------- per-frame host calls
 * For a host (cgo / C++) that looks at ONE frame at the head of a connection's
 * buffer -- e.g. to apply the reference's completeness gate (protocol.go:47)
 * before handing the connection to a device pass.  Plain host memory, no
 * context, no device work. */

/* ws.VirtualReadHeader (plugins/websocket/ws/read.go:19-84) on the `avail`
 * buffered bytes at p.  GEVWS_OK: *out = the header (ws.Header layout),
 * *hdr_len = its length (2..14); the frame is complete iff avail >= *hdr_len +
 * out->length (protocol.go:47).  GEVWS_NEED_MORE: fewer than 6 bytes
 * (ErrHeaderNotReady, read.go:20-23 -- even for a complete 2..5-byte frame) or
 * the extended header is not complete yet (Appendix A U1); *hdr_len = the
 * header length when at least 2 bytes are buffered, else 0.
 * GEVWS_ERR_LEN_MSB: ErrHeaderLengthMSB (read.go:71-73).  *out is written only
 * on GEVWS_OK. */
int gevws_parse_header(const uint8_t *p, uint64_t avail, gevws_header *out, uint32_t *hdr_len);

/* The same over a ring buffer's PeekAll() segments (first, end): the header may
 * straddle the wrap, as the virtual reads of read.go:27,63 allow. */
int gevws_parse_header_ring(const uint8_t *seg0, uint64_t n0, const uint8_t *seg1, uint64_t n1,
                            gevws_header *out, uint32_t *hdr_len);

/* ws.Cipher(p[:n], mask, offset) (plugins/websocket/ws/cipher.go:14-53) in host
 * memory, in place: p[i] ^= mask[(offset + i) % 4]. */
void gevws_cipher(uint8_t *p, uint64_t n, const uint8_t mask[4], uint64_t offset);

/* ---------------------------------------------------------------- synthetic batches
 * Device-side frame generator used by the bench and the full-size property
 * tests (no 64 GiB host buffer is ever built).  d_desc describes each frame:
 * header position in the arena, payload length, key, first header byte, and
 * length form (7, 16 or 64 bit).  Payload plaintext byte i of frame g is
 * byte (i & 7) of splitmix64(seed ^ (g * 0x9E3779B97F4A7C15) + (i >> 3)). */
typedef struct gevws_synth_desc {
    uint64_t hdr_off;   /* arena offset of the frame's first header byte */
    uint64_t length;    /* payload length */
    uint32_t mask;      /* key bytes, little-endian (mask[0] = low byte) */
    uint8_t b0;         /* FIN | RSV | opcode */
    uint8_t len_form;   /* 7, 16 or 64 */
    uint8_t masked;
    uint8_t pad;
} gevws_synth_desc;

int gevws_synth_async(gevws_ctx *ctx, void *stream, uint8_t *d_in, const gevws_synth_desc *d_desc,
                      uint64_t n_frames, uint64_t seed);
/* Property check of a decoded batch against the generator: counts mismatching
 * header fields, payload bytes (decode(mask(P)) == P) and non-zero pad bytes
 * into *d_mismatch (device uint64, accumulated).  Frame g of the batch must be
 * frame g of d_desc; records pointing outside [0, payload_cap) count as
 * mismatches and are not dereferenced. */
int gevws_synth_verify_async(gevws_ctx *ctx, void *stream, const gevws_synth_desc *d_desc,
                             uint64_t n_frames, uint64_t seed, const gevws_frame *d_frames,
                             const uint8_t *d_payload, uint64_t payload_cap, uint64_t *d_mismatch);

/* ---------------------------------------------------------------- host mirror
 * C++ host side above the device ABI, mirroring the reference's plugin
 * surface for this path (gev.Protocol, protocol.go:10-13; websocket.Protocol,
 * plugins/websocket/protocol.go:16-69; ringbuffer.RingBuffer as used at
 * read.go:20,27,63, protocol.go:47-60, connection.go:232-242). */
typedef struct gevws_ring gevws_ring;
typedef struct gevws_conn gevws_conn;
typedef struct gevws_protocol gevws_protocol;

/* ringbuffer.New(size) / Write / Length / PeekAll / Retrieve / IsEmpty. */
gevws_ring *gevws_ring_new(uint64_t size);
void gevws_ring_free(gevws_ring *r);
uint64_t gevws_ring_write(gevws_ring *r, const uint8_t *p, uint64_t n);
uint64_t gevws_ring_length(const gevws_ring *r);
uint64_t gevws_ring_capacity(const gevws_ring *r);
void gevws_ring_peek_all(const gevws_ring *r, const uint8_t **first, uint64_t *n_first,
                         const uint8_t **end, uint64_t *n_end);
void gevws_ring_retrieve(gevws_ring *r, uint64_t n);

/* gev.Connection's KeyValueContext as the websocket plugin uses it
 * (protocol.go:11-14, 28-39): the "gev_ws_upgraded" flag. */
gevws_conn *gevws_conn_new(void);
void gevws_conn_free(gevws_conn *c);
void gevws_conn_set_upgraded(gevws_conn *c, int upgraded);
int gevws_conn_upgraded(const gevws_conn *c);
/* Decoded frames still queued for delivery on this connection. */
uint64_t gevws_conn_pending(const gevws_conn *c);

/* websocket.New(u) (protocol.go:22-24), bound to a device context. */
gevws_protocol *gevws_protocol_new(gevws_ctx *ctx);
void gevws_protocol_free(gevws_protocol *p);

/* websocket.(*Protocol).UnPacket(c, buffer) (protocol.go:27-64): one frame per
 * call.  GEVWS_OK: *ctx_out = the header, (*out, *out_len) = the unmasked
 * payload (protocol-owned, valid until the next UnPacket on this connection),
 * h + L bytes consumed from `ring`.  GEVWS_NEED_MORE: (nil, nil), nothing
 * consumed.  < 0: logged and (nil, nil), as protocol.go:32-34, 41-45.  When the
 * connection has no queued frames the call decodes its buffered bytes on the
 * device first.  On a connection not yet upgraded it runs the handshake
 * (protocol.go:28-37; needs gevws_protocol_set_upgrader): GEVWS_HANDSHAKE with
 * (*out, *out_len) = the 101 response, or GEVWS_ERR_HANDSHAKE with the error
 * response (possibly empty) -- the driver loop (connection.go:208-218) keeps
 * calling while the status is GEVWS_OK or *out_len != 0, sending every `out`
 * that is not a frame payload. */
int gevws_protocol_unpacket(gevws_protocol *p, gevws_conn *c, gevws_ring *ring,
                            gevws_header *ctx_out, const uint8_t **out, uint64_t *out_len);

/* Batched driver for an event loop: one device pass over the buffered bytes of
 * n connections (stage -> H2D -> decode -> D2H); afterwards
 * gevws_protocol_unpacket returns their frames in stream order with no further
 * device work.  A pass still in flight from _begin below is finished (its
 * frames queued) first, as gevws_protocol_unpacket does.  Returns the number
 * of frames decoded, or < 0. */
int64_t gevws_protocol_unpacket_batch(gevws_protocol *p, gevws_conn *const *conns,
                                      gevws_ring *const *rings, uint32_t n);

/* gevws_protocol_unpacket_batch in two halves, so an event loop can read its
 * sockets while the device decodes (connection.go:208-251 runs read and
 * decode back to back; this overlaps them): _begin selects the connections
 * that can make progress, stages their buffered bytes and enqueues the pass
 * without waiting -- it returns the number of connections in the pass (0:
 * nothing to do) or < 0 (GEVWS_ERR_INVALID while a pass is in flight); _end
 * waits for that pass and queues its frames, returning the number of frames
 * decoded (0 when none is in flight) or < 0.  Between the two the rings may
 * take new bytes (gevws_ring_write; the pass decodes its staged copy) but must
 * not be read or retrieved; gevws_protocol_unpacket, _unpacket_batch and
 * gevws_decode_host_batch end a pass in flight first.  The protocol keeps the
 * `conns` and `rings` pointers (not the arrays) until _end: every connection
 * and ring listed must stay alive until then. */
int64_t gevws_protocol_unpacket_batch_begin(gevws_protocol *p, gevws_conn *const *conns,
                                            gevws_ring *const *rings, uint32_t n);
int64_t gevws_protocol_unpacket_batch_end(gevws_protocol *p);

/* Counters of a protocol's host ingress (not on the reference path):
 * device passes run, connections staged into them, bytes staged, UnPacket
 * calls answered NEED_MORE by the host-side gate without a device pass (the
 * first frame's h + L is not buffered yet, protocol.go:47), and the passes run
 * zero-copy (below). */
typedef struct gevws_protocol_stats {
    uint64_t device_passes;
    uint64_t conns_staged;
    uint64_t bytes_staged;
    uint64_t gated;
    uint64_t zero_copy_passes;
    uint64_t handler_passes;  /* passes that ran the device handler step */
    uint64_t chained_handler_passes; /* of those, enqueued behind a zero-copy
                                      * decode (one synchronisation per pass) */
    uint64_t signalled_passes;       /* waits answered by the kernels' completion
                                      * flag (gevws_ctx_set_completion_flag)
                                      * instead of a stream synchronisation */
    uint64_t service_passes;  /* passes posted to the resident decode service */
    uint64_t service_misses;  /* of those, launched again after the instance
                               * ended without them (not expected) */
} gevws_protocol_stats;
void gevws_protocol_get_stats(const gevws_protocol *p, gevws_protocol_stats *out);

/* Where a batched pass's time goes (measurement, not on the reference path):
 * host nanoseconds summed over the batched passes so far -- selecting the
 * ready connections (the host gate, protocol.go:47), staging their bytes into
 * pinned memory, enqueuing the launches (and copies), waiting for the
 * completion flag or the stream, and queueing the frames on their
 * connections -- and, for passes answered by the completion flag, the
 * one-launch kernels' own GPU time from their tick stamps.  ns_wait minus the
 * GPU time is the launch and completion latency. */
typedef struct gevws_protocol_timeline {
    uint64_t passes;
    uint64_t signalled;        /* passes whose wait was the completion flag (GPU times below) */
    uint64_t ns_select;
    uint64_t ns_stage;
    uint64_t ns_launch;
    uint64_t ns_wait;
    uint64_t ns_deliver;
    uint64_t ns_gpu_decode;    /* signalled passes: k_decode_small's start -> end */
    uint64_t ns_gpu_handler;   /* signalled passes with the handler step: k_handle_small's */
    uint64_t ns_gpu_gap;       /* signalled passes with the handler: decode end -> handler start */
} gevws_protocol_timeline;
void gevws_protocol_get_timeline(const gevws_protocol *p, gevws_protocol_timeline *out);

/* Batched passes over at most `bytes` of buffered input (default
 * GEVWS_ZERO_COPY_MAX_DEFAULT; 0 = never) run zero-copy: the kernels read the
 * pinned staging block and write records, payload and results into mapped
 * pinned host memory, so the pass is its launches and one synchronisation
 * with no H2D / D2H copies (a small pass is latency, not bytes).  Larger
 * passes copy in and out (DMA at the PCIe rate). */
#define GEVWS_ZERO_COPY_MAX_DEFAULT (256u * 1024u)

/* websocket.HandlerWrap.OnMessage (plugins/websocket/wrap.go:38-90) on the
 * device for every frame a pass decodes: policy GEVWS_HANDLER_* (-1 = off, the
 * default).  Each pass then also runs gevws_dispatch_async + encode over its
 * frames (close -> util.HandleClose reply, ping -> pong, pong -> ping, data ->
 * the policy's echo as a binary / text frame; FrameToBytes of each) and one
 * more synchronisation; gevws_protocol_reply hands out the answer. */
int gevws_protocol_set_handler(gevws_protocol *p, int policy);
/* The handler's answer for the frame gevws_protocol_unpacket last returned on
 * c: *reply / *len = the reply frame's wire bytes (the `out` OnMessage returns;
 * len 0 = none), *shutdown_write = 1 for a close frame (c.ShutdownWrite() after
 * sending the reply, wrap.go:52-56).  Valid until the next UnPacket on c.
 * GEVWS_ERR_INVALID when no frame was returned yet or the returned frame's
 * pass did not run the handler (decoded while it was off). */
int gevws_protocol_reply(const gevws_protocol *p, const gevws_conn *c, const uint8_t **reply, uint64_t *len,
                         int *shutdown_write);
void gevws_protocol_set_zero_copy_max(gevws_protocol *p, uint64_t bytes);
/* The protocol's zero-copy passes without a handler step go to its context's
 * resident decode service (gevws_ctx_set_service, gevws_decode_batch_post):
 * no launch call on the loop's path.  on = 0 stops it (the default). */
int gevws_protocol_set_service(gevws_protocol *p, int on);
/* The same for direct dispatch (gevws_ctx_set_direct): the protocol's
 * zero-copy passes without a handler step are written into its context's
 * own queue.  on = 0 turns it off (the default). */
int gevws_protocol_set_direct(gevws_protocol *p, int on);

/* One connection's buffered bytes in host memory, as ringbuffer.PeekAll()
 * returns them (first, end) -- e.g. two Go slices passed through cgo. */
typedef struct gevws_host_conn {
    const uint8_t *seg0;
    uint64_t n0;
    const uint8_t *seg1;
    uint64_t n1;
} gevws_host_conn;

/* Host-memory form of the batch decode for FFI callers (cgo): the segments of
 * n connections are staged into pinned memory, decoded on the device and the
 * results copied into the caller's buffers (frames, 16-byte-aligned payload
 * arena, per-connection results).  frames[i].src_off is relative to its own
 * connection's joined segments.  Returns the frame count, GEVWS_ERR_CAPACITY
 * (with *summary holding the sizes needed), or < 0.  Nothing is retained. */
int64_t gevws_decode_host_batch(gevws_protocol *p, const gevws_host_conn *conns, uint32_t n,
                                gevws_frame *frames, uint64_t max_frames, uint8_t *payload,
                                uint64_t payload_cap, gevws_conn_out *conn_out,
                                gevws_summary *summary);

/* One connection, segments as plain arguments (cgo may pass Go slice pointers
 * as arguments but not inside a struct): repeated UnPacket over
 * seg0 || seg1, i.e. ringbuffer.PeekAll()'s (first, end). */
int64_t gevws_decode_host_stream(gevws_protocol *p, const uint8_t *seg0, uint64_t n0,
                                 const uint8_t *seg1, uint64_t n1, gevws_frame *frames,
                                 uint64_t max_frames, uint8_t *payload, uint64_t payload_cap,
                                 gevws_conn_out *conn_out, gevws_summary *summary);

/* ---------------------------------------------------------------- handshake
 * ws.Upgrader (plugins/websocket/ws/ws.go:49-154) and Upgrader.Upgrade
 * (ws.go:158-343) with its HTTP helpers (http.go, nonce.go, util.go) -- host
 * code, once per connection. */
enum {
    GEVWS_HS_OK = 0,
    GEVWS_HS_MALFORMED_REQUEST = 1, /* ErrMalformedRequest (errors.go:60-64); also the
                                       head not yet complete (ws.go:176-198: nothing read) */
    GEVWS_HS_BAD_PROTOCOL = 2,      /* ErrHandshakeBadProtocol (errors.go:26-29) */
    GEVWS_HS_BAD_METHOD = 3,        /* ErrHandshakeBadMethod (errors.go:30-33) */
    GEVWS_HS_BAD_HOST = 4,          /* errors.go:34-37 */
    GEVWS_HS_BAD_UPGRADE = 5,       /* errors.go:38-41 */
    GEVWS_HS_BAD_CONNECTION = 6,    /* errors.go:42-45 */
    GEVWS_HS_BAD_SEC_ACCEPT = 7,    /* errors.go:46-49 (client side; never produced here) */
    GEVWS_HS_BAD_SEC_KEY = 8,       /* errors.go:50-53 */
    GEVWS_HS_BAD_SEC_VERSION = 9,   /* errors.go:54-57 */
    GEVWS_HS_UPGRADE_REQUIRED = 10, /* ErrHandshakeUpgradeRequired (errors.go:66-79): 426 */
    GEVWS_HS_HOOK = 11              /* an Upgrader hook returned an error */
};

/* What a hook returns with a non-zero result: RejectConnectionError(
 * RejectionStatus(code), RejectionReason(reason), RejectionHeader(header))
 * (errors.go:81-129), or with plain = 1 an ordinary Go error whose Error() is
 * `reason` (answered 500 without extra header, ws.go:325-333). */
typedef struct gevws_reject {
    int32_t code;            /* 0 -> 500 (ws.go:331-333) */
    int32_t plain;
    const char *reason;
    uint64_t reason_len;
    const uint8_t *header;   /* raw "Key: value\r\n" lines */
    uint64_t header_len;
} gevws_reject;

/* One parameter of a Sec-WebSocket-Extensions option (httphead.Option). */
typedef struct gevws_ext_param {
    const uint8_t *key;
    uint64_t key_len;
    const uint8_t *value;    /* NULL when the parameter has no value */
    uint64_t value_len;
} gevws_ext_param;

/* The Upgrader's function fields (ws.go:51-153); any may be NULL.  Every
 * argument is valid only until the hook returns.  Hooks returning int: 0 =
 * accept, non-zero = reject with *rej filled (strings copied before return). */
typedef struct gevws_upgrader_hooks {
    void *user;
    /* Protocol (ws.go:51-56): non-zero selects the offered token. */
    int (*protocol)(void *user, const uint8_t *token, uint64_t n);
    /* ProtocolCustom (ws.go:58-61): returns ok; *sel = the selected protocol. */
    int (*protocol_custom)(void *user, gevws_conn *c, const uint8_t *value, uint64_t n,
                           const uint8_t **sel, uint64_t *sel_n);
    /* Extension (ws.go:63-79): non-zero accepts the option. */
    int (*extension)(void *user, const uint8_t *name, uint64_t n, const gevws_ext_param *params,
                     uint32_t n_params);
    /* ExtensionCustom (ws.go:81-84): the header value and the extensions selected
     * so far (response text form) -> ok, *sel = the new selection's text. */
    int (*extension_custom)(void *user, gevws_conn *c, const uint8_t *value, uint64_t n,
                            const uint8_t *cur, uint64_t cur_n, const uint8_t **sel, uint64_t *sel_n);
    /* OnRequest (ws.go:97-106), OnHost (ws.go:108-121), OnHeader (ws.go:123-133). */
    int (*on_request)(void *user, gevws_conn *c, const uint8_t *uri, uint64_t n, gevws_reject *rej);
    int (*on_host)(void *user, gevws_conn *c, const uint8_t *host, uint64_t n, gevws_reject *rej);
    int (*on_header)(void *user, gevws_conn *c, const uint8_t *key, uint64_t kn, const uint8_t *value,
                     uint64_t vn, gevws_reject *rej);
    /* OnBeforeUpgrade (ws.go:135-153): 0 and optionally extra response header
     * lines in (*hdr, *hdr_len), or non-zero + *rej. */
    int (*on_before_upgrade)(void *user, gevws_conn *c, const uint8_t **hdr, uint64_t *hdr_len,
                             gevws_reject *rej);
} gevws_upgrader_hooks;

/* Upgrade's result: ws.Handshake (ws.go:40-47) plus the error.  Pointers are
 * owned by the connection and valid until its next handshake call. */
typedef struct gevws_handshake {
    const uint8_t *protocol;
    uint64_t protocol_len;
    const uint8_t *extensions;   /* as written in Sec-WebSocket-Extensions */
    uint64_t extensions_len;
    int32_t error;               /* GEVWS_HS_* */
    int32_t http_code;           /* 101, the error response status, or 0: nothing written */
    const char *reason;          /* err.Error(); "" on success */
} gevws_handshake;

typedef struct gevws_upgrader gevws_upgrader;

/* &ws.Upgrader{} -- immutable once configured, so one upgrader may serve every loop. */
gevws_upgrader *gevws_upgrader_new(void);
void gevws_upgrader_free(gevws_upgrader *u);
/* Upgrader.Header (ws.go:88-95) as raw header lines. */
void gevws_upgrader_set_header(gevws_upgrader *u, const uint8_t *hdr, uint64_t n);
void gevws_upgrader_set_hooks(gevws_upgrader *u, const gevws_upgrader_hooks *hooks);
/* Upgrader.Upgrade(c, in) (ws.go:158-343): consumes the request head from `in`
 * once it is complete; (*out, *out_len) = the 101 or error response (owned by
 * `c`; empty when the reference writes none).  GEVWS_OK or GEVWS_ERR_HANDSHAKE. */
int gevws_upgrader_upgrade(const gevws_upgrader *u, gevws_conn *c, gevws_ring *in, const uint8_t **out,
                           uint64_t *out_len, gevws_handshake *hs);
/* The connection's last handshake result (after UnPacket ran the upgrade). */
int gevws_conn_handshake(const gevws_conn *c, gevws_handshake *hs);
const char *gevws_handshake_error_string(int hs_error);
/* initAcceptFromNonce (nonce.go:23-39): 24-byte key -> 28-byte Sec-WebSocket-Accept. */
void gevws_accept_key(const uint8_t nonce[24], char accept[28]);
/* websocket.New(u) (protocol.go:22-24): UnPacket on a connection that is not
 * upgraded runs the handshake (protocol.go:28-37). */
void gevws_protocol_set_upgrader(gevws_protocol *p, const gevws_upgrader *u);

/* websocket.(*Protocol).Packet (protocol.go:67-69): identity. */
const uint8_t *gevws_protocol_packet(gevws_protocol *p, gevws_conn *c, const uint8_t *data,
                                     uint64_t n, uint64_t *out_len);

/* ---------------------------------------------------------------- multi-GPU in one process
 * A gev server drives all its event loops from one process (server.go:80-91):
 * with NumLoops loops placed on the node's GPUs round-robin (loop l on device
 * devices[l % n], one gevws_ctx per loop, load_balance.go:7-14 deals
 * connections to loops), each device decodes only its own loops' connections
 * and the one collective is the all-reduce(sum) of the decoded counts
 *  over RCCL / xGMI -- payloads never cross GPUs.
 * gevws_comm_create: ncclCommInitAll over `devices` (RCCL is loaded on first
 * use; NULL when it is absent or a device is not visible). */
typedef struct gevws_comm gevws_comm;
gevws_comm *gevws_comm_create(const int *devices, int n);
void gevws_comm_destroy(gevws_comm *comm);
int gevws_comm_size(const gevws_comm *comm);
/* For every device i of the communicator: d_counts[i] (int64[3], device
 * memory on device i) = the sum over all devices of {frames, payload_len,
 * errors} of their decode summaries d_summaries[i], enqueued on ctxs[i]'s
 * stream after whatever it holds and after ctxs[i]'s last decode, whichever
 * stream that ran on (one RCCL group, ncclAllReduce in place).
 * ctxs[i] must be on the communicator's device i.  The synchronous form
 * waits and also returns the totals in h_total. */
int gevws_counts_allreduce_async(gevws_comm *comm, gevws_ctx *const *ctxs, const gevws_summary *const *d_summaries,
                                 int64_t *const *d_counts);
int gevws_counts_allreduce(gevws_comm *comm, gevws_ctx *const *ctxs, const gevws_summary *const *d_summaries,
                           int64_t *const *d_counts, int64_t h_total[3]);

#if defined(__GNUC__)
#pragma GCC visibility pop
#endif
#ifdef __cplusplus
}
#endif
#endif /* GEVWS_H */
