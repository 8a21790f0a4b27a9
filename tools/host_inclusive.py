#!/usr/bin/env python3
"""Host-inclusive rate of the decode path: the bytes start and end in host
memory, as they do in gev (socket -> ringbuffer.RingBuffer -> user buffer).

Input frames sit in pinned host memory (hipHostMalloc via torch pin_memory),
split into chunks of whole connections; each chunk goes H2D -> decode ->
D2H (payload arena + frame records + per-connection results) on one of S
streams, so copies in both directions overlap the device work.  Reports payload
GiB/s host-to-host next to the raw pinned H2D / D2H copy rates on this box.

With --direct-out the payload arena is mapped pinned host memory
(gevws_pinned_alloc): the unmask kernel writes the plaintext over PCIe and no
payload D2H copy is issued.  With --zero-copy-in the input frames sit in
mapped pinned host memory too and the kernels read them over PCIe (no H2D
copy): with both, a chunk is its launches only -- the large-chunk form of the
live server's zero-copy pass.

    python tools/host_inclusive.py [--gib 8] [--chunk-mib 64] [--streams 2] [--reps 3] [--sweep 64:2,128:3]
                                   [--direct-out] [--zero-copy-in]

The report carries the pinned copy rates one way at a time and both ways at
once (two streams): the last is the bound of the overlapped pipeline
(`frac_of_bidirectional`).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=8.0, help="payload GiB per pass")
    ap.add_argument("--frame", type=int, default=65536)
    ap.add_argument("--chunk-mib", type=int, default=64)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--sweep", default="", help="comma list of chunk_mib:streams to measure, e.g. 64:2,128:3")
    ap.add_argument("--direct-out", action="store_true",
                    help="the unmask kernel writes the payload straight into mapped pinned host memory "
                         "(gevws_pinned_alloc) instead of a device arena + D2H copy")
    ap.add_argument("--zero-copy-in", action="store_true",
                    help="the kernels read the input frames straight from mapped pinned host memory (no H2D copy)")
    args = ap.parse_args()

    import numpy as np
    import torch

    import gev_amd
    from gev_amd import workloads as w

    dev = torch.device("cuda", 0)
    eng = gev_amd.Engine(0)
    n_frames = int(args.gib * 2**30) // args.frame
    lay = w.uniform(max(1, n_frames // 64), 64, args.frame, name=f"{n_frames} x {args.frame} B masked binary")
    stream_bytes = int(lay.conns[0, 1])
    fpc = 64
    # build the batch on the device and stage it into pinned host memory
    d_all = torch.empty(lay.arena_bytes + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    d_all[lay.arena_bytes:] = 0
    eng.synth(d_all, torch.from_numpy(lay.desc.view(np.uint8).copy()).to(dev), lay.n_frames, lay.seed)
    if args.zero_copy_in:
        in_arena = gev_amd.PinnedArena(lay.arena_bytes + gev_amd.IN_PAD)
        h_in = torch.from_numpy(in_arena.host)  # CPU view of the mapped pages
    else:
        h_in = torch.empty(lay.arena_bytes + gev_amd.IN_PAD, dtype=torch.uint8, pin_memory=True)
    h_in.copy_(d_all)
    del d_all
    torch.cuda.empty_cache()
    pay_frame = (args.frame + 15) // 16 * 16
    if args.direct_out:
        arena = gev_amd.PinnedArena(lay.n_frames * pay_frame + 64)
        h_pay = torch.from_numpy(arena.host)  # CPU view of the mapped pages
    else:
        h_pay = torch.empty(lay.n_frames * pay_frame, dtype=torch.uint8, pin_memory=True)
    h_frames = torch.empty((lay.n_frames, 32), dtype=torch.uint8, pin_memory=True)
    h_cout = torch.empty((lay.n_conns, 32), dtype=torch.uint8, pin_memory=True)

    def run(chunk_mib: int, S: int):
        cpc = max(1, (chunk_mib << 20) // stream_bytes)          # connections per chunk
        n_chunks = (lay.n_conns + cpc - 1) // cpc
        chunk_in = cpc * stream_bytes
        chunk_frames = cpc * fpc
        chunk_pay = chunk_frames * pay_frame
        streams = [torch.cuda.Stream(dev) for _ in range(S)]
        engs = [gev_amd.Engine(0) for _ in range(S)]  # one context (scratch) per stream
        d_in = [None if args.zero_copy_in else torch.zeros(chunk_in + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
                for _ in range(S)]
        outs = [eng.alloc_batch(cpc, chunk_frames, 0 if args.direct_out else chunk_pay) for _ in range(S)]
        conn_tab = np.stack([np.arange(cpc, dtype=np.int64) * stream_bytes,
                             np.full(cpc, stream_bytes, np.int64)], 1)
        d_conns = torch.from_numpy(conn_tab).to(dev)

        def one_pass():
            for c in range(n_chunks):
                k = c % S
                s = streams[k]
                nconn = min(cpc, lay.n_conns - c * cpc)
                nin, nfr = nconn * stream_bytes, nconn * fpc
                with torch.cuda.stream(s):
                    if args.zero_copy_in:
                        src = in_arena.at(c * chunk_in)  # the kernels read the mapped host pages
                    else:
                        d_in[k][:nin].copy_(h_in[c * chunk_in:c * chunk_in + nin], non_blocking=True)
                        src = d_in[k]
                    f0 = c * chunk_frames
                    if args.direct_out:
                        o = outs[k]
                        direct = gev_amd.Batch(frames=o.frames, payload=arena.at(f0 * pay_frame),
                                               conn_out=o.conn_out, summary=o.summary, n_conns=o.n_conns)
                        engs[k].decode_async(src, nin, d_conns, nconn, direct, chunk_frames,
                                             nfr * pay_frame, stream=s)
                    else:
                        engs[k].decode_async(src, nin, d_conns, nconn, outs[k], chunk_frames, chunk_pay,
                                             stream=s)
                        h_pay[f0 * pay_frame:(f0 + nfr) * pay_frame].copy_(outs[k].payload[:nfr * pay_frame],
                                                                           non_blocking=True)
                    h_frames[f0:f0 + nfr].copy_(outs[k].frames[:nfr], non_blocking=True)
                    h_cout[c * cpc:c * cpc + nconn].copy_(outs[k].conn_out[:nconn], non_blocking=True)
            torch.cuda.synchronize()

        one_pass()  # warm
        fr = h_frames[:4].numpy().reshape(-1).view(gev_amd.FRAME_DTYPE)
        for g in range(4):
            o = int(fr["payload_off"][g])
            assert h_pay[o:o + args.frame].numpy().tobytes() == w.plaintext(lay.seed, g, args.frame)
        last = lay.n_frames - 1
        assert h_pay[last * pay_frame:last * pay_frame + args.frame].numpy().tobytes() == \
            w.plaintext(lay.seed, last, args.frame)
        times = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            one_pass()
            times.append(time.perf_counter() - t0)
        t = min(times)
        del outs, d_in
        for e in engs:
            e.close()
        torch.cuda.empty_cache()
        return {"chunk_mib": chunk_mib, "streams": S, "chunks": n_chunks, "seconds": round(t, 4),
                "payload_GiBps": round(lay.payload_len / t / 2**30, 2), "frames_per_s": round(lay.n_frames / t, 1)}

    # raw pinned copy rates of the same byte counts: one direction at a time,
    # and both at once on two streams -- the bound of an overlapped pipeline,
    # whose every payload byte crosses PCIe once each way
    n_tmp = min(2 << 30, lay.arena_bytes, h_pay.numel())
    d_tmp = torch.empty(n_tmp, dtype=torch.uint8, device=dev)
    d_tmp2 = torch.empty(n_tmp, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        d_tmp.copy_(h_in[:n_tmp], non_blocking=True)
    torch.cuda.synchronize()
    h2d = 3 * n_tmp / (time.perf_counter() - t0)
    t0 = time.perf_counter()
    for _ in range(3):
        h_pay[:n_tmp].copy_(d_tmp, non_blocking=True)
    torch.cuda.synchronize()
    d2h = 3 * n_tmp / (time.perf_counter() - t0)
    s_up, s_down = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        with torch.cuda.stream(s_up):
            d_tmp.copy_(h_in[:n_tmp], non_blocking=True)
        with torch.cuda.stream(s_down):
            h_pay[:n_tmp].copy_(d_tmp2, non_blocking=True)
    torch.cuda.synchronize()
    bidir = 3 * n_tmp / (time.perf_counter() - t0)  # bytes each way per second, both at once
    del d_tmp, d_tmp2
    configs = [(args.chunk_mib, args.streams)]
    if args.sweep:
        configs = [tuple(int(x) for x in item.split(":")) for item in args.sweep.split(",")]
    runs = [run(cm, S) for cm, S in configs]
    best = max(runs, key=lambda r: r["payload_GiBps"])
    src_mode = "decode reading mapped host memory" if args.zero_copy_in else "pinned H2D -> decode"
    dst_mode = "writing the payload into mapped host memory" if args.direct_out else "-> D2H, overlapped"
    mode = f"host-inclusive ({src_mode} {dst_mode})"
    res = {"mode": mode,
           "workload": lay.name, "payload_bytes": lay.payload_len, "input_bytes": lay.arena_bytes,
           "payload_GiBps": best["payload_GiBps"], "frames_per_s": best["frames_per_s"], "best": best,
           "runs": runs, "pinned_h2d_GBps": round(h2d / 1e9, 2), "pinned_d2h_GBps": round(d2h / 1e9, 2),
           "pinned_bidirectional_GBps_each_way": round(bidir / 1e9, 2),
           # the pipeline moves about one input byte in and one payload byte out per payload byte
           "frac_of_bidirectional": round(best["payload_GiBps"] * 2**30 / bidir, 3)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
