#!/usr/bin/env python3
"""Where a live pass's ~9 us goes: the one-launch decode of the C1 loop's pass
shape (100 connections, one masked 128-byte frame each) with its input and
its outputs placed in device memory or in mapped pinned host memory (the live
server's zero-copy form), launched or written directly into the context's own
AQL queue.  Per placement: the kernel's own time from its start / end ticks
(s_memrealtime, the ticks' rate calibrated against the host clock over the
run) and the host's post -> completion-word latency, medians over --reps;
with GEVWS_PHASE_TICKS=1 also the kernel's phases (input in LDS, lane 0's
chain parsed, the workgroup's scan, the last output store issued).

    python tools/live_pass_probe.py [--reps 300] [--conns 100] [--msg 128]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--conns", type=int, default=100)
    ap.add_argument("--msg", type=int, default=128)
    args = ap.parse_args()
    import numpy as np
    import torch

    import gev_amd
    from oracle import ref
    from oracle import ws_oracle as wo

    rng = np.random.default_rng(7)
    ss = [wo.encode_frame(bytes(rng.integers(0, 256, args.msg, dtype=np.uint8)), 1, True, 0, True,
                          bytes(rng.integers(0, 256, 4, dtype=np.uint8))) for _ in range(args.conns)]
    a = np.frombuffer(b"".join(ss), np.uint8).copy()
    lens = np.array([len(s) for s in ss], np.int64)
    conns = np.stack([np.concatenate([[0], np.cumsum(lens)[:-1]]), lens], 1).astype(np.int64)
    n, nbytes = conns.shape[0], a.size
    max_frames, payload_cap = n + 1, nbytes + 16 * n + 64
    want = ref.decode_batch(a, conns[:, 0], conns[:, 1])

    dev = torch.device("cuda", 0)
    eng = gev_amd.Engine(0)
    sig = gev_amd.PinnedArena(4096)  # [64] completion word, [128] ticks
    eng.set_completion_flag(sig, 64)
    eng.set_timeline_ticks(sig, 128)
    word = sig.host[64:68].view(np.uint32)
    ticks = sig.host[128:176].view(np.uint64)  # [0] / [1] the kernel, [2..5] its phases

    # inputs: device tensors or pinned host memory (input + conn table)
    d_in = torch.zeros(nbytes + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    d_in[:nbytes] = torch.from_numpy(a).to(dev)
    d_conns = torch.from_numpy(conns.copy()).to(dev)
    h_inp = gev_amd.PinnedArena(nbytes + gev_amd.IN_PAD + 16 * n + 256)
    h_inp.host[:] = 0
    h_inp.host[:nbytes] = a
    coff = (nbytes + gev_amd.IN_PAD + 255) // 256 * 256
    h_inp.host[coff:coff + 16 * n] = conns.reshape(-1).view(np.uint8)
    inputs = {"dev": (d_in, d_conns), "host": (h_inp.at(0), h_inp.at(coff))}

    # outputs: a device Batch or the same four regions in pinned host memory
    d_out = eng.alloc_batch(n, max_frames, payload_cap)
    fb, pb, cb = 32 * max_frames, payload_cap + 16, 32 * n
    h_outp = gev_amd.PinnedArena(fb + pb + cb + 64 + 1024)
    o_pay = (fb + 255) // 256 * 256
    o_co = (o_pay + pb + 255) // 256 * 256
    o_sum = (o_co + cb + 255) // 256 * 256
    h_out = types.SimpleNamespace(frames=h_outp.at(0), payload=h_outp.at(o_pay), conn_out=h_outp.at(o_co),
                                  summary=h_outp.at(o_sum))
    outputs = {"dev": d_out, "host": h_out}
    torch.cuda.synchronize()

    def check(where_out):
        if where_out == "dev":
            got = d_out.payload[:want["total_payload"]].cpu().numpy()
        else:
            got = h_outp.host[o_pay:o_pay + want["total_payload"]]
        assert np.array_equal(got, want["payload"]), "payload differs from the oracle"

    rows = []
    for mode in ("launch", "direct"):
        eng.set_direct(mode == "direct")
        for where_in in ("dev", "host"):
            for where_out in ("dev", "host"):
                d_i, d_c = inputs[where_in]
                out = outputs[where_out]
                k_ticks, lat_ns, host_ns, ph = [], [], [], []
                t_first = None
                for r in range(args.reps + 20):
                    t0 = time.perf_counter_ns()
                    eng.decode_post(d_i, nbytes, d_c, n, out, max_frames, payload_cap)
                    t1 = time.perf_counter_ns()
                    seq = eng.completion_seq
                    while int(word[0]) != seq:
                        pass
                    t2 = time.perf_counter_ns()
                    if r >= 20:
                        k_ticks.append(int(ticks[1]) - int(ticks[0]))
                        if int(ticks[2]) and int(ticks[5]):  # GEVWS_PHASE_TICKS=1: staged/parsed/scanned/stored
                            t = [int(ticks[i]) for i in (0, 2, 3, 4, 5, 1)]
                            ph.append(tuple(t[i + 1] - t[i] for i in range(5)))
                        lat_ns.append(t2 - t0)
                        host_ns.append(t1 - t0)
                        if t_first is None:
                            t_first, tk_first = t2, int(ticks[1])
                        t_last, tk_last = t2, int(ticks[1])
                check(where_out)
                ns_per_tick = (t_last - t_first) / max(tk_last - tk_first, 1)
                rows.append({"mode": mode, "input": where_in, "outputs": where_out,
                             "kernel_us": round(statistics.median(k_ticks) * ns_per_tick / 1e3, 2),
                             "post_to_signal_us": round(statistics.median(lat_ns) / 1e3, 2),
                             "host_call_us": round(statistics.median(host_ns) / 1e3, 2),
                             "ns_per_tick": round(ns_per_tick, 3)})
                if ph:  # the kernel's phases: staged, decoded + stored, fenced + signalled
                    for i, name in enumerate(("stage_us", "parse_us", "scan_us", "store_us", "to_signal_us")):
                        rows[-1][name] = round(statistics.median(p[i] for p in ph) * ns_per_tick / 1e3, 2)
                print(json.dumps(rows[-1]), flush=True)
    eng.set_direct(False)
    eng.synchronize()
    eng.set_timeline_ticks(None)
    eng.set_completion_flag(None)
    print(json.dumps({"probe": "live_pass", "conns": n, "bytes": nbytes, "reps": args.reps, "rows": rows}))


if __name__ == "__main__":
    main()
