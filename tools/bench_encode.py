#!/usr/bin/env python3
"""Measure the outbound encode (ws.FrameToBytes for the echo server's
NewBinaryFrame replies, benchmarks/websocket/server.go:22-29) on a decoded
batch: decode once, then time gevws_encode_batch_async with HIP events.
Algorithmic bytes per frame: read L payload + write hlen + L wire bytes.

    python tools/bench_encode.py [--config c3|c2|c4|c5] [--reps 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="0", help="encode variants to A/B, e.g. 0,1 (interleaved rounds)")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--unverified", default="", help="variants timed without the equal-bytes check "
                                                      "(measurement-only upper bounds)")
    ap.add_argument("--decode-reps", type=int, default=0,
                    help="decode the batch this many more times after the encode timing (the same "
                         "process's unmask for a kernel-trace ratio)")
    ap.add_argument("--grids", default="0", help="encode grid caps to A/B (GEVWS_TUNE_UNMASK_GRID; 0 = the default)")
    ap.add_argument("--warmup", type=int, default=3,
                    help="untimed encodes before the timed rounds (the clocks ramp back up after the host-side "
                         "set-up, profiles/r06/README.md r06o/r06p)")
    args = ap.parse_args()
    import numpy as np
    import torch

    import bench
    import gev_amd

    dev = torch.device("cuda", 0)
    eng = gev_amd.Engine(0)
    lay, _ = bench.build_layout(args.config, 0, None)
    arena = torch.empty(lay.arena_bytes + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    arena[lay.arena_bytes:] = 0
    eng.synth(arena, torch.from_numpy(lay.desc.view(np.uint8).copy()).to(dev), lay.n_frames, lay.seed)
    conns = torch.from_numpy(lay.conns.copy()).to(dev)
    out = eng.decode(arena, lay.arena_bytes, conns, lay.n_conns, lay.n_frames, lay.payload_padded)
    if not args.decode_reps:
        del arena
        torch.cuda.empty_cache()
    f = out.frames[: lay.n_frames].cpu().numpy().reshape(-1).view(gev_amd.FRAME_DTYPE)
    rep = np.zeros(lay.n_frames, gev_amd.OUT_FRAME_DTYPE)
    rep["fin"], rep["opcode"] = 1, 2
    rep["length"] = f["length"]
    rep["payload_off"], rep["payload_len"] = f["payload_off"], f["length"]
    L = rep["length"].astype(np.int64)
    hl = np.where(L <= 125, 2, np.where(L <= 0xFFFF, 4, 10))
    wire_total = int((hl + L).sum())
    alg = int(L.sum()) + wire_total
    d_rep = torch.from_numpy(rep.view(np.uint8).reshape(-1, 32).copy()).to(dev)
    wire = torch.empty(wire_total + gev_amd._abi.OUT_PAD, dtype=torch.uint8, device=dev)
    off = torch.empty(lay.n_frames, dtype=torch.int64, device=dev)
    summ = torch.zeros(64, dtype=torch.uint8, device=dev)
    eng.encode_async(d_rep, lay.n_frames, out.payload, wire, wire_total, off, summ)
    torch.cuda.synchronize()
    s = summ.cpu().numpy().view(gev_amd.SUMMARY_DTYPE)[0]
    assert int(s["status"]) == 0 and int(s["payload_bytes"]) == wire_total
    # spot check frame 0 and the last frame against the decoded payloads
    for g in (0, lay.n_frames - 1):
        o = int(off[g].item())
        h = 2 if L[g] <= 125 else (4 if L[g] <= 0xFFFF else 10)
        po = int(rep["payload_off"][g])
        assert torch.equal(wire[o + h:o + h + int(L[g])], out.payload[po:po + int(L[g])])
    variants = [int(x) for x in args.variants.split(",")]
    if len(variants) > 1:
        # every variant's whole wire equals the first one's
        ref_wire = wire.clone()
        unverified = {int(x) for x in filter(None, args.unverified.split(","))}
        for v in variants[1:]:
            if v in unverified:
                continue
            eng.set_tuning(gev_amd._abi.TUNE_ENCODE_VARIANT, v)
            eng.encode_async(d_rep, lay.n_frames, out.payload, wire, wire_total, off, summ)
            torch.cuda.synchronize()
            assert torch.equal(wire[:wire_total], ref_wire[:wire_total]), f"encode variant {v} differs"
        del ref_wire
        torch.cuda.empty_cache()
    grids = [int(x) for x in args.grids.split(",")]
    cfgs = [(v, g) for v in variants for g in grids]
    for _ in range(args.warmup):
        eng.encode_async(d_rep, lay.n_frames, out.payload, wire, wire_total, off, summ)
    torch.cuda.synchronize()
    times = {c: [] for c in cfgs}
    for rnd in range(args.rounds):
        for v, g in (cfgs if rnd % 2 == 0 else cfgs[::-1]):  # alternate the order (position bias)
            eng.set_tuning(gev_amd._abi.TUNE_ENCODE_VARIANT, v)
            eng.set_tuning(gev_amd._abi.TUNE_UNMASK_GRID, g)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                eng.encode_async(d_rep, lay.n_frames, out.payload, wire, wire_total, off, summ)
            e1.record()
            torch.cuda.synchronize()
            times[(v, g)].append(e0.elapsed_time(e1) / args.reps)
    eng.set_tuning(gev_amd._abi.TUNE_ENCODE_VARIANT, 0)
    eng.set_tuning(gev_amd._abi.TUNE_UNMASK_GRID, 0)
    for _ in range(args.decode_reps):  # (rewrites the same payload bytes)
        eng.decode_async(arena, lay.arena_bytes, conns, lay.n_conns, out, lay.n_frames, lay.payload_padded)
    torch.cuda.synchronize()
    for v, g in cfgs:
        ms = sorted(times[(v, g)])[len(times[(v, g)]) // 2]
        print(json.dumps({"path": "encode (FrameToBytes of NewBinaryFrame replies)", "variant": v, "grid": g,
                          "workload": lay.name, "frames": lay.n_frames, "wire_bytes": wire_total,
                          "ms": round(ms, 4), "rounds_ms": [round(t, 4) for t in times[(v, g)]],
                          "warmup": args.warmup,
                          "payload_GiBps": round(int(L.sum()) / (ms / 1e3) / 2**30, 2),
                          "frames_per_s": round(lay.n_frames / ms * 1e3, 1),
                          "algorithmic_GBps": round(alg / ms / 1e6, 1),
                          "frac_of_8TBps": round(alg / ms / 1e6 / 8000, 4)}))


if __name__ == "__main__":
    main()
