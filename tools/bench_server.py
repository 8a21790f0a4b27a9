#!/usr/bin/env python3
"""Device-resident websocket server step: decode the client frames of a batch
(UnPacket), dispatch them as HandlerWrap.OnMessage would with an echo handler
(wrap.go:38-90; control frames answered per util.go), and encode the replies
(FrameToBytes) -- timed with HIP events, all on one stream, nothing on the host
in the timed region.

C1-shaped workload (benchmarks/bench-websocket-pingpong.sh sends masked
128 B text frames; the server echoes binary, benchmarks/websocket/server.go:25):
--config c1 = 65 536 connections x 16 frames x 128 B.  --config c5 = fragmented
text + ping/pong.

    python tools/bench_server.py [--config c1|c5|c2|c3] [--reps 10]
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
    ap.add_argument("--config", default="c1")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="",
                    help="A/B: comma list of wW.eE (header walk variant W, encode variant E), interleaved rounds, "
                         "with per-stage times")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import numpy as np
    import torch

    import bench
    import gev_amd
    from gev_amd import workloads as w

    dev = torch.device("cuda", 0)
    eng = gev_amd.Engine(0)
    if args.config == "c1":
        lay = w.uniform(65536, 16, 128, opcode=0x1, name="C1-shaped: 1048576 x 128 B masked text frames")
    else:
        lay, _ = bench.build_layout(args.config, 0, None)
    arena = torch.empty(lay.arena_bytes + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    arena[lay.arena_bytes:] = 0
    eng.synth(arena, torch.from_numpy(lay.desc.view(np.uint8).copy()).to(dev), lay.n_frames, lay.seed)
    conns = torch.from_numpy(lay.conns.copy()).to(dev)
    n = lay.n_frames
    aux_slots = int((lay.desc["b0"] & 0x0F == 0x8).sum())
    out = eng.alloc_batch(lay.n_conns, n, lay.payload_padded, aux_slots=aux_slots)
    aux_off = (lay.payload_padded + 127) // 128 * 128
    aux_cap = out.payload.numel() - 16 - aux_off
    replies = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    reply_of = torch.empty(n, dtype=torch.int64, device=dev)
    dsum = torch.zeros(64, dtype=torch.uint8, device=dev)
    wire_cap = lay.payload_len + 14 * n
    wire = torch.empty(wire_cap + gev_amd._abi.OUT_PAD, dtype=torch.uint8, device=dev)
    off = torch.empty(n, dtype=torch.int64, device=dev)
    esum = torch.zeros(64, dtype=torch.uint8, device=dev)

    def step():
        eng.decode_async(arena, lay.arena_bytes, conns, lay.n_conns, out, n, lay.payload_padded)
        eng.dispatch_async(out.frames, n, gev_amd._abi.HANDLER_ECHO_BINARY, out.payload, aux_off, aux_cap,
                           replies, reply_of, dsum)
        # every frame of these workloads gets a reply (data echo, pong/ping), so
        # the reply count is n and no host round trip is needed between stages
        eng.encode_async(replies, n, out.payload, wire, wire_cap, off, esum)

    step()
    torch.cuda.synchronize()
    ds = dsum.cpu().numpy().view(gev_amd.SUMMARY_DTYPE)[0]
    es = esum.cpu().numpy().view(gev_amd.SUMMARY_DTYPE)[0]
    assert int(ds["frames"]) == n, "every frame is expected to produce one reply in this workload"
    assert int(es["status"]) == 0
    # check: decode the reply stream back; payload arenas match
    wire_total = int(es["payload_bytes"])
    if n <= 400000:
        # decode the whole reply stream back as one connection, followed by 5
        # bytes of an incomplete 127-form header so even 2-5-byte replies have
        # >= 6 bytes behind them (read.go:20-23); the payload arenas must match
        w2 = torch.zeros(wire_total + 5 + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
        w2[:wire_total] = wire[:wire_total]
        w2[wire_total:wire_total + 5] = torch.tensor([0x82, 0x7F, 0, 0, 0], dtype=torch.uint8, device=dev)
        rc = torch.tensor([[0, wire_total + 5]], dtype=torch.int64, device=dev)
        back = eng.decode(w2, wire_total + 5, rc, 1, n, lay.payload_padded)
        assert int(back.summary_host()["frames"]) == n
        ok = torch.equal(back.payload[: lay.payload_padded], out.payload[: lay.payload_padded])
        assert ok, "reply stream does not decode back to the request payloads"
        del w2, back
    else:
        # HBM holds one more copy at most: spot-check 512 replies' payload bytes
        rng = np.random.default_rng(0)
        fr = out.frames[:n].cpu().numpy().reshape(-1).view(gev_amd.FRAME_DTYPE)
        offs = off.cpu().numpy()
        for g in rng.integers(0, n, 512):
            L = int(fr["length"][g])
            h = 2 if L <= 125 else (4 if L <= 0xFFFF else 10)
            o, po = int(offs[g]), int(fr["payload_off"][g])
            assert torch.equal(wire[o + h:o + h + L], out.payload[po:po + L])
    if args.variants:
        # interleaved A/B with per-stage event times (decode, dispatch, encode)
        from gev_amd import _abi
        combos = [tuple(int(x[1:]) for x in v.split(".")) for v in args.variants.split(",")]
        res = {c: [] for c in combos}
        for _ in range(args.rounds):
            for c in combos:
                eng.set_tuning(_abi.TUNE_WALK_VARIANT, c[0])
                eng.set_tuning(_abi.TUNE_ENCODE_VARIANT, c[1])
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                acc = [0.0, 0.0, 0.0]
                for _r in range(args.reps):
                    ev[0].record()
                    eng.decode_async(arena, lay.arena_bytes, conns, lay.n_conns, out, n, lay.payload_padded)
                    ev[1].record()
                    eng.dispatch_async(out.frames, n, gev_amd._abi.HANDLER_ECHO_BINARY, out.payload, aux_off,
                                       aux_cap, replies, reply_of, dsum)
                    ev[2].record()
                    eng.encode_async(replies, n, out.payload, wire, wire_cap, off, esum)
                    ev[3].record()
                    torch.cuda.synchronize()
                    for k in range(3):
                        acc[k] += ev[k].elapsed_time(ev[k + 1])
                res[c].append([a / args.reps for a in acc])
        eng.set_tuning(_abi.TUNE_WALK_VARIANT, 0)
        eng.set_tuning(_abi.TUNE_ENCODE_VARIANT, 0)
        for c, rows in res.items():
            med = [sorted(r[k] for r in rows)[len(rows) // 2] for k in range(3)]
            print(json.dumps({"workload": lay.name, "walk_variant": c[0], "encode_variant": c[1],
                              "decode_ms": round(med[0], 4), "dispatch_ms": round(med[1], 4),
                              "encode_ms": round(med[2], 4), "sum_ms": round(sum(med), 4)}))
        return
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        step()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.reps
    print(json.dumps({"path": "device server step: decode + dispatch(echo) + encode", "workload": lay.name,
                      "frames": n, "connections": lay.n_conns, "ms": round(ms, 4),
                      "frames_per_s": round(n / ms * 1e3, 1),
                      "payload_GiBps": round(lay.payload_len / (ms / 1e3) / 2**30, 2),
                      "wire_out_bytes": wire_total,
                      "check": "reply stream decoded back" if n <= 400000 else "512 replies spot-checked"}))


if __name__ == "__main__":
    main()
