#!/usr/bin/env python3
"""A/B the unmask kernel variants on one workload, interleaved in one process
(cdna_hip_programming.md §5.4 rule 24), next to a device-to-device copy
ceiling of the same byte count.  Each variant is verified bit-exact first.

    python tools/ab_unmask.py [--config c3] [--rounds 5] [--reps 3] [--variants 0,1,2] [--grids 2048]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--conns", type=int, default=None)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", default="all")
    ap.add_argument("--grids", default="1024")
    ap.add_argument("--emulate-shard", default=None, metavar="R/N", help="rank R's LPT share of an N-way split")
    ap.add_argument("--walk-variants", default="0", help="header walk variants to cross with the unmask variants")
    ap.add_argument("--align-payload", action="store_true",
                    help="experiment: C3-sized frames whose payloads start 16-byte aligned in the input")
    args = ap.parse_args()

    import numpy as np
    import torch

    import gev_amd
    from gev_amd import _abi
    import bench

    dev = torch.device("cuda", 0)
    eng = gev_amd.Engine(0)
    lay, _ = bench.build_layout(args.config, 0, args.conns)
    if args.emulate_shard:  # rank R's LPT share of an N-way strong split (bench.py --emulate-shard)
        from gev_amd import workloads as w
        r, n = (int(x) for x in args.emulate_shard.split("/"))
        lay = w.shard_lpt(lay, r, n)
    if args.align_payload:
        # L = 65538 (16-byte multiple frame size with h = 14) and every stream
        # shifted by 2 bytes: payload starts land on 16-byte boundaries
        from gev_amd import workloads as w
        lay = w.uniform(16384, 64, 65538, name="aligned-payload experiment: 1M x 65538 B")
        lay.desc["hdr_off"] += np.uint64(2)
        lay.conns[:, 0] += 2
        lay.arena_bytes += 2
    arena = torch.empty(lay.arena_bytes + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    arena[lay.arena_bytes:] = 0
    desc = torch.from_numpy(lay.desc.view(np.uint8).copy()).to(dev)
    conns = torch.from_numpy(lay.conns.copy()).to(dev)
    eng.synth(arena, desc, lay.n_frames, lay.seed)
    out = eng.alloc_batch(lay.n_conns, lay.n_frames, lay.payload_padded)
    alg = lay.algorithmic_bytes()
    print(f"[ab] {lay.name}: {lay.n_frames} frames, algorithmic bytes/launch {alg}", file=sys.stderr, flush=True)

    variants = []
    i = 0
    while eng.variant_name(i) is not None:
        variants.append(i)
        i += 1
    if args.variants != "all":
        variants = [int(x) for x in args.variants.split(",")]
    grids = [int(x) for x in args.grids.split(",")]
    walks = [int(x) for x in args.walk_variants.split(",")]
    cfgs = [(v, g, wv) for v in variants for g in grids for wv in walks]

    # verify each configuration once
    for v, g, wv in cfgs:
        eng.set_tuning(_abi.TUNE_UNMASK_VARIANT, v)
        eng.set_tuning(_abi.TUNE_UNMASK_GRID, g)
        eng.set_tuning(_abi.TUNE_WALK_VARIANT, wv)
        out.payload.zero_()
        eng.decode_async(arena, lay.arena_bytes, conns, lay.n_conns, out, lay.n_frames, lay.payload_padded)
        mism = torch.zeros(1, dtype=torch.int64, device=dev)
        eng.verify(desc, lay.n_frames, lay.seed, out, mism)
        torch.cuda.synchronize()
        assert int(mism.item()) == 0, (v, g, wv, int(mism.item()))
    print("[ab] all variants verified bit-exact", file=sys.stderr, flush=True)

    n_copy = min(lay.payload_padded, lay.arena_bytes)
    src = arena[:n_copy]
    dst = out.payload[:n_copy]
    res = {c: [] for c in cfgs}
    copy_ms = []
    for r in range(args.rounds):
        # copy ceiling: same number of bytes read and written
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            dst.copy_(src)
        e1.record()
        torch.cuda.synchronize()
        copy_ms.append(e0.elapsed_time(e1) / args.reps)
        # odd rounds run the configurations in reverse order: the first one
        # after the copy-ceiling kernel measured ~1-2 % slow in every round
        for v, g, wv in (cfgs if r % 2 == 0 else cfgs[::-1]):
            eng.set_tuning(_abi.TUNE_UNMASK_VARIANT, v)
            eng.set_tuning(_abi.TUNE_UNMASK_GRID, g)
            eng.set_tuning(_abi.TUNE_WALK_VARIANT, wv)
            eng.timing()
            eng.set_timing(True)
            for _ in range(args.reps):
                eng.decode_async(arena, lay.arena_bytes, conns, lay.n_conns, out, lay.n_frames, lay.payload_padded)
            eng.set_timing(False)
            ms, calls = eng.timing()
            res[(v, g, wv)].append([x / calls for x in ms])
        print(f"[ab] round {r} done", file=sys.stderr, flush=True)

    cm = statistics.median(copy_ms)
    # same-pattern streaming copy (gevws_copy_async) from the first payload byte
    from gev_amd.workloads import header_len
    so = int(header_len(lay.desc["length"][:1], lay.desc["masked"][:1], lay.desc["len_form"][:1])[0])
    n2 = min(lay.payload_padded, lay.arena_bytes - so) // 16 * 16
    eng.copy_(out.payload, arena, n2, src_offset=so)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(args.reps):
        eng.copy_(out.payload, arena, n2, src_offset=so)
    e1.record()
    torch.cuda.synchronize()
    sm = e0.elapsed_time(e1) / args.reps
    report = {"workload": lay.name, "algorithmic_bytes": alg,
              "copy_ceiling": {"ms": round(cm, 4), "GBps_rw": round(2 * n_copy / cm / 1e6, 1)},
              "stream_copy_ceiling": {"ms": round(sm, 4), "GBps_rw": round(2 * n2 / sm / 1e6, 1)},
              "variants": []}
    for (v, g, wv), rows in res.items():
        um = [row[3] for row in rows]
        med = statistics.median(um)
        report["variants"].append({
            "variant": v, "name": eng.variant_name(v), "grid": g, "walk_variant": wv,
            "unmask_ms_median": round(med, 4), "unmask_ms_min": round(min(um), 4),
            "GBps": round(alg / med / 1e6, 1), "frac_of_8TBps": round(alg / med / 1e6 / 8000, 4),
            "walk_count_ms": round(statistics.median(row[0] for row in rows), 4),
            "walk_emit_ms": round(statistics.median(row[2] for row in rows), 4)})
    print(json.dumps(report, indent=1))


if __name__ == "__main__":
    main()
