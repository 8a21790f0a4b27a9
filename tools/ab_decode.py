#!/usr/bin/env python3
"""Interleaved A/B of decode tuning configurations on one or more workloads,
in one process (cdna_hip_programming.md §5.4 rule 24: interleave, alternate
the order every round).  Every configuration is verified bit-exact on every
workload first (decode(mask(P)) == P on every byte, frame / payload counts).

    python tools/ab_decode.py --workloads c4,c4@0/2,c4@0/4,c4@0/8 \
        --configs 'auto:SPLIT_LANES=0;off:SPLIT_LANES=1;v5:UNMASK_VARIANT=1' --rounds 4 --reps 3

A workload is a bench.py config name, optionally `@R/N` for rank R's LPT share
of an N-way strong split.  A configuration is `name:KEY=VAL,KEY=VAL` with KEY
a gev_amd._abi TUNE_* suffix; keys a configuration does not name are at their
defaults.  Prints one JSON object: per workload x configuration the median
per-phase HIP-event times (walk, scan, emit, unmask, step), the walk's split
lanes and the unmask grid.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEFAULTS = {"SPLIT_LANES": 0, "WALK_VARIANT": 0, "SPLIT_MIN_BYTES": 16384, "SPLIT_LANES_PER_CU": 512,
            "UNMASK_VARIANT": 0, "UNMASK_GRID": 0}


def parse_configs(spec: str):
    out = []
    for part in spec.split(";"):
        part = part.strip()
        if not part:
            continue
        name, _, kv = part.partition(":")
        d = {}
        for item in filter(None, kv.split(",")):
            k, v = item.split("=")
            d[k.strip().upper()] = int(v)
        out.append((name, d))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="c4")
    ap.add_argument("--configs", required=True)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None, help="also append the report as one JSON line to this file")
    ap.add_argument("--unverified", default="",
                    help="comma-separated configuration names that are timed but not verified (measurement-only "
                         "upper bounds whose bytes are wrong by construction); reported with verified: false")
    args = ap.parse_args()

    import numpy as np
    import torch

    import gev_amd
    from gev_amd import _abi
    from gev_amd import workloads as w
    import bench

    dev = torch.device("cuda", 0)
    eng = gev_amd.Engine(0)
    cfgs = parse_configs(args.configs)

    def apply(d):
        for k, dv in DEFAULTS.items():
            eng.set_tuning(getattr(_abi, "TUNE_" + k), d.get(k, dv))
        for k in d:
            if k not in DEFAULTS:
                eng.set_tuning(getattr(_abi, "TUNE_" + k), d[k])

    globals_ = {}
    report = {"rounds": args.rounds, "reps": args.reps, "workloads": []}
    for wspec in args.workloads.split(","):
        name, _, share = wspec.partition("@")
        if name not in globals_:
            globals_[name] = bench.build_layout(name, 0, None)[0]
        lay = globals_[name]
        if share:
            r, n = (int(x) for x in share.split("/"))
            lay = w.shard_lpt(lay, r, n)
        print(f"[ab] {wspec}: {lay.name}: {lay.n_frames} frames, {lay.n_conns} connections", file=sys.stderr,
              flush=True)
        arena = torch.empty(lay.arena_bytes + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
        arena[lay.arena_bytes:] = 0
        desc = torch.from_numpy(lay.desc.view(np.uint8).copy()).to(dev)
        conns = torch.from_numpy(lay.conns.copy()).to(dev)
        eng.synth(arena, desc, lay.n_frames, lay.seed)
        out = eng.alloc_batch(lay.n_conns, lay.n_frames, lay.payload_padded)

        def dec():
            eng.decode_async(arena, lay.arena_bytes, conns, lay.n_conns, out, lay.n_frames, lay.payload_padded)

        mism = torch.zeros(1, dtype=torch.int64, device=dev)
        unverified = set(filter(None, args.unverified.split(",")))
        for cname, d in cfgs:
            if cname in unverified:
                continue
            apply(d)
            for _ in range(2):  # the second decode sees the first one's history (auto choices)
                out.payload.zero_()
                dec()
                torch.cuda.synchronize()
            mism.zero_()
            eng.verify(desc, lay.n_frames, lay.seed, out, mism)
            torch.cuda.synchronize()
            s = out.summary_host()
            assert int(mism.item()) == 0 and int(s["frames"]) == lay.n_frames, (wspec, cname, int(mism.item()))
        print(f"[ab] {wspec}: every verified configuration bit-exact", file=sys.stderr, flush=True)
        res = {c: [] for c, _ in cfgs}
        info = {}
        for r in range(args.rounds):
            for cname, d in (cfgs if r % 2 == 0 else cfgs[::-1]):
                apply(d)
                dec()  # one untimed decode: the history the timed ones see
                torch.cuda.synchronize()
                eng.timing()
                eng.set_timing(True)
                for _ in range(args.reps):
                    dec()
                eng.set_timing(False)
                ms, calls = eng.timing()
                res[cname].append([x / calls for x in ms])
                info[cname] = {"split_lanes": eng.last_split_lanes, "unmask_grid": eng.last_unmask_grid}
            print(f"[ab] {wspec}: round {r} done", file=sys.stderr, flush=True)
        wrep = {"workload": wspec, "name": lay.name, "n_conns": lay.n_conns, "n_frames": lay.n_frames,
                "configs": []}
        for cname, d in cfgs:
            rows = res[cname]
            med = [statistics.median(row[k] for row in rows) for k in range(4)]
            step = statistics.median(sum(row) for row in rows)
            wrep["configs"].append({"config": cname, "tuning": d, "walk_ms": round(med[0], 4),
                                    "scan_ms": round(med[1], 4), "emit_ms": round(med[2], 4),
                                    "unmask_ms": round(med[3], 4), "step_ms": round(step, 4),
                                    "walk_ms_all": [round(row[0], 4) for row in rows], "verified": cname not in unverified,
                                    **info[cname]})
            print(f"[ab] {wspec} {cname}: walk {med[0]:.4f} emit {med[2]:.4f} unmask {med[3]:.4f} "
                  f"step {step:.4f} {info[cname]}", file=sys.stderr, flush=True)
        report["workloads"].append(wrep)
        del arena, desc, conns, out
        torch.cuda.empty_cache()
    print(json.dumps(report))
    if args.out:
        with open(args.out, "a") as f:
            f.write(json.dumps(report) + "\n")


if __name__ == "__main__":
    main()
