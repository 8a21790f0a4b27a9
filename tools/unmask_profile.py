#!/usr/bin/env python3
"""Where the v4 unmask spends its time (measurement): the profiled variant
(GEVWS_TUNE_UNMASK_VARIANT 14) stamps each workgroup's loop phases with
s_memtime, and gevws_unmask_profile returns the cycle sums.  Prints, per
workload, each phase's share of the workgroups' kernel cycles, windows and
streaming steps, frames per window, and the unprofiled kernel's time beside
the profiled one's (the stamps' own cost).

    python tools/unmask_profile.py --workloads c4,c4@0/8,c5 [--reps 3]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["kernel", "stream", "win_barrier1", "win_fill", "win_barrier2", "win_search_issue", "win_decide_next",
          "win_wait_xor_store", "windows", "windows_gt256", "window_frames", "stream_steps", "workgroups",
          "fallback_tiles", "win_load_latency"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="c4")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--variants", default="0:14", help="unprofiled:profiled unmask variant pairs, comma-separated")
    args = ap.parse_args()

    import numpy as np
    import torch

    import gev_amd
    from gev_amd import _abi, lib
    from gev_amd import workloads as w
    import bench

    dev = torch.device("cuda", 0)
    eng = gev_amd.Engine(0)
    rows = []
    for wspec in args.workloads.split(","):
        name, _, share = wspec.partition("@")
        lay = bench.build_layout(name, 0, None)[0]
        if share:
            r, n = (int(x) for x in share.split("/"))
            lay = w.shard_lpt(lay, r, n)
        arena = torch.empty(lay.arena_bytes + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
        arena[lay.arena_bytes:] = 0
        desc = torch.from_numpy(lay.desc.view(np.uint8).copy()).to(dev)
        conns = torch.from_numpy(lay.conns.copy()).to(dev)
        eng.synth(arena, desc, lay.n_frames, lay.seed)
        out = eng.alloc_batch(lay.n_conns, lay.n_frames, lay.payload_padded)

        def dec():
            eng.decode_async(arena, lay.arena_bytes, conns, lay.n_conns, out, lay.n_frames, lay.payload_padded)

        res = {}
        pairs = [tuple(int(x) for x in pv.split(":")) for pv in args.variants.split(",")]
        for variant in sorted({v for pr in pairs for v in pr}):
            eng.set_tuning(_abi.TUNE_UNMASK_VARIANT, variant)
            for _ in range(2):
                dec()
            torch.cuda.synchronize()
            mism = torch.zeros(1, dtype=torch.int64, device=dev)
            eng.verify(desc, lay.n_frames, lay.seed, out, mism)
            torch.cuda.synchronize()
            assert int(mism.item()) == 0, (wspec, variant)
            prof = (ctypes.c_uint64 * 16)()
            lib.gevws_unmask_profile(eng._ctx, prof, 1)
            eng.timing()
            eng.set_timing(True)
            for _ in range(args.reps):
                dec()
            eng.set_timing(False)
            ms, calls = eng.timing()
            lib.gevws_unmask_profile(eng._ctx, prof, 1)
            res[variant] = (ms[3] / calls, [int(x) for x in prof])
        eng.set_tuning(_abi.TUNE_UNMASK_VARIANT, 0)
        for v0, v1 in pairs:
            um0, _ = res[v0]
            um1, p = res[v1]
            k = max(p[0], 1)
            row = {"workload": wspec, "name": lay.name, "variants": [v0, v1], "unmask_ms": round(um0, 4),
                   "unmask_ms_profiled": round(um1, 4),
                   "share_of_kernel_cycles": {PHASES[i]: round(p[i] / k, 4) for i in (1, 2, 3, 4, 5, 14, 6, 7)},
                   "windows": p[8] // args.reps, "windows_gt256_frames": p[9] // args.reps,
                   "frames_per_window": round(p[10] / max(p[8], 1), 1), "stream_steps": p[11] // args.reps,
                   "workgroups": p[12] // args.reps, "fallback_tiles": p[13] // args.reps,
                   "cycles_per_window": round(sum(p[2:8]) / max(p[8], 1), 1),
                   "cycles_per_stream_step": round(p[1] / max(p[11], 1), 1)}
            print(json.dumps(row), flush=True)
            rows.append(row)
        del arena, desc, conns, out
        torch.cuda.empty_cache()
    if args.out:
        with open(args.out, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
