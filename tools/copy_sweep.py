#!/usr/bin/env python3
"""Achievable HBM copy rate on this box: gevws_copy_async (the unmask kernel's
streaming loop without XOR / frame lookup) and torch's device copy, over a
grid-size sweep and two sizes, source offset 14 (unaligned, as C3) and 0.
(Round 1's round-robin "interleaved" tile mapping left the library in round
4; its numbers stay in profiles/r01/r01_copy_sweep*.json.)

    python tools/copy_sweep.py [--gib 64,2] [--grids 256,512,1024,2048] [--reps 5]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", default="64,2")
    ap.add_argument("--grids", default="256,512,1024,2048")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    import gev_amd
    eng = gev_amd.Engine(0)
    dev = torch.device("cuda", 0)
    res = []
    for gib in [float(x) for x in args.gib.split(",")]:
        n = int(gib * 2**30) // 16 * 16
        src = torch.empty(n + 64, dtype=torch.uint8, device=dev)
        dst = torch.empty(n + 64, dtype=torch.uint8, device=dev)
        src.random_(0, 255)

        def timed(fn):
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            return round(2 * n / (e0.elapsed_time(e1) / args.reps / 1e3) / 1e9, 1)

        for off in (14, 0):
            for g in [int(x) for x in args.grids.split(",")]:
                gbps = timed(lambda: eng.copy_(dst, src, n, src_offset=off, grid=g))
                res.append({"GiB": gib, "src_offset": off, "grid": g, "mapping": "contiguous", "GBps": gbps})
                print(json.dumps(res[-1]), flush=True)
        gbps = timed(lambda: dst[:n].copy_(src[:n]))
        res.append({"GiB": gib, "torch_copy": True, "GBps": gbps})
        print(json.dumps(res[-1]), flush=True)
        del src, dst
        torch.cuda.empty_cache()
    print(json.dumps({"copy_sweep": res}))


if __name__ == "__main__":
    main()
