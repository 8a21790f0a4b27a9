#!/usr/bin/env python3
"""Copy rate with a misaligned DESTINATION (measurement for the encode's
scatter layout): aligned 16-byte loads, 16-byte stores at dst offset
0 / 7 / 14, plain vs non-temporal stores, over one size, interleaved rounds.

    python tools/copy_dst_align.py [--gib 16] [--reps 5] [--rounds 3]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=16)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch

    import gev_amd
    eng = gev_amd.Engine(0)
    dev = torch.device("cuda", 0)
    n = int(args.gib * 2**30) // 16 * 16
    src = torch.empty(n + 64, dtype=torch.uint8, device=dev)
    dst = torch.empty(n + 64, dtype=torch.uint8, device=dev)
    src.random_(0, 255)
    cases = [("nt_store_dst0", 0, 0), ("plain_store_dst0", 0, 0x10000000),
             ("plain_store_dst7", 7, 0x10000000), ("plain_store_dst14", 14, 0x10000000),
             ("nt_store_dst7", 7, 0x08000000), ("nt_store_dst14", 14, 0x08000000)]
    res = {c[0]: [] for c in cases}
    for r in range(args.rounds):
        for name, off, flag in (cases if r % 2 == 0 else cases[::-1]):
            fn = lambda: eng.copy_(dst, src, n, dst_offset=off, grid=flag)  # noqa: E731
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(2 * n / (e0.elapsed_time(e1) / args.reps / 1e3) / 1e9)
    # correctness of the misaligned stores: the copied bytes equal the source
    eng.copy_(dst, src, n, dst_offset=7, grid=0x10000000)
    torch.cuda.synchronize()
    ok = bool(torch.equal(dst[7:7 + n], src[:n]))
    out = {"copy_dst_alignment": {k: round(statistics.median(v), 1) for k, v in res.items()},
           "GiB": args.gib, "unit": "GB/s (read + write)", "bytes_equal_at_dst7": ok}
    print(json.dumps(out))
    if args.out:
        with open(args.out, "a") as f:
            f.write(json.dumps(out) + "\n")


if __name__ == "__main__":
    main()
