"""The header walk's roofline: random 128-byte line fetches.

The walk (k_walk_count) reads one ~16-byte header per frame at a data-dependent
position, so every frame costs one L2 line fetch from HBM (128 B, the request
size the TCC issues -- profiles/r02_pmc_split*.json) and one memory latency per
chain step.  gevws_gather_async runs that access pattern without the parsing:
`lanes` lanes each fetch `per_lane` 16-byte windows at random lines of a 16 GiB
buffer, either as a dependent chain (each address waits for the previous
load's data: the walk's latency structure) or 8 independent loads at a time
(the random-line fetch RATE of the memory system: the walk's throughput
ceiling).  Prints one JSON line per case: ms, line fetches per second and the
line bytes per second (128 B x fetches).

    python tools/gather_bench.py [--gib 16] [--reps 5]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--load-kinds", default="0", help="comma list: 0 plain 16 B, 1 / 2 two 8-B system / agent "
                    "scope loads (miss L2), 3 one 4-B system-scope load")
    ap.add_argument("--cases", default="", help="lanes:per_lane:dep,... (default: the C4 set)")
    args = ap.parse_args()
    import torch
    import gev_amd
    dev = torch.device("cuda", 0)
    eng = gev_amd.Engine(0)
    n = args.gib << 30
    buf = torch.empty(n + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    buf[:: 1 << 20] = 0  # touch
    # (lanes, per_lane, dependent): C4's 65 536 chains of mean length 668
    # (43.8 M frames), its 8-way share (8 192 chains; longest 1 104), and the
    # same loads issued independently
    cases = [(65536, 672, True), (65536, 672, False), (262144, 168, False), (8192, 672, True), (8192, 1104, True),
             (8192, 672, False), (131072, 336, True)]
    if args.cases:
        cases = [(int(a), int(b), bool(int(c))) for a, b, c in (x.split(":") for x in args.cases.split(","))]
    kinds = [int(k) for k in args.load_kinds.split(",")]
    cases = [c + (k,) for k in kinds for c in cases]
    sink = torch.empty(max(c[0] for c in cases), dtype=torch.int64, device=dev)
    out = []
    for lanes, per, dep, lk in cases:
        ts = []
        for r in range(args.reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eng.gather_(buf, n, lanes, per, dep, sink, seed=r + 1, load_kind=lk)
            e1.record()
            torch.cuda.synchronize()
            if r:
                ts.append(e0.elapsed_time(e1))
        ms = statistics.median(ts)
        loads = lanes * per
        rec = {"lanes": lanes, "per_lane": per, "dependent": dep, "load_kind": lk, "ms": round(ms, 4),
               "Gloads_per_s": round(loads / ms / 1e6, 2), "line_GBps": round(loads * 128 / ms / 1e6, 1),
               "us_per_step": round(ms * 1e3 / per, 3) if dep else None}
        print(json.dumps(rec), flush=True)
        out.append(rec)
    eng.close()


if __name__ == "__main__":
    main()
