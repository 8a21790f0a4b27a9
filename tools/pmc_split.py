#!/usr/bin/env python3
"""Per-kernel HBM traffic from the request-size counters of
scripts/gpu_pmc_split.sh (rocprofv3 --pmc passes, gpurun_out/<prefix>_<cfg>_{rd,wr}).

gfx950's FETCH_SIZE derived counter tallies 128-byte read requests at 64 B
(it counts TCC_BUBBLE as the 128-B requests; MI355X_MICROARCH.md §HBM: "FETCH_SIZE
reports exactly 1/2 of the bytes of a wide coalesced streaming read"), so it is
calibrated only for wide streaming reads.  Counting the L2->fabric read
requests of each size directly gives the read bytes for any access pattern:

    read bytes  = 32 * TCC_EA0_RDREQ_32B + 64 * TCC_EA0_RDREQ_64B + 128 * TCC_EA0_RDREQ_128B
    write bytes = 64 * TCC_EA0_WRREQ_64B + 32 * (TCC_EA0_WRREQ - TCC_EA0_WRREQ_64B)

(all `_sum` over the TCC instances).  Prints / writes a JSON table: per kernel
the mean per dispatch of every counter and the derived bytes.

    python tools/pmc_split.py --prefix split --configs c4 c3 c5 [--out profiles/r02/r02_pmc_split.json]
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0].strip()


def read_pass(path: str):
    """kernel -> counter -> [value per dispatch]"""
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        per[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def table(src: str, prefix: str, cfg: str):
    out = {}
    merged = collections.defaultdict(dict)
    for p in ("rd", "wr"):
        f = os.path.join(src, f"{prefix}_{cfg}_{p}", "bench_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for k, cs in read_pass(f).items():
            for c, v in cs.items():
                merged[k][c] = statistics.mean(v)
                merged[k]["dispatches"] = len(v)
    for k, c in merged.items():
        g = lambda n: c.get(n + "_sum", c.get(n, 0.0))  # noqa: E731
        n32, n64, n128, nrd = g("TCC_EA0_RDREQ_32B"), g("TCC_EA0_RDREQ_64B"), g("TCC_EA0_RDREQ_128B"), g("TCC_EA0_RDREQ")
        w, w64 = g("TCC_EA0_WRREQ"), g("TCC_EA0_WRREQ_64B")
        hit, miss = g("TCC_HIT"), g("TCC_MISS")
        rd = 32 * n32 + 64 * n64 + 128 * n128
        wr = 64 * w64 + 32 * (w - w64)
        out[k] = {"dispatches": int(c.get("dispatches", 0)),
                  "rdreq": nrd, "rdreq_32B": n32, "rdreq_64B": n64, "rdreq_128B": n128,
                  "rdreq_unsized": nrd - n32 - n64 - n128,
                  "wrreq": w, "wrreq_64B": w64,
                  "read_bytes": rd, "write_bytes": wr, "hbm_bytes": rd + wr,
                  "fetch_size_equiv_bytes": (32 * n32 + 64 * (nrd - n32)),
                  "l2_hit_rate": (hit / (hit + miss)) if hit + miss else None}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--prefix", default="split")
    ap.add_argument("--configs", nargs="+", default=["c4"])
    ap.add_argument("--out", default=None)
    ap.add_argument("--traffic", action="store_true",
                    help="also record the unmask kernel's bytes per launch in profiles/pmc_traffic.json "
                         "(bench.py's roofline.traffic)")
    ap.add_argument("--source", default=None, help="profile file named as the source in pmc_traffic.json")
    ap.add_argument("--commit", default=None,
                    help="the commit the counted kernels were built from (default: this checkout's HEAD)")
    args = ap.parse_args()
    res = {cfg: table(args.src, args.prefix, cfg) for cfg in args.configs}
    if args.traffic and args.commit is None:
        import subprocess
        args.commit = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                                     text=True).stdout.strip() or None
    if args.traffic:
        tj = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        tab = json.load(open(tj)) if os.path.exists(tj) else {}
        for cfg, t in res.items():
            um = [k for k in t if k.startswith("k_unmask")]
            if not um:
                continue
            d = t[um[0]]
            tab[cfg] = {"kernel": um[0], "hbm_bytes_per_launch": int(d["read_bytes"] + d["write_bytes"]),
                        "read_bytes": int(d["read_bytes"]), "write_bytes": int(d["write_bytes"]),
                        "method": "TCC_EA0_RDREQ_{32B,64B,128B} x size + TCC_EA0_WRREQ(_64B) x size, per launch "
                                  "(exact for any access width; FETCH_SIZE tallies 128-B reads at 64 B on gfx950)",
                        "source": args.source or f"gpurun_out/{args.prefix}_{cfg}_rd,_wr",
                        "commit": args.commit}
        json.dump(tab, open(tj, "w"), indent=1)
    for cfg, t in res.items():
        print(f"== {cfg}")
        for k, d in sorted(t.items(), key=lambda kv: -kv[1]["hbm_bytes"]):
            if d["hbm_bytes"] < 1e6:
                continue
            print(f"  {k[:40]:40s} rd {d['read_bytes']/1e9:8.3f} GB (32B {d['rdreq_32B']:.3g} 64B {d['rdreq_64B']:.3g} "
                  f"128B {d['rdreq_128B']:.3g} unsized {d['rdreq_unsized']:.3g})  wr {d['write_bytes']/1e9:8.3f} GB "
                  f"(64B {d['wrreq_64B']:.3g} of {d['wrreq']:.3g})  L2 hit {d['l2_hit_rate'] if d['l2_hit_rate'] is None else round(d['l2_hit_rate'], 3)}")
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
