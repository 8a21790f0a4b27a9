#!/usr/bin/env python3
"""Turn rocprofv3 outputs (gpurun_out/prof_*) into the committed profile
summaries under profiles/:

* profiles/<tag>_kernel_stats.csv   -- rocprofv3 --kernel-trace --stats summary
* profiles/<tag>_pmc.csv            -- per-kernel mean FETCH_SIZE / WRITE_SIZE
* profiles/pmc_traffic.json         -- HBM bytes per unmask launch per config,
  read by bench.py as roofline.traffic.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in
KiB; FETCH_SIZE reports half of the bytes of a wide coalesced streaming read,
so the read side is doubled for the streaming kernel (k_unmask*); WRITE_SIZE is
exact for 16-B-per-lane streaming stores.

    python tools/pmc_traffic.py --tag r01_c3 --config c3 [--src gpurun_out]
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import shutil
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0].strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--config", required=True)
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--prefix", default="prof", help="gpurun_out/<prefix>_trace, <prefix>_pmc_* (scripts/archive/gpu_profile.sh PREFIX)")
    args = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(args.src, f"{args.prefix}_trace", "bench_kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, f"{args.tag}_kernel_stats.csv"))
    per = collections.defaultdict(dict)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        p = os.path.join(args.src, f"{args.prefix}_pmc_{c}", "bench_counter_collection.csv")
        vals = collections.defaultdict(list)
        for r in csv.DictReader(open(p)):
            vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for k, v in vals.items():
            per[k][c] = statistics.mean(v)
            per[k]["dispatches"] = len(v)
    out_csv = os.path.join(prof, f"{args.tag}_pmc.csv")
    with open(out_csv, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "dispatches", "FETCH_SIZE_KiB_mean", "WRITE_SIZE_KiB_mean",
                    "hbm_bytes_corrected"])
        for k, d in sorted(per.items()):
            fetch = d.get("FETCH_SIZE", 0.0)
            write = d.get("WRITE_SIZE", 0.0)
            corr = (2 * fetch if k.startswith("k_unmask") else fetch) * 1024 + write * 1024
            w.writerow([k, d.get("dispatches", 0), round(fetch, 1), round(write, 1), int(corr)])
    unmask = [k for k in per if k.startswith("k_unmask")]
    assert unmask, "no unmask kernel in the PMC data"
    d = per[unmask[0]]
    hbm = int((2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024)
    tj = os.path.join(prof, "pmc_traffic.json")
    table = json.load(open(tj)) if os.path.exists(tj) else {}
    table[args.config] = {"kernel": unmask[0], "hbm_bytes_per_launch": hbm,
                          "fetch_kib": d["FETCH_SIZE"], "write_kib": d["WRITE_SIZE"],
                          "correction": "read side x2 (gfx950 FETCH_SIZE halves wide streaming reads); KiB x 1024",
                          "source": f"profiles/{args.tag}_pmc.csv"}
    json.dump(table, open(tj, "w"), indent=1)
    print(json.dumps(table[args.config], indent=1))


if __name__ == "__main__":
    main()
