#!/usr/bin/env python3
"""Per-kernel PMC counter means from rocprofv3 --pmc results databases
(rocpd SQLite): each dispatch's counter values summed over their instances,
then averaged over the kernel's dispatches, with the mean duration and the
wait / issue fractions of the SQ wave cycles when those counters are present.

    python tools/pmc_sq.py gpurun_out/pmc_x/*_results.db [--out x.json] [--match encode]
"""
import argparse
import glob
import json
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"^void ", "", name)
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    return re.sub(r"\(.*$", "", n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--out", default=None)
    ap.add_argument("--match", default=None, help="only kernels whose name matches this regex")
    ap.add_argument("--source", default="", help="command line recorded in the output")
    a = ap.parse_args()
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    dur = {}
    for pat in a.dbs:
        for db in glob.glob(pat):
            cur = sqlite3.connect(db).cursor()
            for d, k, c, v, du in cur.execute(
                    "select dispatch_id, kernel_name, counter_name, value, duration from counters_collection"):
                key = (db, short(k), d)
                per[key][c] += v
                dur[key] = du
    agg = defaultdict(lambda: defaultdict(list))
    for (db, k, d), cs in per.items():
        if a.match and not re.search(a.match, k):
            continue
        for c, v in cs.items():
            agg[k][c].append(v)
        agg[k]["duration_ns"].append(dur[(db, k, d)])
    res = {}
    for k, cs in agg.items():
        r = {c: round(sum(v) / len(v), 1) for c, v in sorted(cs.items())}
        r["dispatches"] = len(cs["duration_ns"])
        wc = r.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in r:
                    r["frac_" + c[3:].lower()] = round(r[c] / wc, 3)
        res[k] = r
    out = {"source": a.source, "kernels": res}
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        open(a.out, "w").write(s + "\n")


if __name__ == "__main__":
    main()
