#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 results database (rocpd SQLite, what
rocprofv3 writes when no CSV output is asked for): name, calls, mean / min /
max / total duration, in the order of total time.  Optionally the sequence of
kernels matching a pattern (to attribute phases of an A/B run).

    python tools/prof_db.py gpurun_out/prof_x/x_results.db [--csv out.csv] [--seq walk]
"""
import argparse
import re
import sqlite3
import statistics
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"^void ", "", name)
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    return re.sub(r"\((const|unsigned|int|long|char|float|double|gevws|void|bool|u|st|ui)[^()]*\)$", "", n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default=None)
    ap.add_argument("--seq", default=None, help="print the launch sequence of kernels matching this regex")
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = list(cur.execute("select name, start, end from kernels order by start"))
    agg = defaultdict(list)
    for n, s, e in rows:
        agg[short(n)].append((e - s) / 1e3)
    out = []
    for n, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
        out.append((n, len(v), statistics.mean(v), min(v), max(v), sum(v)))
    for n, c, m, lo, hi, t in out[:40]:
        print(f"{c:5d} mean {m:10.2f} us  min {lo:10.2f}  max {hi:10.2f}  total {t / 1e3:9.3f} ms  {n[:110]}")
    if a.csv:
        with open(a.csv, "w") as f:
            f.write("Name,Calls,AverageNs,MinNs,MaxNs,TotalNs\n")
            for n, c, m, lo, hi, t in out:
                f.write(f"\"{n}\",{c},{m * 1e3:.0f},{lo * 1e3:.0f},{hi * 1e3:.0f},{t * 1e3:.0f}\n")
    if a.seq:
        pat = re.compile(a.seq)
        for n, s, e in rows:
            sn = short(n)
            if pat.search(sn):
                print(f"{(e - s) / 1e3:10.2f} us  {sn[:120]}")


if __name__ == "__main__":
    main()
