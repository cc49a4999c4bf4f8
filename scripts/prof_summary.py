#!/usr/bin/env python3
"""Per-kernel summary (calls, total, average, share) of a rocprofv3 --kernel-trace run, from either
its kernel_stats.csv (--output-format csv) or its rocpd SQLite database (ROCm 7.2 default)."""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                     "from kernels group by name order by 3 desc").fetchall()
    return [(r[0], r[1], r[2], r[3], r[4], r[5]) for r in rows]


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
                        float(r["MinNs"]), float(r["MaxNs"])))
    return out


def main(d, out=None):
    csvs = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    rows = from_csv(csvs[0]) if csvs else from_db(dbs[0])
    tot = sum(r[2] for r in rows)
    lines = [f"# rocprofv3 --kernel-trace --stats summary ({csvs[0] if csvs else dbs[0]})",
             f"# total kernel time {tot / 1e6:.3f} ms",
             "share%,calls,total_ms,avg_us,min_us,max_us,kernel"]
    for n, k, t, a, mn, mx in rows:
        short = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        lines.append(f"{100 * t / tot:.2f},{k},{t / 1e6:.4f},{a / 1e3:.2f},{mn / 1e3:.2f},{mx / 1e3:.2f},{short}")
    txt = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
