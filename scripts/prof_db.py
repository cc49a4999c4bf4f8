#!/usr/bin/env python3
"""Kernel summary of a rocprofv3 --kernel-trace database (rocpd sqlite, the default output format):
per kernel name total ms, dispatches, mean us -- the rocprofv3 --stats table. Usage: prof_db.py <dir|db> [n]"""
import glob
import os
import sqlite3
import sys


def summary(path):
    dbs = [path] if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    rows = {}
    for db in dbs:
        c = sqlite3.connect(db)
        for name, n, tot in c.execute("select name, count(*), sum(duration) from kernels group by name"):
            r = rows.setdefault(name, [0, 0.0])
            r[0] += n
            r[1] += tot
    return sorted(((v[1] / 1e6, v[0], v[1] / v[0] / 1e3, k) for k, v in rows.items()), reverse=True)


if __name__ == "__main__":
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    s = summary(sys.argv[1])
    for ms, cnt, us, name in s[:n]:
        print(f"{ms:9.2f} ms {cnt:6d} x {us:8.1f} us  {name[:100]}")
    print("total ms", sum(r[0] for r in s))
